#!/bin/bash
# CI build (no GPU needed: hipcc cross-compiles gfx950). Reference: ci/build.sh (Travis, build only).
set -euo pipefail
cd "$(dirname "$0")/.."
python -c "import __graft_entry__ as g; g.build()"
ls build/bin
