#!/bin/bash
# CPU test job: native unit tests (host backend) + pytest without the GPU marker (multi-process over TCP ranks).
# Reference: ci/test.sh (never wired into .travis.yml); here it is the CI gate.
set -euo pipefail
cd "$(dirname "$0")/.."
./build/bin/stencil_ctest --cpu
python -m pytest tests -q -m "not gpu"
