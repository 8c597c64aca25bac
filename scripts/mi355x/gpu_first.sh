#!/bin/bash
# first GPU bring-up: native ctest (GPU cases), smoke, short bench
set -o pipefail
export STENCIL_SKIP_BUILD=1 STENCIL_PLAN_FILE=0 PYTHONPATH=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 120 ./build/bin/stencil_ctest --all > gpurun_out/ctest.log 2>&1; echo "ctest rc=$?" >> gpurun_out/ctest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/bench1.log 2>&1
echo "done rc=$?"
