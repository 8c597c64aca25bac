#!/bin/bash
# iteration loop: correctness, tuning sweep, bench, kernel profile
export STENCIL_SKIP_BUILD=1 STENCIL_PLAN_FILE=0 PYTHONPATH=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 120 ./build/bin/stencil_ctest --all > gpurun_out/ctest.log 2>&1 || { echo "ctest failed"; tail gpurun_out/ctest.log; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo smoke failed; tail gpurun_out/smoke.log; exit 1; }
timeout -k 10 600 python scripts/mi355x/tune_jacobi.py 512 > gpurun_out/tune.log 2>&1 || { echo tune failed; tail gpurun_out/tune.log; exit 1; }
timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/bench1.log 2>&1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --exchange-iters 5 > gpurun_out/prof/bench.log 2>&1
echo "done rc=$?"
