#!/bin/bash
# In-kernel periodic wrap of the fused pairs: targeted tests, bench wrap on/off, per-GPU shapes of the ladder,
# then the whole GPU suite. Each GPU step has its own time limit; stops at the first failure.
set -o pipefail
export STENCIL_SKIP_BUILD=1 STENCIL_PLAN_FILE=0 PYTHONPATH=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
step() { local name=$1 lim=$2; shift 2; echo "== $name"; timeout -k 10 $lim "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -4 gpurun_out/$name.log; return $rc; }
step wrap_tests 300 python -u -m pytest tests/test_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "in_kernel_wrap or temporal2" &&
step bench_wrap1 200 python bench.py --steps 64 --warmup 16 &&
step bench_wrap0 200 python bench.py --steps 64 --warmup 16 --wrap 0 &&
step bench_wrap1b 200 python bench.py --steps 64 --warmup 16 &&
step shapes 300 python scripts/mi355x/shape_sweep.py --steps 32 &&
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
echo "done rc=$?"
