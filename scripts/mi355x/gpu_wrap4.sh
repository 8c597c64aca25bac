#!/bin/bash
# ragged-x in-kernel wrap (WRAP 3): correctness subset, ladder shapes, bench
set -o pipefail
export STENCIL_SKIP_BUILD=1 STENCIL_PLAN_FILE=0 PYTHONPATH=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
step() { local name=$1 lim=$2; shift 2; echo "== $name"; timeout -k 10 $lim "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -4 gpurun_out/$name.log | cut -c1-300; return $rc; }
step w4_tests 300 python -u -m pytest tests/test_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "in_kernel_wrap or temporal2 or prepare" &&
step w4_shapes 300 python scripts/mi355x/shape_sweep.py --steps 32 &&
STENCIL_WRAP_AXES=6 step w4_shapes_nox 300 python scripts/mi355x/shape_sweep.py --steps 32 --shapes 645x323x645,813x407x407 &&
step w4_bench 200 python bench.py --steps 64 --warmup 16
echo "done rc=$?"
