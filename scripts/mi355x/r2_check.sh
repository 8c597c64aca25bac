#!/bin/bash
# round-2 GPU check: native ctest, GPU pytest, smoke, 1-GPU bench, kernel-trace profile of the bench
set -o pipefail
export STENCIL_SKIP_BUILD=1 STENCIL_PLAN_FILE=0 PYTHONPATH=$GRAFT_REPO_ROOT
D=gpurun_out/${R2TAG:-r2check}; mkdir -p $D
step() { local name=$1 lim=$2; shift 2; echo "== $name"; timeout -k 10 $lim "$@" > $D/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -3 $D/$name.log | cut -c1-700; return $rc; }
step ctest 180 ./build/bin/stencil_ctest --all &&
step pytest_gpu 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread &&
step smoke 200 python -c "import __graft_entry__ as g; g.smoke()" &&
step bench_a 200 python bench.py &&
step bench_b 200 python bench.py --steps 64 --warmup 16 &&
{ cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT;
  step prof 300 rocprofv3 --kernel-trace --stats -d $D/prof -o run --output-format csv -- python3 bench.py --steps 20 --warmup 2; }
echo "done rc=$?"
