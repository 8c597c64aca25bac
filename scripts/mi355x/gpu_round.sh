#!/bin/bash
# Full round check on one MI355X: native ctest, pytest -m gpu, smoke, bench, rocprofv3 kernel stats.
# Each GPU step has its own time limit; the script stops at the first failure.
set -o pipefail
export STENCIL_SKIP_BUILD=1 STENCIL_PLAN_FILE=0 PYTHONPATH=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
step() { local name=$1 lim=$2; shift 2; echo "== $name"; timeout -k 10 $lim "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -5 gpurun_out/$name.log; return $rc; }
step ctest 180 ./build/bin/stencil_ctest --all &&
step pytest_gpu 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider &&
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" &&
step bench1 300 python bench.py --steps 50 --warmup 5 &&
{ cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/prof;
  step prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 20 --warmup 2 --exchange-iters 5; }
echo "done rc=$?"
