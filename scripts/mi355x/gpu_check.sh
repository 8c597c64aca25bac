#!/bin/bash
# Full check on one MI355X: native ctest, pytest -m gpu, smoke, exchange probe, bench, rocprofv3 kernel stats.
# Every GPU step has its own time limit; the script stops at the first failure. OUT=<dir under gpurun_out>.
set -o pipefail
export STENCIL_SKIP_BUILD=1 STENCIL_PLAN_FILE=0 PYTHONPATH=$GRAFT_REPO_ROOT STENCIL_WAIT_TIMEOUT=30
O=gpurun_out/${OUT:-check}
mkdir -p $O
step() { local name=$1 lim=$2; shift 2; echo "== $name"; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -${TAILN:-3} $O/$name.log; return $rc; }
step ctest 180 ./build/bin/stencil_ctest --all &&
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider &&
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" &&
TAILN=6 step xchg 120 ./build/bin/bench_stencil --only xchg &&
step bench1 300 python bench.py --steps 64 --warmup 16 &&
{ cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT;
  step prof 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --steps 32 --warmup 4 --exchange-iters 5; }
echo "done rc=$?"
