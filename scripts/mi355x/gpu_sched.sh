#!/bin/bash
# fused-pair work split A/B (balanced segments vs fixed z-chunks): temporal tests, x2pp sweep, bench, kernel trace
set -o pipefail
export STENCIL_SKIP_BUILD=1 STENCIL_PLAN_FILE=0 PYTHONPATH=$GRAFT_REPO_ROOT
mkdir -p gpurun_out/sched
step() { local name=$1 lim=$2; shift 2; echo "== $name"; timeout -k 10 $lim "$@" > gpurun_out/sched/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -4 gpurun_out/sched/$name.log; return $rc; }
step t2 300 python -u -m pytest tests/test_gpu.py -x -q -k "temporal2" --timeout 120 --timeout-method thread -p no:cacheprovider &&
step x2pp 300 ./build/bin/bench_stencil --only x2pp &&
step bench 300 python bench.py --steps 64 --warmup 16 &&
{ cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT;
  step prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/sched/prof -o run --output-format csv -- python3 bench.py --steps 32 --warmup 4 --exchange-iters 5; }
echo "done rc=$?"
