#!/bin/bash
# round-2 baseline: 1-GPU bench twice + kernel stats of the bench
set -o pipefail
export STENCIL_SKIP_BUILD=1 STENCIL_PLAN_FILE=0 PYTHONPATH=$GRAFT_REPO_ROOT
mkdir -p gpurun_out/r2base
step() { local name=$1 lim=$2; shift 2; echo "== $name"; timeout -k 10 $lim "$@" > gpurun_out/r2base/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -3 gpurun_out/r2base/$name.log | cut -c1-600; return $rc; }
step bench_a 200 python bench.py &&
step bench_b 200 python bench.py --steps 64 --warmup 16 &&
{ cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT;
  step prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r2base/prof -o run --output-format csv -- python3 bench.py --steps 20 --warmup 2 --exchange-iters 5; } &&
head -20 gpurun_out/r2base/prof/run_kernel_stats.csv | cut -c1-200
echo "done rc=$?"
