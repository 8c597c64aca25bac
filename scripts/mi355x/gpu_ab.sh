#!/bin/bash
# same-box A/B of the fused-pair work split: tests, x2pp sweep, bench with x2sched 1 / 0 (twice, interleaved)
set -o pipefail
export STENCIL_SKIP_BUILD=1 STENCIL_PLAN_FILE=0 PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/${OUT:-ab}; mkdir -p $O
step() { local name=$1 lim=$2; shift 2; echo "== $name"; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -${TAILN:-2} $O/$name.log; return $rc; }
step t2 300 python -u -m pytest tests/test_gpu.py -x -q -k "temporal2" --timeout 120 --timeout-method thread -p no:cacheprovider || exit 1
TAILN=30 step x2pp 300 ./build/bin/bench_stencil --only x2pp || exit 1
for r in 1 2; do for sc in 1 0; do
  step bench_s${sc}_$r 300 python bench.py --steps 64 --warmup 16 --x2sched $sc || exit 1
  grep -o '"value": [0-9.]*' $O/bench_s${sc}_$r.log
done; done
echo done
