#!/bin/bash
set -o pipefail
export STENCIL_SKIP_BUILD=1 STENCIL_PLAN_FILE=0 PYTHONPATH=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
step() { local name=$1 lim=$2; shift 2; echo "== $name"; timeout -k 10 $lim "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; grep -v amdgpu.ids gpurun_out/$name.log | tail -${TAILN:-3} | cut -c1-300; return $rc; }
TAILN=8 step pytest_x2 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider -k "temporal2" &&
TAILN=20 step x2sweep 200 ./build/bin/bench_stencil --only x2 &&
step bench_t2 300 python bench.py --steps 64 --warmup 16
echo "done rc=$?"
