#!/bin/bash
# correctness (ctest + pytest -m gpu), kernel sweep, bench
set -o pipefail
export STENCIL_SKIP_BUILD=1 STENCIL_PLAN_FILE=0 PYTHONPATH=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
step() { local name=$1 lim=$2; shift 2; echo "== $name"; timeout -k 10 $lim "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; grep -v amdgpu.ids gpurun_out/$name.log | tail -${TAILN:-3} | cut -c1-600; return $rc; }
step ctest 180 ./build/bin/stencil_ctest --all &&
step pytest_gpu 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider &&
TAILN=40 step sweep 300 ./build/bin/bench_stencil --only lds &&
TAILN=8 step xchg 100 ./build/bin/bench_stencil --only xchg &&
step bench 300 python bench.py --steps 50 --warmup 5
echo "done rc=$?"
