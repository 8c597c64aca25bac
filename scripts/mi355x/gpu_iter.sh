#!/bin/bash
# one iteration on the GPU: selected GPU tests (PYTEST_K), kernel sweep (SWEEP, bench_stencil --only), bench
set -o pipefail
export STENCIL_SKIP_BUILD=1 STENCIL_PLAN_FILE=0 PYTHONPATH=$GRAFT_REPO_ROOT
mkdir -p gpurun_out/iter
step() { local name=$1 lim=$2; shift 2; echo "== $name"; timeout -k 10 $lim "$@" > gpurun_out/iter/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; grep -v amdgpu.ids gpurun_out/iter/$name.log | tail -${TAILN:-4} | cut -c1-400; return $rc; }
step pytest 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "${PYTEST_K:-temporal or special}" &&
for s in ${SWEEP:-x2 x2pp}; do TAILN=40 step sweep_$s 200 ./build/bin/bench_stencil --only $s || exit 1; done &&
step bench 300 python bench.py --steps 64 --warmup 16
echo "done rc=$?"
