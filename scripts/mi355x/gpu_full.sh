#!/bin/bash
# full GPU validation: native ctest, pytest -m gpu, smoke, bench (x2), multi-rank rehearsal on one GPU
set -o pipefail
export STENCIL_SKIP_BUILD=1 STENCIL_PLAN_FILE=0 PYTHONPATH=$GRAFT_REPO_ROOT
mkdir -p gpurun_out/full
step() { local name=$1 lim=$2; shift 2; echo "== $name"; timeout -k 10 $lim "$@" > gpurun_out/full/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; grep -v amdgpu.ids gpurun_out/full/$name.log | tail -${TAILN:-3} | cut -c1-600; return $rc; }
step ctest 180 ./build/bin/stencil_ctest --all &&
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread &&
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" &&
step bench_a 300 python bench.py --steps 64 --warmup 16 &&
step bench_b 300 python bench.py --steps 64 --warmup 16 &&
TAILN=12 step rehearse 700 bash scripts/mi355x/rehearse_mp.sh
echo "done rc=$?"
