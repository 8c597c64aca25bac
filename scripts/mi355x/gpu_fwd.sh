#!/bin/bash
# halo forwarding: GPU tests, then bench with/without forwarding (interleaved)
set -o pipefail
export STENCIL_SKIP_BUILD=1 STENCIL_PLAN_FILE=0 PYTHONPATH=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
step() { local name=$1 lim=$2; shift 2; echo "== $name"; timeout -k 10 $lim "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; grep -v amdgpu.ids gpurun_out/$name.log | tail -3 | cut -c1-400; return $rc; }
step pytest_gpu 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider -k "forwarding or jacobi or astaroth or smoke" &&
step bench_fwd 300 python bench.py --steps 50 --warmup 5 &&
STENCIL_NO_FORWARD=1 step bench_nofwd 300 python bench.py --steps 50 --warmup 5 &&
step bench_fwd2 300 python bench.py --steps 50 --warmup 5 &&
STENCIL_NO_FORWARD=1 step bench_nofwd2 300 python bench.py --steps 50 --warmup 5
echo "done rc=$?"
