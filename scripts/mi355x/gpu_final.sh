#!/bin/bash
# round check: full GPU suite, smoke, 1-GPU bench (x2), ladder shapes, multi-rank bench rehearsal on one GPU
set -o pipefail
export STENCIL_SKIP_BUILD=1 STENCIL_PLAN_FILE=0 PYTHONPATH=$GRAFT_REPO_ROOT
mkdir -p gpurun_out/mp
step() { local name=$1 lim=$2; shift 2; echo "== $name"; timeout -k 10 $lim "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -3 gpurun_out/$name.log | cut -c1-400; return $rc; }
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread &&
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" &&
step bench_a 200 python bench.py &&
step bench_b 200 python bench.py --steps 64 --warmup 16 &&
step shapes 300 python scripts/mi355x/shape_sweep.py --steps 32 &&
for n in 2 4; do
  STENCIL_WAIT_TIMEOUT=30 step rehearse_$n 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29600+n)) bench.py --gpus $n --steps 32 --warmup 8 --per-gpu 256 || exit 1
done
echo "done rc=$?"
