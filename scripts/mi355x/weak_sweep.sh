#!/bin/bash
# Weak-scaling sweep on one MI355X node: Jacobi3D 512^3 per GPU (bench.py) and the reference's exchange-only
# weak driver (radius 3, 4 quantities) at 1/2/4/8 GPUs, one process per GPU.
# Mirrors reference scripts/summit/weak_256n.sh / scripts/hal/run_weak_*.sb. Usage: weak_sweep.sh [per_gpu] [gpus...]
set -o pipefail
cd "$(dirname "$0")/../.."
PER=${1:-512}; shift || true
NS=${*:-1 2 4 8}
export STENCIL_PLAN_FILE=0
mkdir -p gpurun_out/weak
for n in $NS; do
  if [ "$n" = 1 ]; then
    timeout -k 10 600 python bench.py --gpus 1 --per-gpu $PER | tee gpurun_out/weak/jacobi_$n.json || exit 1
  else
    timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
      --master-port $((29500 + n)) bench.py --gpus $n --per-gpu $PER | tee gpurun_out/weak/jacobi_$n.json || exit 1
  fi
  timeout -k 10 600 python -m stencil2_amd.launch -n $n build/bin/weak $PER $PER $PER 30 | tee gpurun_out/weak/exchange_$n.csv || exit 1
done
