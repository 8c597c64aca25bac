#!/bin/bash
# Halo-exchange GB/s (reference bin/bench_exchange.cu, 5 radius patterns) for a 1024^3 global grid at 1/2/4/8 GPUs
# (512^3 per GPU at 8) and the astaroth proxy (8 quantities, radius 3, 26 directions).
set -o pipefail
cd "$(dirname "$0")/../.."
NS=${*:-1 2 4 8}
export STENCIL_PLAN_FILE=0
mkdir -p gpurun_out/bx
for n in $NS; do
  timeout -k 10 600 python -m stencil2_amd.launch -n $n build/bin/bench_exchange --x 1024 --y 1024 --z 1024 --fr 2 | tee gpurun_out/bx/bench_exchange_$n.csv || exit 1
  timeout -k 10 600 python -m stencil2_amd.launch -n $n build/bin/astaroth_sim --x 1024 --y 1024 --z 1024 --q 8 | tee gpurun_out/bx/astaroth_$n.csv || exit 1
done
