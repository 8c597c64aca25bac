#!/bin/bash
# Strong-scaling sweep: fixed global grid (default 1024^3), exchange-only driver and Jacobi3D (jacobi3d app with
# --strong semantics via explicit sizes) at 1/2/4/8 GPUs. Mirrors reference scripts/summit/run_256node_strong_spec.sh.
set -o pipefail
cd "$(dirname "$0")/../.."
L=${1:-1024}; shift || true
NS=${*:-1 2 4 8}
export STENCIL_PLAN_FILE=0
mkdir -p gpurun_out/strong
for n in $NS; do
  timeout -k 10 600 python -m stencil2_amd.launch -n $n build/bin/weak $L $L $L 30 --strong | tee gpurun_out/strong/exchange_$n.csv || exit 1
done
