#!/bin/bash
# fused two-step kernel: standalone sweep + end-to-end bench over (waves per block, z lookahead, z chunk)
set -o pipefail
export STENCIL_SKIP_BUILD=1 STENCIL_PLAN_FILE=0 PYTHONPATH=$GRAFT_REPO_ROOT
mkdir -p gpurun_out/tune
timeout -k 10 200 ./build/bin/bench_stencil --only x2 > gpurun_out/tune/x2sweep.log 2>&1 || exit 1
for cfg in "16 2 0" "12 2 0" "12 3 0" "16 3 0" "8 2 0" "16 2 64" "16 2 128"; do
  set -- $cfg
  timeout -k 10 120 python bench.py --steps 64 --warmup 8 --exchange-iters 4 --x2nw $1 --x2pf $2 --zchunk $3 > gpurun_out/tune/bench_$1_$2_$3.log 2>&1 || exit 1
  echo "$cfg $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/tune/bench_$1_$2_$3.log)"
done
