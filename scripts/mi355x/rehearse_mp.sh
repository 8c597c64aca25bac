#!/bin/bash
# multi-rank rehearsal of the bench on ONE GPU (ranks share the device through HIP IPC; harness uses gloo)
export STENCIL_SKIP_BUILD=1 STENCIL_PLAN_FILE=0 PYTHONPATH=$GRAFT_REPO_ROOT STENCIL_WAIT_TIMEOUT=30
mkdir -p gpurun_out
for n in 2 4; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29600+n)) bench.py --gpus $n --steps 10 --warmup 3 --per-gpu 256 > gpurun_out/rehearse_$n.log 2>&1
  echo "n=$n rc=$?"
  grep metric gpurun_out/rehearse_$n.log | cut -c1-400
done
