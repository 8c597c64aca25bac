#!/bin/bash
# 8 ranks sharing one GPU: does the time follow the number of active streams / cross-process device flags?
set -o pipefail
export STENCIL_SKIP_BUILD=1 STENCIL_PLAN_FILE=0 PYTHONPATH=$GRAFT_REPO_ROOT STENCIL_WAIT_TIMEOUT=30
D=gpurun_out/${TAG:-r2s3_mp8c}; mkdir -p $D
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $D/$name.log 2>&1; local rc=$?; echo "$name rc=$rc $(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"methods": "[a-z/]*"\|"overlap": [a-z]*' $D/$name.log | tr '\n' ' ')"; return $rc; }
MP="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1"
step off 300 $MP --nproc-per-node 8 --master-port 29608 bench.py --gpus 8 --steps 16 --warmup 4 --per-gpu 128 --overlap off &&
step staged 300 $MP --nproc-per-node 8 --master-port 29609 bench.py --gpus 8 --steps 16 --warmup 4 --per-gpu 128 --overlap off --methods staged,kernel &&
step mp4_128 300 $MP --nproc-per-node 4 --master-port 29610 bench.py --gpus 4 --steps 16 --warmup 4 --per-gpu 128 --overlap off
echo "done rc=$?"
