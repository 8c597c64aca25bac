#!/bin/bash
# warm-up overlap choice with five candidates (2 ranks sharing one GPU) + the 1-GPU bench
set -o pipefail
export STENCIL_SKIP_BUILD=1 STENCIL_PLAN_FILE=0 PYTHONPATH=$GRAFT_REPO_ROOT STENCIL_WAIT_TIMEOUT=30
D=gpurun_out/${TAG:-r2s3_tuner}; mkdir -p $D
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $D/$name.log 2>&1; local rc=$?; echo "$name rc=$rc $(grep -o '"value": [0-9.]*\|"overlap_tuned": {[^}]*}' $D/$name.log | tr '\n' ' ')"; return $rc; }
step mp2_512 300 python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1 --nproc-per-node 2 --master-port 29602 bench.py --gpus 2 --steps 20 --warmup 5 &&
step bench 200 python bench.py
echo "done rc=$?"
