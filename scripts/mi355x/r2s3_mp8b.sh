#!/bin/bash
# 8-rank and 2-rank (512^3 each) rehearsals of the bench on one GPU with the final defaults, plus the fallback path
set -o pipefail
export STENCIL_SKIP_BUILD=1 STENCIL_PLAN_FILE=0 PYTHONPATH=$GRAFT_REPO_ROOT STENCIL_WAIT_TIMEOUT=30
D=gpurun_out/${TAG:-r2s3_mp8b}; mkdir -p $D
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $D/$name.log 2>&1; local rc=$?; echo "$name rc=$rc $(grep -o '"value": [0-9.]*\|"decomposition": "[0-9x]*"\|"preflight": "[^"]*"\|"overlap_tuned": {[^}]*}' $D/$name.log | tr '\n' ' ')"; return $rc; }
MP="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1"
step mp8_128 300 $MP --nproc-per-node 8 --master-port 29608 bench.py --gpus 8 --steps 16 --warmup 4 --per-gpu 128 &&
step mp2_512 300 $MP --nproc-per-node 2 --master-port 29602 bench.py --gpus 2 --steps 20 --warmup 5 &&
step mp4_256_cbrt 300 $MP --nproc-per-node 4 --master-port 29604 bench.py --gpus 4 --steps 16 --warmup 4 --per-gpu 256 --grid cbrt &&
step fallback 300 env STENCIL_PREFLIGHT_FORCE_FAIL=1 $MP --nproc-per-node 2 --master-port 29620 bench.py --gpus 2 --steps 8 --warmup 2 --per-gpu 128
echo "done rc=$?"
