#!/bin/bash
# overlap toggle: multi-rank tests over HIP IPC on one GPU and the bench's warm-up choice in 2/4-rank rehearsals
set -o pipefail
export STENCIL_SKIP_BUILD=1 STENCIL_PLAN_FILE=0 PYTHONPATH=$GRAFT_REPO_ROOT STENCIL_WAIT_TIMEOUT=30
D=gpurun_out/${TAG:-r2s3_toggle}; mkdir -p $D
step() { local name=$1 lim=$2; shift 2; echo "== $name"; timeout -k 10 $lim "$@" > $D/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"overlap": [a-z]*\|"overlap_tuned": {[^}]*}\|"wrap_axes": "[a-z]*"\|[0-9]* passed.*\|[0-9]* failed.*' $D/$name.log | tr '\n' ' '; echo; return $rc; }
MP="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1"
step tests 400 python -u -m pytest tests/test_gpu.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread -k "colocated" &&
step mp2_512 300 $MP --nproc-per-node 2 --master-port 29602 bench.py --gpus 2 --steps 16 --warmup 4 &&
step mp2_512_on 300 $MP --nproc-per-node 2 --master-port 29603 bench.py --gpus 2 --steps 16 --warmup 4 --overlap on &&
step mp2_512_off 300 $MP --nproc-per-node 2 --master-port 29605 bench.py --gpus 2 --steps 16 --warmup 4 --overlap off &&
step mp4_256 300 $MP --nproc-per-node 4 --master-port 29604 bench.py --gpus 4 --steps 16 --warmup 4 --per-gpu 256
echo "done rc=$?"
