#!/bin/bash
# GPU suite + 8-rank rehearsal of the bench on one GPU (ranks share it over HIP IPC; 1x2x4 exact grid, warm-up
# overlap choice) + the pre-flight fallback path
set -o pipefail
export STENCIL_SKIP_BUILD=1 STENCIL_PLAN_FILE=0 PYTHONPATH=$GRAFT_REPO_ROOT STENCIL_WAIT_TIMEOUT=30
D=gpurun_out/${TAG:-r2s3_mp8}; mkdir -p $D
step() { local name=$1 lim=$2; shift 2; echo "== $name"; timeout -k 10 $lim "$@" > $D/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"decomposition": "[0-9x]*"\|"methods": "[a-z/]*"\|"preflight": "[^"]*"\|"overlap": [a-z]*\|"overlap_tuned": {[^}]*}\|"wrap_axes": "[a-z]*"\|[0-9]* passed.*\|[0-9]* failed.*' $D/$name.log | tr '\n' ' '; echo; return $rc; }
MP="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1"
step pytest_gpu 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread &&
step mp8_128 300 $MP --nproc-per-node 8 --master-port 29608 bench.py --gpus 8 --steps 16 --warmup 4 --per-gpu 128 &&
step mp2_fallback 300 env STENCIL_PREFLIGHT_FORCE_FAIL=1 $MP --nproc-per-node 2 --master-port 29620 bench.py --gpus 2 --steps 8 --warmup 2 --per-gpu 128 &&
step bench 200 python bench.py
echo "done rc=$?"
