#!/bin/bash
# round-2 session-3 check: native ctest, GPU pytest, smoke, 1-GPU bench, 2/4-rank rehearsal of the exact weak grid
# (ranks sharing the one GPU through HIP IPC), kernel-trace profile of the 1-GPU bench
set -o pipefail
export STENCIL_SKIP_BUILD=1 STENCIL_PLAN_FILE=0 PYTHONPATH=$GRAFT_REPO_ROOT STENCIL_WAIT_TIMEOUT=30
D=gpurun_out/${R2TAG:-r2s3}; mkdir -p $D
step() { local name=$1 lim=$2; shift 2; echo "== $name"; timeout -k 10 $lim "$@" > $D/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -3 $D/$name.log | cut -c1-900; return $rc; }
MP="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1"
step ctest 180 ./build/bin/stencil_ctest --all &&
step pytest_gpu 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread &&
step smoke 200 python -c "import __graft_entry__ as g; g.smoke()" &&
step bench_a 200 python bench.py &&
step bench_b 200 python bench.py --steps 64 --warmup 16 &&
step mp2_512 300 $MP --nproc-per-node 2 --master-port 29602 bench.py --gpus 2 --steps 16 --warmup 4 &&
step mp4_256 300 $MP --nproc-per-node 4 --master-port 29604 bench.py --gpus 4 --steps 16 --warmup 4 --per-gpu 256 &&
{ cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT;
  step prof 300 rocprofv3 --kernel-trace --stats -d $D/prof -o run --output-format csv -- python3 bench.py --steps 20 --warmup 2 &&
  step prof_mp2 300 rocprofv3 --kernel-trace --stats -d $D/prof_mp2 -o run --output-format csv -- python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29612 bench.py --gpus 2 --steps 16 --warmup 4; }
echo "done rc=$?"
