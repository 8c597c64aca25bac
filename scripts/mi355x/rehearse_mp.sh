#!/bin/bash
# multi-rank rehearsal of the bench on ONE GPU (ranks share the device through HIP IPC; harness uses gloo)
set -o pipefail
export STENCIL_SKIP_BUILD=1 STENCIL_PLAN_FILE=0 PYTHONPATH=$GRAFT_REPO_ROOT STENCIL_WAIT_TIMEOUT=30
mkdir -p gpurun_out/mp
for n in 2 4; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29600+n)) bench.py --gpus $n --steps 32 --warmup 8 --per-gpu ${PERGPU:-256} > gpurun_out/mp/rehearse_$n.log 2>&1
  rc=$?
  echo "n=$n rc=$rc"
  grep metric gpurun_out/mp/rehearse_$n.log | cut -c1-700
  [ $rc -ne 0 ] && { tail -20 gpurun_out/mp/rehearse_$n.log; exit 1; }
done
# the pre-flight fallback path (co-located IPC rejected -> staged on a shared GPU)
STENCIL_PREFLIGHT_FORCE_FAIL=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29620 bench.py --gpus 2 --steps 8 --warmup 2 --per-gpu 128 > gpurun_out/mp/rehearse_fallback.log 2>&1
rc=$?
echo "fallback rc=$rc"
grep -o '"methods": "[^"]*", "preflight": "[^"]*"' gpurun_out/mp/rehearse_fallback.log
[ $rc -ne 0 ] && { tail -20 gpurun_out/mp/rehearse_fallback.log; exit 1; }
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/mp/prof -o run --output-format csv -- python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --steps 16 --warmup 4 --per-gpu 256 > gpurun_out/mp/prof.log 2>&1
echo "prof rc=$?"
find gpurun_out/mp/prof -name "*kernel_stats.csv" | head -3
