#!/bin/bash
# remote-only overlap of fused pairs: GPU tests (single- and multi-rank), 2/4-rank rehearsal auto vs off, 1-GPU bench
set -o pipefail
export STENCIL_SKIP_BUILD=1 STENCIL_PLAN_FILE=0 PYTHONPATH=$GRAFT_REPO_ROOT STENCIL_WAIT_TIMEOUT=30
mkdir -p gpurun_out/ovl2
step() { local name=$1 lim=$2; shift 2; echo "== $name"; timeout -k 10 $lim "$@" > gpurun_out/ovl2/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -3 gpurun_out/ovl2/$name.log; return $rc; }
step tests 600 python -u -m pytest tests/test_gpu.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -k "temporal2 or colocated or canary" || exit 1
for n in 2 4; do
  for ov in ${OVS:-auto off}; do
    step r${n}_$ov 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29600+n)) bench.py --gpus $n --steps 32 --warmup 8 --per-gpu 256 --overlap $ov || exit 1
    grep -o '"value": [0-9.]*\|"overlap": [a-z]*\|"preflight": "[^"]*"' gpurun_out/ovl2/r${n}_$ov.log | tr '\n' ' '; echo
  done
done
step bench1 300 python bench.py --steps 64 --warmup 16 || exit 1
grep -o '"value": [0-9.]*' gpurun_out/ovl2/bench1.log
echo done
