#!/bin/bash
# fused pair as the model runs it (ping-pong) + PMC counters of one launch of each default kernel
set -o pipefail
export STENCIL_SKIP_BUILD=1 STENCIL_PLAN_FILE=0 PYTHONPATH=$GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmc
timeout -k 10 200 ./build/bin/bench_stencil --only x2pp > gpurun_out/pmc/x2pp.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
i=0
for pmc in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
           "FETCH_SIZE WRITE_SIZE" "SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"; do
  i=$((i+1))
  timeout -s KILL 60 rocprofv3 --pmc $pmc --output-format csv -d gpurun_out/pmc/p$i -o run -- ./build/bin/bench_stencil --only one --iters 2 > gpurun_out/pmc/p$i.log 2>&1 || exit 1
done
echo ok
