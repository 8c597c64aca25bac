#!/bin/bash
# PMC counters of the default single-step kernel and the fused-pair kernel (bench_stencil --only one, 2 launches each)
export STENCIL_SKIP_BUILD=1 STENCIL_PLAN_FILE=0 PYTHONPATH=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmc
i=0
for set in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU" "SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 60 rocprofv3 --pmc $set -d gpurun_out/pmc/p$i -o pmc --output-format csv -- ./build/bin/bench_stencil --only one --iters 1 > gpurun_out/pmc/p$i.log 2>&1 || { echo "pmc $i rc=$?"; grep -i error gpurun_out/pmc/p$i.log | head -3; exit 1; }
done
python3 scripts/mi355x/summarize_prof.py gpurun_out/pmc
