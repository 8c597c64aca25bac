#!/bin/bash
# PMC counters of the fused sweep per wrap mode (bench.py, few steps; one counter group per pass)
export STENCIL_SKIP_BUILD=1 STENCIL_PLAN_FILE=0 PYTHONPATH=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for w in 1 0; do
  mkdir -p gpurun_out/pmcw$w
  i=0
  for set in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU" "SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $set -d gpurun_out/pmcw$w/p$i -o pmc --output-format csv -- python3 bench.py --steps 4 --warmup 0 --exchange-iters 1 --wrap $w > gpurun_out/pmcw$w/p$i.log 2>&1 || { echo "pmc w$w $i rc=$?"; tail -3 gpurun_out/pmcw$w/p$i.log; exit 1; }
  done
  echo "== wrap $w"
  python3 scripts/mi355x/summarize_pmc.py gpurun_out/pmcw$w | tee gpurun_out/pmcw$w/summary.txt
done
