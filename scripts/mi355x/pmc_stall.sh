#!/bin/bash
# Stall breakdown of the fused-pair sweep (bench.py, 4 steps): one counter group per rocprofv3 pass
export STENCIL_SKIP_BUILD=1 STENCIL_PLAN_FILE=0 PYTHONPATH=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
D=gpurun_out/${PMCTAG:-pmcstall}; mkdir -p $D
i=0
SETS=${PMC_SETS:-12345}
for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM" \
           "SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_BUSY_CYCLES" \
           "TA_TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT" \
           "TCC_HIT TCC_MISS TCC_EA0_RDREQ TCC_EA0_WRREQ" \
           "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_WAVES SQ_INSTS_BRANCH"; do
  i=$((i+1))
  case $SETS in *$i*) ;; *) continue ;; esac
  # PMC_CMD: the program to count (default: bench.py, 4 steps)
  timeout -s KILL 90 rocprofv3 --pmc $set -d $D/p$i -o pmc --output-format csv -- ${PMC_CMD:-python3 bench.py --steps 4 --warmup 0 --exchange-iters 1 $BENCH_ARGS} > $D/p$i.log 2>&1 || { echo "pmc $i rc=$?"; tail -5 $D/p$i.log; exit 1; }
done
python3 scripts/mi355x/summarize_pmc.py $D | tee $D/summary.txt
