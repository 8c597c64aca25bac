#!/bin/bash
# fetched / written bytes and stall split of the whole-row fused pair (bench.py, 4 steps)
export PMC_SETS=${PMC_SETS:-1245} PMCTAG=pmc_row
bash scripts/mi355x/pmc_stall.sh > /dev/null || exit 1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmc_row
for set in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 90 rocprofv3 --pmc $set -d gpurun_out/pmc_row/p_$set -o pmc --output-format csv -- python3 bench.py --steps 4 --warmup 0 --exchange-iters 1 > gpurun_out/pmc_row/p_$set.log 2>&1 || { echo "pmc $set rc=$?"; exit 1; }
done
python3 scripts/mi355x/summarize_pmc.py gpurun_out/pmc_row | tee gpurun_out/pmc_row/summary.txt | grep -A40 row_kernel
