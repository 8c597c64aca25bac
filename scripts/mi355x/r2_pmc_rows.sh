export PMC_SETS=15
PMCTAG=pmc_r2_8_1 BENCH_ARGS="--x2rows 2 --x2nw 8 --x2pf 1" bash scripts/mi355x/pmc_stall.sh > /dev/null && \
PMCTAG=pmc_r1 BENCH_ARGS="" bash scripts/mi355x/pmc_stall.sh > /dev/null
for d in pmc_r2_8_1 pmc_r1; do echo "## $d"; grep -A12 "stencil7x2" gpurun_out/$d/summary.txt; done
