#!/bin/bash
# kernel-level profile of the 1-GPU bench (kernel trace + stats)
export STENCIL_SKIP_BUILD=1 STENCIL_PLAN_FILE=0 PYTHONPATH=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 20 --warmup 2 --exchange-iters 5 > gpurun_out/prof/bench.log 2>&1
echo "rc=$?"
cat gpurun_out/prof/run_kernel_stats.csv | cut -c1-160
