#!/bin/bash
export STENCIL_SKIP_BUILD=1 STENCIL_PLAN_FILE=0 PYTHONPATH=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof gpurun_out/pmc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --exchange-iters 5 > gpurun_out/prof/bench.log 2>&1 || { echo "prof rc=$?"; tail -5 gpurun_out/prof/bench.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE WRITE_SIZE TCC_HIT_sum TCC_MISS_sum -d gpurun_out/pmc -o pmc --output-format csv -- python3 bench.py --steps 3 --warmup 1 --exchange-iters 2 > gpurun_out/pmc/bench.log 2>&1 || { echo "pmc rc=$?"; tail -5 gpurun_out/pmc/bench.log; exit 1; }
echo done
