#!/bin/bash
export STENCIL_SKIP_BUILD=1 STENCIL_PLAN_FILE=0 PYTHONPATH=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
rm -rf gpurun_out/prof2; mkdir -p gpurun_out/prof2
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof2/kt -o kt --output-format csv -- python3 scripts/mi355x/jacobi_steps.py 512 5 ${OVERLAP:-0} ${TUNE:-0,4,32} > gpurun_out/prof2/kt.log 2>&1 || echo "kt failed"
timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof2/p1 -o pmc --output-format csv -- python3 scripts/mi355x/jacobi_steps.py 512 2 ${OVERLAP:-0} ${TUNE:-0,4,32} > gpurun_out/prof2/p1.log 2>&1 || echo "p1 failed"
timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE TCC_HIT_sum TCC_MISS_sum -d gpurun_out/prof2/p2 -o pmc --output-format csv -- python3 scripts/mi355x/jacobi_steps.py 512 2 ${OVERLAP:-0} ${TUNE:-0,4,32} > gpurun_out/prof2/p2.log 2>&1 || echo "p2 failed"
timeout -k 10 240 python3 scripts/mi355x/jacobi_steps.py 512 2 0 > gpurun_out/prof2/copy.log 2>&1
echo done
