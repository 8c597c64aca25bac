#!/bin/bash
export STENCIL_SKIP_BUILD=1 STENCIL_PLAN_FILE=0 PYTHONPATH=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
rm -rf gpurun_out/prof3; mkdir -p gpurun_out/prof3
timeout -k 10 240 rocprofv3 --kernel-trace -d gpurun_out/prof3/ov -o kt --output-format csv -- python3 scripts/mi355x/jacobi_steps.py 512 6 1 0,4,0 > gpurun_out/prof3/ov.log 2>&1 || echo "ov failed"
timeout -k 10 240 rocprofv3 --kernel-trace -d gpurun_out/prof3/no -o kt --output-format csv -- python3 scripts/mi355x/jacobi_steps.py 512 6 0 0,4,0 > gpurun_out/prof3/no.log 2>&1 || echo "no failed"
echo done
