#!/bin/bash
export STENCIL_SKIP_BUILD=1 STENCIL_PLAN_FILE=0 PYTHONPATH=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python scripts/mi355x/tune_jacobi.py 512 > gpurun_out/tune.log 2>&1; echo "tune rc=$?"
