#!/bin/bash
set -o pipefail
export STENCIL_SKIP_BUILD=1 STENCIL_PLAN_FILE=0 PYTHONPATH=$GRAFT_REPO_ROOT
mkdir -p gpurun_out/shapes
timeout -k 10 300 python scripts/mi355x/shape_sweep.py --x2sched 1,0 > gpurun_out/shapes/shapes.log 2>&1
rc=$?; cat gpurun_out/shapes/shapes.log; exit $rc
