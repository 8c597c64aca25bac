#!/bin/bash
# 512-cell column kernel: tests, then the ladder shapes (one GPU) with x2row on/off and the headline bench
set -o pipefail
export STENCIL_SKIP_BUILD=1 STENCIL_PLAN_FILE=0 PYTHONPATH=$GRAFT_REPO_ROOT
D=gpurun_out/r2col2; mkdir -p $D
step() { local name=$1 lim=$2; shift 2; echo "== $name"; timeout -k 10 $lim "$@" > $D/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -3 $D/$name.log | cut -c1-300; return $rc; }
step tests 600 python -u -m pytest tests/test_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "col512 or whole_row or temporal2 or special_values" &&
step shapes 400 python scripts/mi355x/shape_sweep.py --shapes 1024x256x512,512x512x512,1024x512x256 &&
step bench 120 python bench.py
echo "done rc=$?"
