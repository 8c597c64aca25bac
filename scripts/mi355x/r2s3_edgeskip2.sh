#!/bin/bash
# edge-wave skip in the column (256-cell) and 512-column fused-pair kernels: tests + shape A/B
set -o pipefail
export STENCIL_SKIP_BUILD=1 STENCIL_PLAN_FILE=0 PYTHONPATH=$GRAFT_REPO_ROOT
D=gpurun_out/${TAG:-r2s3_edgeskip2}; mkdir -p $D
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $D/$name.log 2>&1; local rc=$?; echo "$name rc=$rc $(grep -o '[0-9]* passed.*\|[0-9]* failed.*' $D/$name.log | tr '\n' ' ')"; return $rc; }
step tests 500 python -u -m pytest tests/test_gpu.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread -k "temporal2 or col512 or whole_row or wide_rows or special_values" || exit 1
for sk in 1 0 1 0; do
  STENCIL_X2_EDGE_SKIP=$sk timeout -k 10 300 python scripts/mi355x/shape_sweep.py --shapes 512x512x512,1024x512x256,813x407x407 --x2row 1,0 --steps 32 > $D/shapes_skip$sk.log 2>&1 || exit 1
  echo "skip=$sk"; grep -o '"shape": "[0-9x]*"\|"x2row": [0-9]\|"gcells": [0-9.]*\|"value": [0-9.]*' $D/shapes_skip$sk.log | paste -sd' ' | fold -w 400
done
echo done
