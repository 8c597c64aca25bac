#!/bin/bash
# lockstep z parts in the column / 512-column fused-pair kernels: tests + shape A/B (interleaved)
set -o pipefail
export STENCIL_SKIP_BUILD=1 STENCIL_PLAN_FILE=0 PYTHONPATH=$GRAFT_REPO_ROOT
D=gpurun_out/${TAG:-r2s3_colparts}; mkdir -p $D
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $D/$name.log 2>&1; local rc=$?; echo "$name rc=$rc $(grep -o '[0-9]* passed.*\|[0-9]* failed.*' $D/$name.log | tr '\n' ' ')"; return $rc; }
step tests 500 python -u -m pytest tests/test_gpu.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread -k "temporal2 or col512 or whole_row or wide_rows or lockstep or special_values" || exit 1
for ls in 1 0 1 0; do
  STENCIL_X2_LOCKSTEP=$ls timeout -k 10 300 python scripts/mi355x/shape_sweep.py --shapes 512x512x512,1024x512x256,1024x256x512 --x2row 1,0 --steps 32 > $D/shapes_ls$ls.log 2>&1 || exit 1
  echo "lockstep=$ls"; grep -o '"shape": "[0-9x]*"\|"x2row": [0-9]\|"gcells": [0-9.]*' $D/shapes_ls$ls.log | paste -sd' ' | fold -w 400
done
for ls in 1 0; do
  STENCIL_X2_LOCKSTEP=$ls timeout -k 10 300 ./build/bin/astaroth_sim --x 512 --y 512 --z 512 --q 2 --fp64 -n 6 --temporal 2 > $D/ast_fp64_ls$ls.log 2>&1 || exit 1
  echo "astaroth fp64 t2 lockstep=$ls: $(grep '^astaroth' $D/ast_fp64_ls$ls.log)"
done
echo done
