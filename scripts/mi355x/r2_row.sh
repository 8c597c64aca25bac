#!/bin/bash
# whole-row fused pair: correctness tests, then bench A/B against the column kernel
set -o pipefail
export STENCIL_SKIP_BUILD=1 STENCIL_PLAN_FILE=0 PYTHONPATH=$GRAFT_REPO_ROOT
D=gpurun_out/${R2TAG:-r2row}; mkdir -p $D
step() { local name=$1 lim=$2; shift 2; echo "== $name"; timeout -k 10 $lim "$@" > $D/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -2 $D/$name.log | cut -c1-300; return $rc; }
step tests 400 python -u -m pytest tests/test_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "whole_row or special_values or in_kernel_wrap" &&
for r in 1 2; do
  step b_col_$r 120 python bench.py --steps 50 --x2row 0 &&
  step b_row3_$r 120 python bench.py --steps 50 &&
  step b_row2_$r 120 python bench.py --steps 50 --x2pf 2 &&
  step b_row1_$r 120 python bench.py --steps 50 --x2pf 1 || exit 1
done
grep -Ho '"value": [0-9.]*' $D/b_*.log
echo done
