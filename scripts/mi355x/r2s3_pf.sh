#!/bin/bash
# fused-pair lookahead depth after the edge-wave skip (interleaved), plus the fused-pair tests
set -o pipefail
export STENCIL_SKIP_BUILD=1 STENCIL_PLAN_FILE=0 PYTHONPATH=$GRAFT_REPO_ROOT
D=gpurun_out/${TAG:-r2s3_pf}; mkdir -p $D
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $D/$name.log 2>&1; local rc=$?; echo "$name rc=$rc $(grep -o '"value": [0-9.]*\|[0-9]* passed.*\|[0-9]* failed.*' $D/$name.log | tr '\n' ' ')"; return $rc; }
step tests 500 python -u -m pytest tests/test_gpu.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread -k "temporal2 or col512 or whole_row or wide_rows or lockstep" || exit 1
for i in 1 2; do for pf in 3 2 1; do
  step pf${pf}_$i 200 python bench.py --steps 100 --x2pf $pf || exit 1
done; done
STENCIL_X2_EDGE_SKIP=0 step skip0 200 python bench.py --steps 100 || exit 1
echo done
