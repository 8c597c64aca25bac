#!/bin/bash
# bench.py over the fused kernel's block shape (waves per block x planes of lookahead), same box
set -o pipefail
export STENCIL_SKIP_BUILD=1 STENCIL_PLAN_FILE=0 PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/${OUT:-nw}; mkdir -p $O
for r in 1 2; do for nw in ${NWS:-8 12 16}; do for pf in ${PFS:-1 2}; do
  timeout -k 10 200 python bench.py --steps 64 --warmup 16 --x2nw $nw --x2pf $pf > $O/b_${nw}_${pf}_$r.log 2>&1 || { tail $O/b_${nw}_${pf}_$r.log; exit 1; }
  echo "nw=$nw pf=$pf r=$r $(grep -o '"value": [0-9.]*' $O/b_${nw}_${pf}_$r.log)"
done; done; done
