#!/bin/bash
# bench.py option A/B on one box (default fused kernel shape): store policy, z-march alternation, work split
set -o pipefail
export STENCIL_SKIP_BUILD=1 STENCIL_PLAN_FILE=0 PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/${OUT:-opts}; mkdir -p $O
i=0
for r in 1 2; do
  while read -r name args; do
    i=$((i+1))
    timeout -k 10 200 python bench.py --steps 64 --warmup 16 $args > $O/b_${name}_$r.log 2>&1 || { tail $O/b_${name}_$r.log; exit 1; }
    echo "$name r=$r $(grep -o '"value": [0-9.]*' $O/b_${name}_$r.log)"
  done <<LIST
default
nt0 --nt 0
altz0 --altz 0
chunks --x2sched 0
nw12pf1 --x2pf 1
LIST
done
