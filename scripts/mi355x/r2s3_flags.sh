#!/bin/bash
# headline flags re-checked after the edge-wave skip / lockstep changes (interleaved on one box)
set -o pipefail
export STENCIL_SKIP_BUILD=1 STENCIL_PLAN_FILE=0 PYTHONPATH=$GRAFT_REPO_ROOT
D=gpurun_out/${TAG:-r2s3_flags}; mkdir -p $D
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $D/$name.log 2>&1; local rc=$?; echo "$name rc=$rc $(grep -o '"value": [0-9.]*' $D/$name.log)"; return $rc; }
for i in 1 2; do
  step default_$i 200 python bench.py --steps 100 || exit 1
  step nt0_$i 200 python bench.py --steps 100 --nt 0 || exit 1
  step altz0_$i 200 python bench.py --steps 100 --altz 0 || exit 1
  step pf2_$i 200 python bench.py --steps 100 --x2pf 2 || exit 1
  STENCIL_X2_QMAJOR=0 step qmajor0_$i 200 python bench.py --steps 100 || exit 1
done
echo done
