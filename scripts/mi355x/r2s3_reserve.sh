#!/bin/bash
# overlapped fused pairs on one GPU with fake remote faces: CUs left to the transports (x2reserve) and z-slab kernel
set -o pipefail
export STENCIL_SKIP_BUILD=1 STENCIL_PLAN_FILE=0 PYTHONPATH=$GRAFT_REPO_ROOT
D=gpurun_out/${TAG:-r2s3_reserve}; mkdir -p $D
step() { local name=$1 lim=$2; shift 2; echo "== $name"; timeout -k 10 $lim "$@" > $D/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"overlap": [a-z]*\|"wrap_axes": "[a-z]*"' $D/$name.log | tr '\n' ' '; echo; return $rc; }
for ax in 4 6; do
  for rs in 8 4 0; do
    STENCIL_FAKE_REMOTE_AXES=$ax step fake${ax}_res$rs 200 python bench.py --x2reserve $rs || exit 1
    STENCIL_FAKE_REMOTE_AXES=$ax STENCIL_ZSLAB_ROW=0 step fake${ax}_res${rs}_thin 200 python bench.py --x2reserve $rs || exit 1
  done
done
step base 200 python bench.py
