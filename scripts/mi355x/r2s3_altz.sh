#!/bin/bash
# per-step z-direction flip (alternate_z) per kernel: fused pairs (row kernel) and single steps, interleaved
set -o pipefail
export STENCIL_SKIP_BUILD=1 STENCIL_PLAN_FILE=0 PYTHONPATH=$GRAFT_REPO_ROOT
D=gpurun_out/${TAG:-r2s3_altz}; mkdir -p $D
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $D/$name.log 2>&1; local rc=$?; echo "$name rc=$rc $(grep -o '"value": [0-9.]*' $D/$name.log)"; return $rc; }
for i in 1 2; do
  step t2_alt1_$i 200 python bench.py --steps 100 --altz 1 || exit 1
  step t2_alt0_$i 200 python bench.py --steps 100 --altz 0 || exit 1
  step t1_alt1_$i 200 python bench.py --steps 100 --altz 1 --temporal 1 || exit 1
  step t1_alt0_$i 200 python bench.py --steps 100 --altz 0 --temporal 1 || exit 1
  STENCIL_FAKE_REMOTE_AXES=4 step f4_alt1_$i 200 python bench.py --altz 1 || exit 1
  STENCIL_FAKE_REMOTE_AXES=4 step f4_alt0_$i 200 python bench.py --altz 0 || exit 1
done
echo done
