#!/bin/bash
# non-persistent fused-pair sweeps (fixed z chunks) vs balanced persistent segments: N=1 and the fake-remote split
set -o pipefail
export STENCIL_SKIP_BUILD=1 STENCIL_PLAN_FILE=0 PYTHONPATH=$GRAFT_REPO_ROOT
D=gpurun_out/${TAG:-r2s3_sched}; mkdir -p $D
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $D/$name.log 2>&1; local rc=$?; echo "$name rc=$rc $(grep -o '"value": [0-9.]*' $D/$name.log)"; return $rc; }
step base 200 python bench.py || exit 1
for zc in 32 64 128; do step base_zc$zc 200 python bench.py --x2sched 0 --zchunk $zc || exit 1; done
for m in 1 2; do
  for rs in 0 8; do
    STENCIL_FAKE_REMOTE_AXES=4 STENCIL_OVERLAP_MODE=$m step fake4_m${m}_r${rs}_bal 200 python bench.py --x2reserve $rs || exit 1
    for zc in 32 64 127; do
      STENCIL_FAKE_REMOTE_AXES=4 STENCIL_OVERLAP_MODE=$m step fake4_m${m}_r${rs}_zc$zc 200 python bench.py --x2reserve $rs --x2sched 0 --zchunk $zc || exit 1
    done
  done
done
echo "done"
