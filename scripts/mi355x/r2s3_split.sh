#!/bin/bash
# cost of the overlapped fused-pair split on one GPU: faces of the masked axes treated as remote (local interior
# sweep, then the slabs), everything else as in the bench; z slabs by the whole-row kernel (default) or the thin kernel
set -o pipefail
export STENCIL_SKIP_BUILD=1 STENCIL_PLAN_FILE=0 PYTHONPATH=$GRAFT_REPO_ROOT
D=gpurun_out/${TAG:-r2s3_split}; mkdir -p $D
step() { local name=$1 lim=$2; shift 2; echo "== $name"; timeout -k 10 $lim "$@" > $D/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"overlap": [a-z]*\|"wrap_axes": "[a-z]*"\|passed.*\|failed.*' $D/$name.log | tr '\n' ' '; echo; return $rc; }
step tests 400 python -u -m pytest tests/test_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "zslab_row or temporal2_overlapped" &&
step base 200 python bench.py &&
STENCIL_FAKE_REMOTE_AXES=4 step fake_z 200 python bench.py &&
STENCIL_FAKE_REMOTE_AXES=4 STENCIL_ZSLAB_ROW=0 step fake_z_thin 200 python bench.py &&
STENCIL_FAKE_REMOTE_AXES=6 step fake_yz 200 python bench.py &&
STENCIL_FAKE_REMOTE_AXES=6 STENCIL_ZSLAB_ROW=0 step fake_yz_thin 200 python bench.py &&
{ cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT;
  STENCIL_FAKE_REMOTE_AXES=4 step prof_z 200 rocprofv3 --kernel-trace --stats -d $D/prof_z -o run --output-format csv -- python3 bench.py --steps 20 --warmup 2 &&
  STENCIL_FAKE_REMOTE_AXES=4 STENCIL_ZSLAB_ROW=0 step prof_z_thin 200 rocprofv3 --kernel-trace --stats -d $D/prof_z_thin -o run --output-format csv -- python3 bench.py --steps 20 --warmup 2 &&
  STENCIL_FAKE_REMOTE_AXES=6 step prof_yz 200 rocprofv3 --kernel-trace --stats -d $D/prof_yz -o run --output-format csv -- python3 bench.py --steps 20 --warmup 2; }
echo "done rc=$?"
