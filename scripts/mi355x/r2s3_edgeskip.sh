#!/bin/bash
# row kernel: edge waves skip the unused u1/u2 (STENCIL_X2_EDGE_SKIP=1, default) vs computing them (0), interleaved A/B
set -o pipefail
export STENCIL_SKIP_BUILD=1 STENCIL_PLAN_FILE=0 PYTHONPATH=$GRAFT_REPO_ROOT
D=gpurun_out/${TAG:-r2s3_edgeskip}; mkdir -p $D
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $D/$name.log 2>&1; local rc=$?; echo "$name rc=$rc $(grep -o '"value": [0-9.]*\|[0-9]* passed.*\|[0-9]* failed.*' $D/$name.log | tr '\n' ' ')"; return $rc; }
step tests 400 python -u -m pytest tests/test_gpu.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread -k "lockstep or zslab_row or whole_row or wide_rows or temporal2_in_kernel_wrap" || exit 1
for i in 1 2 3; do
  STENCIL_X2_EDGE_SKIP=1 step skip1_$i 200 python bench.py --steps 100 || exit 1
  STENCIL_X2_EDGE_SKIP=0 step skip0_$i 200 python bench.py --steps 100 || exit 1
done
STENCIL_FAKE_REMOTE_AXES=4 STENCIL_X2_EDGE_SKIP=1 step fake4_skip1 200 python bench.py || exit 1
STENCIL_FAKE_REMOTE_AXES=4 STENCIL_X2_EDGE_SKIP=0 step fake4_skip0 200 python bench.py || exit 1
echo done
