#!/bin/bash
# lockstep quarter-column schedule of the whole-row fused pair: tests, N=1 bench, fake-remote split per reserve
set -o pipefail
export STENCIL_SKIP_BUILD=1 STENCIL_PLAN_FILE=0 PYTHONPATH=$GRAFT_REPO_ROOT
D=gpurun_out/${TAG:-r2s3_lockstep}; mkdir -p $D
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $D/$name.log 2>&1; local rc=$?; echo "$name rc=$rc $(grep -o '"value": [0-9.]*\|[0-9]* passed.*\|[0-9]* failed.*' $D/$name.log | tr '\n' ' ')"; return $rc; }
step tests 400 python -u -m pytest tests/test_gpu.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread -k "lockstep or zslab_row or whole_row" || exit 1
step base 200 python bench.py || exit 1
STENCIL_X2_LOCKSTEP=0 step base_bal 200 python bench.py || exit 1
for ax in 4 6; do for rs in 8 4; do for m in 1 2; do
  STENCIL_FAKE_REMOTE_AXES=$ax STENCIL_OVERLAP_MODE=$m step fake${ax}_m${m}_r${rs} 200 python bench.py --x2reserve $rs || exit 1
done; done; done
STENCIL_FAKE_REMOTE_AXES=4 STENCIL_X2_LOCKSTEP=0 step fake4_m1_r8_bal 200 python bench.py || exit 1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
STENCIL_FAKE_REMOTE_AXES=4 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $D/prof_z -o run --output-format csv -- python3 bench.py --steps 20 --warmup 2 > $D/prof_z.log 2>&1
echo "done rc=$?"
