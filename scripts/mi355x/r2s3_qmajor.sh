#!/bin/bash
# lockstep quarters in quarter-major block order (an XCD's blocks take y-adjacent columns of one quarter) vs
# column-major: tests, interleaved bench, fake-remote split, FETCH_SIZE of the row kernel
set -o pipefail
export STENCIL_SKIP_BUILD=1 STENCIL_PLAN_FILE=0 PYTHONPATH=$GRAFT_REPO_ROOT
D=gpurun_out/${TAG:-r2s3_qmajor}; mkdir -p $D
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $D/$name.log 2>&1; local rc=$?; echo "$name rc=$rc $(grep -o '"value": [0-9.]*\|[0-9]* passed.*\|[0-9]* failed.*' $D/$name.log | tr '\n' ' ')"; return $rc; }
step tests 500 python -u -m pytest tests/test_gpu.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread -k "temporal2 or whole_row or lockstep or wide_rows" || exit 1
for i in 1 2; do
  STENCIL_X2_QMAJOR=1 step q1_$i 200 python bench.py --steps 100 || exit 1
  STENCIL_X2_QMAJOR=0 step q0_$i 200 python bench.py --steps 100 || exit 1
done
STENCIL_FAKE_REMOTE_AXES=4 STENCIL_X2_QMAJOR=1 step fake4_q1 200 python bench.py || exit 1
STENCIL_FAKE_REMOTE_AXES=4 STENCIL_X2_QMAJOR=0 step fake4_q0 200 python bench.py || exit 1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for q in 1 0; do
  STENCIL_X2_QMAJOR=$q timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE WRITE_SIZE -d $D/pmc_q$q -o run --output-format csv -- python3 bench.py --steps 4 --warmup 0 > $D/pmc_q$q.log 2>&1 || exit 1
done
echo done
