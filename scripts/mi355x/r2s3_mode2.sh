#!/bin/bash
# overlap mode 2 (slabs after the interior sweep): tests, fake-remote split timing vs mode 1, 2-rank tuner rehearsal
set -o pipefail
export STENCIL_SKIP_BUILD=1 STENCIL_PLAN_FILE=0 PYTHONPATH=$GRAFT_REPO_ROOT STENCIL_WAIT_TIMEOUT=30
D=gpurun_out/${TAG:-r2s3_mode2}; mkdir -p $D
step() { local name=$1 lim=$2; shift 2; echo "== $name"; timeout -k 10 $lim "$@" > $D/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"overlap": [a-z]*\|"overlap_tuned": {[^}]*}\|"wrap_axes": "[a-z]*"\|[0-9]* passed.*\|[0-9]* failed.*' $D/$name.log | tr '\n' ' '; echo; return $rc; }
MP="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1"
step tests 500 python -u -m pytest tests/test_gpu.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread -k "zslab_row or overlap_toggle or temporal2_overlapped" &&
for ax in 4 6; do for rs in 8 4; do
  STENCIL_FAKE_REMOTE_AXES=$ax STENCIL_OVERLAP_MODE=1 step fake${ax}_m1_res$rs 200 python bench.py --x2reserve $rs || exit 1
  STENCIL_FAKE_REMOTE_AXES=$ax STENCIL_OVERLAP_MODE=2 step fake${ax}_m2_res$rs 200 python bench.py --x2reserve $rs || exit 1
done; done
step mp2_512 300 $MP --nproc-per-node 2 --master-port 29602 bench.py --gpus 2 --steps 16 --warmup 4 &&
{ cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT;
  STENCIL_FAKE_REMOTE_AXES=4 STENCIL_OVERLAP_MODE=2 step prof_z_m2 200 rocprofv3 --kernel-trace --stats -d $D/prof_z_m2 -o run --output-format csv -- python3 bench.py --steps 20 --warmup 2; }
echo "done rc=$?"
