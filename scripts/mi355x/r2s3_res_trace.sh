#!/bin/bash
# interior-sweep duration vs CUs left to the transports (fake remote z faces, slabs after the sweep: the sweep alone)
set -o pipefail
export STENCIL_SKIP_BUILD=1 STENCIL_PLAN_FILE=0 PYTHONPATH=$GRAFT_REPO_ROOT
D=gpurun_out/${TAG:-r2s3_res_trace}; mkdir -p $D
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for rs in 8 4 2 0; do
  STENCIL_FAKE_REMOTE_AXES=4 STENCIL_OVERLAP_MODE=2 timeout -k 10 200 rocprofv3 --kernel-trace -d $D/res$rs -o run --output-format csv -- python3 bench.py --steps 20 --warmup 2 --x2reserve $rs > $D/res$rs.log 2>&1 || exit 1
  grep -o '"value": [0-9.]*' $D/res$rs.log
done
timeout -k 10 200 rocprofv3 --kernel-trace -d $D/base -o run --output-format csv -- python3 bench.py --steps 20 --warmup 2 > $D/base.log 2>&1
echo "done rc=$?"
