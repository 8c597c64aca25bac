#!/bin/bash
# FETCH_SIZE of the fused-pair kernels, quarter-major vs column-major lockstep order (one counter pass each)
set -o pipefail
export STENCIL_SKIP_BUILD=1 STENCIL_PLAN_FILE=0 PYTHONPATH=$GRAFT_REPO_ROOT
D=gpurun_out/${TAG:-r2s3_fetch}; mkdir -p $D
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for q in 1 0; do
  STENCIL_X2_QMAJOR=$q timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $D/pmc_q$q -o run --output-format csv -- python3 bench.py --steps 4 --warmup 0 > $D/pmc_q$q.log 2>&1 || exit 1
done
echo done
