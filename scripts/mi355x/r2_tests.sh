#!/bin/bash
# GPU test suite + native ctest on one MI355X (each step time-limited, stop at the first failure)
set -o pipefail
export STENCIL_SKIP_BUILD=1 STENCIL_PLAN_FILE=0 PYTHONPATH=$GRAFT_REPO_ROOT
D=gpurun_out/${R2TAG:-r2tests}; mkdir -p $D
step() { local name=$1 lim=$2; shift 2; echo "== $name"; timeout -k 10 $lim "$@" > $D/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -4 $D/$name.log | cut -c1-400; return $rc; }
step ctest 180 ./build/bin/stencil_ctest --all &&
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} &&
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
echo "done rc=$?"
