#!/bin/bash
# graph pre-instantiation: new tests, bench with default and short step counts
set -o pipefail
export STENCIL_SKIP_BUILD=1 STENCIL_PLAN_FILE=0 PYTHONPATH=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
step() { local name=$1 lim=$2; shift 2; echo "== $name"; timeout -k 10 $lim "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; grep -h '^{' gpurun_out/$name.log | cut -c100-260 || tail -3 gpurun_out/$name.log; return $rc; }
step prep_tests 300 python -u -m pytest tests/test_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "prepare or in_kernel_wrap or temporal2_matches" &&
step bp_default 200 python bench.py &&
step bp_20 200 python bench.py --steps 20 --warmup 2 &&
step bp_64 200 python bench.py --steps 64 --warmup 16 &&
step bp_default2 200 python bench.py
echo "done rc=$?"
