#!/bin/bash
# wrap as a kernel template flag: correctness subset, bench wrap on/off (twice), kernel traces
set -o pipefail
export STENCIL_SKIP_BUILD=1 STENCIL_PLAN_FILE=0 PYTHONPATH=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
step() { local name=$1 lim=$2; shift 2; echo "== $name"; timeout -k 10 $lim "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; grep -h '^{' gpurun_out/$name.log | cut -c1-120 || tail -3 gpurun_out/$name.log; return $rc; }
step w2_tests 300 python -u -m pytest tests/test_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "in_kernel_wrap or temporal2" &&
step b_w1 200 python bench.py --steps 64 --warmup 16 &&
step b_w0 200 python bench.py --steps 64 --warmup 16 --wrap 0 &&
step b_w1b 200 python bench.py --steps 64 --warmup 16 &&
step b_w0b 200 python bench.py --steps 64 --warmup 16 --wrap 0 &&
bash scripts/mi355x/prof_wrap.sh
echo "done rc=$?"
