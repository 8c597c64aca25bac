#!/bin/bash
# fused-pair column order (x-major vs y-major) with and without in-kernel wrap; correctness subset first
set -o pipefail
export STENCIL_SKIP_BUILD=1 STENCIL_PLAN_FILE=0 PYTHONPATH=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
step() { local name=$1 lim=$2; shift 2; echo "== $name"; timeout -k 10 $lim "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; grep -h '^{' gpurun_out/$name.log | python3 -c "import sys,json; [print(json.dumps({k: (d.get(k) if k in d else d['config'].get(k)) for k in ('value','ms_per_step','x2xfast','wrap_axes')})) for d in map(json.loads, sys.stdin)]" 2>/dev/null || tail -3 gpurun_out/$name.log; return $rc; }
step xf_tests 300 python -u -m pytest tests/test_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "in_kernel_wrap or temporal2" &&
step b_xf1_w1 200 python bench.py --steps 64 --warmup 16 --x2xfast 1 &&
step b_xf0_w1 200 python bench.py --steps 64 --warmup 16 --x2xfast 0 &&
step b_xf1_w0 200 python bench.py --steps 64 --warmup 16 --x2xfast 1 --wrap 0 &&
step b_xf0_w0 200 python bench.py --steps 64 --warmup 16 --x2xfast 0 --wrap 0 &&
step b_xf1_w1b 200 python bench.py --steps 64 --warmup 16 --x2xfast 1 &&
step b_xf0_w1b 200 python bench.py --steps 64 --warmup 16 --x2xfast 0 &&
step shapes_xf 300 python scripts/mi355x/shape_sweep.py --steps 32 && cat gpurun_out/shapes_xf.log
echo "done rc=$?"
