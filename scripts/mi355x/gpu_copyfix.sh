#!/bin/bash
# copy-kernel check: full GPU suite, exchange probe, bench, kernel trace of the probe
set -o pipefail
export STENCIL_SKIP_BUILD=1 STENCIL_PLAN_FILE=0 PYTHONPATH=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
step() { local name=$1 lim=$2; shift 2; echo "== $name"; timeout -k 10 $lim "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -3 gpurun_out/$name.log | cut -c1-600; return $rc; }
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread &&
step xprobe 120 python scripts/mi355x/xchg_probe.py &&
step bench_a 200 python bench.py &&
step bench_b 200 python bench.py --steps 64 --warmup 16 &&
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT &&
step xprof 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/xprof2 -o xp -- python3 scripts/mi355x/xchg_probe.py
echo "done rc=$?"
