#!/bin/bash
# kernel traces of the 1-GPU bench with and without in-kernel wrap (sweep kernel time vs halo copy)
export STENCIL_SKIP_BUILD=1 STENCIL_PLAN_FILE=0 PYTHONPATH=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/profw
for w in 1 0 6; do
  if [ $w = 6 ]; then export STENCIL_WRAP_AXES=6; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/profw/w$w -o run --output-format csv -- python3 bench.py --steps 32 --warmup 4 --exchange-iters 4 --wrap $((w != 0)) > gpurun_out/profw/bench_w$w.log 2>&1 || { echo "prof w$w rc=$?"; exit 1; }
  echo "== wrap $w"; grep -h '^{' gpurun_out/profw/bench_w$w.log | cut -c1-140
  find gpurun_out/profw/w$w -name '*kernel_stats.csv' -exec cut -d, -f1-7 {} \; | cut -c1-200
done
