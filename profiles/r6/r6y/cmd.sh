#!/bin/bash
# does the driver window (20 steps after 5 warm-up steps) sit below the steady state because of warm-up? bench with
# longer warm-ups and longer timed loops, plus a kernel trace of the driver command
O=gpurun_out/$1; mkdir -p $O
for i in 1 2; do
  for w in 5 50 500; do
    timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup $w --transport-sweep off > $O/w${w}_$i.json 2> $O/w${w}_$i.err || exit 1
  done
  timeout -k 10 300 python bench.py --gpus 1 --steps 200 --warmup 5 --transport-sweep off > $O/s200_$i.json 2> $O/s200_$i.err || exit 1
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/tr -o p -- python bench.py --gpus 1 --steps 20 --warmup 5 --transport-sweep off > $O/tr.json 2> $O/tr.err || exit 1
