#!/bin/bash
# kernel trace of the driver command (per-dispatch durations of the timed window) + driver command x2
O=gpurun_out/$1; mkdir -p $O
for i in 1 2; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --transport-sweep off > $O/b_$i.json 2> $O/b_$i.err || exit 1
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/tr -o p -- python bench.py --gpus 1 --steps 20 --warmup 5 --transport-sweep off > $O/tr.json 2> $O/tr.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/trp -o p -- python scripts/mi355x/x3_probe.py --kinds jacobi --wraps 1 --steps 180 --rounds 1 > $O/trp.log 2>&1 || exit 1
