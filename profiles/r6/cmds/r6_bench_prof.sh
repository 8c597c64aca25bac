#!/bin/bash
# driver command twice + one kernel trace of it: gpurun_out/$1/
O=gpurun_out/$1; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for i in 1 2; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_$i.json 2> $O/bench_$i.err || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python bench.py --gpus 1 --steps 20 --warmup 5 > $O/prof.log 2>&1 || exit 1
find $O/prof -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats.csv \;
