#!/bin/bash
# levelled leftover slices: sphere weight 0.45 .. 1.0 (driver command, interleaved) + block clocks
O=gpurun_out/$1; mkdir -p $O
for i in 1 2 3; do
  for w in 0.45 0.6 0.8 1.0; do
    timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --transport-sweep off --tune x3sphw=$w > $O/w${w}_$i.json 2> $O/w${w}_$i.err || exit 1
  done
done
for w in 0.6 0.8; do
PYTHONPATH=$GRAFT_REPO_ROOT timeout -k 10 200 python scripts/mi355x/lab/x3_blocks.py jacobi 512 20 $w > $O/blocks_$w.log 2>&1 || exit 1
done
timeout -k 10 300 python scripts/mi355x/x3_probe.py --kinds jacobi --steps 108 > $O/probe.log 2>&1 || exit 1
