#!/bin/bash
# leftover-queue chunk sweep (same build, interleaved driver command) -> gpurun_out/$1/
O=gpurun_out/$1; mkdir -p $O
for i in 1 2; do
  for c in 0 1 2 4; do
    timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --transport-sweep off --with-exchange off --tune x3dyn=$c > $O/dyn${c}_$i.json 2> $O/dyn${c}_$i.err || exit 1
  done
done
for c in 0 1 2 4; do
  timeout -k 10 300 python scripts/mi355x/x3_probe.py --kinds jacobi,astaroth --wraps 1 --steps 108 --tune x3dyn=$c > $O/probe_dyn$c.log 2>&1 || exit 1
done
