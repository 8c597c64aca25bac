#!/bin/bash
# levelled leftover slices: sphere weight and part count around the default (driver command, interleaved)
O=gpurun_out/$1; mkdir -p $O
for i in 1 2; do
  for t in x3sphw=0.3 x3sphw=0.45 x3sphw=0.6 x3parts=3 x3parts=5 x3parts=5,x3sphw=0; do
    timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --transport-sweep off --tune $t > $O/${t//[=,]/_}_$i.json 2> $O/${t//[=,]/_}_$i.err || exit 1
  done
done
PYTHONPATH=$GRAFT_REPO_ROOT timeout -k 10 200 python scripts/mi355x/lab/x3_blocks.py jacobi 512 20 0.45 > $O/blocks_045.log 2>&1 || exit 1
PYTHONPATH=$GRAFT_REPO_ROOT timeout -k 10 200 python scripts/mi355x/lab/x3_blocks.py jacobi 512 20 0.3 x3parts=5 > $O/blocks_p5.log 2>&1 || exit 1
