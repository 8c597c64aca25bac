#!/bin/bash
# same-box A/B of the driver command: current tree vs lab_alt/$2 (interleaved, 3 rounds) -> gpurun_out/$1/
O=gpurun_out/$1; mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --transport-sweep off > $O/cur_$i.json 2> $O/cur_$i.err || exit 1
  cp bench.py lab_alt/$2/bench.py && STENCIL_ALLOW_STALE=1 timeout -k 10 300 python lab_alt/$2/bench.py --gpus 1 --steps 20 --warmup 5 --transport-sweep off > $O/alt_$i.json 2> $O/alt_$i.err || exit 1
done
