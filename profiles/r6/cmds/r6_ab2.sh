#!/bin/bash
# same-box A/B (current tree vs lab_alt/$2): driver command x3 interleaved + steady-state probe + block clocks
O=gpurun_out/$1; mkdir -p $O
cp bench.py lab_alt/$2/bench.py
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --transport-sweep off > $O/cur_$i.json 2> $O/cur_$i.err || exit 1
  STENCIL_ALLOW_STALE=1 timeout -k 10 300 python lab_alt/$2/bench.py --gpus 1 --steps 20 --warmup 5 --transport-sweep off > $O/alt_$i.json 2> $O/alt_$i.err || exit 1
done
timeout -k 10 300 python scripts/mi355x/x3_probe.py --kinds jacobi --steps 108 > $O/probe_cur.log 2>&1 || exit 1
STENCIL_ALLOW_STALE=1 PYTHONPATH=lab_alt/$2 timeout -k 10 300 python scripts/mi355x/x3_probe.py --kinds jacobi --steps 108 > $O/probe_alt.log 2>&1 || exit 1
PYTHONPATH=$GRAFT_REPO_ROOT timeout -k 10 200 python scripts/mi355x/lab/x3_blocks.py jacobi 512 20 0.3 > $O/blocks_cur.log 2>&1 || exit 1
STENCIL_ALLOW_STALE=1 PYTHONPATH=lab_alt/$2 timeout -k 10 200 python scripts/mi355x/lab/x3_blocks.py jacobi 512 20 0.3 > $O/blocks_alt.log 2>&1 || exit 1
