#!/bin/bash
# second lockstep phase (x3left 3 = auto: Jacobi P = 4 + lockstep leftover, Astaroth P = 3): sphere weight, driver
# command interleaved, probes, block clocks
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -q --timeout 300 --timeout-method thread -k "temporal3 or headline_config or prepare" > $O/tests.log 2>&1 || exit 1
for i in 1 2; do
  for w in 0.3 0.45 0.6; do
    timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --transport-sweep off --tune x3sphw=$w > $O/w${w}_$i.json 2> $O/w${w}_$i.err || exit 1
  done
done
for w in 0.3 0.45; do
  timeout -k 10 300 python scripts/mi355x/x3_probe.py --kinds jacobi --steps 108 --tune x3sphw=$w > $O/probe_w$w.log 2>&1 || exit 1
  PYTHONPATH=$GRAFT_REPO_ROOT timeout -k 10 200 python scripts/mi355x/lab/x3_blocks.py jacobi 512 20 $w > $O/blocks_w$w.log 2>&1 || exit 1
done
timeout -k 10 300 python scripts/mi355x/x3_probe.py --kinds astaroth --steps 108 > $O/probe_ast.log 2>&1 || exit 1
