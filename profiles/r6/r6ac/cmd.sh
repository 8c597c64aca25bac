#!/bin/bash
# leftover plans (StencilTune.x3left: 1 levelled slices, 2 second lockstep phase, 3 auto) x parts: tests, driver
# command interleaved, steady-state probes, block clocks
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -q --timeout 300 --timeout-method thread -k "temporal3 or headline_config or prepare" > $O/tests.log 2>&1 || exit 1
for i in 1 2; do
  for t in x3left=1,x3parts=4 x3left=2,x3parts=4 x3left=2,x3parts=7 x3left=3 x3left=1,x3parts=3; do
    timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --transport-sweep off --tune $t > $O/${t//[=,]/_}_$i.json 2> $O/${t//[=,]/_}_$i.err || exit 1
  done
done
for t in x3left=1,x3parts=4 x3left=2,x3parts=4 x3left=2,x3parts=7 x3left=3; do
  timeout -k 10 300 python scripts/mi355x/x3_probe.py --kinds jacobi,astaroth --steps 108 --tune $t > $O/probe_${t//[=,]/_}.log 2>&1 || exit 1
done
PYTHONPATH=$GRAFT_REPO_ROOT timeout -k 10 200 python scripts/mi355x/lab/x3_blocks.py jacobi 512 20 0.6 x3left=2 x3parts=4 > $O/blocks_l2p4.log 2>&1 || exit 1
PYTHONPATH=$GRAFT_REPO_ROOT timeout -k 10 200 python scripts/mi355x/lab/x3_blocks.py jacobi 512 20 0.6 x3left=2 x3parts=7 > $O/blocks_l2p7.log 2>&1 || exit 1
