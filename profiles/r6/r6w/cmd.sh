#!/bin/bash
# leftover slices levelled against the lockstep parts (StencilTune.x3balance): triple tests, block clocks on / off,
# driver command interleaved on / off, steady-state probe
O=gpurun_out/$1; mkdir -p $O
: timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -q --timeout 300 --timeout-method thread -k "temporal3 or headline_config" > $O/tests.log 2>&1 || exit 1
PYTHONPATH=$GRAFT_REPO_ROOT timeout -k 10 200 python scripts/mi355x/lab/x3_blocks.py jacobi 512 20 0.3 > $O/blocks_on.log 2>&1 || exit 1
PYTHONPATH=$GRAFT_REPO_ROOT timeout -k 10 200 python scripts/mi355x/lab/x3_blocks.py jacobi 512 20 0.3 x3balance=0 > $O/blocks_off.log 2>&1 || exit 1
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --transport-sweep off > $O/on_$i.json 2> $O/on_$i.err || exit 1
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --transport-sweep off --tune x3balance=0 > $O/off_$i.json 2> $O/off_$i.err || exit 1
done
timeout -k 10 300 python scripts/mi355x/x3_probe.py --kinds jacobi --steps 108 > $O/probe_on.log 2>&1 || exit 1
