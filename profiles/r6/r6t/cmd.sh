#!/bin/bash
# triple tests + leftover queue on/off (same build) + A/B vs lab_alt/$2 -> gpurun_out/$1/
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu.py -k "temporal3 or headline_config or triples or smoke" > $O/pytest.log 2>&1
tail -2 $O/pytest.log
grep -q " passed" $O/pytest.log && ! grep -q "failed\|error" $O/pytest.log || exit 1
cp bench.py lab_alt/$2/bench.py
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --transport-sweep off > $O/cur_$i.json 2> $O/cur_$i.err || exit 1
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --transport-sweep off --tune x3dyn=0 > $O/nodyn_$i.json 2> $O/nodyn_$i.err || exit 1
  STENCIL_ALLOW_STALE=1 timeout -k 10 300 python lab_alt/$2/bench.py --gpus 1 --steps 20 --warmup 5 --transport-sweep off > $O/alt_$i.json 2> $O/alt_$i.err || exit 1
done
timeout -k 10 300 python scripts/mi355x/x3_probe.py --kinds jacobi,astaroth --wraps 1 --steps 108 > $O/probe_cur.log 2>&1 || exit 1
timeout -k 10 300 python scripts/mi355x/x3_probe.py --kinds jacobi,astaroth --wraps 1 --steps 108 --tune x3dyn=0 > $O/probe_nodyn.log 2>&1 || exit 1
PYTHONPATH=$GRAFT_REPO_ROOT timeout -k 10 200 python scripts/mi355x/lab/x3_blocks.py jacobi 512 20 0.3 > $O/blocks_cur.log 2>&1 || exit 1
