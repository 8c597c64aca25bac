#!/bin/bash
# x-face forwarding: triple GPU tests + driver command x3 + probe with forwarding on/off -> gpurun_out/$1/
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu.py -k "temporal3 or headline_config or triples or smoke" > $O/pytest.log 2>&1
tail -2 $O/pytest.log
grep -q " passed" $O/pytest.log && ! grep -q "failed\|error" $O/pytest.log || exit 1
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_$i.json 2> $O/bench_$i.err || exit 1
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o p -- python bench.py --gpus 1 --steps 20 --warmup 5 > $O/prof.log 2>&1 || exit 1
