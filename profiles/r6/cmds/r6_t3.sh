#!/bin/bash
# triple GPU tests + config 5b pairs vs triples -> gpurun_out/$1/
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu.py -k "temporal3 or headline_config or triples or smoke" > $O/pytest.log 2>&1
tail -3 $O/pytest.log
grep -q " passed" $O/pytest.log && ! grep -q "failed\|error" $O/pytest.log || exit 1
for t in 2 3; do
  timeout -k 10 400 build/bin/astaroth_sim --x 1024 --y 1024 --z 1024 --q 8 --fp64 -n 3 --temporal $t > $O/c5b_t$t.log 2>&1 || exit 1
done
