#!/bin/bash
# triple GPU tests + same-box A/B against lab_alt/$2 -> gpurun_out/$1/
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu.py -k "temporal3 or headline_config or triples or smoke" > $O/pytest.log 2>&1
tail -2 $O/pytest.log
grep -q " passed" $O/pytest.log && ! grep -q "failed\|error" $O/pytest.log || exit 1
bash scripts/mi355x/r6_ab2.sh $1 $2
