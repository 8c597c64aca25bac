#!/bin/bash
# full GPU suite + smoke + the driver command -> gpurun_out/$1/
export STENCIL_PLAN_FILE=0
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 1300 python -u -m pytest -v --timeout 240 --timeout-method thread tests/ -m gpu > $O/pytest.log 2>&1
tail -3 $O/pytest.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || exit 1
