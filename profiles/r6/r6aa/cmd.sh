#!/bin/bash
# whole-run graphs (prepare(runs)): tests, then the driver command x3
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -q --timeout 300 --timeout-method thread -k "prepare or temporal3_matches or headline_config" > $O/tests.log 2>&1 || exit 1
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --transport-sweep off > $O/b_$i.json 2> $O/b_$i.err || exit 1
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/tr -o p -- python bench.py --gpus 1 --steps 20 --warmup 5 --transport-sweep off > $O/tr.json 2> $O/tr.err || exit 1
