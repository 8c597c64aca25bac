#!/bin/bash
# x-halo triples across ranks + 2 / 4-rank rehearsals on one GPU (phase times), one traced 4-rank run -> gpurun_out/$1/
export STENCIL_PLAN_FILE=0
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu.py -k "x_halo_triples_across or triples_across" > $O/pytest.log 2>&1 || exit 1
tail -2 $O/pytest.log
timeout -k 10 400 python bench.py --gpus 2 > $O/bench2.json 2> $O/bench2.err || exit 1
timeout -k 10 500 python bench.py --gpus 4 > $O/bench4.json 2> $O/bench4.err || exit 1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 500 python scripts/mi355x/launch_ranks.py -n 4 --timeout 480 -- rocprofv3 --kernel-trace -d $O/rank{rank} -o p -- python bench.py --gpus 4 --transport-sweep off > $O/bench4_traced.json 2> $O/bench4_traced.err || exit 1
