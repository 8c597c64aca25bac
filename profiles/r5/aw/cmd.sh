# triples with remote halos (multi-rank on one GPU) + bench rehearsals at 2 / 4 ranks
export STENCIL_PLAN_FILE=0 TMPDIR=/tmp
set -o pipefail
O=gpurun_out/r5/${TAG:-z}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_gpu.py -k "triples_across or two_rank_triples or two_rank_exact" > $O/pytest.log 2>&1 || exit 1
timeout -k 10 400 python bench.py --gpus 2 > $O/bench2.json 2> $O/bench2.err || exit 1
timeout -k 10 500 python bench.py --gpus 4 > $O/bench4.json 2> $O/bench4.err || exit 1
timeout -k 10 120 python bench.py --steps 20 --warmup 5 > $O/bench1.json 2> $O/bench1.err
