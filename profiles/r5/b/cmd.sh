set -o pipefail
O=gpurun_out/r5/b
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu.py -k "temporal3" > $O/pytest.log 2>&1 &&
for i in 1 2; do
  timeout -k 10 120 python bench.py --temporal 3 > $O/bench_t3_$i.json 2> $O/bench_t3_$i.err &&
  timeout -k 10 120 python bench.py --temporal 3 --x3pf 2 > $O/bench_t3pf2_$i.json 2> $O/bench_t3pf2_$i.err &&
  timeout -k 10 120 python bench.py > $O/bench_t2_$i.json 2> $O/bench_t2_$i.err || exit 1
done &&
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT &&
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/prof -o t3 -- python bench.py --temporal 3 --steps 36 --with-exchange off > $O/prof_t3.log 2>&1
