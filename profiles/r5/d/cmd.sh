set -o pipefail
O=gpurun_out/r5/d
mkdir -p $O
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_gpu.py -k "temporal3" > $O/pytest.log 2>&1;
for i in 1 2; do
  timeout -k 10 120 python bench.py --temporal 3 --x3stagger 1 > $O/bench_t3s_$i.json 2> $O/bench_t3s_$i.err &&
  timeout -k 10 120 python bench.py --temporal 3 > $O/bench_t3_$i.json 2> $O/bench_t3_$i.err &&
  timeout -k 10 120 python bench.py > $O/bench_t2_$i.json 2> $O/bench_t2_$i.err || exit 1
done &&
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT &&
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/prof -o t3s -- python bench.py --temporal 3 --x3stagger 1 --steps 36 --with-exchange off > $O/prof_t3s.log 2>&1 &&
PMC_TAG=d/pmc PMC_TEMPORALS="2 3" bash scripts/mi355x/r5_pmc.sh &&
PMC_TAG=d/pmcs PMC_TEMPORALS="3" PMC_ARGS="--x3stagger 1" bash scripts/mi355x/r5_pmc.sh
