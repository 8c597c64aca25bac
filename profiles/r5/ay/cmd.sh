# round-end sequence: full GPU suite, smoke, driver command x3, pairs, kernel trace of the driver command
export STENCIL_PLAN_FILE=0 TMPDIR=/tmp
set -o pipefail
O=gpurun_out/r5/${FULL_TAG:-final}
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/steps.txt; [ $rc -le 1 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
echo "smoke rc=0" >> $O/steps.txt
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/bench_$i.json 2> $O/bench_$i.err || exit 1
done
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --temporal 2 > $O/bench_t2.json 2> $O/bench_t2.err || exit 1
echo "bench rc=0" >> $O/steps.txt
cd /tmp && cd $GRAFT_REPO_ROOT &&
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/prof -o drv -- python bench.py --steps 20 --warmup 5 > $O/prof.log 2>&1
