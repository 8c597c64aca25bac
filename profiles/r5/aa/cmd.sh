# full GPU suite + smoke + driver bench (the round-end sequence); stops after a crash, abort or time limit
export STENCIL_PLAN_FILE=0 TMPDIR=/tmp
set -o pipefail
O=gpurun_out/r5/${FULL_TAG:-h}
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/steps.txt; [ $rc -le 1 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
echo "smoke rc=0" >> $O/steps.txt
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || exit 1
echo "bench rc=0" >> $O/steps.txt
