export STENCIL_PLAN_FILE=0 TMPDIR=/tmp
set -o pipefail
O=gpurun_out/r5/${TAG:-r}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_gpu.py -k "temporal3 or temporal2" > $O/pytest.log 2>&1 || exit 1
for i in 1 2 3; do
  timeout -k 10 120 python bench.py --steps 20 --warmup 5 --temporal 2 > $O/drv_t2_$i.json 2> $O/drv_t2_$i.err || exit 1
  timeout -k 10 120 python bench.py --steps 20 --warmup 5 > $O/drv_t3_$i.json 2> $O/drv_t3_$i.err || exit 1
done
cd /tmp && cd $GRAFT_REPO_ROOT &&
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/prof -o t3 -- python bench.py --steps 36 --with-exchange off > $O/prof_t3.log 2>&1 &&
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/prof2 -o t2 -- python bench.py --steps 36 --temporal 2 --with-exchange off > $O/prof_t2.log 2>&1
