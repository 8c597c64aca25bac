# triple: all LDS reads at the top of the step (x3var 15) vs 7
export STENCIL_PLAN_FILE=0 TMPDIR=/tmp
set -o pipefail
O=gpurun_out/r5/${TAG:-y}
mkdir -p $O
timeout -k 10 500 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_gpu.py -k "temporal3" > $O/pytest.log 2>&1 || exit 1
for i in 1 2 3 4; do
  for v in 7 15; do
    timeout -k 10 120 python bench.py --steps 20 --warmup 5 --x3var $v > $O/drv_v${v}_$i.json 2> $O/drv_v${v}_$i.err || exit 1
  done
  timeout -k 10 120 python bench.py --steps 20 --warmup 5 --x3var 15 --x3pf 2 > $O/drv_v15p2_$i.json 2> $O/drv_v15p2_$i.err || exit 1
done
cd /tmp && cd $GRAFT_REPO_ROOT &&
for v in 7 15; do
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/prof$v -o v$v -- python bench.py --steps 36 --with-exchange off --x3var $v > $O/prof_v$v.log 2>&1 || exit 1
done
