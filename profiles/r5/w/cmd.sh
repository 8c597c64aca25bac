# triple lookahead / layout A/B on the early-publish variant (x3var 7)
export STENCIL_PLAN_FILE=0 TMPDIR=/tmp
set -o pipefail
O=gpurun_out/r5/${TAG:-w}
mkdir -p $O
timeout -k 10 500 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_gpu.py -k "temporal3" > $O/pytest.log 2>&1 || exit 1
for i in 1 2 3; do
  for c in "1 0" "2 0" "1 1" "2 1"; do
    set -- $c
    timeout -k 10 120 python bench.py --steps 20 --warmup 5 --x3pf $1 --x3layout $2 > $O/drv_p$1l$2_$i.json 2> $O/drv_p$1l$2_$i.err || exit 1
  done
done
cd /tmp && cd $GRAFT_REPO_ROOT &&
for p in 1 2; do
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/prof$p -o p$p -- python bench.py --steps 36 --with-exchange off --x3pf $p > $O/prof_p$p.log 2>&1 || exit 1
done
