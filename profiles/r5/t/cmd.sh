# triple lane layouts A/B (x3layout 1: 8 adjacent cells per lane; 0: chunks 256 apart) + pairs, kernel traces
export STENCIL_PLAN_FILE=0 TMPDIR=/tmp
set -o pipefail
O=gpurun_out/r5/${TAG:-s}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_gpu.py -k "temporal3 or temporal2_whole_row or temporal2_in_kernel_wrap" > $O/pytest.log 2>&1 || exit 1
for i in 1 2 3 4; do
  timeout -k 10 120 python bench.py --steps 20 --warmup 5 --x3var 0 > $O/drv_v0_$i.json 2> $O/drv_v0_$i.err || exit 1
  timeout -k 10 120 python bench.py --steps 20 --warmup 5 --x3var 5 > $O/drv_v5_$i.json 2> $O/drv_v5_$i.err || exit 1
  timeout -k 10 120 python bench.py --steps 20 --warmup 5 --x3var 7 > $O/drv_v7_$i.json 2> $O/drv_v7_$i.err || exit 1
  timeout -k 10 120 python bench.py --steps 20 --warmup 5 --x3var 1 > $O/drv_v1_$i.json 2> $O/drv_v1_$i.err || exit 1
done
cd /tmp && cd $GRAFT_REPO_ROOT &&
for v in 0 1 5 7; do
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/prof$v -o v$v -- python bench.py --steps 36 --with-exchange off --x3var $v > $O/prof_v$v.log 2>&1 || exit 1
done
