# early LDS publication A/B: triples (x3var 0/1/5/7) and pairs (x2early 0/1, row + col2 kernels)
export STENCIL_PLAN_FILE=0 TMPDIR=/tmp
set -o pipefail
O=gpurun_out/r5/${TAG:-v}
mkdir -p $O
timeout -k 10 500 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_gpu.py -k "temporal3 or temporal2_whole_row or temporal2_in_kernel_wrap or col512" > $O/pytest.log 2>&1 || exit 1
for i in 1 2 3; do
  for v in 0 1 5 7; do
    timeout -k 10 120 python bench.py --steps 20 --warmup 5 --x3var $v > $O/drv_v${v}_$i.json 2> $O/drv_v${v}_$i.err || exit 1
  done
  for e in 0 1; do
    timeout -k 10 120 python bench.py --steps 20 --warmup 5 --temporal 2 --x2early $e > $O/drv_e${e}_$i.json 2> $O/drv_e${e}_$i.err || exit 1
  done
done
cd /tmp && cd $GRAFT_REPO_ROOT &&
for e in 0 1; do
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/profe$e -o e$e -- python bench.py --steps 36 --temporal 2 --x2early $e > $O/prof_e$e.log 2>&1 || exit 1
done
