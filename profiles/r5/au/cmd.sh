# sphere-weighted z parts for the pair kernels (row, col2): bitwise tests, driver command per weight
export STENCIL_PLAN_FILE=0 TMPDIR=/tmp
set -o pipefail
O=gpurun_out/r5/${TAG:-at}
mkdir -p $O
timeout -k 10 500 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_gpu.py -k "temporal2_whole or col512" > $O/pytest.log 2>&1 || exit 1
for i in 1 2 3; do
  for w in 0 0.15; do
    timeout -k 10 120 python bench.py --steps 20 --warmup 5 --x2sphw $w > $O/drv_w${w}_$i.json 2> $O/drv_w${w}_$i.err || exit 1
    timeout -k 10 120 python bench.py --steps 20 --warmup 5 --temporal 2 --with-exchange off --x2sphw $w > $O/t2_w${w}_$i.json 2> $O/t2_w${w}_$i.err || exit 1
  done
done
