# leftover row groups only on the lightest blocks (x3leftover): bitwise tests, per-block times, driver command A/B
export PYTHONPATH=. TMPDIR=/tmp STENCIL_PLAN_FILE=0
set -o pipefail
O=gpurun_out/r5/${TAG:-az}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_gpu.py -k "temporal3" > $O/pytest.log 2>&1 || exit 1
timeout -k 10 120 python scripts/mi355x/lab/x3_blocks.py jacobi 512 4 0.3 > $O/blocks_512.txt 2>&1 || exit 1
for i in 1 2 3; do
  for l in 0 1; do
    timeout -k 10 120 python bench.py --steps 20 --warmup 5 --x3leftover $l > $O/drv_l${l}_$i.json 2> $O/drv_l${l}_$i.err || exit 1
  done
done
