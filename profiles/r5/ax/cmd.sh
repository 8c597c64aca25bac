# sphere-weighted z parts of the Jacobi triple: bitwise tests, per-block times, driver command per weight
export PYTHONPATH=. TMPDIR=/tmp STENCIL_PLAN_FILE=0
set -o pipefail
O=gpurun_out/r5/${TAG:-an}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_gpu.py -k "temporal3" > $O/pytest.log 2>&1 || exit 1
for c in "512 0.4" "512 0.6"; do
  set -- $c
  timeout -k 10 120 python scripts/mi355x/lab/x3_blocks.py jacobi $1 4 $2 > $O/blocks_$1_$2.txt 2>&1 || exit 1
done
for i in 1 2 3; do
  for w in 0.3 0.4 0.5 0.6; do
    timeout -k 10 120 python bench.py --steps 20 --warmup 5 --x3sphw $w > $O/drv_w${w}_$i.json 2> $O/drv_w${w}_$i.err || exit 1
  done
done
