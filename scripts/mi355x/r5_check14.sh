# sphere interval test in the triple: bitwise tests, row-count sweep, driver command
export PYTHONPATH=. TMPDIR=/tmp STENCIL_PLAN_FILE=0
set -o pipefail
O=gpurun_out/r5/${TAG:-ai}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_gpu.py -k "temporal3" > $O/pytest.log 2>&1 || exit 1
cd /tmp && cd $GRAFT_REPO_ROOT
run() { timeout -k 10 120 rocprofv3 --kernel-trace -d $O/k_$1 -o k -- python scripts/mi355x/lab/x3_radius.py $2 $3 $4 3 36 $5 > $O/k_$1.log 2>&1 || exit 1; }
for y in 510 512; do run j$y 512 $y 512 jacobi; run a$y 512 $y 512 astaroth; done
for i in 1 2 3; do
  timeout -k 10 120 python bench.py --steps 20 --warmup 5 > $O/drv_$i.json 2> $O/drv_$i.err || exit 1
done
for c in "jacobi 512" "jacobi 510"; do
  set -- $c
  timeout -k 10 120 python scripts/mi355x/lab/x3_blocks.py $1 $2 > $O/blocks_$1_$2.txt 2>&1 || exit 1
done
