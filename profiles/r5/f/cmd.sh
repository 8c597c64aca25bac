# shared halo lines: GPU tests, then interleaved A/B (off / on) of the exchange-bound configs
export STENCIL_SKIP_BUILD=1 STENCIL_PLAN_FILE=0 PYTHONPATH=$GRAFT_REPO_ROOT TMPDIR=/tmp
set -o pipefail
O=gpurun_out/r5/f
mkdir -p $O
timeout -k 10 400 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_gpu.py -k "shared_halo" > $O/pytest.log 2>&1;
for i in 1 2; do
  for sh in "" "--shared-halo-line"; do
    if [ -n "$sh" ]; then t=on; v=1; else t=off; v=0; fi
    timeout -k 10 120 ./build/bin/bench_exchange --x 512 --y 512 --z 512 --fr 2 --iters 30 $sh > $O/c3_${t}_$i.log 2>&1 || exit 1
    timeout -k 10 200 ./build/bin/astaroth_sim --x 512 --y 512 --z 512 --q 8 -n 5 --no-wrap $sh > $O/c4_${t}_$i.log 2>&1 || exit 1
    timeout -k 10 300 ./build/bin/weak 1024 1024 1024 10 --q 4 --fp64 $sh > $O/c5a_${t}_$i.log 2>&1 || exit 1
    timeout -k 10 120 python bench.py --steps 20 --warmup 5 --shared-halo-line $v > $O/bench_${t}_$i.json 2> $O/bench_${t}_$i.err || exit 1
  done
done
