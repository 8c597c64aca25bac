set -o pipefail
O=gpurun_out/r5/e
mkdir -p $O
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_gpu.py -k "temporal3" > $O/pytest.log 2>&1;
for i in 1 2; do
  for cfg in "t2:--temporal 2" "t3:--temporal 3" "t3_s0p0:--temporal 3 --x3sched 0 --x3permute 0" "t3_s1p0:--temporal 3 --x3permute 0" "t3_s0p1:--temporal 3 --x3sched 0" "t3stag:--temporal 3 --x3stagger 1"; do
    n=${cfg%%:*}; a=${cfg#*:}
    timeout -k 10 120 python bench.py $a --with-exchange off > $O/bench_${n}_$i.json 2> $O/bench_${n}_$i.err || exit 1
  done
done
