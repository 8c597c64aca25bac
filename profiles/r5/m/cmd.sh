export STENCIL_PLAN_FILE=0 TMPDIR=/tmp
set -o pipefail
O=gpurun_out/r5/${TAG:-m}
mkdir -p $O
for i in 1 2; do
  for cfg in "t3:" "t3nt0:--nt 0" "t3alt0:--altz 0" "t3s0:--x3sched 0"; do
    n=${cfg%%:*}; a=${cfg#*:}
    timeout -k 10 120 python bench.py --steps 20 --warmup 5 --with-exchange off $a > $O/${n}_$i.json 2> $O/${n}_$i.err || exit 1
  done
done
