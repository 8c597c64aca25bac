O=gpurun_out/r6ai; mkdir -p $O
cp bench.py lab_alt/head/bench.py
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --transport-sweep off > $O/cur_$i.json 2> $O/cur_$i.err || exit 1
  STENCIL_ALLOW_STALE=1 timeout -k 10 300 python lab_alt/head/bench.py --gpus 1 --steps 20 --warmup 5 --transport-sweep off > $O/alt_$i.json 2> $O/alt_$i.err || exit 1
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --transport-sweep off --tune x3sphchunk=0 > $O/nochunk_$i.json 2> $O/nochunk_$i.err || exit 1
done
timeout -k 10 300 python scripts/mi355x/x3_probe.py --kinds jacobi --wraps 1 --steps 108 > $O/probe_cur.log 2>&1 || exit 1
STENCIL_ALLOW_STALE=1 PYTHONPATH=lab_alt/head timeout -k 10 300 python scripts/mi355x/x3_probe.py --kinds jacobi --wraps 1 --steps 108 > $O/probe_alt.log 2>&1 || exit 1
timeout -k 10 300 python scripts/mi355x/x3_probe.py --kinds jacobi --wraps 1 --steps 108 > $O/probe_cur2.log 2>&1 || exit 1
STENCIL_ALLOW_STALE=1 PYTHONPATH=lab_alt/head timeout -k 10 300 python scripts/mi355x/x3_probe.py --kinds jacobi --wraps 1 --steps 108 > $O/probe_alt2.log 2>&1 || exit 1
