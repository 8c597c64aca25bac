O=gpurun_out/r6as; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -q --timeout 300 --timeout-method thread -k "temporal3_matches or headline_config or set_triple" > $O/tests.log 2>&1 || exit 1
cp bench.py lab_alt/head/bench.py
for i in 1 2; do
timeout -k 10 300 python scripts/mi355x/x3_probe.py --kinds jacobi --wraps 1 --steps 108 > $O/probe_cur$i.log 2>&1 || exit 1
STENCIL_ALLOW_STALE=1 PYTHONPATH=lab_alt/head timeout -k 10 300 python scripts/mi355x/x3_probe.py --kinds jacobi --wraps 1 --steps 108 > $O/probe_alt$i.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --transport-sweep off > $O/cur_$i.json 2> $O/cur_$i.err || exit 1
STENCIL_ALLOW_STALE=1 timeout -k 10 300 python lab_alt/head/bench.py --gpus 1 --steps 20 --warmup 5 --transport-sweep off > $O/alt_$i.json 2> $O/alt_$i.err || exit 1
done
