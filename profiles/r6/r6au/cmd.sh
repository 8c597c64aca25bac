O=gpurun_out/r6au; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -q --timeout 300 --timeout-method thread -k "temporal3_x_halos or field_beyond or headline_config" > $O/tests.log 2>&1 || exit 1
for i in 1 2; do
timeout -k 10 300 python scripts/mi355x/x3_probe.py --kinds jacobi,astaroth --wraps 0 --steps 108 > $O/probe_cur$i.log 2>&1 || exit 1
STENCIL_ALLOW_STALE=1 PYTHONPATH=lab_alt/head timeout -k 10 300 python scripts/mi355x/x3_probe.py --kinds jacobi,astaroth --wraps 0 --steps 108 > $O/probe_alt$i.log 2>&1 || exit 1
done
timeout -k 10 400 build/bin/astaroth_sim --x 1024 --y 1024 --z 1024 --q 8 --fp64 -n 3 --temporal 3 > $O/c5b_t3.log 2>&1 || exit 1
