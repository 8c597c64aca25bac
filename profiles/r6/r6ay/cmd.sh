O=gpurun_out/r6ay; mkdir -p $O
for i in 1 2; do
timeout -k 10 300 python scripts/mi355x/x3_probe.py --kinds jacobi --wraps 0 --steps 108 > $O/probe_on$i.log 2>&1 || exit 1
timeout -k 10 300 python scripts/mi355x/x3_probe.py --kinds jacobi --wraps 0 --steps 108 --tune x3sphchunk=0 > $O/probe_off$i.log 2>&1 || exit 1
done
