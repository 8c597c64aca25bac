O=gpurun_out/r6bg; mkdir -p $O
for i in 1 2; do
for t in x3left=3 x3left=1 x3sphw=0.3 x3sphw=0.6 x3left=2,x3sphw=0.3; do
timeout -k 10 300 python scripts/mi355x/x3_probe.py --kinds jacobi --wraps 0 --steps 108 --tune $t > $O/probe_${t//[=,]/_}_$i.log 2>&1 || exit 1
done; done
