O=gpurun_out/r6bd; mkdir -p $O
for i in 1 2; do
for t in nontemporal=1 nontemporal=0 alternate_z=0 xcd_remap=0; do
timeout -k 10 300 python scripts/mi355x/x3_probe.py --kinds jacobi --steps 108 --tune $t > $O/probe_${t/=/_}_$i.log 2>&1 || exit 1
done; done
