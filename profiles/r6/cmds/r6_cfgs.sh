#!/bin/bash
# fused-triple probes + BASELINE configs 4 / 5b with pairs vs triples -> gpurun_out/$1/
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 300 python scripts/mi355x/x3_probe.py > $O/probe.log 2>&1 || exit 1
timeout -k 10 300 python scripts/mi355x/x3_probe.py --wraps 0 --tune nontemporal=0 > $O/probe_nt0.log 2>&1 || exit 1
timeout -k 10 300 python scripts/mi355x/x3_probe.py --shape 1024,512,256 --kinds jacobi,astaroth --wraps 1 > $O/probe_1024.log 2>&1 || exit 1
for t in 2 3; do
  timeout -k 10 300 build/bin/astaroth_sim --q 8 --no-wrap --temporal $t -n 9 > $O/c4_t$t.log 2>&1 || exit 1
done
for t in 2 3; do
  timeout -k 10 400 build/bin/astaroth_sim --x 1024 --y 1024 --z 1024 --q 8 --fp64 -n 3 --temporal $t > $O/c5b_t$t.log 2>&1 || exit 1
done
