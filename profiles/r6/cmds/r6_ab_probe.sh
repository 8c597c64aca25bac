#!/bin/bash
# steady-state triple kernel A/B: x3_probe (jacobi, whole rows) on the current tree vs lab_alt/$2, kernel traces
O=gpurun_out/$1; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for i in 1 2; do
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/cur$i -o p -- python scripts/mi355x/x3_probe.py --kinds jacobi --wraps 1 --steps 180 --rounds 1 > $O/cur$i.log 2>&1 || exit 1
STENCIL_ALLOW_STALE=1 PYTHONPATH=lab_alt/$2 timeout -k 10 300 rocprofv3 --kernel-trace -d $O/alt$i -o p -- python scripts/mi355x/x3_probe.py --kinds jacobi --wraps 1 --steps 180 --rounds 1 > $O/alt$i.log 2>&1 || exit 1
done
