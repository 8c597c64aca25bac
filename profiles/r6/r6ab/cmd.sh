#!/bin/bash
# cost of the unsynchronised leftover slices: lockstep parts 3 (one 2-row leftover group) vs 4 (22 leftover groups),
# steady-state probe, both kinds, whole rows and x halos; block clocks for Astaroth (no spheres)
O=gpurun_out/$1; mkdir -p $O
for p in 3 4 5; do
  timeout -k 10 300 python scripts/mi355x/x3_probe.py --kinds jacobi,astaroth --steps 108 --tune x3parts=$p > $O/probe_p$p.log 2>&1 || exit 1
done
for p in 3 4; do
PYTHONPATH=$GRAFT_REPO_ROOT timeout -k 10 200 python scripts/mi355x/lab/x3_blocks.py astaroth 512 20 0.6 x3parts=$p > $O/blocks_ast_p$p.log 2>&1 || exit 1
done
