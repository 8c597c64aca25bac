#!/bin/bash
# BASELINE.json configs 2-5 on ONE MI355X (configs 3-5 name 8 GPUs: these are their single-GPU points; every halo is
# a periodic self-copy on the same GPU). Config 1 (CPU path) runs on the host: profiles/r2/r2_config1_cpu_path.txt
# Usage (gpurun): bash scripts/mi355x/baseline_configs.sh <outdir>
export STENCIL_SKIP_BUILD=1 STENCIL_PLAN_FILE=0 PYTHONPATH=$GRAFT_REPO_ROOT TMPDIR=/tmp
source scripts/mi355x/steps.sh "${1:-baseline_configs}"
step c2_bench 120 python bench.py --steps 20 --warmup 5
step app_jacobi_t2 200 ./build/bin/jacobi3d 512 512 512 -n 20 --temporal 2
step app_jacobi_t1 200 ./build/bin/jacobi3d 512 512 512 -n 20
step c3_bench_exchange 300 ./build/bin/bench_exchange --x 512 --y 512 --z 512 --fr 2 --iters 30
step c4_astaroth_exchange 300 ./build/bin/astaroth_sim --x 512 --y 512 --z 512 --q 8 -n 5 --no-wrap
step c4_astaroth_exchange_t2 300 ./build/bin/astaroth_sim --x 512 --y 512 --z 512 --q 8 -n 6 --temporal 2 --no-wrap
step c4_astaroth_compute_only 300 ./build/bin/astaroth_sim --x 512 --y 512 --z 512 --q 8 -n 5
step c5_weak_fp64 300 ./build/bin/weak 1024 1024 1024 10 --q 4 --fp64
step c5_astaroth_fp64_t2 400 ./build/bin/astaroth_sim --x 1024 --y 1024 --z 1024 --q 8 --fp64 -n 3 --temporal 2
