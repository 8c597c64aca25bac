#!/bin/bash
set -o pipefail
timeout -k 10 120 ./build/bin/stencil_ctest --gpu > gpurun_out/ctest.log 2>&1; tail -6 gpurun_out/ctest.log | grep -v amdgpu
export PYTEST_K="temporal or special or overlap" SWEEP="x2pp"
bash scripts/mi355x/gpu_iter.sh && timeout -k 10 200 python bench.py --steps 64 --warmup 16 --overlap on > gpurun_out/iter/bench_ovl.log 2>&1; grep -o '"value": [0-9.]*\|"overlap": [a-z]*' gpurun_out/iter/bench_ovl.log; bash scripts/mi355x/rehearse_mp.sh
