export PYTEST_K="mfma"; export SWEEP="mfma"
bash scripts/mi355x/gpu_iter.sh && timeout -k 10 200 python bench.py --steps 32 --warmup 8 --temporal 1 --variant 8 > gpurun_out/iter/bench_mfma.log 2>&1 && timeout -k 10 200 python bench.py --steps 32 --warmup 8 --temporal 1 > gpurun_out/iter/bench_t1.log 2>&1 && bash scripts/mi355x/gpu_pmc.sh
