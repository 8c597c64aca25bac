O=gpurun_out/r6az; mkdir -p $O
PYTHONPATH=$GRAFT_REPO_ROOT timeout -k 10 200 python scripts/mi355x/lab/x3_blocks.py jacobi 512 20 0.45 xh=1 P=4 > $O/blocks_xh_j.log 2>&1 || exit 1
PYTHONPATH=$GRAFT_REPO_ROOT timeout -k 10 200 python scripts/mi355x/lab/x3_blocks.py jacobi 512 20 0.45 P=4 > $O/blocks_wrap_j.log 2>&1 || exit 1
PYTHONPATH=$GRAFT_REPO_ROOT timeout -k 10 200 python scripts/mi355x/lab/x3_blocks.py astaroth 512 20 0.45 xh=1 P=3 > $O/blocks_xh_a.log 2>&1 || exit 1
