O=gpurun_out/r6ax; mkdir -p $O; cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/tr -o p -- python bench.py --gpus 1 --steps 20 --warmup 5 --transport-sweep off > $O/tr.json 2> $O/tr.err || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU -d $O/p1 -o p -- python scripts/mi355x/x3_probe.py --kinds jacobi --steps 18 --rounds 1 > $O/p1.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/p2 -o p -- python scripts/mi355x/x3_probe.py --kinds jacobi --steps 18 --rounds 1 > $O/p2.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES -d $O/p3 -o p -- python scripts/mi355x/x3_probe.py --kinds jacobi --steps 18 --rounds 1 > $O/p3.log 2>&1 || exit 1
