O=gpurun_out/r6be; mkdir -p $O; cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/tr -o p -- python scripts/mi355x/lab/xh_after_exchange.py > $O/run.log 2>&1 || exit 1
