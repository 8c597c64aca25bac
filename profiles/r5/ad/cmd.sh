# fused-triple kernel time vs memory layout (row pitch / plane stride), kernel trace only
export PYTHONPATH=. TMPDIR=/tmp
set -o pipefail
O=gpurun_out/r5/${TAG:-ad}
mkdir -p $O
cd /tmp && cd $GRAFT_REPO_ROOT
run() { # name nx ny nz pad shared
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/k_$1 -o k -- python scripts/mi355x/lab/x3_fetch.py $2 $3 $4 1 0 36 $5 $6 > $O/k_$1.log 2>&1 || exit 1
}
for rep in a b; do
run base$rep 512 512 512 0 0
run pad1$rep 512 512 512 1 0
run pad2$rep 512 512 512 2 0
run pad3$rep 512 512 512 3 0
run shared$rep 512 512 512 0 1
run y510$rep 512 510 512 0 0
run y510p1$rep 512 510 512 1 0
done
