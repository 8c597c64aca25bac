# fused-triple kernel time vs plane stride (halo radius 3..6) and row count
export PYTHONPATH=. TMPDIR=/tmp
set -o pipefail
O=gpurun_out/r5/${TAG:-ag}
mkdir -p $O
cd /tmp && cd $GRAFT_REPO_ROOT
run() { timeout -k 10 120 rocprofv3 --kernel-trace -d $O/k_$1 -o k -- python scripts/mi355x/lab/x3_radius.py $2 $3 $4 $5 36 > $O/k_$1.log 2>&1 || exit 1; }
for rep in a b; do
  for r in 3 4 5 6 8; do run r${r}_512$rep 512 512 512 $r; done
  for r in 3 4 5; do run r${r}_510$rep 512 510 512 $r; done
done
