# fused-triple kernel time vs grid rows (row groups of 6: leftover rows 0..5)
export PYTHONPATH=. TMPDIR=/tmp
set -o pipefail
O=gpurun_out/r5/${TAG:-ah}
mkdir -p $O
cd /tmp && cd $GRAFT_REPO_ROOT
run() { timeout -k 10 120 rocprofv3 --kernel-trace -d $O/k_$1 -o k -- python scripts/mi355x/lab/x3_radius.py $2 $3 $4 3 36 $5 > $O/k_$1.log 2>&1 || exit 1; }
for y in 504 506 508 510 511 512 513 514 516; do run j$y 512 $y 512 jacobi; done
for y in 510 512; do run a$y 512 $y 512 astaroth; done
run j512z510 512 512 510 jacobi
