# fused-triple read amplification: FETCH_SIZE and kernel time per schedule / grid (lab/x3_fetch.py)
export PYTHONPATH=. TMPDIR=/tmp
set -o pipefail
O=gpurun_out/r5/${TAG:-ac}
mkdir -p $O
cd /tmp && cd $GRAFT_REPO_ROOT
run() { # name nx ny nz sched parts
  timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/f_$1 -o pmc -- python scripts/mi355x/lab/x3_fetch.py $2 $3 $4 $5 $6 18 > $O/f_$1.log 2>&1 || exit 1
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/k_$1 -o k -- python scripts/mi355x/lab/x3_fetch.py $2 $3 $4 $5 $6 36 > $O/k_$1.log 2>&1 || exit 1
}
run base 512 512 512 1 0
run p2 512 512 512 1 2
run p4 512 512 512 1 4
run s0 512 512 512 0 0
run y510 512 510 512 1 0
run y504 512 504 512 1 0
