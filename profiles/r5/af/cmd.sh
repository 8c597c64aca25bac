export PYTHONPATH=. TMPDIR=/tmp
set -o pipefail
O=gpurun_out/r5/${TAG:-ae}
mkdir -p $O
cd /tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 120 rocprofv3 --kernel-trace -d $O/kj -o k -- python scripts/mi355x/lab/x3_timeline.py jacobi 900 > $O/kj.log 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace -d $O/ka -o k -- python scripts/mi355x/lab/x3_timeline.py jacobi 90 > $O/ka.log 2>&1 || exit 1
