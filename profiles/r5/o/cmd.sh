# triple-kernel ablations (timing only): kernel time per ablation mask under the profiler
export STENCIL_PLAN_FILE=0 TMPDIR=/tmp
set -o pipefail
O=gpurun_out/r5/${TAG:-n}
mkdir -p $O
cd /tmp && cd $GRAFT_REPO_ROOT
for m in 0 1 2 3 4 8 12 16 5 7 15 31; do
  STENCIL_X3_ABLATE=$m timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/a$m -o a -- python bench.py --steps 18 --warmup 18 --exchange-iters 1 --with-exchange off > $O/a$m.log 2>&1 || exit 1
done
