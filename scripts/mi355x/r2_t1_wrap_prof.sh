# kernel times of single steps with in-kernel wrap vs the self-exchange + LDS kernel (jacobi3d 512^3, temporal 1)
set -o pipefail
export STENCIL_SKIP_BUILD=1 STENCIL_PLAN_FILE=0 PYTHONPATH=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/t1wrapp
mkdir -p $out
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $out/wrap -o run -- ./build/bin/jacobi3d 512 512 512 -n 40 > $out/wrap.log 2>&1 || exit 1
STENCIL_NO_WRAP=1 timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $out/nowrap -o run -- ./build/bin/jacobi3d 512 512 512 -n 40 > $out/nowrap.log 2>&1 || exit 1
