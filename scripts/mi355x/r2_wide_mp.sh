set -o pipefail
export STENCIL_SKIP_BUILD=1 STENCIL_PLAN_FILE=0 PYTHONPATH=$GRAFT_REPO_ROOT
mkdir -p gpurun_out/r2wide
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread -k "wide_rows or colocated_ipc_jacobi" > gpurun_out/r2wide/tests.log 2>&1; rc=$?
tail -3 gpurun_out/r2wide/tests.log; exit $rc
