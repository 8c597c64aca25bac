set -o pipefail
export STENCIL_SKIP_BUILD=1 STENCIL_PLAN_FILE=0 PYTHONPATH=$GRAFT_REPO_ROOT
mkdir -p gpurun_out/apps_t2
timeout -k 10 200 ./build/bin/jacobi3d 512 512 512 -n 20 --temporal 2 > gpurun_out/apps_t2/app_jacobi_t2.log 2>&1 &&
timeout -k 10 200 ./build/bin/jacobi3d 512 512 512 -n 20 > gpurun_out/apps_t2/app_jacobi_t1.log 2>&1 &&
timeout -k 10 300 ./build/bin/astaroth_sim --x 512 --y 512 --z 512 --q 8 -n 6 --temporal 2 > gpurun_out/apps_t2/c4_astaroth_t2.log 2>&1
rc=$?; tail -n1 gpurun_out/apps_t2/*.log; exit $rc
