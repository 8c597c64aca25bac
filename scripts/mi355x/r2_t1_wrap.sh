# single steps with in-kernel periodic wrap: targeted GPU tests, then jacobi3d / astaroth apps (temporal 1)
set -o pipefail
export STENCIL_SKIP_BUILD=1 STENCIL_PLAN_FILE=0 PYTHONPATH=$GRAFT_REPO_ROOT
out=gpurun_out/wrap1
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -v --timeout 120 --timeout-method thread -m gpu \
  -k "single_step_in_kernel_wrap or jacobi or astaroth or forward" > $out/pytest.log 2>&1 || { tail -n 30 $out/pytest.log; exit 1; }
tail -n 3 $out/pytest.log
for r in 1 2; do
STENCIL_NO_WRAP=1 timeout -k 10 120 ./build/bin/jacobi3d 512 512 512 -n 60 > $out/jac_nowrap$r.log 2>&1 || exit 1
timeout -k 10 120 ./build/bin/jacobi3d 512 512 512 -n 60 > $out/jac_wrap$r.log 2>&1 || exit 1
done
STENCIL_NO_WRAP=1 timeout -k 10 200 ./build/bin/astaroth_sim --x 512 --y 512 --z 512 --q 8 -n 6 > $out/ast_nowrap.log 2>&1 || exit 1
timeout -k 10 200 ./build/bin/astaroth_sim --x 512 --y 512 --z 512 --q 8 -n 6 > $out/ast_wrap.log 2>&1 || exit 1
for f in $out/*.log; do echo "== $f"; tail -n 1 $f; done
