# ragged whole-row kernel: targeted GPU tests, headline sanity, per-GPU ladder shapes (both cut orders) x2row 1 / 0
set -o pipefail
export STENCIL_SKIP_BUILD=1 STENCIL_PLAN_FILE=0 PYTHONPATH=$GRAFT_REPO_ROOT
out=gpurun_out/ragged
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_gpu.py -x -v --timeout 120 --timeout-method thread -m gpu \
  -k "whole_row or wide_rows or in_kernel_wrap or col512" > $out/pytest.log 2>&1 || { tail -n 40 $out/pytest.log; exit 1; }
tail -n 3 $out/pytest.log
timeout -k 10 120 python bench.py > $out/bench.log 2>&1 || exit 1
timeout -k 10 400 python scripts/mi355x/shape_sweep.py --shapes ${SHAPES:-645x323x645,645x645x323,813x407x407,813x204x813,813x813x204,1024x256x512,1024x512x256} --x2row ${ROWS:-1,0} > $out/shapes.log 2>&1 || exit 1
cat $out/bench.log | tail -n 1 | cut -c1-200; cat $out/shapes.log
