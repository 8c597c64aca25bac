# forced overlap at N=1 (config 4), tests, and the temporal 2 vs 3 driver-command A/B
export STENCIL_SKIP_BUILD=1 STENCIL_PLAN_FILE=0 PYTHONPATH=$GRAFT_REPO_ROOT TMPDIR=/tmp
set -o pipefail
O=gpurun_out/r5/g
mkdir -p $O
timeout -k 10 400 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_gpu.py -k "forced_overlap or jacobi_device_matches_oracle or temporal3 or shared_halo_lines_models" > $O/pytest.log 2>&1;
A=./build/bin/astaroth_sim
for i in 1 2; do
  timeout -k 10 200 $A --q 8 -n 5 --no-wrap > $O/c4_base_$i.log 2>&1 || exit 1
  for r in 8 16 32; do
    timeout -k 10 200 $A --q 8 -n 5 --no-wrap --overlap --reserve $r > $O/c4_ovl_r${r}_$i.log 2>&1 || exit 1
  done
  timeout -k 10 200 $A --q 8 -n 5 --no-wrap --overlap --reserve 0 > $O/c4_ovl_r0_$i.log 2>&1 || exit 1
  timeout -k 10 200 $A --q 8 -n 5 --no-wrap --shared-halo-line > $O/c4_shared_$i.log 2>&1 || exit 1
  timeout -k 10 200 $A --q 8 -n 5 --no-wrap --overlap --reserve 16 --shared-halo-line > $O/c4_ovl_shared_$i.log 2>&1 || exit 1
done
for i in 1 2 3; do
  timeout -k 10 120 python bench.py --steps 20 --warmup 5 --temporal 2 > $O/drv_t2_$i.json 2> $O/drv_t2_$i.err || exit 1
  timeout -k 10 120 python bench.py --steps 20 --warmup 5 --temporal 3 > $O/drv_t3_$i.json 2> $O/drv_t3_$i.err || exit 1
done
