O=gpurun_out/r6av; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -q --timeout 300 --timeout-method thread -k "temporal2 or ragged or col2 or whole_row" > $O/tests.log 2>&1 || exit 1
for i in 1 2; do
PYTHONPATH=$GRAFT_REPO_ROOT timeout -k 10 300 python scripts/mi355x/shape_sweep.py --steps 64 --x2row 1 --shapes 512x512x512,645x323x645,813x407x407 > $O/pairs_cur$i.log 2>&1 || exit 1
STENCIL_ALLOW_STALE=1 PYTHONPATH=lab_alt/head timeout -k 10 300 python scripts/mi355x/shape_sweep.py --steps 64 --x2row 1 --shapes 512x512x512,645x323x645,813x407x407 > $O/pairs_alt$i.log 2>&1 || exit 1
done
cp bench.py lab_alt/head/bench.py
for i in 1 2; do
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --transport-sweep off > $O/cur_$i.json 2> $O/cur_$i.err || exit 1
STENCIL_ALLOW_STALE=1 timeout -k 10 300 python lab_alt/head/bench.py --gpus 1 --steps 20 --warmup 5 --transport-sweep off > $O/alt_$i.json 2> $O/alt_$i.err || exit 1
done
