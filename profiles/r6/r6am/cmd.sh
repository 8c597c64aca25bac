export STENCIL_PLAN_FILE=0
O=gpurun_out/r6am; mkdir -p $O
timeout -k 10 400 python bench.py --gpus 2 > $O/bench2.json 2> $O/bench2.err || exit 1
timeout -k 10 500 python bench.py --gpus 4 > $O/bench4.json 2> $O/bench4.err || exit 1
