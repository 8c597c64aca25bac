# multi-rank rehearsals on one GPU (ranks share the device): the transport warm-up table and every sweep entry
export STENCIL_PLAN_FILE=0 TMPDIR=/tmp
set -o pipefail
O=gpurun_out/r5/${TAG:-k}
mkdir -p $O
timeout -k 10 400 python bench.py --gpus 2 > $O/bench2.json 2> $O/bench2.err || exit 1
timeout -k 10 500 python bench.py --gpus 4 > $O/bench4.json 2> $O/bench4.err || exit 1
timeout -k 10 500 python bench.py --gpus 8 --per-gpu 256 > $O/bench8_256.json 2> $O/bench8_256.err
