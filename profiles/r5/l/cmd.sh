export STENCIL_PLAN_FILE=0 TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT
set -o pipefail
O=gpurun_out/r5/${TAG:-l}
mkdir -p $O
timeout -k 10 300 python scripts/mi355x/copy_items_probe.py --combos 1024:512,2048:512,512:512,1536:512 --rounds 4 > $O/probe_faces.jsonl 2>&1 &&
timeout -k 10 300 python scripts/mi355x/copy_items_probe.py --combos 1024:512,2048:512,512:512 --rounds 4 --edges 1 > $O/probe_edges.jsonl 2>&1
