#!/bin/bash
# kernel traces of the driver command (headline only): current tree vs lab_alt/$2 -> gpurun_out/$1/
O=gpurun_out/$1; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
cp bench.py lab_alt/$2/bench.py
for i in 1 2; do
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/cur$i -o p -- python bench.py --gpus 1 --steps 20 --warmup 5 --with-exchange off > $O/cur$i.log 2>&1 || exit 1
STENCIL_ALLOW_STALE=1 timeout -k 10 300 rocprofv3 --kernel-trace -d $O/alt$i -o p -- python lab_alt/$2/bench.py --gpus 1 --steps 20 --warmup 5 --with-exchange off > $O/alt$i.log 2>&1 || exit 1
done
