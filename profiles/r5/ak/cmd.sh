export PYTHONPATH=. TMPDIR=/tmp
set -o pipefail
O=gpurun_out/r5/${TAG:-ak}
mkdir -p $O
for c in "jacobi 512" "jacobi 510" "astaroth 512" "astaroth 510"; do
  set -- $c
  timeout -k 10 120 python scripts/mi355x/lab/x3_blocks.py $1 $2 > $O/blocks_$1_$2.txt 2>&1 || exit 1
done
