O=gpurun_out/r6bc; mkdir -p $O
for i in 1 2 3 4 5; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/b_$i.json 2> $O/b_$i.err || exit 1
done
