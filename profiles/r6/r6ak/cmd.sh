O=gpurun_out/r6ak; mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/tuned_$i.json 2> $O/tuned_$i.err || exit 1
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --schedule-rounds 0 > $O/fixed_$i.json 2> $O/fixed_$i.err || exit 1
done
