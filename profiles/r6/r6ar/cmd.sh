O=gpurun_out/r6ar; mkdir -p $O
timeout -k 10 300 build/bin/astaroth_sim --q 8 --no-wrap --temporal 3 -n 9 > $O/c4_t3.log 2>&1 || exit 1
timeout -k 10 300 build/bin/astaroth_sim --q 8 --temporal 3 -n 9 > $O/c4wrap_t3.log 2>&1 || exit 1
timeout -k 10 400 build/bin/astaroth_sim --x 1024 --y 1024 --z 1024 --q 8 --fp64 -n 3 --temporal 3 > $O/c5b_t3.log 2>&1 || exit 1
