#!/bin/bash
# host wake-up latency of synchronize(): blocking vs polling
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 300 python scripts/mi355x/lab/sync_latency.py > $O/sync.log 2>&1 || exit 1
