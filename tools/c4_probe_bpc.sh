#!/bin/bash
# C4 with the meet probe's grid at 4-7 blocks per CU (option sp_probe_bpc), twice each
set -e
O=gpurun_out/c4bpc2; mkdir -p $O
for v in 5 6 5 6 5 6 5 6; do
  timeout -k 10 200 python3 bench.py --workload paths --steps 10 --warmup 3 --no-cpu --option sp_probe_bpc=$v > $O/b${v}_$(date +%s%N).json 2> $O/e$v.txt
done
