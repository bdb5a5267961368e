#!/bin/bash
# C3 with the rest passes' non-temporal record / column loads (option bu_rest_nt), interleaved A/B
set -e
O=gpurun_out/c3rnt; mkdir -p $O
for v in 0 1 0 1 0 1 0 1; do
  timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu --option bu_rest_nt=$v > $O/b${v}_$(date +%s%N).json 2> $O/e$v.txt
done
