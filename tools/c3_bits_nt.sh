#!/bin/bash
# C3 with the DISTINCT output kernel's non-temporal vid loads / stores (option bits_nt), A/B
set -e
O=gpurun_out/c3nt2; mkdir -p $O
for v in 1 0 1 0 1 0 1 0; do
  timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu --option bits_nt=$v > $O/b${v}_$(date +%s%N).json 2> $O/e$v.txt
done
