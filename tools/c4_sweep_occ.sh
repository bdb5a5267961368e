#!/bin/bash
# C4 bench with the select's occupancy variants (sp_sel_occ), twice each
set -e
O=gpurun_out/c4occ3; mkdir -p $O
for v in 1 6 8 1 6 8; do
  timeout -k 10 200 python3 bench.py --workload paths --steps 10 --warmup 3 --no-cpu --option sp_sel_occ=$v > $O/b${v}_$(date +%s%N).json 2> $O/e$v.txt
done
