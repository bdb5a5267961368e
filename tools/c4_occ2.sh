#!/bin/bash
# C4: walk scan at 8 waves per SIMD (61 VGPRs) and the sweep select at 8 (44 B spilled), A/B
set -e
O=gpurun_out/c4occ4; mkdir -p $O
for v in "sp_walk_occ=1" "sp_walk_occ=8" "sp_walk_occ=1" "sp_walk_occ=8" "sp_walk_occ=1" "sp_walk_occ=8" "sp_ssel_occ=8" "sp_ssel_occ=8"; do
  timeout -k 10 200 python3 bench.py --workload paths --steps 10 --warmup 3 --no-cpu --option $v > "$O/${v}_$(date +%s%N).json" 2> $O/e.txt
done
