#!/bin/bash
# shortest-path suites, then C4 with the step fused into the expansion (default) and not
set -e
O=gpurun_out/c4fuse; mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_paths.py tests/test_gpu_capacity.py tests/test_gpu_rccl_single.py > $O/pytest.txt 2>&1
for v in 1 0 1 0; do
  timeout -k 10 200 python3 bench.py --workload paths --steps 10 --warmup 3 --no-cpu --option sp_fuse_step=$v > $O/b${v}_$(date +%s%N).json 2> $O/e$v.txt
done
