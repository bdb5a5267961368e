#!/bin/bash
# the GO suites twice after the agent-scope counter reads
set -e
O=gpurun_out/r13j; mkdir -p $O
for i in 1 2; do
  timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_multirank_scale.py \
    tests/test_gpu_parity.py tests/test_gpu_scale.py tests/test_gpu_rccl_single.py > $O/pytest$i.txt 2>&1
done
timeout -k 10 300 python bench.py --no-cpu > $O/bench.json 2> $O/bench.err
