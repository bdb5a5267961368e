#!/bin/bash
# GO suites + the C3 bench after the non-temporal DISTINCT output
set -e
O=gpurun_out/r13i; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py \
  tests/test_gpu_scale.py tests/test_gpu_multirank_scale.py tests/test_gpu_rccl_single.py tests/test_gpu_writes.py > $O/pytest.txt 2>&1
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err
