#!/bin/bash
# C3 bench x3 with coherent publish / gate-word checks but plain gate_open loads; GO suites once
set -e
O=gpurun_out/r13l; mkdir -p $O
for i in 1 2 3; do timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu --no-parity > $O/b$i.json 2> $O/e$i.txt; done
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_multirank_scale.py \
  tests/test_gpu_parity.py tests/test_gpu_scale.py > $O/pytest.txt 2>&1
