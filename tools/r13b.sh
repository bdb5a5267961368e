#!/bin/bash
# round-6 late checks: parity + sharded suites, the one-rank RCCL C3 timeline, C3 benches
set -e
O=gpurun_out/r13b; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py \
  tests/test_gpu_scale.py tests/test_gpu_capacity.py tests/test_gpu_rccl_single.py tests/test_gpu_multirank_scale.py \
  tests/test_gpu_multirank.py > $O/pytest.txt 2>&1
bash tools/kt_timeline.sh r13b 14 --comm-single
timeout -k 10 200 python3 bench.py --comm-single --steps 20 --warmup 5 --no-cpu --option rep1_atomic=1 > $O/atomic_bench.json 2>/dev/null
timeout -k 10 200 python3 bench.py --comm-single --steps 20 --warmup 5 --no-cpu > $O/cs_bench.json 2>/dev/null
timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 > $O/bench.json 2>/dev/null
