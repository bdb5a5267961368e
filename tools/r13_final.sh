#!/bin/bash
# end-of-round check: full GPU suite, smoke, the default bench (C3), C4, and C3 through one RCCL rank
set -e
O=gpurun_out/r13z; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.txt 2>&1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err
timeout -k 10 300 python bench.py --workload paths > $O/c4_bench.json 2> $O/c4.err
timeout -k 10 300 python bench.py --comm-single --no-cpu > $O/comm_single_bench.json 2> $O/cs.err
