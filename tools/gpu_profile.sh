#!/bin/bash
# One GPU-box session: bench line + rocprofv3 kernel stats + HBM PMC passes (separate runs,
# never combined with runtime/sys traces).  Usage: tools/gpu_profile.sh <round-tag> [bench args]
set -e
tag=${1:-r01}; shift || true
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 480 python3 bench.py "$@" > $out/bench.json 2> $out/bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/kt -o run -- \
  python3 bench.py --no-cpu --steps 5 --warmup 1 "$@" > $out/kt_bench.json 2> $out/kt.err
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out/pmc_fetch -o run -- \
  python3 bench.py --no-cpu --steps 2 --warmup 1 "$@" > $out/pmc_fetch_bench.json 2> $out/pmc_fetch.err
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $out/pmc_write -o run -- \
  python3 bench.py --no-cpu --steps 2 --warmup 1 "$@" > $out/pmc_write_bench.json 2> $out/pmc_write.err
echo done
