#!/bin/bash
# rocprofv3 kernel statistics + the kernel timeline of the last query of a bench run.
# Usage: tools/kt_timeline.sh <tag> <timeline launches> [bench args]
tag=$1; n=$2; shift 2
out=gpurun_out/$tag; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/kt -o run -- \
  python3 bench.py --no-cpu --steps 5 --warmup 1 "$@" > $out/kt_bench.json 2> $out/kt.err || exit 1
cp $out/kt/run_kernel_stats.csv $out/kernel_stats.csv
python3 tools/timeline.py $out/kt/run_kernel_trace.csv $n > $out/timeline.txt
cp $out/kt/run_kernel_trace.csv $out/kernel_trace.csv
rm -rf $out/kt
