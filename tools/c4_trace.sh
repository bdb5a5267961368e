#!/bin/bash
# C4 kernel trace + the timeline of one timed-loop query: tools/c4_trace.sh <tag> [bench args]
tag=$1; shift
out=gpurun_out/$tag; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/kt -o run -- \
  python3 bench.py --workload paths --no-cpu --steps 5 --warmup 1 "$@" > $out/kt_bench.json 2> $out/kt.err || exit 1
cp $out/kt/run_kernel_stats.csv $out/kernel_stats.csv
python3 tools/query_timeline.py $out/kt/run_kernel_trace.csv k_dv_begin 3 > $out/timeline.txt
rm -rf $out/kt
