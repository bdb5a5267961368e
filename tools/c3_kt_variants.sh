#!/bin/bash
# C3 kernel timelines under option variants: one rocprofv3 kernel-trace run each (its own time
# limit), printing the middle timed query's launches.  Usage: tools/c3_kt_variants.sh <tag> "<opt=v ...>" ...
tag=$1; shift
out=gpurun_out/$tag; mkdir -p $out
export TMPDIR=/tmp
i=0
for v in "$@"; do
  i=$((i+1))
  args=""
  [ "$v" != "-" ] && for o in $v; do args="$args --option $o"; done
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $out/kt$i -o run -- \
    python3 bench.py --no-cpu --steps 10 --warmup 2 $args > $out/kt$i.json 2> $out/kt$i.err || exit 1
  echo "== $v"
  python3 tools/query_timeline.py $out/kt$i/run_kernel_trace.csv k_starts_small
  rm -rf $out/kt$i
done
