#!/bin/bash
# Per-kernel durations of the bench query under several option sets (rocprofv3 kernel trace,
# one run each).  Usage: tools/prof_sweep.sh <out-dir> "<opts1>" "<opts2>" ...  where an opts
# string is space-separated key=value engine options ("" = defaults).
set -e
out=$1; shift
mkdir -p $out
export TMPDIR=/tmp
i=0
for cfg in "$@"; do
  args=""
  for kv in $cfg; do args="$args --option $kv"; done
  timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d $out/c$i -o run -- \
    python3 tools/run_query.py --reps 4 $args > $out/c$i.json 2> $out/c$i.err
  echo "$i: $cfg" >> $out/configs.txt
  i=$((i+1))
done
echo done
