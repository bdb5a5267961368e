#!/bin/bash
# PMC counter passes over the bench query (one rocprofv3 --pmc run per pass, each under its own
# time limit; stops at the first run that was killed or crashed).  Usage:
#   tools/pmc_diag.sh <out-dir> "<engine opts>" "<pass1 counters>" "<pass2 counters>" ...
out=$1; shift
opts=$1; shift
mkdir -p $out
export TMPDIR=/tmp
args=""
for kv in $opts; do args="$args --option $kv"; done
i=0
for pass in "$@"; do
  timeout -s KILL 90 rocprofv3 --pmc $pass --output-format csv -d $out/p$i -o run -- \
    python3 tools/run_query.py --reps 2 $args > $out/p$i.json 2> $out/p$i.err
  rc=$?
  echo "$i rc=$rc: $pass" >> $out/passes.txt
  case $rc in 124|134|137|139) echo "pass $i ended with $rc, stopping"; exit $rc;; esac
  i=$((i+1))
done
echo done
