#!/bin/bash
# PMC counter passes over any python workload (one rocprofv3 --pmc run per pass, each under its
# own time limit; stops at the first run that was killed or crashed).  Usage:
#   tools/pmc_passes.sh <out-dir> "<pass1 counters>" "<pass2 counters>" ... -- <python args>
out=$1; shift
passes=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do passes+=("$1"); shift; done
shift
mkdir -p $out
export TMPDIR=/tmp
i=0
for pass in "${passes[@]}"; do
  timeout -s KILL 150 rocprofv3 --pmc $pass --output-format csv -d $out/p$i -o run -- python3 "$@" \
    > $out/p$i.out 2> $out/p$i.err
  rc=$?
  echo "$i rc=$rc: $pass" >> $out/passes.txt
  case $rc in 124|134|137|139) echo "pass $i ended with $rc, stopping"; exit $rc;; esac
  i=$((i+1))
done
python3 tools/pmc_summary.py $(find $out -name "*counter_collection.csv") > $out/summary.txt
echo done
