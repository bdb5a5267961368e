#!/bin/bash
# C4 (1024-pair FIND SHORTEST PATH, RMAT-26) evidence for one tree: rocprofv3 kernel statistics,
# then one --pmc pass per counter group (each its own run and time limit), summarised per kernel
# and per dispatch of the scan kernels.  Usage: tools/c4_counters.sh <tag> [bench args]
set -e
tag=${1:-r09a}; shift || true
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/kt -o run -- \
  python3 bench.py --no-cpu --workload paths --steps 5 --warmup 1 "$@" > $out/kt_bench.json 2> $out/kt.err
cp $out/kt/run_kernel_stats.csv $out/c4_kernel_stats.csv
rm -rf $out/kt
bash tools/pmc_passes.sh $out/pmc "FETCH_SIZE" "WRITE_SIZE" \
  "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum" \
  "TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TA_BUSY_avr" \
  -- bench.py --no-cpu --workload paths --steps 1 --warmup 1 "$@"
python3 tools/pmc_summary.py --dispatch 'k_(sp|dv)_(sweep|probe|expand|walk_scan)' $(find $out/pmc -name "*counter_collection.csv" | sort) \
  > $out/pmc/dispatch.txt
find $out/pmc -name "*.db" -delete 2>/dev/null || true
echo done
