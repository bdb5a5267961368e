#!/bin/bash
# One GPU-box session for a round's committed profiles: the default bench line (C3) with
# rocprofv3 kernel stats and the FETCH_SIZE / WRITE_SIZE passes (tools/gpu_profile.sh), then
# kernel stats + bench lines of C2 (RMAT-22 plain rows), C4 (1024 pairs FIND SHORTEST PATH) and
# C5 (RMAT-28 GO 2 STEPS with supernode seeds).  Usage: tools/profile_round.sh <tag>
set -e
tag=${1:-r03p}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
bash tools/gpu_profile.sh $tag
stats() {  # name, bench args...
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/kt_$name -o run -- \
    python3 bench.py --no-cpu "$@" > $out/${name}_bench.json 2> $out/${name}.err
  cp $out/kt_$name/run_kernel_stats.csv $out/${name}_kernel_stats.csv
  rm -rf $out/kt_$name
}
stats c2 --plain --scale 22 --steps 10 --warmup 2
stats c4 --workload paths --steps 5 --warmup 1
stats c5 --plain --scale 28 --hops 2 --hubs 8 --steps 5 --warmup 1
rm -rf $out/kt/*.db $out/pmc_fetch/*.db $out/pmc_write/*.db 2>/dev/null || true
echo done
