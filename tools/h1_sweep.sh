#!/bin/bash
# C3 option sets under rocprofv3 (averaged timed-query timelines) and one C4 batch timeline
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/h1b
cd /tmp && export TMPDIR=/tmp
i=0
for o in "compact_grid=1024" "compact_grid=2048" "compact_grid=4096" "compact_grid=8192"; do
  i=$((i+1))
  opts=""
  for kv in ${o//,/ }; do opts="$opts --option $kv"; done
  timeout -k 10 240 rocprofv3 --kernel-trace -d /tmp/h1p$i -o run -- \
    python3 $R/bench.py --steps 10 --warmup 3 --no-cpu --no-parity $opts > $R/gpurun_out/h1b/b$i.json
  python3 $R/tools/db_timeline.py $(find /tmp/h1p$i -name '*.db' | head -1) nbg::k_publish 4 9 > $R/gpurun_out/h1b/t$i.txt
  rm -rf /tmp/h1p$i
  echo "$i $o" >> $R/gpurun_out/h1b/index.txt
done
timeout -k 10 240 rocprofv3 --kernel-trace -d /tmp/c4p -o run -- \
  python3 $R/bench.py --workload paths --steps 10 --warmup 3 --no-cpu --no-parity > $R/gpurun_out/h1b/c4.json
python3 $R/tools/db_timeline.py $(find /tmp/c4p -name '*.db' | head -1) nbg::k_dv_clear 4 9 > $R/gpurun_out/h1b/c4_t.txt
rm -rf /tmp/c4p
