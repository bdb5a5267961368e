#!/bin/bash
# C4 bench lines under option variants (one bench process each, its own time limit; stops at the
# first failure).  Usage: tools/bench_variants.sh <tag> "<opt=v ...>" "<opt=v ...>" ...
# ("-" = defaults).  Prints ms/query, parity and the per-launch times of each.
tag=$1; shift
out=gpurun_out/$tag; mkdir -p $out
i=0
for v in "$@"; do
  i=$((i+1))
  args=""
  [ "$v" != "-" ] && for o in $v; do args="$args --option $o"; done
  timeout -k 10 300 python3 bench.py --no-cpu --workload paths --steps 10 --warmup 2 $args > $out/v$i.json 2> $out/v$i.err || exit 1
  python3 - "$out/v$i.json" "$v" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
ls = d["config"]["launches"]
print(f"{sys.argv[2]:40s} {d['ms_per_step']:.4f} ms dev {d['roofline']['device_ms_per_query']:.4f} {d['parity']['status']}",
      " ".join(f"{l['kind'][0]}{l['iter']}={l['ms']:.3f}" for l in ls))
PY
done
