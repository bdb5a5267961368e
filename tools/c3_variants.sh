#!/bin/bash
# C3 bench lines under option variants (one bench process each, its own time limit; stops at the
# first failure).  Usage: tools/c3_variants.sh <tag> "<opt=v ...>" ... ("-" = defaults)
tag=$1; shift
out=gpurun_out/$tag; mkdir -p $out
i=0
for v in "$@"; do
  i=$((i+1))
  args=""
  [ "$v" != "-" ] && for o in $v; do args="$args --option $o"; done
  timeout -k 10 300 python3 bench.py --no-cpu --steps 20 --warmup 3 $args > $out/g$i.json 2> $out/g$i.err || exit 1
  python3 - "$out/g$i.json" "$v" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
hs = d["roofline"]["hops"]
print(f"{sys.argv[2]:40s} {d['ms_per_step']:.4f} ms {d['parity']['status']} frac {d['roofline']['frac']:.3f}",
      " ".join(f"{h['mode'][0]}={h['ms']:.4f}/{h['kernel_ms']:.4f}" for h in hs))
PY
done
