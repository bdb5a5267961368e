#!/bin/bash
# A/B bench lines of one workload: tools/r12_ab.sh <tag> <reps> "<variant A args>" "<variant B args>" [common bench args]
# Alternates A and B reps times (box drift hits both), one JSON line per run into gpurun_out/<tag>/ab.jsonl
tag=$1; reps=$2; A=$3; B=$4; shift 4
out=gpurun_out/$tag; mkdir -p $out
for i in $(seq 1 $reps); do
  for v in A B; do
    args=$A; [ $v = B ] && args=$B
    timeout -k 10 200 python3 bench.py --no-cpu --no-parity $args "$@" > $out/ab_$v$i.json 2> $out/ab_$v$i.err || exit 1
    python3 - "$out/ab_$v$i.json" "$v" "$args" >> $out/ab.jsonl <<'PY'
import json, sys
L = [l for l in open(sys.argv[1]) if l.startswith("{")]
d = json.loads(L[-1])
r = d.get("roofline") or {}
print(json.dumps({"variant": sys.argv[2], "args": sys.argv[3], "ms": d["ms_per_step"], "value": d["value"],
                  "device_ms": r.get("device_ms_per_query"), "dom_ms": r.get("launch_ms"),
                  "dom_frac": r.get("frac")}))
PY
  done
done
