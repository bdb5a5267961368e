#!/usr/bin/env python3
"""Print the query kernels' average durations of a tools/prof_sweep.sh run, one block per config."""
import csv
import sys
from pathlib import Path

out = Path(sys.argv[1])
keys = ("k_bu_", "k_bits", "k_reduce", "k_expand", "k_compact", "k_degrees", "k_sp_")
for line in (out / "configs.txt").read_text().splitlines():
    i, cfg = line.split(":", 1)
    f = out / f"c{i}" / "run_kernel_stats.csv"
    print(f"== [{i}] {cfg.strip() or 'defaults'}")
    if not f.exists():
        print("   (no stats)")
        continue
    tot = 0.0
    for r in sorted(csv.DictReader(open(f)), key=lambda r: -float(r["TotalDurationNs"])):
        n = r["Name"]
        if any(k in n for k in keys):
            us = float(r["AverageNs"]) / 1e3
            print(f"   {r['Calls']:>4} x {us:8.1f} us  {n.split('(')[0][:80]}")
