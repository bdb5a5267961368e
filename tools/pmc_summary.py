#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc counter_collection CSVs per kernel (mean per dispatch)."""
import csv
import sys
from collections import defaultdict


def main():
    acc = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    for path in sys.argv[1:]:
        with open(path) as f:
            for r in csv.DictReader(f):
                k = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0][:60]
                acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
                disp[k].add(r["Dispatch_Id"])
    rows = sorted(acc.items(), key=lambda kv: -max(kv[1].values()))
    for k, cs in [r for r in rows if len(sys.argv) < 3 or True][:60]:
        n = len(disp[k])
        print(f"{k:60s} n={n:3d} " + " ".join(f"{c}={v / n:.4g}" for c, v in sorted(cs.items())))


if __name__ == "__main__":
    main()
