#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc counter_collection CSVs per kernel (mean per dispatch).

    pmc_summary.py CSV...                      one row per kernel (template arguments kept)
    pmc_summary.py --dispatch REGEX CSV...     one row per dispatch of the kernels matching REGEX,
                                               in dispatch order, with the dispatch's duration
"""
import csv
import re
import sys
from collections import defaultdict


def kname(raw: str) -> str:
    return raw.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0][:60]


def main():
    args = sys.argv[1:]
    pat = None
    if args and args[0] == "--dispatch":
        pat = re.compile(args[1])
        args = args[2:]
    acc = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    per = defaultdict(lambda: defaultdict(float))  # (dispatch id, kernel) -> counters
    dur = {}
    for path in args:
        with open(path) as f:
            for r in csv.DictReader(f):
                k = kname(r["Kernel_Name"])
                acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
                disp[k].add(r["Dispatch_Id"])
                if pat and pat.search(k):
                    key = (path, int(r["Dispatch_Id"]), k)
                    per[key][r["Counter_Name"]] += float(r["Counter_Value"])
                    dur[key] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    if pat:
        for key in sorted(per):
            path, d, k = key
            cs = per[key]
            print(f"{path.split('/')[-3] if path.count('/') >= 2 else path} d={d:6d} {k:40s} us={dur[key]:9.2f} "
                  + " ".join(f"{c}={v:.6g}" for c, v in sorted(cs.items())))
        return
    rows = sorted(acc.items(), key=lambda kv: -max(kv[1].values()))
    for k, cs in rows[:60]:
        n = len(disp[k])
        print(f"{k:60s} n={n:3d} " + " ".join(f"{c}={v / n:.4g}" for c, v in sorted(cs.items())))


if __name__ == "__main__":
    main()
