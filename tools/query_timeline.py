#!/usr/bin/env python3
"""Kernel timeline of one query of a rocprofv3 --kernel-trace CSV: queries start at each launch of
the marker kernel; prints query q (default: the middle one, a timed-loop query of bench.py, which
runs without per-hop event pairs) with each launch's start offset, idle gap before it and duration.
Usage: python tools/query_timeline.py <kernel_trace.csv> <marker substring> [q]"""
import csv
import sys


def main():
    path, marker = sys.argv[1], sys.argv[2]
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
    q = int(sys.argv[3]) if len(sys.argv) > 3 else len(starts) // 2
    a = starts[q]
    b = starts[q + 1] if q + 1 < len(starts) else len(rows)
    t0 = int(rows[a]["Start_Timestamp"])
    prev = None
    busy = idle = 0.0
    for r in rows[a:b]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        gap = (s - prev) / 1e3 if prev is not None else 0.0
        if prev is not None and gap > 40.0:  # the host's time between two queries
            break
        idle += max(gap, 0.0)
        busy += (e - s) / 1e3
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
        print(f"{(s - t0) / 1e3:9.1f} gap {gap:7.1f} dur {(e - s) / 1e3:8.1f}  {name}")
        prev = e
    print(f"# query {q} of {len(starts)}: busy {busy:.1f} us, idle {idle:.1f} us, span {(prev - t0) / 1e3:.1f} us")


if __name__ == "__main__":
    main()
