"""Kernel timeline of the last N launches of a rocprofv3 --kernel-trace CSV: start offset, the
idle gap before each launch (host round trips show up here) and its duration, in microseconds.
Usage: python tools/timeline.py <kernel_trace.csv> [N] > timeline.txt"""
import csv
import sys


def main():
    path = sys.argv[1]
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 80
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))[-n:]
    t0 = int(rows[0]["Start_Timestamp"])
    prev = None
    busy = idle = 0.0
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        gap = (s - prev) / 1e3 if prev is not None else 0.0
        idle += max(gap, 0.0)
        busy += (e - s) / 1e3
        name = r["Kernel_Name"][:100]
        print(f"{(s - t0) / 1e3:10.1f} gap {gap:8.1f} dur {(e - s) / 1e3:8.1f}  {name}")
        prev = e
    print(f"# busy {busy:.1f} us, idle {idle:.1f} us over the last {len(rows)} launches")


if __name__ == "__main__":
    main()
