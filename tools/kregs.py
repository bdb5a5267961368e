#!/usr/bin/env python3
"""Per-kernel VGPRs / scratch / occupancy from hipcc -Rpass-analysis=kernel-resource-usage output.

    hipcc ... -Rpass-analysis=kernel-resource-usage > remarks.txt 2>&1; python tools/kregs.py remarks.txt [filter]"""
import re
import subprocess
import sys

cur, rows = None, []
for line in open(sys.argv[1]):
    m = re.search(r"remark: Function Name: (\S+)", line)
    if m:
        cur = {"name": m.group(1)}
        rows.append(cur)
        continue
    m = re.search(r"remark:\s+(VGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|TotalSGPRs): (\d+)", line)
    if m and cur is not None:
        cur[m.group(1).split()[0]] = int(m.group(2))
flt = sys.argv[2] if len(sys.argv) > 2 else ""
names = [r["name"] for r in rows]
dem = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True).stdout.split("\n")
for r, d in zip(rows, dem):
    if flt in d:
        print(f"{r.get('VGPRs', '?'):>4} vgpr {r.get('ScratchSize', '?'):>4} scratch occ {r.get('Occupancy', '?')}  {d.split('(')[0]}")
