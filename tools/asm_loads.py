#!/usr/bin/env python3
"""Count memory instruction kinds per kernel in a hipcc -S device assembly file.

    hipcc ... --offload-device-only -S csrc/traverse.hip -o /tmp/tr.s; python tools/asm_loads.py /tmp/tr.s k_bu_quad"""
import re
import sys

text = open(sys.argv[1]).read()
flt = sys.argv[2] if len(sys.argv) > 2 else ""
kinds = ["flat_load", "global_load", "ds_read", "ds_write", "global_store", "flat_store", "s_waitcnt", "scratch_"]
for m in re.finditer(r"\n(_Z\w+):[^\n]*\n(.*?)\n\s+\.size\s", text, re.S):
    name, body = m.group(1), m.group(2)
    if flt not in name:
        continue
    c = {k: len(re.findall(r"\n\s+" + k, body)) for k in kinds}
    print(f"{name[:70]:70s} " + " ".join(f"{k}={v}" for k, v in c.items() if v))
