#!/usr/bin/env python3
"""Debug aid: FIND SHORTEST PATH on `world` in-process ranks (LocalComm, one GPU), the
device-driven batches (sp_dev = 1, walk errors not fatal) against the host-driven path (sp_dev = 0)
pair by pair.  Usage: python tools/sp_debug.py <scale> <world> [pairs] [option=value ...]"""
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "tests"))
from test_gpu_multirank import Group  # noqa: E402
from nebula_amd import synth  # noqa: E402

scale, world = int(sys.argv[1]), int(sys.argv[2])
npairs = int(sys.argv[3]) if len(sys.argv) > 3 else 1024
seq = "seq" in sys.argv[4:]
opts = [a.split("=") for a in sys.argv[4:] if "=" in a]
g = Group(world)
for s in g.sp:
    s.set_edge_schema(1, [("weight", 2)])
g.each(lambda r, s: s.gen_rmat(scale, 16, 1, 1))
g.each(lambda r, s: s.finalize())
src, dst = synth.pairs(scale, 16, 1, npairs)
for k, v in opts:
    g.each(lambda r, s: s.set_option(k, int(v)))
# the first call on every rank together: it assembles the replicated CSRs (collectives)
g.each(lambda r, s: s.shortest_path(src[:1], dst[:1], 1, 8))


def run(dev):
    g.each(lambda r, s: s.set_option("sp_dev", dev))
    g.each(lambda r, s: s.set_option("sp_dv_diag", 4))
    if seq:  # one rank after the other (no concurrent contexts on the device)
        res, tim = [], []
        for s in g.sp:
            res.append(s.shortest_path(src, dst, 1, 8))
            tim.append(s.last_timing())
    else:
        res = g.each(lambda r, s: s.shortest_path(src, dst, 1, 8))
        tim = g.each(lambda r, s: s.last_timing())
    out = {}
    for r, p in enumerate(res):
        for j in range(len(p.hops)):
            out[r + j * world] = (int(p.hops[j]), tuple(int(x) for x in p.paths[j]))
    return out, tim


for rep in range(2):
    a, ta = run(1)
    b, tb = run(0)
    bad = [i for i in range(npairs) if a[i] != b[i]]
    print(f"rep {rep}: {len(bad)} of {npairs} pairs differ; dev batches {[t['spec_hops'] for t in ta]}", flush=True)
    for i in bad[:10]:
        print("  pair", i, "rank", i % world, "dev", a[i], "host", b[i])
g.close()
