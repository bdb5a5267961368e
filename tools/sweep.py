#!/usr/bin/env python3
"""Option sweep of the GO benchmark query on one graph build (tuning aid, GPU box only).

    python tools/sweep.py --scale 26 --config bu_lean_u_final=2 --config bu_rest_steps=2 ...

Each --config is a comma list of engine options applied on top of the defaults; every config
runs the BASELINE query `reps` times and prints one JSON line (median ms, hop stats)."""
import argparse
import json
import statistics
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=int, default=26)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--hops", type=int, default=3)
    ap.add_argument("--where", type=int, default=499)
    ap.add_argument("--config", action="append", default=[])
    args = ap.parse_args()
    from nebula_amd import GraphSpace, synth
    from nebula_amd import expr as X
    sp = GraphSpace(64)
    sp.set_edge_schema(1, [("weight", 2)])
    t0 = time.time()
    sp.gen_rmat(args.scale, 16, 1, 1)
    sp.finalize()
    print(json.dumps({"build_s": time.time() - t0}), flush=True)
    starts = synth.seeds(args.scale, 16, 1, 64)
    where = X.AliasProp("follow", "weight") > args.where
    cfgs = [""] + args.config
    # interleaved: every rep runs each config once, so clock / neighbour drift hits all alike
    ms = {c: [] for c in cfgs}
    hop_ms = {c: [] for c in cfgs}
    kern_ms = {}
    res = {}
    for _ in range(args.reps):
        for cfg in cfgs:
            opts = dict(kv.split("=") for kv in cfg.split(",") if kv)
            for k, v in opts.items():
                sp.set_option(k, int(v))
            t = time.perf_counter()
            r = sp.go(starts, args.hops, 1, where=where, yields=[X.EdgeDst("follow")], distinct=True,
                      keep_on_device=True)
            ms[cfg].append((time.perf_counter() - t) * 1e3)
            tm = sp.last_timing()
            hop_ms[cfg].append([h["ms"] for h in tm["hops"]])
            kern_ms.setdefault(cfg, []).append([h["kernel_ms"] for h in tm["hops"]])
            res[cfg] = (r.n_rows, r.edges_scanned, tm)
            sp.reset_options()  # engine defaults again
    ref = res[""][0]
    for cfg in cfgs:
        rows, edges, tm = res[cfg]
        hops = [round(statistics.median(h[i] for h in hop_ms[cfg]), 4) for i in range(len(hop_ms[cfg][0]))]
        kms = [round(statistics.median(h[i] for h in kern_ms[cfg]), 4) for i in range(len(kern_ms[cfg][0]))]
        print(json.dumps({"config": cfg or "default", "ms_median": statistics.median(ms[cfg]), "ms_min": min(ms[cfg]),
                          "rows": rows, "rows_ok": rows == ref, "edges": edges, "hop_ms_median": hops,
                          "kernel_ms_median": kms,
                          "hops": [(h["mode"], h["c"]) for h in tm["hops"]]}), flush=True)
    sp.close()


if __name__ == "__main__":
    main()
