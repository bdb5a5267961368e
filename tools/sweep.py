#!/usr/bin/env python3
"""Option sweep of the GO benchmark query on one graph build (tuning aid, GPU box only).

    python tools/sweep.py --scale 26 --config bu_r=1,bu_eager_fast=2 --config bu_nt=1 ...

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

# engine defaults of the swept options (traverse.hip / snapshot.hip), restored after each config
DEFAULTS = {"bu_r": 2, "bu_eager_fast": 1, "bu_eager": 1, "bu_nt": 0, "bu_defer": 0, "bu_grid": 4096,
            "bu_tiles_per_wave": 4, "bu_lds_kb": 0, "bu_lds_grid": 512, "bu_div": 4, "bu_slab": 4,
            "bu_lazy": 3, "bu_unroll": 1, "bu_wpe": 8, "bu_kernel": 2, "bu_lean_u": 1, "bu_lean_grid": 2048, "bu_lean_lds_kb": 64, "bu_lean_lds_kb_final": 64, "bu_lean_u_final": 1, "bu_rest_lds_kb": 0, "bu_rest_lds_kb_final": 64, "bu_rest_steps": 4, "bu_pair_eh": 1,
            "bu_pair_lds_kb": 64, "bu_pair_grid": 512, "bu_pair_defer": 1, "bu_pair_defer_final": 1,
            "bu_rest_grid": 512, "bu_pair_r": 1, "bu_rest_occ": 8, "bu_qpred": 1, "bu_pair_diag": 0,
            "bu_ring": 0, "bu_ring_lds_kb": 128, "bu_ring_grid": 256, "fuse_dst": 1, "mark_check": 0,
            "expand_grid": 2048, "rest_grid": 2048}


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
            saved = {k: DEFAULTS.get(k, 0) for k in opts}
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
            for k, v in saved.items():
                sp.set_option(k, v)
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
