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
    ref = None
    for cfg in [""] + args.config:
        opts = dict(kv.split("=") for kv in cfg.split(",") if kv)
        for k, v in opts.items():
            sp.set_option(k, int(v))
        ms, rows = [], None
        for _ in range(args.reps):
            t = time.perf_counter()
            r = sp.go(starts, args.hops, 1, where=where, yields=[X.EdgeDst("follow")], distinct=True,
                      keep_on_device=True)
            ms.append((time.perf_counter() - t) * 1e3)
            rows = r.n_rows
        tm = sp.last_timing()
        if ref is None:
            ref = rows
        print(json.dumps({"config": cfg or "default", "ms_median": statistics.median(ms), "ms_min": min(ms),
                          "rows": rows, "rows_ok": rows == ref, "edges": r.edges_scanned,
                          "hops": [(h["mode"], round(h["ms"], 4), h["c"]) for h in tm["hops"]]}), flush=True)
        for k in opts:  # back to defaults
            sp.set_option(k, {"bu_r": 2, "bu_eager_fast": 1, "bu_eager": 1, "bu_nt": 0, "bu_defer": 0, "bu_grid": 4096,
                              "bu_tiles_per_wave": 4, "bu_lds_kb": 0, "bu_lds_grid": 512, "bu_div": 4, "bu_slab": 4}.get(k, 0))
    sp.close()


if __name__ == "__main__":
    main()
