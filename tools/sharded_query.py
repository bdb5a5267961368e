#!/usr/bin/env python3
"""The bench query on an in-process rank group (LocalComm, N contexts on one GPU): per-rank
host waits, speculated hops, device and exchange time (GPU box only).

    python3 tools/sharded_query.py --world 8 --scale 20 --option wait_trace=1
"""
import argparse
import json
import sys
import time
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--scale", type=int, default=20)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--option", action="append", default=[])
    ap.add_argument("--paths", type=int, default=0, help="also run this many shortest-path pairs")
    args = ap.parse_args()
    import numpy as np
    from nebula_amd import GraphSpace, synth
    from nebula_amd import expr as X
    W = args.world
    sps = [GraphSpace(64, device=0, rank=r, world_size=W) for r in range(W)]
    for s in sps:
        s.comm_init_local(4242)
        for kv in args.option:
            k, v = kv.split("=")
            s.set_option(k, int(v))
        s.set_edge_schema(1, [("weight", 2)])
    pool = ThreadPoolExecutor(max_workers=W)

    def each(fn):
        return [f.result(timeout=600) for f in [pool.submit(fn, r, s) for r, s in enumerate(sps)]]

    t0 = time.time()
    each(lambda r, s: s.gen_rmat(args.scale, 16, 1, 1))
    each(lambda r, s: s.finalize())
    print(f"build {time.time() - t0:.2f} s", flush=True)
    starts = synth.seeds(args.scale, 16, 1, 64)
    w = X.AliasProp("follow", "weight") > 499
    for i in range(args.reps):
        t = time.perf_counter()
        res = each(lambda r, s: s.go(starts, 3, 1, where=w, yields=[X.EdgeDst("follow")], distinct=True))
        wall = (time.perf_counter() - t) * 1e3
        tim = each(lambda r, s: s.last_timing())
        rows = sum(x.n_rows for x in res)
        print(json.dumps({"rep": i, "wall_ms": round(wall, 3), "rows": rows,
                          "host_waits": [x["host_waits"] for x in tim], "spec_hops": [x["spec_hops"] for x in tim],
                          "device_ms": [round(x["total_ms"], 3) for x in tim],
                          "comm_ms": [round(x["comm_ms"], 3) for x in tim],
                          "modes": [h["mode"] for h in tim[0]["hops"]]}), flush=True)
    if args.paths:
        s_, t_ = synth.pairs(args.scale, 16, 1, args.paths)
        for i in range(2):
            t = time.perf_counter()
            each(lambda r, sp: sp.shortest_path(s_, t_, 1, 8))
            tim = each(lambda r, s: s.last_timing())
            print(json.dumps({"paths_rep": i, "wall_ms": round((time.perf_counter() - t) * 1e3, 3),
                              "device_ms": [round(x["total_ms"], 3) for x in tim]}), flush=True)
    for s in sps:
        s.close()


if __name__ == "__main__":
    main()
