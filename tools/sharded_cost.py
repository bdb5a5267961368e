#!/usr/bin/env python3
"""Multi-GPU cost evidence a one-GPU lease can produce (GPU box only).

C3 (GO 3 STEPS ... YIELD DISTINCT, RMAT-26) on an in-process rank group of W contexts on the one
GPU (LocalComm: the RCCL call sequence with device-to-device copies): per rank the hop records
(direction, frontier / found counts, bytes of the byte model), device time, exchange time and
bytes, host waits.  The W ranks share one GPU here, so their kernel times are contention-bound;
the per-rank BYTES are what a rank of a W-GPU run would move.

C4 (1024-pair FIND SHORTEST PATH, RMAT-26): pairs are sharded i % W over replicated CSRs with no
collective in the traversal, so rank r of a W-GPU run answers exactly the pairs r, r + W, ...
on a full replica: timed here on the one GPU, alone, for rank 0's subset at W = 1, 2, 4, 8.

    python3 tools/sharded_cost.py --scale 26 --worlds 2 4 8 > gpurun_out/<tag>/sharded.jsonl
"""
import argparse
import json
import sys
import time
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def emit(d):
    print(json.dumps(d), flush=True)


def c4_subsets(scale, worlds, steps):
    from nebula_amd import GraphSpace, synth
    sp = GraphSpace(64)
    sp.set_edge_schema(1, [("weight", 2)])
    sp.gen_rmat(scale, 16, 1, 1)
    sp.finalize()
    s, t = synth.pairs(scale, 16, 1, 1024)
    for w in [1] + list(worlds):
        for r in sorted({0, w - 1}):
            ss, tt = s[r::w], t[r::w]
            for _ in range(2):
                sp.shortest_path(ss, tt, 1, 8)
            sp.set_option("hop_timing", 0)
            t0 = time.perf_counter()
            for _ in range(steps):
                res = sp.shortest_path(ss, tt, 1, 8)
            wall = (time.perf_counter() - t0) / steps * 1e3
            sp.unset_option("hop_timing")
            sp.shortest_path(ss, tt, 1, 8)
            tm = sp.last_timing()
            emit({"c4": True, "world": w, "rank": r, "pairs": len(ss), "ms_per_batch": round(wall, 4),
                  "device_ms": round(tm["total_ms"], 4), "host_waits": tm["host_waits"],
                  "dev_batches": tm["spec_hops"], "edges_examined": int(res.edges_scanned),
                  "scan_ms": round(sum(h["ms"] for h in tm["hops"]), 4),
                  "launches": [(h["mode"], round(h["ms"], 4), h["c"][1]) for h in tm["hops"]]})
    sp.close()


def c3_group(scale, world, reps):
    from nebula_amd import GraphSpace, synth
    from nebula_amd import expr as X
    sps = [GraphSpace(64, device=0, rank=r, world_size=world) for r in range(world)]
    for s in sps:
        s.comm_init_local(7000 + world)
        s.set_edge_schema(1, [("weight", 2)])
    pool = ThreadPoolExecutor(max_workers=world)

    def each(fn):
        return [f.result(timeout=600) for f in [pool.submit(fn, r, s) for r, s in enumerate(sps)]]

    t0 = time.time()
    each(lambda r, s: s.gen_rmat(scale, 16, 1, 1))
    each(lambda r, s: s.finalize())
    build = time.time() - t0
    infos = each(lambda r, s: s.info(1))
    starts = synth.seeds(scale, 16, 1, 64)
    w = X.AliasProp("follow", "weight") > 499
    for i in range(reps):
        t = time.perf_counter()
        res = each(lambda r, s: s.go(starts, 3, 1, where=w, yields=[X.EdgeDst("follow")], distinct=True,
                                     keep_on_device=True))
        wall = (time.perf_counter() - t) * 1e3
        tim = each(lambda r, s: s.last_timing())
        if i < reps - 1:
            continue
        ranks = []
        for r, (x, inf) in enumerate(zip(tim, infos)):
            ranks.append({"rank": r, "local_vertices": inf["local_vertices"],
                          "local_out_edges": inf["local_out_edges"], "rows": int(res[r].n_rows),
                          "device_ms": round(x["total_ms"], 4), "comm_ms": round(x["comm_ms"], 4),
                          "comm_bytes": int(x["comm_bytes"]), "comm_calls": x.get("comm_calls"),
                          "host_waits": x["host_waits"],
                          "spec_hops": x["spec_hops"],
                          "hops": [{"mode": h["mode"], "final": h["final"], "ms": round(h["ms"], 4),
                                    "kernel_ms": round(h["kernel_ms"], 4), "bytes": h["bytes"],
                                    "kernel_bytes": h["kernel_bytes"], "c": h["c"][:4]} for h in x["hops"]]})
        emit({"c3": True, "world": world, "scale": scale, "build_s": round(build, 2), "wall_ms": round(wall, 3),
              "rows": sum(int(x.n_rows) for x in res), "ranks": ranks})
    for s in sps:
        s.close()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=int, default=26)
    ap.add_argument("--worlds", type=int, nargs="+", default=[2, 4, 8])
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--skip-c3", action="store_true")
    ap.add_argument("--skip-c4", action="store_true")
    args = ap.parse_args()
    if not args.skip_c4:
        c4_subsets(args.scale, args.worlds, args.steps)
    if not args.skip_c3:
        for w in args.worlds:
            c3_group(args.scale, w, args.reps)


if __name__ == "__main__":
    main()
