#!/usr/bin/env python3
"""Run the bench query a few times with engine options (profiling driver, GPU box only).

    rocprofv3 --kernel-trace --stats -d gpurun_out/p -- python3 tools/run_query.py --option bu_rest_steps=2

The graph build happens before the timed queries; rocprof summaries of the run include both, so
tools/profile_summary.py separates query kernels from build kernels by call count."""
import argparse
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=int, default=26)
    ap.add_argument("--reps", type=int, default=6)
    ap.add_argument("--hops", type=int, default=3)
    ap.add_argument("--where", type=int, default=499)
    ap.add_argument("--plain", action="store_true")
    ap.add_argument("--option", action="append", default=[])
    args = ap.parse_args()
    from nebula_amd import GraphSpace, synth
    from nebula_amd import expr as X
    sp = GraphSpace(64)
    for kv in args.option:
        k, v = kv.split("=")
        sp.set_option(k, int(v))
    sp.set_edge_schema(1, [("weight", 2)])
    sp.gen_rmat(args.scale, 16, 1, 1)
    sp.finalize()
    starts = synth.seeds(args.scale, 16, 1, 64)
    where = None if args.plain else X.AliasProp("follow", "weight") > args.where
    ms = []
    for _ in range(args.reps):
        t = time.perf_counter()
        r = sp.go(starts, args.hops, 1, where=where, yields=[X.EdgeDst("follow")], distinct=not args.plain,
                  keep_on_device=True)
        ms.append((time.perf_counter() - t) * 1e3)
    tm = sp.last_timing()
    print(json.dumps({"options": args.option, "ms": ms, "rows": r.n_rows,
                      "hops": [(h["mode"], round(h["ms"], 4), round(h["kernel_ms"], 4), h["c"]) for h in tm["hops"]]}))
    sp.close()


if __name__ == "__main__":
    main()
