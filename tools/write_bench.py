"""Write-path cost on the RMAT snapshot: a writable snapshot takes a batch of
AddEdges puts (out-edge key + weight row, in-edge key + empty row, version INT64_MAX - 1 - 1 so
it is the newest version, AddEdgesProcessor.cpp:15-31) through nbg_snapshot_write_part, then
nbg_snapshot_commit rebuilds the CSRs from the device-resident log.  Prints one JSON line with
the initial build, the write-batch decode and the commit times, and GO 3 STEPS before / after.

    python tools/write_bench.py --scale 24 --edges 1048576
    python tools/write_bench.py --scale 26 --new-frac 0.1 --world 2   # in-process rank group

With --world N the snapshot is sharded part % N over N contexts on one GPU (LocalComm); each
rank takes the batches of its own parts and every rank commits (collective).
"""
import argparse
import json
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nebula_amd import GraphSpace, synth  # noqa: E402

PARTS, FOLLOW, SEED = 64, 1, 1
KEY = np.dtype([("part", "<i4"), ("src", "<i8"), ("type", "<i4"), ("rank", "<i8"), ("dst", "<i8"),
                ("ver", "<i8")])


def varint_rows(w):
    """RowWriter row of schema (weight int): header byte 0 + LEB128 varint (w < 2^14)."""
    lo = (w & 0x7F) | np.where(w >= 128, 0x80, 0)
    hi = w >> 7
    n = np.where(w >= 128, 3, 2).astype(np.uint64)
    out = np.zeros((len(w), 3), np.uint8)
    out[:, 1] = lo
    out[:, 2] = hi
    mask = np.ones((len(w), 3), bool)
    mask[:, 2] = w >= 128
    return out[mask], np.concatenate([[0], np.cumsum(n)]).astype(np.uint64)


def batches(src, dst, w, ver):
    out = {}
    for s, d, et, with_val in ((src, dst, FOLLOW, True), (dst, src, -FOLLOW, False)):
        part = (s.astype(np.uint64) % np.uint64(PARTS) + np.uint64(1)).astype(np.int32)
        for p in np.unique(part):
            sel = part == p
            k = np.zeros(int(sel.sum()), KEY)
            k["part"], k["src"], k["type"], k["dst"], k["ver"] = p, s[sel], et, d[sel], ver
            kb = np.frombuffer(k.tobytes() + b"\0", np.uint8)
            koff = (np.arange(len(k) + 1) * 40).astype(np.uint64)
            if with_val:
                vb, voff = varint_rows(w[sel])
                vb = np.concatenate([vb, [0]]).astype(np.uint8)
            else:
                vb, voff = np.zeros(1, np.uint8), np.zeros(len(k) + 1, np.uint64)
            out.setdefault(int(p), []).append((kb, koff, vb, voff))
    return out


class Ranks:
    """`world` contexts on device 0 (one per rank); every call runs on all ranks in threads."""

    def __init__(self, world):
        self.sp = [GraphSpace(PARTS, device=0, rank=r, world_size=world) for r in range(world)]
        if world > 1:
            for s in self.sp:
                s.comm_init_local(4711)
        self.pool = ThreadPoolExecutor(max_workers=world)

    def each(self, fn):
        return [f.result(timeout=900) for f in [self.pool.submit(fn, r, s) for r, s in enumerate(self.sp)]]


def go3(g, starts):
    g.each(lambda r, s: s.go(starts, 3, FOLLOW))  # warm
    t = time.perf_counter()
    rs = g.each(lambda r, s: s.go(starts, 3, FOLLOW))
    return (time.perf_counter() - t) * 1e3, sum(x.n_rows for x in rs)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=int, default=24)
    ap.add_argument("--edges", type=int, default=1 << 20)
    ap.add_argument("--trace", action="store_true", help="per-phase build / commit times on stderr")
    ap.add_argument("--commits", type=int, default=1, help="successive write batch + commit rounds")
    ap.add_argument("--new-frac", type=float, default=0.0,
                    help="fraction of the batch's edges whose dst is a brand-new vertex (AddEdges to new vids)")
    ap.add_argument("--world", type=int, default=1, help="ranks of an in-process group on device 0")
    a = ap.parse_args()
    W = a.world
    g = Ranks(W)
    for sp in g.sp:
        sp.set_option("writable", 1)
        if a.trace:
            sp.set_option("build_trace", 1)
        sp.set_edge_schema(FOLLOW, [("weight", 2)])
    t0 = time.perf_counter()
    g.each(lambda r, s: s.gen_rmat(a.scale, 16, SEED, FOLLOW))
    g.each(lambda r, s: s.finalize())
    build_s = time.perf_counter() - t0
    info0 = g.each(lambda r, s: s.info(FOLLOW))
    starts = [int(x) for x in synth.seeds(a.scale, 16, SEED, 1)]
    go_before = go3(g, starts)
    rng = np.random.default_rng(3)
    commit_times, write_times = [], []
    for k in range(a.commits):
        s, _ = synth.pairs(a.scale, 16, SEED, a.edges, pick_seed=5 + 2 * k)
        _, d = synth.pairs(a.scale, 16, SEED, a.edges, pick_seed=6 + 2 * k)
        w = rng.integers(1000, 2000, a.edges)
        d = np.asarray(d, np.int64).copy()
        if a.new_frac > 0:
            sel = rng.random(a.edges) < a.new_frac
            d[sel] = rng.integers(1, 2**62, int(sel.sum()))
        bs = batches(np.asarray(s, np.int64), np.asarray(d, np.int64), w, 2**63 - 3 - k)
        t1 = time.perf_counter()

        def write(r, sp):
            for p, lst in bs.items():
                if p % W == r:
                    for blob in lst:
                        sp.write_part(p, blob)
        g.each(write)
        write_times.append(round(time.perf_counter() - t1, 3))
        t2 = time.perf_counter()
        g.each(lambda r, s: s.commit())
        commit_times.append(round(time.perf_counter() - t2, 3))
    write_s, commit_s = write_times[0], commit_times[0]
    info1 = g.each(lambda r, s: s.info(FOLLOW))
    go_after = go3(g, starts)
    print(json.dumps({
        "workload": f"rmat{a.scale} + {a.commits} x AddEdges batch of {a.edges} edges (out + in keys)"
                    + (f", {a.new_frac:.0%} to new vertices" if a.new_frac > 0 else "")
                    + (f", {W} ranks (in-process group)" if W > 1 else ""),
        "world": W,
        "vertices_before": info0[0].get("num_vertices"), "vertices_after": info1[0].get("num_vertices"),
        "initial_build_s": round(build_s, 3), "write_part_s": round(write_s, 3), "commit_s": round(commit_s, 3),
        "commit_s_each": commit_times, "write_part_s_each": write_times,
        "merge_commits": [i.get("merge_commits") for i in info1],
        "out_edges_before": sum(i["local_out_edges"] for i in info0),
        "out_edges_after": sum(i["local_out_edges"] for i in info1),
        "device_bytes_before": sum(i["device_bytes"] for i in info0),
        "device_bytes_after": sum(i["device_bytes"] for i in info1),
        "go3_ms_before": round(go_before[0], 3), "go3_rows_before": go_before[1],
        "go3_ms_after": round(go_after[0], 3), "go3_rows_after": go_after[1],
    }))
    for sp in g.sp:
        sp.close()


if __name__ == "__main__":
    main()
