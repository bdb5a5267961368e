#!/usr/bin/env python3
"""Benchmark: GTEPS of GO 3 STEPS on RMAT-26 on N MI355X (BASELINE.json metric).

Workload (BASELINE.json configs[2], the RMAT-26 query the metric is quoted on):
    GO 3 STEPS FROM <64 seeds> OVER follow WHERE follow.weight > 499 YIELD DISTINCT follow._dst
on a synthetic RMAT graph (scale 26, edge factor 16, Graph500 parameters, seed 1), built on the
device by the snapshot builder.  A "step" of this benchmark is one full query.  TEPS = adjacency
entries scanned over all hops / wall time; the frontier never leaves HBM.

    python bench.py                       # N=1
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md, chip-level parameters)


def hop_kernels(h):
    """rocprof names of the kernels one hop stat times"""
    if h["mode"] == "bottom-up":
        return ["nbg::k_bu_slab<1," if h["final"] else "nbg::k_bu_slab<0,"] + (["nbg::k_bits_compact<1>"] if h["final"] else [])
    return ["nbg::k_expand<"]


def pmc_traffic(workload: str, prefixes):
    """HBM bytes per launch of the given kernels from the newest committed rocprof PMC summary of
    the same workload (profiles/<tag>_summary.json: FETCH_SIZE x2 gfx950 correction + WRITE_SIZE,
    separate --pmc passes, tools/gpu_profile.sh + tools/profile_summary.py).  None if absent."""
    best = None
    # newest round tag last (r01b < r01c < ...); file mtimes are meaningless in a fresh checkout
    for f in sorted((ROOT / "profiles").glob("*_summary.json"), key=lambda p: p.name):
        try:
            d = json.loads(f.read_text())
        except ValueError:
            continue
        b = d.get("bench") or {}
        if (b.get("config") or {}).get("workload") != workload:
            continue
        tot, hit = 0.0, 0
        for pre in prefixes:
            ks = [k for k in d.get("query_kernels", []) if k["kernel"].startswith(pre)
                  and k.get("fetch_bytes_x2") is not None]
            if ks:
                k = max(ks, key=lambda k: k["total_ms"])
                tot += k["fetch_bytes_x2"] + (k.get("write_bytes") or 0.0)
                hit += 1
        if hit == len(prefixes):
            best = {"bytes": tot, "source": f"profiles/{f.name}"}
    return best


def cpu_baseline(scale: int, seeds: int, where_k: int):
    """The oracle (CPU restatement of storaged+graphd, faithful mode: 10 bucket handlers,
    single-threaded graphd loop) on a bounded sample of the same query."""
    sys.path.insert(0, str(ROOT / "tests"))
    import numpy as np  # noqa: F401
    import oracle as O
    from nebula_amd import expr as X
    from nebula_amd import synth

    st = O.Store(64)
    st.set_edge_schema(1, [("weight", O.INT)], name="follow")
    t0 = time.time()
    st.load_rmat(scale, 16, 1, 1, versions=1, threads=min(8, os.cpu_count() or 1))
    load_s = time.time() - t0
    starts = synth.seeds(scale, 16, 1, seeds)
    w = (X.AliasProp("follow", "weight") > where_k).encode()
    y = [X.EdgeDst("follow").encode()]
    best = None
    scanned = 0
    for _ in range(2):
        t0 = time.time()
        r = st.go(starts, 3, 1, where=w, yields=y, distinct=True, hosts=1, handlers=10, min_per_bucket=3)
        dt = time.time() - t0
        scanned = r.edges_scanned
        best = dt if best is None else min(best, dt)
    return {
        "value": scanned / best / 1e9,
        "unit": "GTEPS",
        "cores": min(10, os.cpu_count() or 1),
        "kind": "port",
        "sample": f"oracle GO 3 STEPS WHERE weight>{where_k} YIELD DISTINCT _dst from {seeds} seeds on "
                  f"RMAT-{scale} (ef16), 1 storaged host x 10 handlers, graphd 1 thread; "
                  f"{scanned} edges scanned in {best:.2f}s (best of 2); KV load {load_s:.1f}s",
    }


def cpu_baseline_paths(scale: int, npairs: int, max_steps: int):
    """The oracle's FIND SHORTEST PATH (backward BFS + greedy walk, one thread) on a sample."""
    sys.path.insert(0, str(ROOT / "tests"))
    import oracle as O
    from nebula_amd import synth

    st = O.Store(64)
    st.set_edge_schema(1, [("weight", O.INT)], name="follow")
    st.load_rmat(scale, 16, 1, 1, versions=1, threads=min(8, os.cpu_count() or 1))
    s, t = synth.pairs(scale, 16, 1, npairs)
    t0 = time.time()
    st.shortest_path(s, t, 1, max_steps)
    dt = time.time() - t0
    return {"value": npairs / dt, "unit": "pairs/s", "cores": 1, "kind": "port",
            "sample": f"oracle FIND SHORTEST PATH {npairs} pairs on RMAT-{scale} (ef16) UPTO {max_steps} STEPS "
                      f"in {dt:.2f}s"}


def bench_paths(args, sp, info, build_s, rank, world, dist=None):
    """BASELINE.json configs[3]: FIND SHORTEST PATH, 1024 (src, dst) pairs on RMAT-26.  With
    world > 1 the pairs are sharded i % world over the ranks (each answers its own against the
    replicated CSRs, no collective in the timed region): strong scaling of a fixed pair set."""
    from nebula_amd import synth
    s, t = synth.pairs(args.scale, args.edge_factor, 1, args.pairs)
    for _ in range(args.warmup):
        sp.shortest_path(s, t, 1, args.max_steps)
    if dist is not None:
        dist.barrier()
    t0 = time.perf_counter()
    edges = 0
    exp_ms = exp_bytes = dev_ms = 0.0
    iters = 0
    for _ in range(args.steps):
        r = sp.shortest_path(s, t, 1, args.max_steps)
        tm = sp.last_timing()
        edges += r.edges_scanned
        exp_ms += tm["expand_ms"]
        exp_bytes += tm["expand_bytes"]
        dev_ms += tm["total_ms"]
        iters = tm["steps_run"]
    if dist is not None:
        dist.barrier()
    dt = time.perf_counter() - t0
    hops = r.hops
    if dist is not None:
        import torch
        tt = torch.tensor([dt], dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
        te = torch.tensor([edges], dtype=torch.int64)
        dist.all_reduce(te, op=dist.ReduceOp.SUM)
        edges = int(te.item())
        hl = [None] * world
        dist.all_gather_object(hl, hops.tolist())
        hops = np.array([h for part in hl for h in part], dtype=np.int64)
    achieved = exp_bytes / (exp_ms / 1e3) / 1e9 if exp_ms > 0 else 0.0
    out = {
        "metric": "FIND SHORTEST PATH pairs/s (batched bidirectional BFS) on RMAT-26",
        "value": args.pairs * args.steps / dt,
        "unit": "pairs/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": dt / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "int64",
        "data": "synthetic RMAT (Graph500 a/b/c=0.57/0.19/0.19, seed 1) generated on device",
        "config": {
            "parallelism": f"pairs sharded i % {world} over the ranks, replicated CSRs" if world > 1 else "1 GPU",
            "workload": f"FIND SHORTEST PATH {args.pairs} pairs UPTO {args.max_steps} STEPS OVER follow; "
                        f"RMAT-{args.scale} ef{args.edge_factor}",
            "vertices": info["num_vertices"],
            "edges_examined_per_query": edges // max(args.steps, 1),
            "gteps": edges / dt / 1e9,
            "reachable": int((hops >= 0).sum()),
            "hops_histogram": {int(h): int((hops == h).sum()) for h in sorted(set(hops.tolist()))},
            "bfs_iterations": iters,
            "snapshot_build_s": round(build_s, 2),
        },
        "roofline": {
            "bound": "hbm", "kernel": "k_sp_expand", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS, "traffic": None,
            "expand_ms_per_query": exp_ms / max(args.steps, 1), "device_ms_per_query": dev_ms / max(args.steps, 1),
        },
        "cpu_baseline": None,
    }
    if not args.no_cpu and world == 1:
        try:
            out["cpu_baseline"] = cpu_baseline_paths(args.cpu_scale, 64, args.max_steps)
        except Exception as e:
            out["cpu_baseline"] = {"error": str(e)}
    if rank == 0:
        print(json.dumps(out), flush=True)
    sp.close()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--scale", type=int, default=26)
    ap.add_argument("--edge-factor", type=int, default=16)
    ap.add_argument("--seeds", type=int, default=64)
    ap.add_argument("--where", type=int, default=499)
    ap.add_argument("--hops", type=int, default=3)
    ap.add_argument("--cpu-scale", type=int, default=20)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--option", action="append", default=[], help="engine option key=value")
    ap.add_argument("--workload", choices=["go", "paths"], default="go",
                    help="go: BASELINE metric (GO 3 STEPS); paths: configs[3] FIND SHORTEST PATH")
    ap.add_argument("--pairs", type=int, default=1024)
    ap.add_argument("--plain", action="store_true",
                    help="GO without WHERE / DISTINCT (configs[1]: RMAT-22 3 steps, configs[4]: RMAT-28 2 steps)")
    ap.add_argument("--max-steps", type=int, default=8)
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", str(args.gpus)))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo", rank=rank, world_size=world)

    from nebula_amd import GraphSpace
    from nebula_amd import expr as X
    from nebula_amd import synth

    sp = GraphSpace(64, device=local, rank=rank, world_size=world)
    if world > 1:
        uid = [GraphSpace.comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        sp.comm_init(uid[0])
    for kv in args.option:
        k, v = kv.split("=")
        sp.set_option(k, int(v))
    FOLLOW = 1
    sp.set_edge_schema(FOLLOW, [("weight", 2)])
    t0 = time.time()
    sp.gen_rmat(args.scale, args.edge_factor, 1, FOLLOW)
    sp.finalize()
    build_s = time.time() - t0
    info = sp.info(FOLLOW)
    if args.workload == "paths":
        return bench_paths(args, sp, info, build_s, rank, world, dist)
    starts = synth.seeds(args.scale, args.edge_factor, 1, args.seeds)
    # --plain: no WHERE, default YIELD follow._dst rows without DISTINCT (configs[1] / configs[4])
    where = None if args.plain else X.AliasProp("follow", "weight") > args.where
    yields = [X.EdgeDst("follow")]

    def one():
        return sp.go(starts, args.hops, FOLLOW, where=where, yields=yields, distinct=not args.plain,
                     keep_on_device=True)

    for _ in range(args.warmup):
        one()

    def barrier():
        if dist is not None:
            dist.barrier()

    barrier()
    t0 = time.perf_counter()
    edges = 0
    rows = 0
    exp_ms = 0.0
    exp_bytes = 0
    tot_ms = 0.0
    bu_steps = 0
    hop_ms, hop_bytes = {}, {}
    for _ in range(args.steps):
        r = one()
        t = sp.last_timing()
        edges += r.edges_scanned
        rows = r.n_rows
        exp_ms += t["expand_ms"]
        exp_bytes += t["expand_bytes"]
        tot_ms += t["total_ms"]
        bu_steps = t["bu_steps"]
        hop_stats = t["hops"]
        for i, h in enumerate(hop_stats):
            hop_ms[i] = hop_ms.get(i, 0.0) + h["ms"]
            hop_bytes[i] = hop_bytes.get(i, 0) + h["bytes"]
    barrier()
    dt = time.perf_counter() - t0
    if dist is not None:
        import torch
        tt = torch.tensor([dt], dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
        te = torch.tensor([edges, rows], dtype=torch.int64)
        dist.all_reduce(te, op=dist.ReduceOp.SUM)
        edges, rows = int(te[0].item()), int(te[1].item())
    gteps = edges / dt / 1e9
    achieved = exp_bytes / (exp_ms / 1e3) / 1e9 if exp_ms > 0 else 0.0
    # dominant kernel: the hop with the largest summed time (the final bottom-up hop here)
    dom = max(range(len(hop_stats)), key=lambda i: hop_ms[i]) if hop_stats else None
    workload = (f"GO {args.hops} STEPS FROM {args.seeds} seeds OVER follow WHERE follow.weight > "
                f"{args.where} YIELD DISTINCT follow._dst; RMAT-{args.scale} ef{args.edge_factor}")
    if args.plain:
        workload = (f"GO {args.hops} STEPS FROM {args.seeds} seeds OVER follow (YIELD follow._dst rows); "
                    f"RMAT-{args.scale} ef{args.edge_factor}")
    if dom is not None:
        dh = hop_stats[dom]
        dom_ach = hop_bytes[dom] / (hop_ms[dom] / 1e3) / 1e9 if hop_ms[dom] > 0 else 0.0
        dom_names = hop_kernels(dh)
        tr = pmc_traffic(workload, dom_names)
    if rank == 0:
        out = {
            "metric": "GTEPS for GO 3 STEPS on RMAT-26 at 1/2/4/8 GPUs; % of HBM roofline",
            "value": gteps,
            "unit": "GTEPS",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": dt / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "int64",
            "data": "synthetic RMAT (Graph500 a/b/c=0.57/0.19/0.19, seed 1) generated on device",
            "config": {
                "workload": workload,
                "vertices": info["num_vertices"],
                "edges_after_collapse": info["local_out_edges"] if world == 1 else None,
                "edges_scanned_per_query": edges // max(args.steps, 1),
                "result_rows": rows,
                "snapshot_build_s": round(build_s, 2),
                "parallelism": f"part%{world} sharding, RCCL frontier exchange" if world > 1 else "1 GPU",
            },
            "roofline": {
                "bound": "hbm",
                "kernel": " + ".join(k.rstrip("<,") for k in dom_names) + f" (hop {dom + 1} of {len(hop_stats)})",
                "achieved": dom_ach,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": dom_ach / HBM_PEAK_GBS,
                "traffic": tr["bytes"] if tr else None,
                "traffic_source": tr["source"] + " (FETCH_SIZE x2 + WRITE_SIZE per launch)" if tr else None,
                "algorithmic_bytes_per_launch": hop_bytes[dom] // max(args.steps, 1),
                "launch_ms": hop_ms[dom] / max(args.steps, 1),
                "all_expansion_kernels": {"achieved": achieved, "frac": achieved / HBM_PEAK_GBS},
                "algorithmic_bytes_per_query": exp_bytes // max(args.steps, 1),
                "expand_ms_per_query": exp_ms / max(args.steps, 1),
                "device_ms_per_query": tot_ms / max(args.steps, 1),
                "bottom_up_hops": bu_steps,
                "hops": hop_stats,
            },
            "cpu_baseline": None,
        }
        if world == 1 and not args.no_cpu and not args.plain:
            try:
                out["cpu_baseline"] = cpu_baseline(args.cpu_scale, args.seeds, args.where)
            except Exception as e:  # the baseline must not hide the GPU number
                out["cpu_baseline"] = {"error": str(e)}
        print(json.dumps(out), flush=True)
    sp.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
