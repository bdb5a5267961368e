#!/usr/bin/env python3
"""Benchmark: GTEPS of GO 3 STEPS on RMAT-26 on N MI355X (BASELINE.json metric).

Workload (BASELINE.json configs[2], the RMAT-26 query the metric is quoted on):
    GO 3 STEPS FROM <64 seeds> OVER follow WHERE follow.weight > 499 YIELD DISTINCT follow._dst
on a synthetic RMAT graph (scale 26, edge factor 16, Graph500 parameters, seed 1), built on the
device by the snapshot builder.  A "step" of this benchmark is one full query.  TEPS = adjacency
entries scanned over all hops / wall time; the frontier never leaves HBM.

    python bench.py                       # N=1
    python bench.py --gpus N              # spawns N ranks itself (one process per GPU)
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N
    python bench.py --plain --scale 22    # configs[1] (C2)
    python bench.py --plain --scale 28 --hops 2 --hubs 8   # configs[4] (C5)
    python bench.py --workload paths      # configs[3] (C4)

After the timed region the same query runs once more with its result copied to the host and is
checked against tests/golden/rmat_digests.json (the oracle's digest of that config) -> "parity".
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md, chip-level parameters)
GOLDEN = ROOT / "tests" / "golden" / "rmat_digests.json"


def hop_kernels(h):
    """rocprof names of the kernels one hop stat times, dominant first (reported by the engine)"""
    return h.get("kernels") or ["nbg::k_expand"]


def same_model(a, b, tol=0.01):
    """the profiled run and this run moved the same algorithmic bytes (within tol): the profile's
    counters describe this tree's kernel on this workload, not an older one"""
    return a is not None and b is not None and abs(float(a) - float(b)) <= tol * max(float(a), float(b), 1.0)


def pmc_traffic(workload: str, prefixes, model_bytes=None):
    """HBM bytes per launch of the given kernels from the newest committed rocprof PMC summary of
    the same workload (profiles/<tag>_summary.json: FETCH_SIZE x2 gfx950 correction + WRITE_SIZE,
    separate --pmc passes, tools/gpu_profile.sh + tools/profile_summary.py) whose bench line
    recorded the same algorithmic bytes per launch as this run (model_bytes; a profile of an older
    tree whose kernel moved other bytes is skipped).  None if absent."""
    best = None
    # newest round tag last (r01b < r01c < ... < r02a); file mtimes are meaningless in a checkout
    for f in sorted((ROOT / "profiles").glob("*_summary.json"), key=lambda p: p.name):
        try:
            d = json.loads(f.read_text())
        except ValueError:
            continue
        b = d.get("bench") or {}
        if (b.get("config") or {}).get("workload") != workload:
            continue
        if model_bytes is not None and not same_model((b.get("roofline") or {}).get("algorithmic_bytes_per_launch"),
                                                      model_bytes):
            continue
        tot, raw, hit = 0.0, 0.0, 0
        for pre in prefixes:
            ks = [k for k in d.get("query_kernels", []) if k["kernel"].startswith(pre)
                  and k.get("fetch_bytes_x2") is not None]
            if ks:
                k = max(ks, key=lambda k: k["total_ms"])
                tot += k["fetch_bytes_x2"] + (k.get("write_bytes") or 0.0)
                raw += k["fetch_bytes_x2"] / 2 + (k.get("write_bytes") or 0.0)
                hit += 1
        if hit == len(prefixes):
            best = {"bytes": tot, "raw_bytes": raw, "source": f"profiles/{f.name}"}
    return best


def pmc_traffic_query(workload: str, kind: str, model_bytes=None):
    """HBM bytes per query of one scan kind (all its launches of one query) from the newest
    committed C4 PMC summary of the same workload (profiles/<tag>_c4.json, tools/c4_counters.sh +
    tools/c4_summary.py: FETCH_SIZE x2 + WRITE_SIZE per dispatch) whose byte model of that kind
    equals this run's (model_bytes, within 1 %).  None if absent."""
    best = None
    for f in sorted((ROOT / "profiles").glob("*_c4.json"), key=lambda p: p.name):
        try:
            d = json.loads(f.read_text())
        except ValueError:
            continue
        if ((d.get("bench") or {}).get("config") or {}).get("workload") != workload:
            continue
        k = (d.get("query_kinds") or {}).get(kind)
        if k and k.get("complete") and (model_bytes is None or same_model(k.get("model_bytes"), model_bytes)):
            best = {"bytes": k["fetch_bytes_x2"] + k["write_bytes"],
                    "raw_bytes": k["fetch_bytes_x2"] / 2 + k["write_bytes"],
                    "model_bytes": k["model_bytes"], "launches": k["launches"], "source": f"profiles/{f.name}"}
    return best


# ---- CPU baseline -----------------------------------------------------------------------------
def host_cpu():
    """(usable cores of this process, cores of the machine, CPU model).  The GPU box pins a
    process's CPU share through OMP_NUM_THREADS (16 per GPU) while its affinity mask shows the
    whole machine, so the share is the smaller of the two."""
    try:
        usable = len(os.sched_getaffinity(0))
    except AttributeError:
        usable = os.cpu_count() or 1
    share = os.environ.get("OMP_NUM_THREADS", "")
    if share.isdigit() and int(share) > 0:
        usable = min(usable, int(share))
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return usable, os.cpu_count() or usable, model


def best_of(fn, reps=3):
    """best wall time of `reps` runs after one warm-up"""
    fn()  # warm-up
    best, out = None, None
    for _ in range(reps):
        t0 = time.perf_counter()
        out = fn()
        dt = time.perf_counter() - t0
        best = dt if best is None else min(best, dt)
    return best, out


def cpu_baseline(scale: int, where_k: int, golden: dict, c1_scale: int = 16):
    """The oracle (oracle/refcpu.cpp: the CPU restatement of storaged + graphd over the
    reference's KV layout) timed on this host on a bounded sample, best of 3 after 1 warm-up:
      * faithful: 1 storaged host x max_handlers_per_req = 10 bucket threads, min 3 vertices per
        bucket (QueryBaseProcessor.cpp:9-10), graphd loop single-threaded (GraphFlags.cpp:19);
      * all-cores: the same with one bucket thread per usable core.
    Sample: the bench query's shape (GO 3 STEPS ... WHERE weight > k YIELD DISTINCT _dst, 64
    seeds) on RMAT-`scale`, and configs[0] (C1: GO 2 STEPS FROM 16 seeds) on RMAT-`c1_scale`."""
    sys.path.insert(0, str(ROOT / "tests"))
    import oracle as O
    from nebula_amd import expr as X
    from nebula_amd import synth

    usable, machine, model = host_cpu()
    stores, load_s = {}, 0.0
    for sc in sorted({scale, c1_scale}):
        st = O.Store(64)
        st.set_edge_schema(1, [("weight", O.INT)], name="follow")
        t0 = time.perf_counter()
        st.load_rmat(sc, 16, 1, 1, versions=1, threads=min(16, usable))
        load_s += time.perf_counter() - t0
        stores[sc] = st
    w = (X.AliasProp("follow", "weight") > where_k).encode()
    y = [X.EdgeDst("follow").encode()]
    cases = {
        "c3_shape": dict(scale=scale, starts=synth.seeds(scale, 16, 1, 64), steps=3, where=w, yields=y,
                         distinct=True, golden=f"go3_where{where_k}_distinct_s{scale}"),
        "c1": dict(scale=c1_scale, starts=synth.seeds(c1_scale, 16, 1, 16), steps=2, where=b"", yields=(),
                   distinct=False, golden=f"go2_plain_s{c1_scale}"),
    }
    res = {}
    for name, cs in cases.items():
        st = stores[cs["scale"]]
        row = {}
        # RMAT-20 and up: one timed run after the warm-up (a query takes ~9 s there; the sample
        # stays inside the bench's few-minute budget)
        reps = 3 if cs["scale"] <= 18 else 1
        for mode, handlers in (("faithful", 10), ("all_cores", usable)):
            dt, r = best_of(lambda: st.go(cs["starts"], cs["steps"], 1, where=cs["where"], yields=cs["yields"],
                                          distinct=cs["distinct"], hosts=1, handlers=handlers, min_per_bucket=3),
                            reps)
            row[mode] = {"gteps": r.edges_scanned / dt / 1e9, "seconds": dt, "threads": min(handlers, usable) + 1}
            row["edges_scanned"] = r.edges_scanned
            row["rows"] = r.nrows
            g = golden.get(cs["golden"])
            row["parity"] = ("no golden" if g is None else
                             "digest ok" if O.digest(r.int_col(0)) == g["sha256"] and r.nrows == g["n_rows"]
                             else "mismatch")
        res[name] = row
    c3 = res["c3_shape"]
    return {
        "value": c3["faithful"]["gteps"],
        "unit": "GTEPS",
        "cores": c3["faithful"]["threads"],
        "kind": "port",
        "sample": f"oracle (KV-store restatement of storaged+graphd) GO 3 STEPS WHERE weight>{where_k} YIELD "
                  f"DISTINCT _dst from 64 seeds on RMAT-{scale} (ef16), faithful mode (1 storaged host x 10 bucket "
                  f"threads + 1 graphd thread), {'best of 3' if scale <= 18 else 'one run'} after 1 warm-up; KV load "
                  f"{load_s:.1f}s.  The sample graph is smaller than the GPU's RMAT-26 (the oracle holds the KV bytes "
                  f"in host memory and scans them at 2-4 M edges/s, falling with size: 3.8 / 4.4 / 3.1 / 2.4 MTEPS "
                  f"at RMAT-16/18/20/22, profiles/r10j_cpu_scaling.jsonl): GTEPS of the two are rates on different "
                  f"graph sizes, not a like-for-like speedup",
        "host_cores": usable,
        "machine_cores": machine,
        "cpu_model": model,
        "faithful": {"c3_shape": c3["faithful"], "c1": res["c1"]["faithful"]},
        "all_cores": {"c3_shape": c3["all_cores"], "c1": res["c1"]["all_cores"]},
        "config": {"c3_shape": {"scale": scale, **{k: c3[k] for k in ("edges_scanned", "rows", "parity")}},
                   "c1": {"scale": c1_scale, **{k: res["c1"][k] for k in ("edges_scanned", "rows", "parity")}}},
    }


def cpu_baseline_paths(scale: int, npairs: int, max_steps: int):
    """The oracle's FIND SHORTEST PATH (backward BFS + greedy walk, one thread) on a sample."""
    sys.path.insert(0, str(ROOT / "tests"))
    import oracle as O
    from nebula_amd import synth

    usable, machine, model = host_cpu()
    st = O.Store(64)
    st.set_edge_schema(1, [("weight", O.INT)], name="follow")
    st.load_rmat(scale, 16, 1, 1, versions=1, threads=min(16, usable))
    s, t = synth.pairs(scale, 16, 1, npairs)
    dt, _ = best_of(lambda: st.shortest_path(s, t, 1, max_steps))
    return {"value": npairs / dt, "unit": "pairs/s", "cores": 1, "kind": "port", "host_cores": usable,
            "machine_cores": machine, "cpu_model": model,
            "sample": f"oracle FIND SHORTEST PATH {npairs} pairs on RMAT-{scale} (ef16) UPTO {max_steps} STEPS, "
                      f"best of 3 after 1 warm-up: {dt:.2f}s; a smaller graph than the GPU's RMAT-26, so pairs/s "
                      f"of the two are not a like-for-like speedup"}


# ---- parity of the timed query ----------------------------------------------------------------
def gather_column(col, dist, world):
    if dist is None or world == 1:
        return col
    parts = [None] * world
    dist.all_gather_object(parts, col)
    return np.concatenate(parts)


def parity_go(sp, run_host, key, golden, dist, world, rank, plain_rows_check):
    """re-run the timed query with its result on the host; compare with the committed digest of
    the config, or (no digest committed) the size-independent property of the workload"""
    r = run_host()
    col = gather_column(np.asarray(r.columns[0], dtype=np.int64), dist, world)
    out = {"golden": key}
    g = golden.get(key)
    if g is not None and "msum" in g:  # results too large to sort: order-independent digest
        n, sm, x = msum(col)
        ok = n == g["n_rows"] and [str(sm), str(x)] == g["msum"]
        out.update(status="digest ok" if ok else "mismatch", rows=int(n), digest="msum", msum=[str(sm), str(x)])
        return out
    if g is not None:
        ok = len(col) == g["n_rows"] and O_digest(col) == g["sha256"]
        out.update(status="digest ok" if ok else "mismatch", rows=int(len(col)), sha256=O_digest(col)[:16])
        return out
    # property check: a plain GO's final-hop rows are one per (frontier vertex, edge), i.e. the
    # out-degree sum of the final frontier (hop stat c[1] of a top-down hop, c[1] of the previous
    # bottom-up hop), which the engine reports independently of the rows it wrote
    out["status"] = "no golden"
    if plain_rows_check is not None:
        want = plain_rows_check()
        # weak: a fused plain-_dst expansion writes exactly that many rows by construction, so this
        # only catches a row-count slip, not a wrong frontier -- labelled as such
        out.update(property="rows == out-degree sum of the final frontier (row count only; no digest)",
                   status="unchecked (row count ok)" if want == len(col) else "property mismatch",
                   rows=int(len(col)), expected=int(want))
    return out


def msum(vids, chunk=1 << 26):
    """(rows, sum of splitmix64(vid) mod 2^64, xor of the same): the order-independent digest of
    tests/golden/make_rmat_digests.py's go_msum cases (oracle ora_rmat_graph_go_msum)"""
    v = np.asarray(vids, dtype=np.int64).view(np.uint64)
    s, x = 0, np.uint64(0)
    with np.errstate(over="ignore"):
        for i in range(0, len(v), chunk):
            z = v[i:i + chunk] + np.uint64(0x9E3779B97F4A7C15)
            z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
            z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
            z = z ^ (z >> np.uint64(31))
            s = (s + int(z.sum(dtype=np.uint64))) & ((1 << 64) - 1)
            x ^= np.bitwise_xor.reduce(z)
    return len(v), s, int(x)


def O_digest(vids) -> str:
    a = np.sort(np.asarray(vids, dtype=np.int64)).astype("<i8")
    return hashlib.sha256(a.tobytes()).hexdigest()


# ---- FIND SHORTEST PATH -------------------------------------------------------------------------
def bench_paths(args, sp, info, build_s, rank, world, golden, dist=None):
    """BASELINE.json configs[3]: FIND SHORTEST PATH, 1024 (src, dst) pairs on RMAT-26.  With
    world > 1 the pairs are sharded i % world over the ranks (each answers its own against the
    replicated CSRs, no collective in the timed region): strong scaling of a fixed pair set."""
    from nebula_amd import synth
    s, t = synth.pairs(args.scale, args.edge_factor, 1, args.pairs)
    for _ in range(args.warmup):
        sp.shortest_path(s, t, 1, args.max_steps)
    sp.set_option("hop_timing", 0)  # no event pairs between the timed launches (the stats loop has them)
    if dist is not None:
        dist.barrier()
    t0 = time.perf_counter()
    edges = 0
    for _ in range(args.steps):  # the timed region: K batches of pairs, nothing else
        r = sp.shortest_path(s, t, 1, args.max_steps)
        edges += r.edges_scanned
    if dist is not None:
        dist.barrier()
    dt = time.perf_counter() - t0
    sp.unset_option("hop_timing")
    # per-launch statistics from as many untimed calls again
    exp_ms = exp_bytes = dev_ms = 0.0
    iters = 0
    for _ in range(args.steps):
        r = sp.shortest_path(s, t, 1, args.max_steps)
        tm = sp.last_timing()
        exp_ms += tm["expand_ms"]
        exp_bytes += tm["expand_bytes"]
        dev_ms += tm["total_ms"]
        iters = tm["steps_run"]
    names = {2: "expand", 3: "probe", 4: "sweep", 5: "walk"}
    launches = [{"kind": names.get(h["mode_id"], h["mode"]), "ms": round(h["ms"], 4), "x": h["c"][0], "entries": h["c"][1],
                 "claims": h["c"][2], "iter": h["c"][4],
                 "kernel": h.get("kernels", ["?"])[0].replace("(anonymous namespace)::", "")} for h in tm["hops"]]
    for rec, h in zip(launches, tm["hops"]):
        if rec["kind"] == "probe" and (h["c"][6] or h["c"][7]):
            # option sp_dv_diag bit 3: the meet probe's filter statistics
            rec.update(pair_filter_passes=h["c"][6], distance_bytes_read=h["c"][2], bytes_at_depth=h["c"][7])
    # parity: the last result (host copy) against the committed digest
    hops, paths, srcs = r.hops, r.paths, r.src
    if dist is not None:
        import torch
        tt = torch.tensor([dt], dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
        te = torch.tensor([edges], dtype=torch.int64)
        dist.all_reduce(te, op=dist.ReduceOp.SUM)
        edges = int(te.item())
        hl = [None] * world
        dist.all_gather_object(hl, (hops.tolist(), [p.tolist() for p in paths]))
        # rank q answered pairs q, q + world, ...: back to input order
        hops = np.full(args.pairs, -2, dtype=np.int64)
        paths = [None] * args.pairs
        for q, (hq, pq) in enumerate(hl):
            for j, (h, p) in enumerate(zip(hq, pq)):
                hops[q + j * world] = h
                paths[q + j * world] = np.asarray(p, dtype=np.int64)
    key = f"paths{args.pairs}_s{args.scale}"
    parity = {"golden": key, "status": "no golden"}
    if key in golden:
        h = hashlib.sha256(np.asarray(hops, dtype="<i8").tobytes())
        for p in paths:
            h.update(np.asarray(p, dtype="<i8").tobytes())
        parity["status"] = "digest ok" if h.hexdigest() == golden[key]["sha256"] else "mismatch"
    achieved = exp_bytes / (exp_ms / 1e3) / 1e9 if exp_ms > 0 else 0.0
    # dominant launch kind of one query (its rocprof kernel, the engine's byte models:
    # paths.hip timing.expand_bytes): expand / probe / sweep
    kern = {"expand": "nbg::k_sp_expand", "probe": "nbg::k_sp_probe", "sweep": "nbg::k_sp_sweep",
            "walk": "nbg::k_dv_walk_scan"}
    model = {"expand": lambda l: l["x"] * 32 + l["entries"] * 5 + l["claims"] * 26,
             "probe": lambda l: l["x"] * 24 + l["entries"] * 5,
             "sweep": lambda l: l["x"] * 32 + l["entries"] * 6 + l["claims"] * 18,
             "walk": lambda l: l["x"] * 24 + l["entries"] * 5}
    by_kind = {}
    for l in launches:
        k = by_kind.setdefault(l["kind"], {"ms": 0.0, "bytes": 0.0, "launches": 0})
        k["ms"] += l["ms"]
        k["bytes"] += model.get(l["kind"], lambda _: 0)(l)
        k["launches"] += 1
    dom = max(by_kind, key=lambda k: by_kind[k]["ms"]) if by_kind else "expand"
    dk = by_kind.get(dom, {"ms": 0.0, "bytes": 0.0, "launches": 1})
    dom_ach = dk["bytes"] / (dk["ms"] / 1e3) / 1e9 if dk["ms"] > 0 else 0.0
    workload = (f"FIND SHORTEST PATH {args.pairs} pairs UPTO {args.max_steps} STEPS OVER follow; "
                f"RMAT-{args.scale} ef{args.edge_factor}")
    # the kernel of the dominant kind's longest launch (k_sp_sweep_sets / k_sp_probe_sets run the
    # large steps, the global-test kernels the small ones)
    dl = [l for l in launches if l["kind"] == dom]
    if dl:
        kern[dom] = max(dl, key=lambda l: l["ms"])["kernel"]
    tr = pmc_traffic_query(workload, dom, dk["bytes"])
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
            "parallelism": (f"pairs sharded i % {world} over the ranks, replicated CSRs" if world > 1 else
                            "1 GPU, replicas assembled through a one-rank RCCL communicator" if args.comm_single
                            else "1 GPU"),
            "communicator": sp.comm_info() if world > 1 or args.comm_single else None,
            "workload": workload,
            "vertices": info["num_vertices"],
            "edges_examined_per_query": edges // max(args.steps, 1),
            "gteps": edges / dt / 1e9,
            "reachable": int((np.asarray(hops) >= 0).sum()),
            "hops_histogram": {int(h): int((np.asarray(hops) == h).sum()) for h in sorted(set(np.asarray(hops).tolist()))},
            "bfs_iterations": iters,
            # the last query's batch: host waits and kernel launches (the device-driven chain)
            "host_waits": tm["host_waits"], "kernel_launches": tm.get("launches"),
            "device_driven_batches": tm["spec_hops"],
            "launches": launches,
            "snapshot_build_s": round(build_s, 2),
        },
        "parity": parity,
        "roofline": {
            "bound": "hbm", "kernel": kern.get(dom, dom), "achieved": dom_ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": dom_ach / HBM_PEAK_GBS,
            # PMC HBM bytes of the dominant kind per query (all its launches of one profiled query)
            "traffic": tr["bytes"] if tr else None,
            "traffic_raw_fetch_plus_write": tr["raw_bytes"] if tr else None,
            "traffic_over_model": tr["bytes"] / tr["model_bytes"] if tr and tr["model_bytes"] else None,
            "traffic_source": tr["source"] + " (FETCH_SIZE x2 + WRITE_SIZE summed over the kind's launches "
            "of one query)" if tr else None,
            "algorithmic_bytes_per_query": dk["bytes"], "kernel_ms_per_query": dk["ms"],
            "all_scan_kernels": {"achieved": achieved, "frac": achieved / HBM_PEAK_GBS},
            "expand_ms_per_query": exp_ms / max(args.steps, 1), "device_ms_per_query": dev_ms / max(args.steps, 1),
        },
        "cpu_baseline": None,
    }
    if not args.no_cpu and world == 1:
        try:
            out["cpu_baseline"] = cpu_baseline_paths(min(args.cpu_scale, 16), 64, args.max_steps)
        except Exception as e:
            out["cpu_baseline"] = {"error": str(e)}
    if rank == 0:
        print(json.dumps(out), flush=True)
    sp.close()


def free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def spawn_ranks(n: int) -> int:
    """`bench.py --gpus N` without torch.distributed.run: N child processes of this script with
    RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT set (one per GPU, as the launcher
    sets them); rank 0's stdout (the JSON line) is passed through, the others' discarded.  The
    parent never touches the GPU.  Returns the first non-zero child exit code, else 0."""
    import subprocess
    port = str(free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, str(Path(__file__).resolve())] + sys.argv[1:], env=env,
                                      stdout=None if r == 0 else subprocess.DEVNULL))
    # poll every child: when one fails, the others (possibly blocked in the rendezvous or a
    # collective waiting for it) are ended at once instead of waiting out their timeouts
    import time as _t
    rcs = [None] * n
    while any(rc is None for rc in rcs):
        for i, p in enumerate(procs):
            if rcs[i] is None:
                rcs[i] = p.poll()
        failed = [rc for rc in rcs if rc not in (None, 0)]
        if failed:
            for i, p in enumerate(procs):
                if rcs[i] is None:
                    p.terminate()
            for i, p in enumerate(procs):
                if rcs[i] is None:
                    try:
                        rcs[i] = p.wait(timeout=30)
                    except subprocess.TimeoutExpired:
                        p.kill()
                        rcs[i] = p.wait()
            break
        _t.sleep(0.2)
    bad = [c for c in rcs if c != 0]
    if bad:
        print(f"bench.py: rank exit codes {rcs}", file=sys.stderr)
    return bad[0] if bad else 0


def launch_check(dist, rank, world, local) -> int:
    """--launch-check: the ranks came up with consistent env and can talk (no GPU call)"""
    total = world * (world - 1) // 2
    seen = rank
    if dist is not None:
        import torch
        t = torch.tensor([rank], dtype=torch.int64)
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        seen = int(t.item())
        dist.barrier()
    if rank == 0:
        print(json.dumps({"launch_check": "ok" if seen == total else "mismatch", "world": world,
                          "rank_sum": seen, "master_port": os.environ.get("MASTER_PORT")}), flush=True)
    if dist is not None:
        dist.destroy_process_group()
    return 0 if seen == total else 1


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--scale", type=int, default=26)
    ap.add_argument("--edge-factor", type=int, default=16)
    ap.add_argument("--seeds", type=int, default=64)
    ap.add_argument("--hubs", type=int, default=0,
                    help="replace the first N seeds with the N highest-out-degree vertices (configs[4]: 8)")
    ap.add_argument("--where", type=int, default=499)
    ap.add_argument("--hops", type=int, default=3)
    ap.add_argument("--cpu-scale", type=int, default=20)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-parity", action="store_true")
    ap.add_argument("--option", action="append", default=[], help="engine option key=value")
    ap.add_argument("--workload", choices=["go", "paths"], default="go",
                    help="go: BASELINE metric (GO 3 STEPS); paths: configs[3] FIND SHORTEST PATH")
    ap.add_argument("--pairs", type=int, default=1024)
    ap.add_argument("--plain", action="store_true",
                    help="GO without WHERE / DISTINCT (configs[1]: RMAT-22 3 steps, configs[4]: RMAT-28 2 steps)")
    ap.add_argument("--max-steps", type=int, default=8)
    ap.add_argument("--comm-single", action="store_true",
                    help="one GPU through a one-rank RCCL communicator: the sharded algorithm with every "
                         "exchange issued to RCCL (the rank's own slice sent to itself)")
    ap.add_argument("--launch-check", action="store_true",
                    help="only bring the ranks up (gloo init, barrier, all-reduce) and print one JSON line")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # no external launcher: spawn one process per GPU here, before anything touches the GPU
        return spawn_ranks(args.gpus)
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", str(args.gpus)))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        import datetime
        # a rank that dies before the rendezvous fails the others within minutes, not 30
        dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(minutes=5))
    if args.launch_check:
        return launch_check(dist, rank, world, local)

    from nebula_amd import GraphSpace
    from nebula_amd import expr as X
    from nebula_amd import synth

    golden = json.loads(GOLDEN.read_text()) if GOLDEN.exists() else {}
    sp = GraphSpace(64, device=local, rank=rank, world_size=world)
    for kv in args.option:
        k, v = kv.split("=")
        sp.set_option(k, int(v))
    single = args.comm_single and world == 1
    if world > 1:
        uid = [GraphSpace.comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        sp.comm_init(uid[0])
    elif single:
        sp.set_option("comm_single", 1)
        sp.comm_init(GraphSpace.comm_unique_id())
    FOLLOW = 1
    sp.set_edge_schema(FOLLOW, [("weight", 2)])
    t0 = time.time()
    sp.gen_rmat(args.scale, args.edge_factor, 1, FOLLOW)
    sp.finalize()
    build_s = time.time() - t0
    info = sp.info(FOLLOW)
    sharded = world > 1 or single
    comm_seen = sp.comm_info() if sharded else None  # ncclCommCount of the engine's communicator
    if args.workload == "paths":
        return bench_paths(args, sp, info, build_s, rank, world, golden, dist)
    starts = synth.seeds(args.scale, args.edge_factor, 1, args.seeds)
    hubs = []
    if args.hubs:
        # the top-N out-degree vertices (global: every rank sees the same vid -> degree via its
        # own rows; the owner's answer is the true degree, others report -1 / 0)
        cand = synth.hub_candidates(args.scale, 1)
        deg = np.array([sp.out_degree(FOLLOW, int(v)) for v in cand], dtype=np.int64)
        if dist is not None:
            import torch
            td = torch.tensor(deg)
            dist.all_reduce(td, op=dist.ReduceOp.MAX)
            deg = td.numpy()
        order = np.argsort(-deg, kind="stable")[:args.hubs]
        hubs = [(int(cand[i]), int(deg[i])) for i in order]
        starts = np.concatenate([np.array([h for h, _ in hubs], dtype=np.int64), starts[args.hubs:]])
    # --plain: no WHERE, default YIELD follow._dst rows without DISTINCT (configs[1] / configs[4]).
    # Encoded once, as graphd hands the storage / engine the encoded Expression bytes.
    where = None if args.plain else X.encode(X.AliasProp("follow", "weight") > args.where)
    yields = [X.encode(X.EdgeDst("follow"))]

    def one(keep=True):
        return sp.go(starts, args.hops, FOLLOW, where=where, yields=yields, distinct=not args.plain,
                     keep_on_device=keep)

    for _ in range(args.warmup):
        one()

    def barrier():
        if dist is not None:
            dist.barrier()

    # the timed queries run without the per-hop event pairs (profiling markers a production caller
    # would not record); the statistics loop below turns them back on
    sp.set_option("hop_timing", 0)
    one()
    barrier()
    t0 = time.perf_counter()
    edges = 0
    rows = 0
    for _ in range(args.steps):  # the timed region: K queries, nothing else
        r = one()
        edges += r.edges_scanned
        rows = r.n_rows
    barrier()
    dt = time.perf_counter() - t0
    sp.unset_option("hop_timing")
    # per-kernel statistics (HIP events the engine recorded) from as many untimed queries again,
    # so reading them back does not sit inside the timed region
    exp_ms = 0.0
    exp_bytes = 0
    tot_ms = comm_ms = 0.0
    comm_calls = 0
    tot_each = []
    comm_bytes = 0
    bu_steps = 0
    hop_ms, hop_bytes, k_ms, k_bytes = {}, {}, {}, {}
    for _ in range(args.steps):
        r = one()  # held like the timed loop's, so its buffers cycle the same way
        t = sp.last_timing()
        exp_ms += t["expand_ms"]
        exp_bytes += t["expand_bytes"]
        tot_ms += t["total_ms"]
        tot_each.append(round(t["total_ms"], 3))
        comm_ms += t["comm_ms"]
        comm_bytes += t["comm_bytes"]
        comm_calls += t["comm_calls"]
        bu_steps = t["bu_steps"]
        hop_stats = t["hops"]
        for i, h in enumerate(hop_stats):
            hop_ms[i] = hop_ms.get(i, 0.0) + h["ms"]
            hop_bytes[i] = hop_bytes.get(i, 0) + h["bytes"]
            k_ms[i] = k_ms.get(i, 0.0) + h["kernel_ms"]
            k_bytes[i] = k_bytes.get(i, 0) + h["kernel_bytes"]
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
    K = max(args.steps, 1)
    # dominant kernel: the kernel with the largest summed time (the final bottom-up hop's
    # k_bu_lean for the bench query); its hop (kernel + compaction) is reported beside it
    dom = max(range(len(hop_stats)), key=lambda i: k_ms[i]) if hop_stats else None
    workload = (f"GO {args.hops} STEPS FROM {args.seeds} seeds OVER follow WHERE follow.weight > "
                f"{args.where} YIELD DISTINCT follow._dst; RMAT-{args.scale} ef{args.edge_factor}")
    if args.plain:
        workload = (f"GO {args.hops} STEPS FROM {args.seeds} seeds{' incl. top-%d degree' % args.hubs if args.hubs else ''} "
                    f"OVER follow (YIELD follow._dst rows); RMAT-{args.scale} ef{args.edge_factor}")
    roof = None
    if dom is not None:
        dh = hop_stats[dom]
        dom_names = hop_kernels(dh)
        kach = k_bytes[dom] / (k_ms[dom] / 1e3) / 1e9 if k_ms[dom] > 0 else 0.0
        hach = hop_bytes[dom] / (hop_ms[dom] / 1e3) / 1e9 if hop_ms[dom] > 0 else 0.0
        tr = pmc_traffic(workload, dom_names[:1], k_bytes[dom] // K)
        roof = {
            "bound": "hbm",
            "kernel": dom_names[0] + f" (hop {dom + 1} of {len(hop_stats)})",
            "achieved": kach,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": kach / HBM_PEAK_GBS,
            "traffic": tr["bytes"] if tr else None,
            "traffic_raw_fetch_plus_write": tr["raw_bytes"] if tr else None,
            "traffic_source": tr["source"] + " (FETCH_SIZE x2 + WRITE_SIZE per launch)" if tr else None,
            "algorithmic_bytes_per_launch": k_bytes[dom] // K,
            "launch_ms": k_ms[dom] / K,
            "hop": {"kernels": " + ".join(dom_names), "achieved": hach,
                    "frac": hach / HBM_PEAK_GBS, "bytes": hop_bytes[dom] // K, "ms": hop_ms[dom] / K},
            "all_expansion_kernels": {"achieved": achieved, "frac": achieved / HBM_PEAK_GBS},
            "algorithmic_bytes_per_query": exp_bytes // K,
            "expand_ms_per_query": exp_ms / K,
            "device_ms_per_query": tot_ms / K,
            "device_ms_each": tot_each,
            "bottom_up_hops": bu_steps,
            "hops": hop_stats,
        }
    r = None  # release the last result before the end-to-end and parity queries
    # end to end: the same query with its result copied to the host (what a graphd caller pays);
    # untimed by the contract's clock, reported beside the device-resident ms_per_step
    e2e = []
    for _ in range(3):
        barrier()
        t1 = time.perf_counter()
        r = one(False)
        e2e.append((time.perf_counter() - t1) * 1e3)
        r = None
    e2e_ms = float(np.median(e2e))
    if dist is not None:
        import torch
        te2 = torch.tensor([e2e_ms], dtype=torch.float64)
        dist.all_reduce(te2, op=dist.ReduceOp.MAX)
        e2e_ms = float(te2.item())
    parity = {"status": "skipped"}
    if not args.no_parity:
        key = (f"go{args.hops}_plain_s{args.scale}" if args.plain else
               f"go{args.hops}_where{args.where}_distinct_s{args.scale}")
        if args.hubs or args.seeds != 64:
            key += f"_seeds{args.seeds}_hubs{args.hubs}"

        def plain_check():
            # rows of a plain GO = one per (final frontier vertex, edge): the final hop's
            # out-degree sum, which the engine takes from the CSR offsets (hop stat c[1]),
            # independently of the rows the expansion wrote (summed over ranks)
            v = int(sp.last_timing()["hops"][-1]["c"][1])
            if dist is not None:
                import torch
                tv = torch.tensor([v], dtype=torch.int64)
                dist.all_reduce(tv, op=dist.ReduceOp.SUM)
                v = int(tv.item())
            return v
        try:
            parity = parity_go(sp, lambda: one(False), key, golden, dist, world, rank,
                               plain_check if args.plain else None)
        except Exception as e:  # the check must not hide the GPU number
            parity = {"status": f"error: {e}"}
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
                "edges_scanned_per_query": edges // K,
                "result_rows": rows,
                # the timed queries leave their result in HBM (ms_per_step); with the result
                # copied to host memory a query takes query_end_to_end_ms (median of 3), the
                # difference being the device->host copy of the rows
                "query_end_to_end_ms": round(e2e_ms, 4),
                "result_d2h_ms": round(e2e_ms - dt / args.steps * 1e3, 4),
                "snapshot_build_s": round(build_s, 2),
                "parallelism": (f"part%{world} sharding, RCCL frontier exchange" if world > 1 else
                                "1 GPU, sharded algorithm through a one-rank RCCL communicator" if single else "1 GPU"),
                "hub_seeds": hubs or None,
            },
            "parity": parity,
            "roofline": roof,
            "cpu_baseline": None,
        }
        if sharded:
            out["comm"] = {"backend": "rccl (nbg_comm_init over ncclCommInitRank)", "ranks": world,
                           "communicator": comm_seen,
                           "comm_ms_per_query_rank0": comm_ms / K, "comm_bytes_per_query_rank0": comm_bytes // K,
                           "collectives_per_query_rank0": comm_calls / K,
                           "ms_per_collective_rank0": comm_ms / comm_calls if comm_calls else None}
        if world == 1 and not args.no_cpu and not args.plain:
            try:
                out["cpu_baseline"] = cpu_baseline(args.cpu_scale, args.where, golden)
            except Exception as e:  # the baseline must not hide the GPU number
                out["cpu_baseline"] = {"error": str(e)}
        print(json.dumps(out), flush=True)
    sp.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    sys.exit(main() or 0)
