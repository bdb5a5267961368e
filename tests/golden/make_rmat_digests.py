#!/usr/bin/env python3
"""Generate tests/golden/rmat_digests.json: result digests of the BASELINE configs at their
configured sizes, computed by the oracle's index-space restatement (oracle/rmat_graph.cpp,
pinned to the faithful KV-store restatement by tests/test_oracle_rmat_graph.py).

The GPU tests (tests/test_gpu_scale.py) and bench.py compare the HIP path's results with these
digests: SHA-256 of the result column as sorted little-endian int64 (oracle.digest), plus the
row count and the edges scanned (the TEPS numerator).  FIND SHORTEST PATH digests hash the hops
array (int64, input order) and the concatenated paths.

    python tests/golden/make_rmat_digests.py [case ...]     # default: all cases
"""
from __future__ import annotations

import hashlib
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))

import oracle as O  # noqa: E402
from nebula_amd import synth  # noqa: E402

OUT = Path(__file__).resolve().parent / "rmat_digests.json"

# name -> (scale, kind, params).  Seeds / pairs are the bench's (nebula_amd.synth, seeds 7 / 11).
CASES = {
    # configs[0] (C1): GO 2 STEPS FROM 16 seeds OVER follow on RMAT-16
    "go2_plain_s16": (16, "go", dict(seeds=16, steps=2, where=None, distinct=False)),
    # configs[1] (C2): GO 3 STEPS FROM 64 seeds OVER follow on RMAT-22
    "go3_plain_s18": (18, "go", dict(seeds=64, steps=3, where=None, distinct=False)),
    "go3_plain_s22": (22, "go", dict(seeds=64, steps=3, where=None, distinct=False)),
    # configs[2] (C3, the bench query): GO 3 STEPS ... WHERE follow.weight > 499 YIELD DISTINCT
    "go3_where499_distinct_s16": (16, "go", dict(seeds=64, steps=3, where=499, distinct=True)),
    "go3_where499_distinct_s18": (18, "go", dict(seeds=64, steps=3, where=499, distinct=True)),
    "go3_where499_distinct_s20": (20, "go", dict(seeds=64, steps=3, where=499, distinct=True)),
    "go3_where499_distinct_s22": (22, "go", dict(seeds=64, steps=3, where=499, distinct=True)),
    "go3_where499_distinct_s24": (24, "go", dict(seeds=64, steps=3, where=499, distinct=True)),
    "go3_where499_distinct_s26": (26, "go", dict(seeds=64, steps=3, where=499, distinct=True)),
    # configs[3] (C4): FIND SHORTEST PATH, 1024 pairs, UPTO 8 STEPS
    "paths1024_s18": (18, "paths", dict(pairs=1024, max_steps=8)),
    "paths1024_s22": (22, "paths", dict(pairs=1024, max_steps=8)),
    "paths1024_s26": (26, "paths", dict(pairs=1024, max_steps=8)),
    # configs[4] (C5): GO 2 STEPS FROM 64 seeds incl. the top-8 out-degree vertices on RMAT-28
    # (2.7 G rows: order-independent digest, oracle.msum)
    "go2_plain_s28_seeds64_hubs8": (28, "go_msum", dict(seeds=64, hubs=8, steps=2)),
    "go2_plain_s16_seeds64_hubs8": (16, "go_msum", dict(seeds=64, hubs=8, steps=2)),
}


def hub_starts(g, scale, seeds, hubs):
    """bench.py --hubs: the top-N out-degree vertices among synth.hub_candidates (collapsed
    degrees, stable order) replace the first N seeds"""
    starts = synth.seeds(scale, 16, 1, seeds)
    idx = [0] + [1 << k for k in range(scale)]
    cand = synth.hub_candidates(scale, 1)
    deg = np.array([g.out_degree(i) for i in idx], dtype=np.int64)
    order = np.argsort(-deg, kind="stable")[:hubs]
    return np.concatenate([cand[order].astype(np.int64), starts[hubs:]]), [(int(cand[i]), int(deg[i])) for i in order]


def paths_digest(hops, paths) -> str:
    h = hashlib.sha256(np.asarray(hops, dtype="<i8").tobytes())
    for p in paths:
        h.update(np.asarray(p, dtype="<i8").tobytes())
    return h.hexdigest()


def run_case(g, name, kind, prm, scale):
    if kind == "go_msum":
        starts, hubs = hub_starts(g, scale, prm["seeds"], prm["hubs"])
        t0 = time.time()
        ms, scanned = g.go_msum(starts, prm["steps"])
        return {"scale": scale, **prm, "n_rows": ms[0], "msum": [str(ms[1]), str(ms[2])], "hub_seeds": hubs,
                "edges_scanned": int(scanned), "oracle_s": round(time.time() - t0, 2)}
    if kind == "go":
        starts = synth.seeds(scale, 16, 1, prm["seeds"])
        t0 = time.time()
        res, scanned = g.go(starts, prm["steps"], where_gt=prm["where"], distinct=prm["distinct"])
        return {"scale": scale, **prm, "n_rows": int(len(res)), "sha256": O.digest(res),
                "edges_scanned": int(scanned), "oracle_s": round(time.time() - t0, 2)}
    s, t = synth.pairs(scale, 16, 1, prm["pairs"])
    t0 = time.time()
    hops, paths = g.shortest_path(s, t, prm["max_steps"])
    hist = {int(k): int((hops == k).sum()) for k in sorted(set(hops.tolist()))}
    return {"scale": scale, **prm, "sha256": paths_digest(hops, paths), "hops_histogram": hist,
            "hops_sha256": hashlib.sha256(np.asarray(hops, dtype="<i8").tobytes()).hexdigest(),
            "oracle_s": round(time.time() - t0, 2)}


def main():
    names = sys.argv[1:] or list(CASES)
    data = json.loads(OUT.read_text()) if OUT.exists() else {}
    by_scale = {}
    for n in names:
        by_scale.setdefault(CASES[n][0], []).append(n)
    for scale in sorted(by_scale):
        t0 = time.time()
        g = O.RmatGraph(scale, 16, 1)
        info = g.info()
        print(f"RMAT-{scale}: {info} built in {time.time() - t0:.1f}s", flush=True)
        for n in by_scale[scale]:
            _, kind, prm = CASES[n]
            data[n] = {**run_case(g, n, kind, prm, scale), "graph": info}
            print(n, json.dumps(data[n]), flush=True)
            OUT.write_text(json.dumps(data, indent=1, sort_keys=True) + "\n")
        del g


if __name__ == "__main__":
    main()
