"""Streamed RMAT build (snapshot.hip finalize_rmat_stream): the one-rank builder for graphs past
the tuple stage's 2^32 cap (BASELINE.json configs[4], RMAT-28).  It regenerates the samples per
src-gidx bucket instead of staging them, so it must give the staged build's snapshot exactly:
same vertex numbering, same rows in the same (RocksDB key) order, same weights.

Checked here with the bucket size forced small (many buckets per direction) against the staged
build (getBound rows in order, GO results, shortest paths) and against the oracle's index-space
restatement and the committed digests.
"""
import json
from pathlib import Path

import numpy as np
import pytest

import oracle as O
from nebula_amd import GraphSpace
from nebula_amd import expr as X
from nebula_amd import synth

pytestmark = pytest.mark.gpu

FOLLOW = 1
GOLD = json.loads((Path(__file__).resolve().parent / "golden" / "rmat_digests.json").read_text())
W499 = X.AliasProp("follow", "weight") > 499


def space(scale, **opts):
    sp = GraphSpace(64)
    for k, v in opts.items():
        sp.set_option(k, v)
    sp.set_edge_schema(FOLLOW, [("weight", O.INT)])
    sp.gen_rmat(scale, 16, 1, FOLLOW)
    sp.finalize()
    return sp


@pytest.fixture(scope="module")
def pair16():
    staged = space(16, rmat_stream=0)
    streamed = space(16, rmat_stream=1, rmat_bucket=1 << 16)  # ~16 buckets per direction
    yield staged, streamed
    staged.close()
    streamed.close()


def test_info_matches_staged(pair16):
    a, b = pair16
    ia, ib = a.info(FOLLOW), b.info(FOLLOW)
    for k in ("num_vertices", "local_out_edges", "local_in_edges"):
        assert ia[k] == ib[k], k


def test_get_bound_rows_in_key_order(pair16):
    """getBound returns each vertex's rows in RocksDB key order: the streamed CSR's row order,
    dst columns and weights equal the staged build's, for hubs and ordinary vertices"""
    a, b = pair16
    vids = np.concatenate([synth.hub_candidates(16, 1)[:8], synth.seeds(16, 16, 1, 56)])
    parts = np.array([a.part_of(int(v)) for v in vids], dtype=np.int32)
    cols = ["_dst", "weight"]
    for et in (FOLLOW, -FOLLOW):
        ra = a.get_bound(et, parts, vids, cols if et > 0 else ["_dst"])
        rb = b.get_bound(et, parts, vids, cols if et > 0 else ["_dst"])
        assert ra.n_rows == rb.n_rows and ra.n_rows > 0
        for ca, cb in zip(ra.columns, rb.columns):
            assert np.array_equal(np.asarray(ca), np.asarray(cb))
        assert np.array_equal(np.asarray(ra.vertex_ids), np.asarray(rb.vertex_ids))


@pytest.mark.parametrize("steps", [1, 2, 3])
def test_go_plain_matches_oracle(pair16, steps):
    _, b = pair16
    g = O.RmatGraph(16, 16, 1)
    starts = synth.seeds(16, 16, 1, 16)
    r = b.go(starts, steps, FOLLOW)
    want, scanned = g.go(starts, steps)
    assert np.array_equal(np.sort(r.columns[0]), want)
    assert r.edges_scanned == scanned


def test_bench_query_top_down_only(pair16):
    """no transposed CSR in a streamed snapshot: every hop runs top-down, same answer"""
    _, b = pair16
    starts = synth.seeds(16, 16, 1, 64)
    r = b.go(starts, 3, FOLLOW, where=W499, yields=[X.EdgeDst("follow")], distinct=True)
    g = GOLD["go3_where499_distinct_s16"]
    assert len(r.columns[0]) == g["n_rows"]
    assert O.digest(r.columns[0]) == g["sha256"]
    assert r.edges_scanned == g["edges_scanned"]
    assert b.last_timing()["bu_steps"] == 0


def test_shortest_paths_match_staged(pair16):
    a, b = pair16
    s, t = synth.pairs(16, 16, 1, 256)
    ra, rb = a.shortest_path(s, t, FOLLOW, 8), b.shortest_path(s, t, FOLLOW, 8)
    assert np.array_equal(ra.hops, rb.hops)
    for i in range(len(s)):
        assert np.array_equal(ra.paths[i], rb.paths[i]), i


def test_configs1_rmat22_streamed_digest():
    """configs[1] (GO 3 STEPS plain rows, RMAT-22) on a streamed snapshot, by digest"""
    sp = space(22, rmat_stream=1, rmat_bucket=1 << 24)  # 4 buckets per direction
    try:
        r = sp.go(synth.seeds(22, 16, 1, 64), 3, FOLLOW)
        g = GOLD["go3_plain_s22"]
        assert len(r.columns[0]) == g["n_rows"]
        assert O.digest(r.columns[0]) == g["sha256"]
        assert r.edges_scanned == g["edges_scanned"]
    finally:
        sp.close()


def test_streamed_snapshot_is_read_only():
    sp = GraphSpace(64)
    try:
        sp.set_option("rmat_stream", 1)
        sp.set_option("writable", 1)
        sp.set_edge_schema(FOLLOW, [("weight", O.INT)])
        with pytest.raises(Exception):
            sp.gen_rmat(12, 16, 1, FOLLOW)
    finally:
        sp.close()


def hub_starts(sp, scale, seeds=64, hubs=8):
    """bench.py --hubs: the top-N out-degree vertices among synth.hub_candidates replace the
    first N seeds (configs[4]'s supernode seeds)"""
    cand = synth.hub_candidates(scale, 1)
    deg = np.array([sp.out_degree(FOLLOW, int(v)) for v in cand], dtype=np.int64)
    order = np.argsort(-deg, kind="stable")[:hubs]
    return np.concatenate([cand[order].astype(np.int64), synth.seeds(scale, 16, 1, seeds)[hubs:]])


def check_msum(name, col, scanned):
    g = GOLD[name]
    n, sm, x = O.msum(col)
    assert n == g["n_rows"]
    assert [str(sm), str(x)] == g["msum"]
    assert scanned == g["edges_scanned"]


def test_configs4_shape_rmat16(pair16):
    """configs[4]'s query shape (GO 2 STEPS, supernode seeds, plain rows) on both builds"""
    a, b = pair16
    for sp in (a, b):
        r = sp.go(hub_starts(sp, 16), 2, FOLLOW)
        check_msum("go2_plain_s16_seeds64_hubs8", r.columns[0], r.edges_scanned)


@pytest.mark.skipif("go2_plain_s28_seeds64_hubs8" not in GOLD, reason="digest not generated")
def test_configs4_rmat28_digest():
    """configs[4] at its size on one GPU: RMAT-28 (2^32 samples, 4.26 G edges) through the
    streamed build, GO 2 STEPS from the top-8 hubs + 56 seeds: 2.7 G rows by order-free digest"""
    sp = space(28)  # rmat_stream is automatic past 2^31 samples on one rank
    try:
        r = sp.go(hub_starts(sp, 28), 2, FOLLOW)
        check_msum("go2_plain_s28_seeds64_hubs8", r.columns[0], r.edges_scanned)
    finally:
        sp.close()
