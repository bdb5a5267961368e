"""The index-space restatement (oracle/rmat_graph.cpp) against the faithful KV-store restatement
(oracle/refcpu.cpp: storaged + graphd over the reference byte layout) at small scales.

The index-space restatement is what checks the HIP path at the configured sizes (RMAT-18..26,
tests/test_gpu_scale.py and the committed digests); this pins it to the faithful one on the
same graph: identical result multisets, identical edges_scanned, identical shortest paths.
"""
import numpy as np
import pytest

import oracle as O
from nebula_amd import expr as X
from nebula_amd import synth

FOLLOW = 1


@pytest.fixture(scope="module", params=[12, 14])
def both(request):
    scale = request.param
    st = O.Store(64)
    st.set_edge_schema(FOLLOW, [("weight", O.INT)], name="follow")
    st.load_rmat(scale, 16, 1, FOLLOW)
    g = O.RmatGraph(scale, 16, 1, threads=4)
    return scale, st, g


def test_graph_size_matches_kv_store(both):
    scale, st, g = both
    # every distinct (src, dst) writes one out key and one in key
    assert st.num_keys() == 2 * g.info()["num_edges"]


@pytest.mark.parametrize("steps", [1, 2, 3])
def test_go_distinct_where_matches_faithful(both, steps):
    scale, st, g = both
    starts = synth.seeds(scale, 16, 1, 64)
    w = X.AliasProp("follow", "weight") > 499
    r = st.go(starts, steps, FOLLOW, where=w.encode(), yields=[X.EdgeDst("follow").encode()], distinct=True)
    got, scanned = g.go(starts, steps, where_gt=499, distinct=True)
    assert np.array_equal(got, np.sort(r.int_col(0)))
    assert scanned == r.edges_scanned


@pytest.mark.parametrize("op", [">", ">=", "<", "<=", "==", "!="])
def test_go_distinct_every_operator_matches_faithful(both, op):
    """every relational operator (Expressions.cpp:891-933) at constants below, on the edges of,
    inside and above the weight range [0, 999]"""
    scale, st, g = both
    starts = synth.seeds(scale, 16, 1, 48)
    wcol = X.AliasProp("follow", "weight")
    mk = {">": lambda k: wcol > k, ">=": lambda k: wcol >= k, "<": lambda k: wcol < k,
          "<=": lambda k: wcol <= k, "==": lambda k: wcol.eq(k), "!=": lambda k: wcol.ne(k)}[op]
    for k in (-5, 0, 499, 998, 999, 1000):
        w = mk(k)
        r = st.go(starts, 2, FOLLOW, where=w.encode(), yields=[X.EdgeDst("follow").encode()], distinct=True)
        got, scanned = g.go(starts, 2, distinct=True, where=(op, k))
        assert np.array_equal(got, np.sort(r.int_col(0))), (op, k)
        assert scanned == r.edges_scanned


@pytest.mark.parametrize("steps", [1, 2, 3])
def test_go_plain_rows_match_faithful(both, steps):
    scale, st, g = both
    starts = list(synth.seeds(scale, 16, 1, 16))
    starts += starts[:3]  # duplicates rescan at hop 1 (P14)
    r = st.go(starts, steps, FOLLOW)
    got, scanned = g.go(starts, steps)
    assert np.array_equal(got, np.sort(r.int_col(0)))
    assert scanned == r.edges_scanned
    assert O.digest(got) == O.digest(r.int_col(0))


def test_go_empty_and_unknown_start(both):
    scale, st, g = both
    got, scanned = g.go([12345678901], 2)
    assert len(got) == 0 and scanned == 0
    got, scanned = g.go([], 3, where_gt=10, distinct=True)
    assert len(got) == 0 and scanned == 0


def test_shortest_path_matches_faithful(both):
    scale, st, g = both
    s, t = synth.pairs(scale, 16, 1, 48)
    s = np.concatenate([s, s[:2], [7]])
    t = np.concatenate([t, s[:2], [7]])  # src == dst (a vertex, and a vid that is none)
    r = st.shortest_path(s, t, FOLLOW, 8)
    hops, paths = g.shortest_path(s, t, 8)
    rows = r.rows()
    for i in range(len(s)):
        assert hops[i] == rows[i][2]
        assert list(paths[i]) == [v for v in rows[i][3:] if v is not None]


def test_grouped_build_and_msum(both, monkeypatch):
    """the grouped CSR build (bucket groups of ORA_RMAT_GROUP_KEYS samples, one generator pass
    each: how RMAT-28 fits the build host) gives the single-pass build's graph, and the order-free
    msum digest of a plain GO equals the msum of its materialised rows"""
    scale, st, g = both
    monkeypatch.setenv("ORA_RMAT_GROUP_KEYS", str(1 << 12))
    g2 = O.RmatGraph(scale, 16, 1, threads=4)
    assert g2.info() == g.info()
    starts = synth.seeds(scale, 16, 1, 16)
    for steps in (1, 2, 3):
        r1, s1 = g.go(starts, steps)
        r2, s2 = g2.go(starts, steps)
        assert np.array_equal(r1, r2) and s1 == s2
        ms, sc = g2.go_msum(starts, steps)
        assert ms == O.msum(r1) and sc == s1
    # msum is order-free and sensitive to the multiset
    r1, _ = g.go(starts, 2)
    assert O.msum(r1[::-1]) == O.msum(r1)
    assert O.msum(r1[1:]) != O.msum(r1)
