"""GPU parity of outBoundStats / inBoundStats against the oracle's
QueryStatsProcessor restatement, which is pinned by the reference's QueryStatsTest
(src/storage/test/QueryStatsTest.cpp) in tests/test_oracle_storage.py.

The device path takes the getBound scan with its filter push-down and reduces the kept edges on
the GPU (k_bound_stats); SOURCE/DEST tag columns reduce the request entries' vertex rows
(QueryStatsProcessor.cpp:69-82).  Known answers: QueryStatsTest's checkResponse (AVG of
tag_3001_col_0 = 0.0 and of tag_3003_col_2 = 2.0; SUM of col_2i over 210 edges = 2i * 210).
"""
import numpy as np
import pytest

import fixtures as F
import oracle as O
from nebula_amd import AVG, COUNT, SUM, GetNeighborsRequest, GraphSpace, NbgError, PropDef, QueryStatsProcessor
from nebula_amd.engine import IN_BOUND
from nebula_amd import expr as X

pytestmark = pytest.mark.gpu

FOLLOW = 1
SEED = 1


def same(a, b):
    assert len(a) == len(b)
    for x, y in zip(a, b):
        if isinstance(x, float) or isinstance(y, float):
            assert (np.isnan(x) and np.isnan(y)) or x == y, (a, b)
        else:
            assert x == y, (a, b)


@pytest.fixture(scope="module")
def qs():
    sp = GraphSpace(6)
    sp.set_edge_schema(F.EDGE_TYPE, F.qb_edge_schema())
    for tag in range(3001, 3010):
        sp.set_tag_schema(tag, str(tag), F.qb_tag_schema(tag))
    for part, data in F.qs_kv_parts().items():
        sp.load_part(part, data)
    sp.finalize()
    st = F.qs_oracle_store()
    yield sp, st
    sp.close()


def test_stats_fixture_edge_columns(qs):
    """QueryStatsTest's edge columns: SUM(col_2i) = 2i * 210 (QueryStatsTest.cpp:88-135)"""
    sp, st = qs
    parts, vids, cols, stats = F.qs_request()
    cols, stats = cols[2:], stats[2:]
    g = sp.bound_stats(F.EDGE_TYPE, parts, vids, cols, stats)
    assert g.failed == [] and g.n_rows == 1
    assert g.rows()[0] == tuple(i * 2 * 210 for i in range(5))
    r = st.bound_stats(F.EDGE_TYPE, parts, vids, cols, stats)
    same(g.rows()[0], r.rows()[0])


def test_stats_mixed_columns_and_filter(qs):
    sp, st = qs
    parts, vids, _, _ = F.qs_request()
    cols = [("col_1", O.EDGE, 0), ("_dst", O.EDGE, 0), ("_rank", O.EDGE, 0),
            ("col_10", O.EDGE, 0), ("_src", O.EDGE, 0), ("col_9", O.EDGE, 0)]
    stats = [AVG, COUNT, SUM, COUNT, SUM, AVG]
    for f in (b"", (X.AliasProp("e101", "col_3") > 2).encode(), (X.AliasProp("e101", "col_5") < 3).encode()):
        g = sp.bound_stats(F.EDGE_TYPE, parts, vids, cols, stats, f)
        r = st.bound_stats(F.EDGE_TYPE, parts, vids, cols, stats, filt=f)
        if r.code:
            pytest.skip(f"oracle rejects the filter: {r.error}")
        same(g.rows()[0], r.rows()[0])
        assert g.types == [O.DOUBLE, O.INT, O.INT, O.INT, O.INT, O.DOUBLE]


def test_stats_validation(qs):
    sp, st = qs
    parts, vids, _, _ = F.qs_request()
    g = sp.bound_stats(F.EDGE_TYPE, parts, vids, [("col_10", O.EDGE, 0)], [SUM])
    r = st.bound_stats(F.EDGE_TYPE, parts, vids, [("col_10", O.EDGE, 0)], [SUM])
    assert g.n_rows == 0 and sorted(g.failed) == sorted(r.failed()) == [(0, -23), (1, -23), (2, -23)]
    g = sp.bound_stats(F.EDGE_TYPE, parts, vids, [("no_such", O.EDGE, 0)], [COUNT])
    assert sorted(g.failed) == [(0, -23), (1, -23), (2, -23)]
    # tag columns: unknown tag, unknown prop, SUM / AVG over a STRING prop (validOperation)
    for cols, stats in (([("tag_3001_col_0", O.SOURCE, 4242)], [AVG]),
                        ([("no_such", O.SOURCE, 3001)], [COUNT]),
                        ([("tag_3001_col_3", O.SOURCE, 3001)], [SUM]),
                        ([("col_0", O.EDGE, 0), ("tag_3001_col_4", O.DEST, 3001)], [SUM, AVG])):
        g = sp.bound_stats(F.EDGE_TYPE, parts, vids, cols, stats)
        r = st.bound_stats(F.EDGE_TYPE, parts, vids, cols, stats)
        assert g.n_rows == 0 and sorted(g.failed) == sorted(r.failed()), cols
        assert len(g.failed) == 3


def test_stats_fixture_all_columns(qs):
    """QueryStatsTest StatsSimpleTest's full request (2 SOURCE tag columns with AVG + 5 edge
    columns with SUM) and checkResponse's expected values (QueryStatsTest.cpp:88-135)"""
    sp, st = qs
    parts, vids, cols, stats = F.qs_request()
    g = sp.bound_stats(F.EDGE_TYPE, parts, vids, cols, stats)
    assert g.failed == [] and g.n_rows == 1
    assert g.types == [O.DOUBLE, O.DOUBLE] + [O.INT] * 5
    assert g.rows()[0] == (0.0, 2.0) + tuple(i * 2 * 210 for i in range(5))
    r = st.bound_stats(F.EDGE_TYPE, parts, vids, cols, stats)
    same(g.rows()[0], r.rows()[0])


def test_stats_tag_columns_vs_oracle(qs):
    """tag columns mixed with edge columns and a filter, every stat, SOURCE and DEST owners,
    duplicate entries, a vertex without rows, entries whose part does not hold the vertex's row,
    a part out of range (failed, its entries not counted)"""
    sp, st = qs
    parts, vids, _, _ = F.qs_request()
    parts = list(parts) + [0, 0, 1, 2, 1, 9]
    vids = list(vids) + [3, 3, 5, 999, 20, 4]
    cols = [("tag_3002_col_1", O.SOURCE, 3002), ("col_3", O.EDGE, 0), ("tag_3005_col_2", O.DEST, 3005),
            ("tag_3007_col_5", O.SOURCE, 3007), ("tag_3002_col_1", O.SOURCE, 3002), ("_dst", O.EDGE, 0)]
    stats = [SUM, AVG, AVG, COUNT, COUNT, COUNT]
    for f in (b"", (X.AliasProp("e101", "col_3") > 2).encode()):
        g = sp.bound_stats(F.EDGE_TYPE, parts, vids, cols, stats, f)
        r = st.bound_stats(F.EDGE_TYPE, parts, vids, cols, stats, filt=f)
        assert sorted(g.failed) == sorted(r.failed())
        same(g.rows()[0], r.rows()[0])
        assert g.types == [O.INT, O.DOUBLE, O.DOUBLE, O.INT, O.INT, O.INT]


def test_stats_empty_request_and_no_rows(qs):
    sp, st = qs
    cols, stats = [("col_1", O.EDGE, 0), ("col_1", O.EDGE, 0), ("col_1", O.EDGE, 0)], [SUM, COUNT, AVG]
    g = sp.bound_stats(F.EDGE_TYPE, [], [], cols, stats)
    r = st.bound_stats(F.EDGE_TYPE, [], [], cols, stats)
    same(g.rows()[0], r.rows()[0])  # 0, 0, NaN
    g = sp.bound_stats(F.EDGE_TYPE, [0, 1], [999, 998], cols, stats)
    r = st.bound_stats(F.EDGE_TYPE, [0, 1], [999, 998], cols, stats)
    same(g.rows()[0], r.rows()[0])


@pytest.fixture(scope="module")
def rmat12():
    sp = GraphSpace(64)
    sp.set_edge_schema(FOLLOW, [("weight", O.INT)])
    sp.gen_rmat(12, 16, SEED, FOLLOW)
    sp.finalize()
    st = O.Store(64)
    st.set_edge_schema(FOLLOW, [("weight", O.INT)], name="follow")
    st.load_rmat(12, 16, SEED, FOLLOW)
    yield sp, st
    sp.close()


@pytest.mark.parametrize("k", [-1, 499, 990])
def test_rmat_stats_out_and_in_bound(rmat12, k):
    sp, st = rmat12
    s, _, _ = O.rmat_edges(12, 16, SEED)
    rng = np.random.default_rng(k + 5)
    vids = [int(x) for x in s[rng.integers(0, len(s), 300)]] + [123456789]
    parts = [O.part_of(v, 64) for v in vids]
    cols = [("weight", O.EDGE, 0), ("weight", O.EDGE, 0), ("weight", O.EDGE, 0), ("_dst", O.EDGE, 0),
            ("_src", O.EDGE, 0), ("_rank", O.EDGE, 0)]
    stats = [SUM, COUNT, AVG, SUM, SUM, COUNT]
    f = (X.AliasProp("follow", "weight") > k).encode()
    g = sp.bound_stats(FOLLOW, parts, vids, cols, stats, f)
    r = st.bound_stats(FOLLOW, parts, vids, cols, stats, filt=f)
    same(g.rows()[0], r.rows()[0])
    # in-bound: edge props are skipped, key props stay (QueryBaseProcessor.inl:80-99)
    g = sp.bound_stats(-FOLLOW, parts, vids, cols, stats)
    r = st.bound_stats(-FOLLOW, parts, vids, cols, stats, in_bound=True)
    assert len(g.rows()[0]) == 3
    same(g.rows()[0], r.rows()[0])


def test_query_stats_processor_shape(qs):
    """QueryStatsProcessor::instance(space).process(req) -> schema + one row"""
    sp, _ = qs
    parts, vids, _, _ = F.qs_request()
    req_parts = {}
    for p, v in zip(parts, vids):
        req_parts.setdefault(p, []).append(v)
    req = GetNeighborsRequest(0, req_parts, F.EDGE_TYPE,
                              return_columns=[(PropDef(O.EDGE, "col_4"), SUM), (PropDef(O.EDGE, "_dst"), COUNT)])
    resp = QueryStatsProcessor.instance(sp).process(req)
    assert resp.failed_codes == []
    assert [n for n, _ in resp.schema] == ["col_4", "_dst"]
    assert resp.row == (4 * 210, 210)


def test_query_stats_processor_in_bound():
    """IN_BOUND: the request carries -edge_type (StorageClient.cpp:116) and is scanned as is
    (QueryBaseProcessor.inl:39-40); QueryBoundTest's fixture has 5 in-edges x 3 versions each"""
    sp = GraphSpace(6)
    sp.set_edge_schema(F.EDGE_TYPE, F.qb_edge_schema())
    for part, data in F.qb_kv_parts().items():
        sp.load_part(part, data)
    sp.finalize()
    try:
        parts, vids, _ = F.qb_request(False)
        req_parts = {}
        for p, v in zip(parts, vids):
            req_parts.setdefault(p, []).append(v)
        req = GetNeighborsRequest(0, req_parts, -F.EDGE_TYPE, return_columns=[(PropDef(O.EDGE, "_dst"), COUNT)])
        resp = QueryStatsProcessor.instance(sp, IN_BOUND).process(req)
        assert resp.failed_codes == []
        assert resp.row == (30 * 5,)
    finally:
        sp.close()
