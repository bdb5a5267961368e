"""GPU parity: the HIP path (through the C ABI) against the oracle and the reference fixtures.

Every comparison is bit-exact on integer/byte results; rows are compared as multisets after
sorting (the reference's own result check, src/graph/test/TestBase.h:182-222).
"""
from collections import Counter

import numpy as np
import pytest

import fixtures as F
import oracle as O
from nebula_amd import GraphSpace, NbgError
from nebula_amd import expr as X

pytestmark = pytest.mark.gpu

FOLLOW = 1
SEED = 1


def ms(rows):
    return Counter(tuple(r) for r in rows)


# ------------------------------------------------------------------------------------------
# NBA dataset (GoTest)
# ------------------------------------------------------------------------------------------
@pytest.fixture(scope="module")
def nba():
    sp = GraphSpace(1)
    for et, (name, fields) in F.NBA_EDGE_SCHEMAS.items():
        sp.set_edge_schema(et, fields)
    parts, vid = F.nba_kv()
    for p, kv in parts.items():
        sp.load_part(p, kv)
    sp.finalize()
    st, _ = F.nba_oracle_store()
    yield sp, st, vid, F.nba()
    sp.close()


def names(vid, rows):
    inv = {v: k for k, v in vid.items()}
    return Counter(tuple(inv.get(c, c) if isinstance(c, int) and c in inv else c for c in r) for r in rows)


def golden(d, key):
    return Counter(tuple(r) for r in d["expect"][key]["rows"])


def gpu_pipe(sp, starts, etypes, distinct_last=False, ylast=()):
    cur = list(starts)
    rs = None
    for i, et in enumerate(etypes):
        last = i == len(etypes) - 1
        rs = sp.go(cur, 1, et, yields=ylast if last else (), distinct=distinct_last and last)
        cur = [r[0] for r in rs.rows()]
    return rs


def test_nba_one_step(nba):
    sp, st, vid, d = nba
    rs = sp.go([vid["Tim Duncan"]], 1, F.NBA_SERVE)
    assert names(vid, rs.rows()) == golden(d, "one_step_serve_tim")


def test_nba_yield_props_and_where(nba):
    sp, st, vid, d = nba
    ys = [X.AliasProp("serve", "start_year"), X.AliasProp("serve", "end_year"), X.EdgeDst("serve")]
    rs = sp.go([vid["Boris Diaw"]], 1, F.NBA_SERVE, yields=ys)
    assert names(vid, rs.rows()) == golden(d, "serve_boris_years")
    w = (X.AliasProp("serve", "start_year") >= 2013) & (X.AliasProp("serve", "end_year") <= 2018)
    rs = sp.go([vid["Rajon Rondo"]], 1, F.NBA_SERVE, where=w, yields=ys)
    assert names(vid, rs.rows()) == golden(d, "serve_rondo_where")
    ref = st.go([vid["Rajon Rondo"]], 1, F.NBA_SERVE, where=w.encode(), yields=[y.encode() for y in ys])
    assert ms(rs.rows()) == ms(ref.rows())


def test_nba_pipes(nba):
    sp, st, vid, d = nba
    rs = gpu_pipe(sp, [vid["Boris Diaw"]], [F.NBA_LIKE, F.NBA_LIKE, F.NBA_SERVE])
    assert names(vid, rs.rows()) == golden(d, "pipe_boris_like_like_serve")
    rs = gpu_pipe(sp, [vid["Tracy McGrady"]], [F.NBA_LIKE, F.NBA_LIKE])
    assert names(vid, rs.rows()) == golden(d, "var_tracy_like_like")
    rs = gpu_pipe(sp, [vid["Tracy McGrady"]], [F.NBA_LIKE] * 3)
    assert names(vid, rs.rows()) == golden(d, "var_pipe_tracy")
    rs = gpu_pipe(sp, [vid["Boris Diaw"]], [F.NBA_LIKE, F.NBA_LIKE, F.NBA_SERVE], distinct_last=True,
                  ylast=[X.EdgeDst("serve")])
    assert names(vid, rs.rows()) == golden(d, "distinct_boris_serve_dst")


def test_nba_steps_and_empty(nba):
    sp, st, vid, d = nba
    rs = sp.go([vid["Boris Diaw"]], 3, F.NBA_LIKE)
    assert names(vid, rs.rows()) == golden(d, "derived_go3_boris_like")
    assert sp.go([d["nonexist_hash"]], 1, F.NBA_SERVE).n_rows == 0
    assert sp.go([d["nonexist_hash"]], 3, F.NBA_LIKE).n_rows == 0
    assert sp.go([], 2, F.NBA_LIKE).n_rows == 0


def test_nba_expression_semantics(nba):
    sp, st, vid, d = nba
    tim = [vid["Tim Duncan"], vid["Tony Parker"], vid["Dejounte Murray"]]
    cases = [
        X.AliasProp("like", "likeness") > 10.5,        # int vs double: variant index order
        X.AliasProp("like", "likeness") < 10.5,
        X.AliasProp("like", "likeness").eq(95.0),      # almostEqual
        X.AliasProp("like", "likeness").ne(95),
        (X.AliasProp("like", "likeness") % 7) > 2,
        ~(X.AliasProp("like", "likeness") >= 95) | X.Primary(False),
        X.Primary("x") > X.AliasProp("like", "likeness"),   # string vs int
        X.Unary(X.NOT, X.Primary("")),                       # asBool(string) is empty()
        (X.AliasProp("like", "likeness") * 2 - 100) / 3 > 20,
        X.EdgeDst("like") > 0,
        X.EdgeRank("like").eq(0),
    ]
    for w in cases:
        g = sp.go(tim, 1, F.NBA_LIKE, where=w, yields=[X.EdgeDst("like"), X.AliasProp("like", "likeness")])
        r = st.go(tim, 1, F.NBA_LIKE, where=w.encode(),
                  yields=[X.EdgeDst("like").encode(), X.AliasProp("like", "likeness").encode()])
        assert r.code == 0
        assert ms(g.rows()) == ms(r.rows()), w.encode()


def test_nba_eval_error_fails_query(nba):
    sp, st, vid, d = nba
    with pytest.raises(NbgError) as e:
        sp.go([vid["Tim Duncan"]], 1, F.NBA_LIKE, where=X.AliasProp("like", "nope") > 1)
    assert e.value.code == -23  # E_IMPROPER_DATA_TYPE
    with pytest.raises(NbgError):
        sp.go([vid["Tim Duncan"]], 1, F.NBA_LIKE, where=(X.AliasProp("like", "likeness") / 0) > 1)
    # the deferred error is not raised when the frontier empties first (onEmptyInputs)
    assert sp.go([d["nonexist_hash"]], 2, F.NBA_LIKE, where=X.AliasProp("like", "nope") > 1).n_rows == 0


def test_nba_yield_distinct_multicol(nba):
    sp, st, vid, d = nba
    starts = [p["vid"] for p in d["players"]]
    ys = [X.AliasProp("serve", "end_year"), X.AliasProp("serve", "end_year") > 2015]
    g = sp.go(starts, 1, F.NBA_SERVE, yields=ys, distinct=True)
    r = st.go(starts, 1, F.NBA_SERVE, yields=[y.encode() for y in ys], distinct=True)
    assert ms(g.rows()) == ms(r.rows())
    g = sp.go(starts, 2, F.NBA_LIKE, distinct=False)
    r = st.go(starts, 2, F.NBA_LIKE)
    assert ms(g.rows()) == ms(r.rows())


# ------------------------------------------------------------------------------------------
# QueryBoundTest fixture (storage getBound)
# ------------------------------------------------------------------------------------------
@pytest.fixture(scope="module")
def qb():
    sp = GraphSpace(6)
    sp.set_edge_schema(F.EDGE_TYPE, F.qb_edge_schema())
    for tag in range(3001, 3010):
        sp.set_tag_schema(tag, str(tag), F.qb_tag_schema(tag))
    for part, data in F.qb_kv_parts().items():
        sp.load_part(part, data)
    sp.finalize()
    st = F.qb_oracle_store()
    yield sp, st
    sp.close()


def edge_cols():
    return [("_dst", O.EDGE, 0), ("_rank", O.EDGE, 0)] + [(f"col_{i * 2}", O.EDGE, 0) for i in range(10)]


def by_vertex(rs):
    out = {}
    rows = rs.rows()
    for i, v in enumerate(rs.vertex_ids):
        out[int(v)] = rows[rs.vertex_row_offsets[i]:rs.vertex_row_offsets[i + 1]]
    return out


def oracle_by_vertex(res):
    out = {}
    for r, row in enumerate(res.rows()):
        out.setdefault(res.row_vertex(r), []).append(row)
    return out


@pytest.mark.parametrize("filt", [
    None,
    X.Relational(X.GE, X.AliasProp("e101", "col_0"), X.Primary(10007)),
    X.Relational(X.LT, X.AliasProp("e101", "col_2"), X.Primary(10005)) | (X.AliasProp("e101", "col_14").eq("string_col_14_2")),
    X.AliasProp("e101", "col_11") > X.Primary("string_col_11_1"),
    # firstLoop (QueryBaseProcessor.inl:349-402): the newest version (2) fails, so the scan keeps
    # reading versions until one passes and emits it -- one older-version row per vertex
    X.AliasProp("e101", "col_14").eq("string_col_14_1"),
    X.AliasProp("e101", "col_14").eq("string_col_14_0"),
    X.Relational(X.GE, X.AliasProp("e101", "col_0"), X.Primary(10003)) & X.AliasProp("e101", "col_10").eq("string_col_10_0"),
    X.Relational(X.GE, X.AliasProp("e101", "col_0"), X.Primary(10006)) | X.AliasProp("e101", "col_12").eq("string_col_12_1"),
])
def test_get_bound_matches_reference(qb, filt):
    sp, st = qb
    parts, vids, _ = F.qb_request()
    cols = edge_cols()
    f = X.encode(filt)
    g = sp.get_bound(F.EDGE_TYPE, parts, vids, cols, f)
    r = st.get_bound(F.EDGE_TYPE, parts, vids, cols, filt=f)
    assert g.failed == r.failed() == []
    gv, rv = by_vertex(g), oracle_by_vertex(r)
    assert gv == rv  # same vertices, same rows, same per-vertex order (bytewise key order)
    if filt is None:  # checkResponse expectations (QueryBoundTest.cpp:111-178), edge part
        assert len(gv) == 30
        for vid, rows in gv.items():
            assert [row[0] for row in rows] == list(range(10001, 10008))
            for row in rows:
                assert row[1] == 0
                assert list(row[2:7]) == [row[0] + 2 * i for i in range(5)]
                assert list(row[7:]) == [f"string_col_{(i + 5) * 2}_2" for i in range(5)]


@pytest.mark.parametrize("out_bound", [True, False])
def test_get_bound_tag_props(qb, out_bound):
    # checkResponse's vertex part (QueryBoundTest.cpp:111-178): SOURCE tag props of every vertex,
    # read from the request's part (the fixture stores vertices outside their hash part)
    sp, st = qb
    parts, vids, cols = F.qb_request(out_bound)
    et = F.EDGE_TYPE if out_bound else -F.EDGE_TYPE
    g = sp.get_bound(et, parts, vids, cols)
    r = st.get_bound(et, parts, vids, cols, in_bound=not out_bound)
    assert g.failed == r.failed() == []
    assert len(g.vertex_ids) == 30 and len(g.vertex_columns) == 3
    ref = dict(r.vertices())
    for i, vid in enumerate(g.vertex_ids):
        vals = [col[i] for col in g.vertex_columns]
        assert vals == [int(vid) + 3001, int(vid) + 3003 + 2, "tag_string_col_4"]
        assert tuple(vals) == tuple(ref[int(vid)])
    assert by_vertex(g) == oracle_by_vertex(r)
    # the same vertices asked under their hash part: only those whose fixture part happens to be
    # their hash part have rows there (edges and tags alike)
    hp = [O.part_of(v, 6) for v in vids]
    g = sp.get_bound(et, hp, vids, cols)
    r = st.get_bound(et, hp, vids, cols, in_bound=not out_bound)
    ref = dict(r.vertices())
    assert sorted(int(v) for v in g.vertex_ids) == sorted(ref)
    for i, vid in enumerate(g.vertex_ids):
        assert tuple(col[i] for col in g.vertex_columns) == tuple(ref[int(vid)])
    assert by_vertex(g) == oracle_by_vertex(r)


@pytest.mark.parametrize("case", ["only_tag", "tag_and_edge", "tag_string", "tag_or_edge"])
def test_get_bound_tag_filters(qb, case):
    # QueryBoundTest FilterOnlyTag (:260-291) / FilterTagAndEdge (:345-385): the push-down filter
    # reads $^ props of the request part's vertex row; an evaluation error keeps the edge
    sp, st = qb
    parts, vids, cols = F.qb_request()
    tag = X.Relational(X.GE, X.SourceProp("3001", "tag_3001_col_0"), X.Primary(20 + 3001))
    edge = X.Relational(X.GE, X.AliasProp("e101", "col_0"), X.Primary(10007))
    filt = {"only_tag": tag, "tag_and_edge": X.Logical(X.AND, tag, edge),
            "tag_string": X.SourceProp("3005", "tag_3005_col_4").eq("tag_string_col_4"),
            "tag_or_edge": X.Logical(X.OR, X.SourceProp("3002", "tag_3002_col_1") < 3010, edge)}[case]
    g = sp.get_bound(F.EDGE_TYPE, parts, vids, cols, filt)
    r = st.get_bound(F.EDGE_TYPE, parts, vids, cols, filt=filt.encode())
    assert g.failed == r.failed() == []
    assert by_vertex(g) == oracle_by_vertex(r)
    ref = dict(r.vertices())
    for i, vid in enumerate(g.vertex_ids):
        assert tuple(col[i] for col in g.vertex_columns) == tuple(ref[int(vid)])
    if case == "only_tag":  # check_response(res, 10, 12, 10001, 7, True)
        assert len(g.vertex_ids) == 10 and all(len(v) == 7 for v in by_vertex(g).values())
    if case == "tag_and_edge":  # check_response(res, 10, 12, 10007, 1, True)
        assert len(g.vertex_ids) == 10 and all(len(v) == 1 for v in by_vertex(g).values())
    # $$ and unknown tag props are invalid storage filters (checkExp)
    for bad in (X.DestProp("3001", "tag_3001_col_0") > 1, X.SourceProp("3001", "nope") > 1,
                X.SourceProp("9999", "tag_3001_col_0") > 1):
        g = sp.get_bound(F.EDGE_TYPE, parts, vids, cols, bad)
        assert sorted(g.failed) == [(0, -31), (1, -31), (2, -31)]


def test_get_bound_tag_prop_errors(qb):
    sp, st = qb
    parts, vids, _ = F.qb_request()
    g = sp.get_bound(F.EDGE_TYPE, parts, vids, edge_cols() + [("tag_3001_col_0", O.SOURCE, 4242)])
    assert sorted(g.failed) == [(0, -22), (1, -22), (2, -22)]
    g = sp.get_bound(F.EDGE_TYPE, parts, vids, edge_cols() + [("nope", O.SOURCE, 3001)])
    assert sorted(g.failed) == [(0, -23), (1, -23), (2, -23)]


def test_get_bound_in_bound(qb):
    sp, st = qb
    parts, vids, _ = F.qb_request(False)
    cols = edge_cols()
    g = sp.get_bound(-F.EDGE_TYPE, parts, vids, cols)
    r = st.get_bound(-F.EDGE_TYPE, parts, vids, cols, in_bound=True)
    gv = by_vertex(g)
    assert gv == oracle_by_vertex(r)
    assert len(gv) == 30 and all([row[0] for row in rows] == list(range(20001, 20006)) for rows in gv.values())


def test_get_bound_invalid_filter(qb):
    sp, st = qb
    parts, vids, _ = F.qb_request()
    g = sp.get_bound(F.EDGE_TYPE, parts, vids, edge_cols(), X.InputProp("tag_3001_col_0"))
    assert sorted(g.failed) == [(0, -31), (1, -31), (2, -31)]
    g = sp.get_bound(F.EDGE_TYPE, parts, vids, edge_cols() + [("nope", O.EDGE, 0)])
    assert sorted(g.failed) == [(0, -23), (1, -23), (2, -23)]


def test_get_bound_wrong_part_and_dups(qb):
    sp, st = qb
    # vertex 5 lives in part 0; asking part 1 scans an empty prefix. Duplicates repeat rows.
    parts, vids = [1, 0, 0], [5, 5, 5]
    cols = edge_cols()
    g = sp.get_bound(F.EDGE_TYPE, parts, vids, cols)
    r = st.get_bound(F.EDGE_TYPE, parts, vids, cols)
    assert g.n_rows == r.nrows == 14
    assert ms(g.rows()) == ms(r.rows())


# ------------------------------------------------------------------------------------------
# synthetic RMAT: device generator + KV ingest vs the oracle
# ------------------------------------------------------------------------------------------
def oracle_rmat(scale, versions=1, parts=64):
    st = O.Store(parts)
    st.set_edge_schema(FOLLOW, [("weight", O.INT)], name="follow")
    st.load_rmat(scale, 16, SEED, FOLLOW, versions=versions)
    return st


def seeds_from(scale, n, seed=7):
    s, d, w = O.rmat_edges(scale, 16, SEED)
    rng = np.random.default_rng(seed)
    return [int(x) for x in s[rng.integers(0, len(s), n)]]


@pytest.fixture(scope="module")
def rmat12():
    sp = GraphSpace(64)
    sp.set_edge_schema(FOLLOW, [("weight", O.INT)])
    sp.gen_rmat(12, 16, SEED, FOLLOW)
    sp.finalize()
    st = oracle_rmat(12)
    yield sp, st
    sp.close()


@pytest.mark.parametrize("steps", [1, 2, 3])
def test_rmat_go_steps(rmat12, steps):
    sp, st = rmat12
    starts = seeds_from(12, 16)
    g = sp.go(starts, steps, FOLLOW)
    r = st.go(starts, steps, FOLLOW)
    assert g.n_rows == r.nrows
    assert np.array_equal(np.sort(g.columns[0]), np.sort(r.int_col(0)))
    assert g.edges_scanned == r.edges_scanned


@pytest.mark.parametrize("small", [1, 0])
def test_rmat_start_frontier_edge_cases(rmat12, small):
    """the one-launch start frontier of a top-down first hop (k_starts_small, option starts_small)
    and the multi-kernel path against the oracle: duplicate starts, vids not in the graph, starts
    without out-edges, DISTINCT or not (hop-1 rows of a non-DISTINCT query rescan duplicate
    starts), 4096 starts (the most the one-block kernel takes) and 4097 (the fallback path)"""
    sp, st = rmat12
    sp.set_option("starts_small", small)
    s, d, _ = O.rmat_edges(12, 16, SEED)
    no_out = sorted(set(d.tolist()) - set(s.tolist()))[:8]
    assert no_out
    base = seeds_from(12, 40, seed=31)
    starts = base + base[:10] + [123456789, -5] + no_out
    w = X.AliasProp("follow", "weight") > 499
    y = [X.EdgeDst("follow")]
    for steps in (2, 3):
        g = sp.go(starts, steps, FOLLOW)
        r = st.go(starts, steps, FOLLOW)
        assert np.array_equal(np.sort(g.columns[0]), np.sort(r.int_col(0)))
        assert g.edges_scanned == r.edges_scanned
        g = sp.go(starts, steps, FOLLOW, where=w, yields=y, distinct=True)
        r = st.go(starts, steps, FOLLOW, where=w.encode(), yields=[y[0].encode()], distinct=True)
        assert np.array_equal(np.sort(g.columns[0]), np.sort(r.int_col(0)))
        assert g.edges_scanned == r.edges_scanned
    # only starts without out-edges: an empty first frontier
    g = sp.go(no_out, 2, FOLLOW)
    assert g.n_rows == 0 and st.go(no_out, 2, FOLLOW).nrows == 0
    sp.set_option("bottom_up", 0)  # a top-down first hop is then certain at any start count
    for n in (4096, 4097):
        many = seeds_from(12, n, seed=n)
        g = sp.go(many, 2, FOLLOW)
        r = st.go(many, 2, FOLLOW)
        assert np.array_equal(np.sort(g.columns[0]), np.sort(r.int_col(0)))
        assert g.edges_scanned == r.edges_scanned


@pytest.mark.parametrize("bu_div", [1, 2, 4, 16, 256])
def test_rmat_speculative_hops(rmat12, bu_div):
    """speculative bottom-up hops (bu_spec: the hops after a top-down compaction enqueued as gated
    bottom-up hops before one counter fetch) take exactly the directions the host's choice takes
    without speculation -- same hop modes and counters -- and return the oracle's rows, at
    thresholds where the gate passes everywhere, only for some hops, or nowhere"""
    sp, st = rmat12
    sp.set_option("bu_div", bu_div)
    starts = sorted(set(seeds_from(12, 24, seed=41)))
    w = X.AliasProp("follow", "weight") > 499
    y = [X.EdgeDst("follow")]
    for steps in (2, 3, 4):
        for where, distinct in ((w, True), (None, True), (None, False)):
            runs = []
            for spec in (1, 0):
                sp.set_option("bu_spec", spec)
                g = sp.go(starts, steps, FOLLOW, where=where, yields=y if distinct else (), distinct=distinct)
                t = sp.last_timing()
                hops = t["hops"]
                if spec:
                    # a bottom-up hop right after a top-down hop ran behind its device gate
                    # (the final DISTINCT hop included), never re-run by the host
                    tr = [i for i in range(1, len(hops))
                          if hops[i - 1]["mode"] == "top-down" and hops[i]["mode"] == "bottom-up"]
                    assert t["spec_hops"] >= len(tr), (steps, distinct, t["spec_hops"], tr)
                else:
                    assert t["spec_hops"] == 0
                runs.append((np.sort(g.columns[0]), g.edges_scanned, [(h["mode"], h["c"]) for h in hops]))
            assert np.array_equal(runs[0][0], runs[1][0]) and runs[0][1] == runs[1][1]
            assert runs[0][2] == runs[1][2], (steps, distinct)
            r = st.go(starts, steps, FOLLOW, where=w.encode() if where is not None else b"",
                      yields=[y[0].encode()] if distinct else (), distinct=distinct)
            assert np.array_equal(runs[0][0], np.sort(r.int_col(0)))
            assert runs[0][1] == r.edges_scanned
    sp.set_option("bu_spec", 1)
    sp.set_option("bu_div", 4)


def test_rmat_speculative_hops_ran(rmat12):
    """the gated path itself is exercised: over the thresholds above, some non-final and some
    final (DISTINCT _dst) hops ran behind their gates (nbg_timing.spec_hops)"""
    sp, _ = rmat12
    starts = sorted(set(seeds_from(12, 24, seed=41)))
    w = X.AliasProp("follow", "weight") > 499
    nonfinal = final = 0
    try:
        for bu_div in (1, 2, 4, 16, 256):
            sp.set_option("bu_div", bu_div)
            for steps in (2, 3, 4):
                sp.go(starts, steps, FOLLOW, where=w, yields=[X.EdgeDst("follow")], distinct=True)
                t = sp.last_timing()
                hops = t["hops"]
                if t["spec_hops"] and hops[-1]["final"] and hops[-1]["mode"] == "bottom-up":
                    # speculated hops are the last ones of the query
                    final += 1
                    nonfinal += t["spec_hops"] - 1
                else:
                    nonfinal += t["spec_hops"]
    finally:
        sp.set_option("bu_div", 4)
    assert nonfinal > 0 and final > 0, (nonfinal, final)


def test_rmat_go_where_distinct(rmat12):
    sp, st = rmat12
    starts = seeds_from(12, 64)
    w = X.AliasProp("follow", "weight") > 499
    y = [X.EdgeDst("follow")]
    g = sp.go(starts, 3, FOLLOW, where=w, yields=y, distinct=True)
    r = st.go(starts, 3, FOLLOW, where=w.encode(), yields=[y[0].encode()], distinct=True)
    assert np.array_equal(np.sort(g.columns[0]), np.sort(r.int_col(0)))
    assert len(set(g.columns[0].tolist())) == g.n_rows
    # non-distinct with a VM predicate and computed yields
    w2 = (X.AliasProp("follow", "weight") % 3).eq(1) & (X.EdgeSrc("follow") > 0)
    y2 = [X.EdgeSrc("follow"), X.EdgeDst("follow"), X.AliasProp("follow", "weight") * 2]
    g = sp.go(starts, 2, FOLLOW, where=w2, yields=y2)
    r = st.go(starts, 2, FOLLOW, where=w2.encode(), yields=[y.encode() for y in y2])
    assert ms(g.rows()) == ms(r.rows())


def test_rmat_kv_ingest_equals_generator(rmat12):
    sp, st = rmat12
    kv = GraphSpace(64)
    kv.set_edge_schema(FOLLOW, [("weight", O.INT)])
    for p in range(1, 65):
        kv.load_part(p, st.dump_part(p))
    kv.finalize()
    a, b = sp.info(FOLLOW), kv.info(FOLLOW)
    assert a["num_vertices"] == b["num_vertices"] and a["local_out_edges"] == b["local_out_edges"]
    assert a["local_in_edges"] == b["local_in_edges"]
    starts = seeds_from(12, 32, seed=3)
    for steps in (1, 3):
        ga = sp.go(starts, steps, FOLLOW, yields=[X.EdgeDst("f"), X.AliasProp("f", "weight")])
        gb = kv.go(starts, steps, FOLLOW, yields=[X.EdgeDst("f"), X.AliasProp("f", "weight")])
        assert ms(ga.rows()) == ms(gb.rows())
    kv.close()


def test_rmat_multiversion_first_version_wins():
    st = oracle_rmat(10, versions=3)
    sp = GraphSpace(64)
    sp.set_edge_schema(FOLLOW, [("weight", O.INT)])
    for p in range(1, 65):
        sp.load_part(p, st.dump_part(p))
    sp.finalize()
    starts = seeds_from(10, 32)
    for steps in (1, 2, 3):
        w = X.AliasProp("follow", "weight") > 499
        y = [X.EdgeDst("follow"), X.AliasProp("follow", "weight")]
        g = sp.go(starts, steps, FOLLOW, where=w, yields=y)
        r = st.go(starts, steps, FOLLOW, where=w.encode(), yields=[x.encode() for x in y])
        assert ms(g.rows()) == ms(r.rows())
    sp.close()


@pytest.mark.parametrize("k", [0, 500, 900, 998])
def test_rmat_multiversion_get_bound_first_loop(k):
    """push-down filters over 3-version data (older versions carry other weights): the fast typed
    compare and the VM both follow collectEdgeProps' firstLoop rule, in getBound and in stats"""
    st = oracle_rmat(10, versions=3)
    sp = GraphSpace(64)
    sp.set_edge_schema(FOLLOW, [("weight", O.INT)])
    for p in range(1, 65):
        sp.load_part(p, st.dump_part(p))
    sp.finalize()
    starts = seeds_from(10, 48, seed=13)
    parts = [O.part_of(v, 64) for v in starts]
    cols = [("_dst", O.EDGE, 0), ("weight", O.EDGE, 0), ("_rank", O.EDGE, 0)]
    for f in (X.AliasProp("follow", "weight") > k,                       # fast typed compare
              (X.AliasProp("follow", "weight") % 7).eq(k % 7) | (X.AliasProp("follow", "weight") > k)):  # VM
        g = sp.get_bound(FOLLOW, parts, starts, cols, f)
        r = st.get_bound(FOLLOW, parts, starts, cols, filt=f.encode())
        assert vertex_groups_gpu(g) == vertex_groups_oracle(r)
        gs = sp.bound_stats(FOLLOW, parts, starts, [("weight", O.EDGE, 0), ("_dst", O.EDGE, 0)], [1, 2], f)
        rs = st.bound_stats(FOLLOW, parts, starts, [("weight", O.EDGE, 0), ("_dst", O.EDGE, 0)], [1, 2],
                            filt=f.encode())
        assert gs.rows() == rs.rows()
    sp.close()


def vertex_groups_gpu(g):
    rows = g.rows()
    return Counter((int(v), tuple(rows[g.vertex_row_offsets[i]:g.vertex_row_offsets[i + 1]]))
                   for i, v in enumerate(g.vertex_ids))


def vertex_groups_oracle(r):
    rows = r.rows()
    out = Counter()
    pos = 0
    for i, (vid, _) in enumerate(r.vertices()):
        n = r.vertex_nrows(i)
        out[(vid, tuple(rows[pos:pos + n]))] += 1
        pos += n
    return out


def test_rmat_get_bound_matches_oracle(rmat12):
    sp, st = rmat12
    starts = seeds_from(12, 40, seed=5)
    parts = [O.part_of(v, 64) for v in starts]
    cols = [("_dst", O.EDGE, 0), ("weight", O.EDGE, 0), ("_rank", O.EDGE, 0), ("_src", O.EDGE, 0)]
    f = X.AliasProp("follow", "weight") >= 300
    g = sp.get_bound(FOLLOW, parts, starts, cols, f)
    r = st.get_bound(FOLLOW, parts, starts, cols, filt=f.encode())
    # one VertexData per request entry (duplicates repeat), rows in key order within each
    assert vertex_groups_gpu(g) == vertex_groups_oracle(r)


@pytest.mark.parametrize("force", [1, -1])
def test_rmat_direction_modes_agree(rmat12, force):
    """bottom-up (forced) and top-down (forced) steps give the oracle's results"""
    sp, st = rmat12
    sp.set_option("bu_force", force)
    try:
        starts = sorted(set(seeds_from(12, 48, seed=9)))  # unique: the reference rescans duplicates
        w = X.AliasProp("follow", "weight") > 499
        for steps in (2, 3):
            g = sp.go(starts, steps, FOLLOW, where=w, yields=[X.EdgeDst("follow")], distinct=True)
            r = st.go(starts, steps, FOLLOW, where=w.encode(), yields=[X.EdgeDst("follow").encode()], distinct=True)
            assert np.array_equal(np.sort(g.columns[0]), np.sort(r.int_col(0)))
            g = sp.go(starts, steps, FOLLOW)
            r = st.go(starts, steps, FOLLOW)
            assert np.array_equal(np.sort(g.columns[0]), np.sort(r.int_col(0)))
            assert g.edges_scanned == r.edges_scanned
        t = sp.last_timing()
        assert (t["bu_steps"] > 0) == (force > 0)
    finally:
        sp.set_option("bu_force", 0)


@pytest.fixture(autouse=True)
def _reset_rmat12_options(request):
    """rmat12 is module-scoped: engine options a test sets on it end with that test"""
    yield
    if "rmat12" in request.fixturenames:
        request.getfixturevalue("rmat12")[0].reset_options()


def final_bu_kernels(sp):
    """rocprof names of the last query's final bottom-up hop (dominant first)"""
    hops = [h for h in sp.last_timing()["hops"] if h["mode"] == "bottom-up" and h["final"]]
    assert hops, "the final hop did not run bottom-up"
    return hops[-1]["kernels"]


@pytest.mark.parametrize("fin", [0, 1])
@pytest.mark.parametrize("lds,rest_lds,rsteps,unroll,cap", [(64, 64, 4, 1, 36 * 1024), (64, 0, 1, 2, 36 * 1024),
                                                          (0, 64, 2, 1, 36 * 1024), (1, 1, 4, 2, 8)])
def test_rmat_bottom_up_shapes(rmat12, lds, rest_lds, rsteps, unroll, cap, fin):
    """the bottom-up kernels (k_bu_lean / k_bu_fin first pass + k_bu_rest_lean) for every tile / LDS hub /
    rest-chunk shape, non-final and final hops, thresholds that leave rows pending past the slab,
    against the oracle; the hop stats name the kernels that ran"""
    sp, st = rmat12
    for k, v in {"bu_force": 1, "bu_lean_lds_kb": lds,
                 "bu_lean_lds_kb_final": lds, "bu_rest_lds_kb": rest_lds, "bu_rest_lds_kb_final": rest_lds,
                 "bu_rest_steps": rsteps, "bu_unroll": unroll, "bu_hub_cap": cap, "bu_fin": fin}.items():
        sp.set_option(k, v)
    # the final hop's first pass: k_bu_fin (the default) or k_bu_lean (bu_fin = 0; its
    # non-temporal instantiation carries a fifth argument)
    first = "nbg::k_bu_fin<" if fin else f"nbg::k_bu_lean<1, 1, {1 if lds else 0}, 0"
    starts = sorted(set(seeds_from(12, 48, seed=23)))
    pending = 0
    for k in (0, 499, 990):
        w = X.AliasProp("follow", "weight") > k
        for steps in (2, 3):
            g = sp.go(starts, steps, FOLLOW, where=w, yields=[X.EdgeDst("follow")], distinct=True)
            r_ = st.go(starts, steps, FOLLOW, where=w.encode(), yields=[X.EdgeDst("follow").encode()], distinct=True)
            assert np.array_equal(np.sort(g.columns[0]), np.sort(r_.int_col(0)))
            assert g.edges_scanned == r_.edges_scanned
            ks = final_bu_kernels(sp)
            assert ks[0].startswith(first), ks
            assert ks[1].startswith("nbg::k_bu_rest_lean<1, "), ks
            pending += sum(h["c"][3] for h in sp.last_timing()["hops"] if h["mode"] == "bottom-up")
    assert pending > 0  # the rest pass had rows to scan
    # DISTINCT _dst without WHERE: the final-hop kernels with every bucket passing
    g = sp.go(starts, 3, FOLLOW, yields=[X.EdgeDst("follow")], distinct=True)
    r_ = st.go(starts, 3, FOLLOW, yields=[X.EdgeDst("follow").encode()], distinct=True)
    assert np.array_equal(np.sort(g.columns[0]), np.sort(r_.int_col(0)))
    assert final_bu_kernels(sp)[0].startswith(first)
    g = sp.go(starts, 3, FOLLOW)
    r_ = st.go(starts, 3, FOLLOW)
    assert np.array_equal(np.sort(g.columns[0]), np.sort(r_.int_col(0)))
    hops = [h for h in sp.last_timing()["hops"] if h["mode"] == "bottom-up"]
    assert hops and hops[0]["kernels"][0].startswith(f"nbg::k_bu_lean<0, 1, {1 if lds else 0}, 0")


OPS = {">": lambda c, k: c > k, ">=": lambda c, k: c >= k, "<": lambda c, k: c < k, "<=": lambda c, k: c <= k,
       "==": lambda c, k: c.eq(k), "!=": lambda c, k: c.ne(k)}


@pytest.mark.parametrize("fin", [0, 1])
@pytest.mark.parametrize("qpred", [1, 0])
@pytest.mark.parametrize("hub_cap", [36 * 1024, 16])
def test_rmat_bottom_up_packed_predicate(rmat12, qpred, hub_cap, fin):
    """the final bottom-up hop (first pass k_bu_lean<1,..> or, bu_fin = 1, k_bu_fin<..>, then
    k_bu_rest_lean<1,..>, asserted by name) with the quantised predicate (slot words carry the
    bucket of follow.weight): every compare op, constants below, inside, on the edges of and above
    the value range; bu_qpred=0 reads every value of a frontier hit instead (the path a predicate
    on an unpacked column takes); hub_cap 16 leaves all but the first 512 vertices to the global
    (L2) probe branch"""
    sp, st = rmat12
    starts = sorted(set(seeds_from(12, 48, seed=29)))
    wcol = X.AliasProp("follow", "weight")
    sp.set_option("bu_force", 1)
    sp.set_option("bu_qpred", qpred)
    sp.set_option("bu_hub_cap", hub_cap)
    sp.set_option("bu_fin", fin)
    first = "nbg::k_bu_fin<" if fin else "nbg::k_bu_lean<1, "
    for k in (-5, 0, 1, 3, 4, 255, 499, 500, 998, 999, 1000, 5000):
        for op, mk in OPS.items():
            w = mk(wcol, k)
            g = sp.go(starts, 2, FOLLOW, where=w, yields=[X.EdgeDst("follow")], distinct=True)
            r_ = st.go(starts, 2, FOLLOW, where=w.encode(), yields=[X.EdgeDst("follow").encode()], distinct=True)
            assert np.array_equal(np.sort(g.columns[0]), np.sort(r_.int_col(0))), (k, op)
            assert g.edges_scanned == r_.edges_scanned, (k, op, [(h["mode"], h["c"][:6]) for h in sp.last_timing()["hops"]])
            ks = final_bu_kernels(sp)
            assert ks[0].startswith(first) and ks[1].startswith("nbg::k_bu_rest_lean<1, "), ks


@pytest.mark.parametrize("spec,force", [(1, 0), (0, 0), (1, 1), (1, -1)])
def test_host_direct_distinct_output(rmat12, spec, force):
    """option host_direct: the DISTINCT _dst output kernel writes the vids straight into pinned
    host memory (no device->host copy); same rows as the default path and the oracle, on the
    speculated final hop, the host-driven bottom-up hop and the top-down hop (device column)"""
    sp, st = rmat12
    starts = seeds_from(12, 64)
    w = X.AliasProp("follow", "weight") > 499
    y = [X.EdgeDst("follow")]
    r = st.go(starts, 3, FOLLOW, where=w.encode(), yields=[y[0].encode()], distinct=True)
    want = np.sort(r.int_col(0))
    sp.set_option("bu_spec", spec)
    sp.set_option("bu_force", force)
    sp.set_option("bu_div", 16)
    try:
        for hd in (1, 0, 1):
            sp.set_option("host_direct", hd)
            g = sp.go(starts, 3, FOLLOW, where=w, yields=y, distinct=True)
            col = np.array(g.columns[0])
            del g  # the pinned block returns to the cache while `col` keeps its copy
            assert np.array_equal(np.sort(col), want)
    finally:
        for k in ("bu_spec", "bu_force", "bu_div", "host_direct"):
            sp.unset_option(k)


@pytest.mark.parametrize("bu_div", [2, 16])
def test_atomic_hop_sums_match(rmat12, bu_div):
    """option bu_atomic_sums: the bottom-up passes add their block sums into the hop counters
    with no-return atomics instead of partials + k_reduce_partials; same rows and the same hop
    counters (found, out-degree sum, slab words, pending rows), speculated hops included"""
    sp, st = rmat12
    starts = sorted(set(seeds_from(12, 24, seed=43)))
    w = X.AliasProp("follow", "weight") > 499
    y = [X.EdgeDst("follow")]
    sp.set_option("bu_div", bu_div)
    try:
        for steps in (2, 3, 4):
            runs = []
            for atomic in (0, 1):
                sp.set_option("bu_atomic_sums", atomic)
                g = sp.go(starts, steps, FOLLOW, where=w, yields=y, distinct=True)
                hops = sp.last_timing()["hops"]
                runs.append((np.sort(g.columns[0]), [(h["mode"], h["c"][:4]) for h in hops]))
            assert np.array_equal(runs[0][0], runs[1][0])
            assert runs[0][1] == runs[1][1], steps
    finally:
        sp.unset_option("bu_atomic_sums")
        sp.set_option("bu_div", 4)
