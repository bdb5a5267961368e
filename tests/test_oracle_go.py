"""Pin the oracle's graphd restatement against the reference's GoTest expectations
(src/graph/test/GoTest.cpp; data src/graph/test/TraverseTestBase.h, via tests/golden/nba.json)."""
from collections import Counter

import pytest

import fixtures as F
import oracle as O
from nebula_amd import expr as X


@pytest.fixture(scope="module")
def nba(oracle):
    st, vid = F.nba_oracle_store()
    return st, vid, F.nba()


def names(vid, rows):
    inv = {v: k for k, v in vid.items()}
    return Counter(tuple(inv.get(c, c) if isinstance(c, int) and c in inv else c for c in r) for r in rows)


def expect(data, key):
    return Counter(tuple(r) for r in data["expect"][key]["rows"])


def test_one_step_serve(nba):
    st, vid, d = nba
    r = st.go([vid["Tim Duncan"]], 1, F.NBA_SERVE)
    assert r.code == 0
    assert names(vid, r.rows()) == expect(d, "one_step_serve_tim")


def test_serve_years(nba):
    st, vid, d = nba
    ys = [X.AliasProp("serve", "start_year").encode(), X.AliasProp("serve", "end_year").encode(),
          X.EdgeDst("serve").encode()]
    r = st.go([vid["Boris Diaw"]], 1, F.NBA_SERVE, yields=ys)
    assert names(vid, r.rows()) == expect(d, "serve_boris_years")


def test_serve_where(nba):
    st, vid, d = nba
    w = ((X.AliasProp("serve", "start_year") >= 2013) & (X.AliasProp("serve", "end_year") <= 2018)).encode()
    ys = [X.AliasProp("serve", "start_year").encode(), X.AliasProp("serve", "end_year").encode(),
          X.EdgeDst("serve").encode()]
    r = st.go([vid["Rajon Rondo"]], 1, F.NBA_SERVE, where=w, yields=ys)
    assert names(vid, r.rows()) == expect(d, "serve_rondo_where")


def pipe(st, starts, etypes, distinct_last=False, ylast=()):
    cur = starts
    r = None
    for i, et in enumerate(etypes):
        last = i == len(etypes) - 1
        r = st.go(cur, 1, et, yields=ylast if last else (), distinct=distinct_last and last)
        assert r.code == 0, r.error
        cur = [row[0] for row in r.rows()]
    return r


def test_pipe_keeps_duplicates(nba):
    st, vid, d = nba
    r = pipe(st, [vid["Boris Diaw"]], [F.NBA_LIKE, F.NBA_LIKE, F.NBA_SERVE])
    assert names(vid, r.rows()) == expect(d, "pipe_boris_like_like_serve")


def test_variable_two_hops(nba):
    st, vid, d = nba
    r = pipe(st, [vid["Tracy McGrady"]], [F.NBA_LIKE, F.NBA_LIKE])
    assert names(vid, r.rows()) == expect(d, "var_tracy_like_like")
    r = pipe(st, [vid["Tracy McGrady"]], [F.NBA_LIKE, F.NBA_LIKE, F.NBA_LIKE])
    assert names(vid, r.rows()) == expect(d, "var_pipe_tracy")


def test_distinct(nba):
    st, vid, d = nba
    r = pipe(st, [vid["Boris Diaw"]], [F.NBA_LIKE, F.NBA_LIKE, F.NBA_SERVE], distinct_last=True,
             ylast=[X.EdgeDst("serve").encode()])
    assert names(vid, r.rows()) == expect(d, "distinct_boris_serve_dst")


def test_vertex_not_exist(nba):
    st, vid, d = nba
    nid = d["nonexist_hash"]
    assert st.go([nid], 1, F.NBA_SERVE).nrows == 0
    assert pipe(st, [nid], [F.NBA_LIKE, F.NBA_LIKE, F.NBA_SERVE]).nrows == 0


def test_go_three_steps_derived(nba):
    st, vid, d = nba
    r = st.go([vid["Boris Diaw"]], 3, F.NBA_LIKE)
    assert names(vid, r.rows()) == expect(d, "derived_go3_boris_like")
    # the step form dedups the intermediate frontier (P12); the pipe form keeps duplicates (P14)
    assert pipe(st, [vid["Boris Diaw"]], [F.NBA_LIKE] * 3).nrows == 9


def test_relational_type_order(nba):
    # P8: int vs double compares by variant index -> int < double always; == uses almostEqual
    st, vid, d = nba
    w = (X.AliasProp("like", "likeness") > 10.5).encode()
    assert st.go([vid["Tim Duncan"]], 1, F.NBA_LIKE, where=w).nrows == 0
    w = (X.AliasProp("like", "likeness") < 10.5).encode()
    assert st.go([vid["Tim Duncan"]], 1, F.NBA_LIKE, where=w).nrows == 2
    w = X.AliasProp("like", "likeness").eq(95.0).encode()
    assert st.go([vid["Tim Duncan"]], 1, F.NBA_LIKE, where=w).nrows == 2


def test_where_error_fails_query(nba):
    st, vid, d = nba
    w = (X.AliasProp("like", "nope") > 1).encode()
    r = st.go([vid["Tim Duncan"]], 1, F.NBA_LIKE, where=w)
    assert r.code != 0


# ---- $^ / $$ tag props (GoExecutor::getStepOutProps / fetchVertexProps) ----------
def tag_yields():
    return [X.SourceProp("player", "name").encode(), X.AliasProp("serve", "start_year").encode(),
            X.AliasProp("serve", "end_year").encode(), X.DestProp("team", "name").encode()]


def test_tag_props_yield(nba):
    st, vid, d = nba
    r = st.go([vid["Boris Diaw"]], 1, F.NBA_SERVE, yields=tag_yields())
    assert r.code == 0, r.error
    assert names(vid, r.rows()) == expect(d, "tag_serve_boris")
    w = ((X.AliasProp("serve", "start_year") >= 2013) & (X.AliasProp("serve", "end_year") <= 2018)).encode()
    r = st.go([vid["Rajon Rondo"]], 1, F.NBA_SERVE, where=w, yields=tag_yields())
    assert names(vid, r.rows()) == expect(d, "tag_serve_rondo_where")


def test_tag_props_distinct(nba):
    st, vid, d = nba
    ys = [X.SourceProp("player", "name").encode(), X.DestProp("team", "name").encode()]
    r = st.go([vid["Nobody"]], 1, F.NBA_SERVE, yields=ys, distinct=True)
    assert r.code == 0 and names(vid, r.rows()) == expect(d, "tag_distinct_nobody")
    r = pipe(st, [vid["Boris Diaw"]], [F.NBA_LIKE, F.NBA_LIKE, F.NBA_SERVE], distinct_last=True,
             ylast=[X.EdgeDst("serve").encode(), X.DestProp("team", "name").encode()])
    assert names(vid, r.rows()) == expect(d, "tag_distinct_pipe_dst_team")


def test_tag_props_vertex_not_exist(nba):
    st, vid, d = nba
    nid = d["nonexist_hash"]
    for distinct in (False, True):
        r = st.go([nid], 1, F.NBA_SERVE, yields=tag_yields(), distinct=distinct)
        assert r.code == 0 and names(vid, r.rows()) == expect(d, "tag_vertex_not_exist")


def test_tag_props_where_and_errors(nba):
    st, vid, d = nba
    # WHERE over both ends' tags: teammates older than 35 liking each other
    w = ((X.SourceProp("player", "age") > 35) & (X.DestProp("player", "age") > 35)).encode()
    ys = [X.SourceProp("player", "name").encode(), X.DestProp("player", "name").encode()]
    r = st.go([vid["Tim Duncan"], vid["Tony Parker"], vid["Manu Ginobili"]], 1, F.NBA_LIKE, where=w, yields=ys)
    assert r.code == 0, r.error
    ages = {p["name"]: p["age"] for p in d["players"]}
    likes = {(a, b) for a, b, _ in d["like"]}
    want = sorted((a, b) for a, b in likes if a in ("Tim Duncan", "Tony Parker", "Manu Ginobili")
                  and ages[a] > 35 and ages.get(b, 0) > 35)
    assert sorted(r.rows()) == want
    # unknown tag name -> "No schema found" (GoExecutor.cpp:475-478)
    r = st.go([vid["Tim Duncan"]], 1, F.NBA_LIKE, yields=[X.DestProp("coach", "name").encode()])
    assert r.code != 0
    # $$.team.name on a player vertex: the dst has no team row -> evaluation error fails the query
    r = st.go([vid["Tim Duncan"]], 1, F.NBA_LIKE, yields=[X.DestProp("team", "name").encode()])
    assert r.code != 0


# ---- $-.prop / $var.prop (GoExecutor::getPropFromInterim, InterimResult index) -----
def ref_first(st, vid):
    """GO FROM Tim Duncan, Chris Paul OVER like YIELD $^.player.name AS name, like._dst AS id"""
    r = st.go([vid["Tim Duncan"], vid["Chris Paul"]], 1, F.NBA_LIKE,
              yields=[X.SourceProp("player", "name").encode(), X.EdgeDst("like").encode()])
    assert r.code == 0, r.error
    rows = r.rows()
    return [row[1] for row in rows], [("name", O.STRING, [row[0] for row in rows]),
                                      ("id", O.VID, [row[1] for row in rows])]


def test_reference_input_and_variable(nba):
    st, vid, d = nba
    ys = lambda ref: [ref, X.SourceProp("player", "name"), X.DestProp("player", "name")]
    for ref in (X.InputProp("name"), X.VariableProp("var", "name")):
        starts, inputs = ref_first(st, vid)
        r = st.go(starts, 1, F.NBA_LIKE, yields=[y.encode() for y in ys(ref)], inputs=inputs)
        assert r.code == 0, r.error
        assert names(vid, r.rows()) == expect(d, "ref_input_yield")
        w = ref.ne(X.DestProp("player", "name")).encode()
        r = st.go(starts, 1, F.NBA_LIKE, where=w, yields=[y.encode() for y in ys(ref)], inputs=inputs)
        assert names(vid, r.rows()) == expect(d, "ref_input_where")
    # without an input table the reference path is not restated
    assert st.go(starts, 1, F.NBA_LIKE, yields=[X.InputProp("name").encode()]).code != 0


def test_reference_input_multistep_rule(nba):
    """STEPS > 1: $-.prop is the input row of the vertex's root start (VertexBackTracker); a
    vertex reached from several starts takes the smallest root vid (the build's order-free rule).
    Checked against the rule applied to single-start GO 1 STEPS results."""
    st, vid, d = nba
    who = ["Tim Duncan", "Tony Parker", "Chris Paul", "Manu Ginobili"]
    starts = [vid[w] for w in who]
    inputs = [("tag", O.STRING, who)]
    one = lambda v: [row[0] for row in st.go([v], 1, F.NBA_LIKE).rows()]
    root = {s: s for s in starts}
    nxt = {}
    for v, r in root.items():
        for dd in one(v):
            nxt[dd] = min(nxt.get(dd, r), r)
    want = Counter((who[starts.index(r)], dd) for v, r in nxt.items() for dd in one(v))
    r = st.go(starts, 2, F.NBA_LIKE, yields=[X.InputProp("tag").encode(), X.EdgeDst("like").encode()],
              inputs=inputs)
    assert r.code == 0, r.error
    assert Counter(tuple(x) for x in r.rows()) == want
    # a vertex reached from two starts exists in this case, so the rule is exercised
    reach = Counter(dd for v in starts for dd in set(one(v)))
    assert max(reach.values()) > 1
