"""GPU parity for $^ / $$ vertex tag props in GO (GoExecutor::getStepOutProps,
fetchVertexProps + VertexHolder, GoExecutor.cpp:454-569, 785-828; storage collectVertexProps,
QueryBaseProcessor.inl:309-333) and STRING YIELD columns.

Pinned by the reference's GoTest expectations over the NBA data (tests/golden/nba.json, tag_*
cases) and compared with the oracle on a random graph with multi-version / misplaced tag rows.
Rows are compared as multisets (src/graph/test/TestBase.h:182-222).
"""
import random
from collections import Counter

import pytest

import fixtures as F
import oracle as O
from nebula_amd import GraphSpace, NbgError
from nebula_amd import expr as X

pytestmark = pytest.mark.gpu

NBA_TAGS = {F.NBA_PLAYER: ("player", [("name", O.STRING), ("age", O.INT)]),
            F.NBA_TEAM: ("team", [("name", O.STRING)])}


def ms(rows):
    return Counter(tuple(r) for r in rows)


def names(vid, rows):
    inv = {v: k for k, v in vid.items()}
    return Counter(tuple(inv.get(c, c) if isinstance(c, int) and c in inv else c for c in r) for r in rows)


def golden(d, key):
    return Counter(tuple(r) for r in d["expect"][key]["rows"])


@pytest.fixture(scope="module")
def nba():
    sp = GraphSpace(1)
    for et, (name, fields) in F.NBA_EDGE_SCHEMAS.items():
        sp.set_edge_schema(et, fields)
    for tag, (name, fields) in NBA_TAGS.items():
        sp.set_tag_schema(tag, name, fields)
    parts, vid = F.nba_kv()
    for p, kv in parts.items():
        sp.load_part(p, kv)
    sp.finalize()
    st, _ = F.nba_oracle_store()
    yield sp, st, vid, F.nba()
    sp.close()


def tag_yields():
    return [X.SourceProp("player", "name"), X.AliasProp("serve", "start_year"),
            X.AliasProp("serve", "end_year"), X.DestProp("team", "name")]


def test_nba_tag_yield(nba):
    sp, st, vid, d = nba
    rs = sp.go([vid["Boris Diaw"]], 1, F.NBA_SERVE, yields=tag_yields())
    assert names(vid, rs.rows()) == golden(d, "tag_serve_boris")
    w = (X.AliasProp("serve", "start_year") >= 2013) & (X.AliasProp("serve", "end_year") <= 2018)
    rs = sp.go([vid["Rajon Rondo"]], 1, F.NBA_SERVE, where=w, yields=tag_yields())
    assert names(vid, rs.rows()) == golden(d, "tag_serve_rondo_where")


def test_nba_tag_distinct(nba):
    sp, st, vid, d = nba
    ys = [X.SourceProp("player", "name"), X.DestProp("team", "name")]
    rs = sp.go([vid["Nobody"]], 1, F.NBA_SERVE, yields=ys, distinct=True)
    assert names(vid, rs.rows()) == golden(d, "tag_distinct_nobody")
    cur = [vid["Boris Diaw"]]
    for et in (F.NBA_LIKE, F.NBA_LIKE):
        cur = [r[0] for r in sp.go(cur, 1, et).rows()]
    rs = sp.go(cur, 1, F.NBA_SERVE, yields=[X.EdgeDst("serve"), X.DestProp("team", "name")], distinct=True)
    assert names(vid, rs.rows()) == golden(d, "tag_distinct_pipe_dst_team")


def test_nba_tag_vertex_not_exist(nba):
    sp, st, vid, d = nba
    for distinct in (False, True):
        rs = sp.go([d["nonexist_hash"]], 1, F.NBA_SERVE, yields=tag_yields(), distinct=distinct)
        assert names(vid, rs.rows()) == golden(d, "tag_vertex_not_exist")
        # frontier empties before the final step (onEmptyInputs): typed empty STRING columns
        rs = sp.go([d["nonexist_hash"], vid["Spurs"]], 2, F.NBA_LIKE, yields=[X.DestProp("player", "name")],
                   distinct=distinct)
        assert rs.n_rows == 0 and rs.rows() == []


@pytest.mark.parametrize("steps", [1, 2, 3])
def test_nba_tag_where_both_ends(nba, steps):
    sp, st, vid, d = nba
    w = (X.SourceProp("player", "age") > 33) & (X.DestProp("player", "age") < 40)
    ys = [X.SourceProp("player", "name"), X.DestProp("player", "name"), X.DestProp("player", "age"),
          X.AliasProp("like", "likeness")]
    starts = [vid[n] for n in ("Tim Duncan", "Tony Parker", "Manu Ginobili", "Boris Diaw", "Tracy McGrady")]
    for distinct in (False, True):
        rs = sp.go(starts, steps, F.NBA_LIKE, where=w, yields=ys, distinct=distinct)
        ref = st.go(starts, steps, F.NBA_LIKE, where=w.encode(), yields=[y.encode() for y in ys], distinct=distinct)
        assert ref.code == 0, ref.error
        assert ms(rs.rows()) == ms(ref.rows())
        assert rs.n_rows > 0


def test_nba_tag_errors(nba):
    sp, st, vid, d = nba
    tim = [vid["Tim Duncan"]]
    # unknown tag: graphd "No schema found" (GoExecutor.cpp:475-478)
    with pytest.raises(NbgError) as e:
        sp.go(tim, 1, F.NBA_LIKE, yields=[X.DestProp("coach", "name")])
    assert e.value.code == -22
    assert st.go(tim, 1, F.NBA_LIKE, yields=[X.DestProp("coach", "name").encode()]).code != 0
    # unknown prop of a known tag: E_IMPROPER_DATA_TYPE on every part -> query fails
    with pytest.raises(NbgError) as e:
        sp.go(tim, 1, F.NBA_LIKE, yields=[X.DestProp("player", "height")])
    assert e.value.code == -23
    # $$.team.name of a player: no team row -> VertexHolder miss -> evaluation error
    with pytest.raises(NbgError) as e:
        sp.go(tim, 1, F.NBA_LIKE, yields=[X.DestProp("team", "name")])
    assert e.value.code == -1004
    assert st.go(tim, 1, F.NBA_LIKE, yields=[X.DestProp("team", "name").encode()]).code != 0
    # the error is raised only by rows that are evaluated: WHERE false everywhere -> no rows
    w = X.AliasProp("like", "likeness") > 1000
    rs = sp.go(tim, 1, F.NBA_LIKE, where=w, yields=[X.DestProp("team", "name")])
    assert rs.n_rows == 0


# ------------------------------------------------------------------------------------------
# random graph with tag rows: several versions, identical keys (last write wins), rows in a
# foreign part (invisible), strings with equal content at different vertices
# ------------------------------------------------------------------------------------------
PARTS = 8
ET = 1
PERSON = 5


def random_space_kv(seed, n_vertices=400, n_edges=4000, missing=0.0):
    rng = random.Random(seed)
    vids = sorted({rng.randrange(-2**62, 2**62) for _ in range(n_vertices)})
    parts = {p: [] for p in range(1, PARTS + 1)}

    def part(v):
        return O.part_of(v, PARTS)

    ver = 2**63 - 2
    for _ in range(n_edges):
        s, t = rng.choice(vids), rng.choice(vids)
        wgt = rng.randrange(1000)
        parts[part(s)].append((O.edge_key(part(s), s, ET, 0, t, ver), O.encode_row([wgt])))
        parts[part(t)].append((O.edge_key(part(t), t, -ET, 0, s, ver), b""))
    for v in vids:
        if rng.random() < missing:
            continue
        p = part(v)
        row = [f"p{abs(v) % 37}", rng.randrange(100), rng.random() * 10]
        parts[p].append((O.vertex_key(p, v, PERSON, 1000), O.encode_row(row)))
        if rng.random() < 0.3:  # older version (larger LE bytes at byte 0 -> later in order)
            parts[p].append((O.vertex_key(p, v, PERSON, 1001), O.encode_row(["old", -1, -1.0])))
        if rng.random() < 0.2:  # identical key written again: the last write wins
            parts[p].append((O.vertex_key(p, v, PERSON, 1000), O.encode_row([f"q{abs(v) % 11}", 7, 0.5])))
        if rng.random() < 0.1:  # a row under a foreign part: never reached by the prefix scan
            q = p % PARTS + 1
            parts[q].append((O.vertex_key(q, v, PERSON, 0), O.encode_row(["foreign", 999, 9.0])))
    return parts, vids


def build_pair(seed, missing=0.0):
    parts, vids = random_space_kv(seed, missing=missing)
    fields = [("name", O.STRING), ("score", O.INT), ("wt", O.DOUBLE)]
    sp = GraphSpace(PARTS)
    sp.set_edge_schema(ET, [("weight", O.INT)])
    sp.set_tag_schema(PERSON, "person", fields)
    st = O.Store(PARTS)
    st.set_edge_schema(ET, [("weight", O.INT)], name="e")
    st.set_tag_schema(PERSON, fields, name="person")
    for p, kv in parts.items():
        if kv:
            sp.load_part(p, kv)
            st.put(p, kv)
    sp.finalize()
    st.finalize()
    return sp, st, vids


@pytest.fixture(scope="module")
def rnd():
    sp, st, vids = build_pair(3)
    yield sp, st, vids
    sp.close()


QUERIES = [
    (1, None, [X.SourceProp("person", "name"), X.DestProp("person", "score"), X.AliasProp("e", "weight")], False),
    (2, (X.DestProp("person", "score") > 50) & (X.AliasProp("e", "weight") < 700),
     [X.DestProp("person", "name"), X.SourceProp("person", "wt")], False),
    (3, None, [X.DestProp("person", "name")], True),
    (2, X.SourceProp("person", "name").eq("p3") | X.DestProp("person", "name").eq("q4"),
     [X.EdgeDst("e"), X.SourceProp("person", "score") + X.DestProp("person", "score")], False),
    (1, X.DestProp("person", "wt") > X.SourceProp("person", "wt"),
     [X.SourceProp("person", "name"), X.DestProp("person", "name")], True),
]


@pytest.mark.parametrize("qi", range(len(QUERIES)))
def test_random_tag_parity(rnd, qi):
    sp, st, vids = rnd
    steps, where, ys, distinct = QUERIES[qi]
    starts = vids[::23]
    rs = sp.go(starts, steps, ET, where=where, yields=ys, distinct=distinct)
    ref = st.go(starts, steps, ET, where=X.encode(where), yields=[y.encode() for y in ys], distinct=distinct)
    assert ref.code == 0, ref.error
    assert ms(rs.rows()) == ms(ref.rows())
    assert rs.n_rows > 0


def test_random_tag_missing_rows_error():
    sp, st, vids = build_pair(5, missing=0.2)
    try:
        starts = vids[::17]
        ys = [X.DestProp("person", "name")]
        ref = st.go(starts, 1, ET, yields=[y.encode() for y in ys])
        assert ref.code != 0  # some dst has no person row
        with pytest.raises(NbgError) as e:
            sp.go(starts, 1, ET, yields=ys)
        assert e.value.code == -1004
        # edge-only YIELD is unaffected by the missing tag rows
        rs = sp.go(starts, 1, ET, yields=[X.AliasProp("e", "weight")])
        ref = st.go(starts, 1, ET, yields=[X.AliasProp("e", "weight").encode()])
        assert ms(rs.rows()) == ms(ref.rows())
    finally:
        sp.close()


# ------------------------------------------------------------------------------------------
# $-.prop / $var.prop: GoTest ReferencePipeInYieldAndWhere /
# ReferenceVariableInYieldAndWhere, input rows = the first GO's (name, id) rows
# ------------------------------------------------------------------------------------------
def test_nba_reference_input_and_variable(nba):
    sp, st, vid, d = nba
    first = sp.go([vid["Tim Duncan"], vid["Chris Paul"]], 1, F.NBA_LIKE,
                  yields=[X.SourceProp("player", "name"), X.EdgeDst("like")])
    rows = first.rows()
    starts = [r[1] for r in rows]
    inputs = [("name", O.STRING, [r[0] for r in rows]), ("id", O.VID, starts)]
    for ref in (X.InputProp("name"), X.VariableProp("var", "name")):
        ys = [ref, X.SourceProp("player", "name"), X.DestProp("player", "name")]
        rs = sp.go(starts, 1, F.NBA_LIKE, yields=ys, inputs=inputs)
        assert names(vid, rs.rows()) == golden(d, "ref_input_yield")
        w = ref.ne(X.DestProp("player", "name"))
        rs = sp.go(starts, 1, F.NBA_LIKE, where=w, yields=ys, inputs=inputs)
        assert names(vid, rs.rows()) == golden(d, "ref_input_where")
        ref_rs = st.go(starts, 1, F.NBA_LIKE, where=w.encode(), yields=[y.encode() for y in ys], inputs=inputs)
        assert ms(rs.rows()) == ms(ref_rs.rows())


def test_nba_reference_input_duplicates_and_types(nba):
    sp, st, vid, d = nba
    # a vid piped twice: its LAST input row supplies $-.props (InterimResult::buildIndex);
    # numeric / bool / double input columns in WHERE and YIELD arithmetic
    starts = [vid["Tim Duncan"], vid["Tony Parker"], vid["Tim Duncan"], vid["Boris Diaw"]]
    inputs = [("tag", O.STRING, ["a", "b", "c", "d"]), ("n", O.VID, [10, 20, 30, 40]),
              ("x", O.DOUBLE, [0.5, 1.5, 2.5, 3.5]), ("f", O.BOOL, [True, False, False, True])]
    ys = [X.InputProp("tag"), X.InputProp("n") + X.AliasProp("like", "likeness"), X.InputProp("x"),
          X.InputProp("f"), X.EdgeDst("like")]
    for distinct in (False, True):
        for w in (None, X.InputProp("n") > 15, X.InputProp("f")):
            rs = sp.go(starts, 1, F.NBA_LIKE, where=w, yields=ys, distinct=distinct, inputs=inputs)
            ref = st.go(starts, 1, F.NBA_LIKE, where=X.encode(w), yields=[y.encode() for y in ys],
                        distinct=distinct, inputs=inputs)
            assert ref.code == 0, ref.error
            assert ms(rs.rows()) == ms(ref.rows())
            assert all(r[0] != "a" for r in rs.rows())  # Tim's last row is "c"


def test_nba_reference_input_errors(nba):
    sp, st, vid, d = nba
    starts = [vid["Tim Duncan"]]
    inputs = [("name", O.STRING, ["x"])]
    with pytest.raises(NbgError) as e:  # no input table
        sp.go(starts, 1, F.NBA_LIKE, yields=[X.InputProp("name")])
    assert e.value.code == -1003
    with pytest.raises(NbgError) as e:  # unknown input column
        sp.go(starts, 1, F.NBA_LIKE, yields=[X.InputProp("nope")], inputs=inputs)
    assert e.value.code == -1001


# ------------------------------------------------------------------------------------------
# $-.prop / $var.prop with STEPS > 1 (VertexBackTracker, GoExecutor.h:174-193): the input row of
# the vertex's root start; several roots -> the smallest root vid (the build's order-free rule,
# DESIGN.md; the reference picks by RPC response order there)
# ------------------------------------------------------------------------------------------
def expected_multistep(sp, starts, names_in, steps, et):
    """the rule restated from single-start GO results: root(v) after each non-final hop =
    min vid over the roots of v's in-edge srcs in the previous frontier"""
    name_of = {}
    for s_, n_ in zip(starts, names_in):
        name_of[s_] = n_  # the last input row of a vid wins (InterimResult::buildIndex)
    root = {s_: s_ for s_ in starts}
    for _ in range(steps - 1):
        nxt = {}
        for v, r in root.items():
            rs = sp.go([v], 1, et)
            for d in rs.columns[0]:
                d = int(d)
                nxt[d] = min(nxt.get(d, r), r)
        root = nxt
    rows = []
    for v, r in root.items():
        rs = sp.go([v], 1, et)
        rows += [(name_of[r], int(d)) for d in rs.columns[0]]
    return Counter(rows)


@pytest.mark.parametrize("steps", [2, 3])
def test_nba_multistep_input(nba, steps):
    sp, st, vid, d = nba
    who = ["Tim Duncan", "Tony Parker", "Chris Paul", "Manu Ginobili", "Tim Duncan"]
    starts = [vid[w] for w in who]
    tags = [f"row{i}" for i in range(len(who))]
    inputs = [("tag", O.STRING, tags), ("n", O.INT, list(range(len(who))))]
    ys = [X.InputProp("tag"), X.EdgeDst("like")]
    rs = sp.go(starts, steps, F.NBA_LIKE, yields=ys, inputs=inputs)
    assert ms(rs.rows()) == expected_multistep(sp, starts, tags, steps, F.NBA_LIKE)
    for ref in (X.InputProp("n"), X.VariableProp("v", "n")):
        for w in (None, ref > 1):
            ys2 = [ref, X.InputProp("tag"), X.SourceProp("player", "name"), X.EdgeDst("like")]
            rs = sp.go(starts, steps, F.NBA_LIKE, where=w, yields=ys2, inputs=inputs)
            ref_rs = st.go(starts, steps, F.NBA_LIKE, where=X.encode(w), yields=[y.encode() for y in ys2],
                           inputs=inputs)
            assert ref_rs.code == 0, ref_rs.error
            assert ms(rs.rows()) == ms(ref_rs.rows())


@pytest.mark.parametrize("steps", [2, 3])
def test_rmat_multistep_input_vs_oracle(steps):
    """random graph, many starts sharing descendants (the tie rule decides most roots)"""
    from nebula_amd import synth
    scale = 11
    sp = GraphSpace(16)
    try:
        sp.set_edge_schema(1, [("weight", O.INT)])
        sp.gen_rmat(scale, 8, 3, 1)
        sp.finalize()
        st = O.Store(16)
        st.set_edge_schema(1, [("weight", O.INT)], name="e")
        st.load_rmat(scale, 8, 3, 1)
        starts = list(synth.seeds(scale, 8, 3, 24))
        inputs = [("n", O.INT, [int(i * 7 % 11) for i in range(len(starts))])]
        ys = [X.InputProp("n"), X.AliasProp("e", "weight"), X.EdgeDst("e")]
        for w in (None, X.InputProp("n") > 4, (X.InputProp("n") + X.AliasProp("e", "weight")) > 600):
            for distinct in (False, True):
                rs = sp.go(starts, steps, 1, where=w, yields=ys, distinct=distinct, inputs=inputs)
                ref = st.go(starts, steps, 1, where=X.encode(w), yields=[y.encode() for y in ys],
                            distinct=distinct, inputs=inputs)
                assert ref.code == 0, ref.error
                assert ms(rs.rows()) == ms(ref.rows())
                assert rs.n_rows > 0
    finally:
        sp.close()
