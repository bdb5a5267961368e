"""FLOAT edge props: RowWriter stores a FLOAT column as 4 bytes, RowReader::getFloat
reads it and collectProps widens it to double and collects 8 bytes (QueryBaseProcessor.inl:285-290,
Collector collectDouble), while the response's edge schema still names the column FLOAT
(QueryBoundProcessor.cpp:94-100) -- so the reference's own response rows, decoded with that schema,
are garbage past the column (the oracle restates exactly that).  The device returns what the
collector computes: the widened double, typed DOUBLE (DESIGN.md divergence 3).  Checked against
the oracle over the same edges stored with a DOUBLE column holding the widened values: getBound
rows in key order, a push-down filter, GO WHERE / YIELD over the prop.
"""
import random
from collections import Counter

import numpy as np
import pytest

import oracle as O
from nebula_amd import GraphSpace
from nebula_amd import expr as X

pytestmark = pytest.mark.gpu

PARTS, ET = 8, 3
FIELDS = [("f", O.FLOAT), ("w", O.INT)]


def ms(rows):
    return Counter(tuple(r) for r in rows)


@pytest.fixture(scope="module")
def spaces():
    rng = random.Random(41)
    vids = sorted({rng.randrange(-2**40, 2**40) for _ in range(300)})
    parts = {p: [] for p in range(1, PARTS + 1)}
    dparts = {p: [] for p in range(1, PARTS + 1)}  # the same edges, f as the widened double
    for _ in range(2500):
        s, d = rng.choice(vids), rng.choice(vids)
        f = np.float32(rng.uniform(-2.0, 2.0))
        w = rng.randrange(100)
        ps, pd = O.part_of(s, PARTS), O.part_of(d, PARTS)
        for tgt, row in ((parts, O.encode_row([f, w])), (dparts, O.encode_row([float(f), w]))):
            tgt[ps].append((O.edge_key(ps, s, ET, 0, d, 2**63 - 2), row))
            tgt[pd].append((O.edge_key(pd, d, -ET, 0, s, 2**63 - 2), b""))
    sp = GraphSpace(PARTS)
    sp.set_edge_schema(ET, FIELDS)
    st = O.Store(PARTS)
    st.set_edge_schema(ET, [("f", O.DOUBLE), ("w", O.INT)], name="e")
    for p, kv in parts.items():
        if kv:
            sp.load_part(p, kv)
    for p, kv in dparts.items():
        if kv:
            st.put(p, kv)
    sp.finalize()
    st.finalize()
    yield sp, st, vids
    sp.close()


def test_float_get_bound_rows(spaces):
    sp, st, vids = spaces
    q = vids[::3]
    parts = [O.part_of(v, PARTS) for v in q]
    cols = [("_dst", O.EDGE, 0), ("f", O.EDGE, 0), ("w", O.EDGE, 0)]
    for filt in (None, X.AliasProp("e", "f") > 0.5):
        g = sp.get_bound(ET, parts, q, cols, filter=filt)
        r = st.get_bound(ET, parts, q, cols, filt=X.encode(filt))
        rows = g.rows()
        got = {int(v): rows[g.vertex_row_offsets[i]:g.vertex_row_offsets[i + 1]] for i, v in enumerate(g.vertex_ids)}
        want = {}
        for i, row in enumerate(r.rows()):
            want.setdefault(r.row_vertex(i), []).append(row)
        assert got == want
        assert len(rows) > 100
        # widened float values: exactly representable in float32
        assert all(float(np.float32(x[1])) == x[1] for x in rows)


@pytest.mark.parametrize("steps", [1, 2])
def test_float_go_where_yield(spaces, steps):
    sp, st, vids = spaces
    starts = vids[::11]
    w = X.AliasProp("e", "f") > 0.25
    ys = [X.AliasProp("e", "f"), X.AliasProp("e", "w"), X.EdgeDst("e")]
    for distinct in (False, True):
        rs = sp.go(starts, steps, ET, where=w, yields=ys, distinct=distinct)
        ref = st.go(starts, steps, ET, where=w.encode(), yields=[y.encode() for y in ys], distinct=distinct)
        assert ref.code == 0, ref.error
        assert ms(rs.rows()) == ms(ref.rows())
        assert rs.n_rows > 0
