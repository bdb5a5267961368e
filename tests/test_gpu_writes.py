"""GPU parity of the write path: AddEdges / AddVertices KV batches applied to a
finalized snapshot (nbg_snapshot_write_part + nbg_snapshot_commit).

The reference writes `edgeKey(part, src, type, rank, dst, INT64_MAX - now_us)` /
`vertexKey(part, vid, tag, INT64_MAX - now_us)` puts per part (AddEdgesProcessor.cpp:15-31,
AddVerticesProcessor.cpp:16-38), so a later write of the same edge carries a smaller version and
is read first by the prefix scan, and an identical key overwrites.  The oracle is the same
store built from base + write batches in write order; after each commit GO, getBound and
FIND SHORTEST PATH must match it exactly, and before the commit queries must still see the
previous commit.
"""
import random
from collections import Counter

import numpy as np
import pytest

import oracle as O
from nebula_amd import GraphSpace, NbgError, synth
from nebula_amd import expr as X
from test_gpu_tags import ET, PARTS, PERSON, random_space_kv

pytestmark = pytest.mark.gpu

FIELDS = [("name", O.STRING), ("score", O.INT), ("wt", O.DOUBLE)]
BASE_VER = 2**63 - 2


def ms(rows):
    return Counter(tuple(r) for r in rows)


def write_batch(rng, vids, new_vids, ver, tags=True, ends=None):
    """One AddEdges + AddVertices round: new edges (also to brand-new vertices), newer versions
    of existing edges, identical-key rewrites, new / updated tag rows (tags=False: edges only).
    ends: a set collecting the edges' endpoints (the vertices the snapshot numbers)."""
    part = lambda v: O.part_of(v, PARTS)  # noqa: E731
    batch = {p: [] for p in range(1, PARTS + 1)}
    every = vids + new_vids
    for _ in range(600):
        s, t = rng.choice(every), rng.choice(every)
        if ends is not None:
            ends.update((s, t))
        kind = rng.random()
        v = BASE_VER if kind < 0.2 else ver  # 20%: identical key of a base edge -> overwrite
        w = rng.randrange(1000, 2000)
        batch[part(s)].append((O.edge_key(part(s), s, ET, 0, t, v), O.encode_row([w])))
        batch[part(t)].append((O.edge_key(part(t), t, -ET, 0, s, v), b""))
    for v in (new_vids + rng.sample(vids, 40)) if tags else []:
        p = part(v)
        batch[p].append((O.vertex_key(p, v, PERSON, ver), O.encode_row([f"w{abs(v) % 13}", rng.randrange(100), 1.5])))
    return batch


def fresh_oracle(history):
    st = O.Store(PARTS)
    st.set_edge_schema(ET, [("weight", O.INT)], name="e")
    st.set_tag_schema(PERSON, FIELDS, name="person")
    merged = {p: [] for p in range(1, PARTS + 1)}
    for parts in history:
        for p, kv in parts.items():
            merged[p].extend(kv)
    for p, kv in merged.items():
        if kv:
            st.put(p, kv)
    st.finalize()
    return st


QUERIES = [
    (1, None, [X.SourceProp("person", "name"), X.DestProp("person", "score"), X.AliasProp("e", "weight")], False),
    (2, X.AliasProp("e", "weight") > 900, [X.EdgeDst("e"), X.DestProp("person", "name")], False),
    (3, None, [X.EdgeDst("e")], True),
]


def check_go(sp, st, starts):
    for steps, where, ys, distinct in QUERIES:
        rs = sp.go(starts, steps, ET, where=where, yields=ys, distinct=distinct)
        ref = st.go(starts, steps, ET, where=X.encode(where), yields=[y.encode() for y in ys], distinct=distinct)
        assert ref.code == 0, ref.error
        assert ms(rs.rows()) == ms(ref.rows())


def check_bound(sp, st, vids):
    q = vids[::7]
    parts = [O.part_of(v, PARTS) for v in q]
    cols = [("_dst", O.EDGE, 0), ("weight", O.EDGE, 0)]
    g = sp.get_bound(ET, parts, q, cols)
    r = st.get_bound(ET, parts, q, cols)
    assert g.failed == r.failed() == []
    rows = g.rows()
    got = {int(v): rows[g.vertex_row_offsets[i]:g.vertex_row_offsets[i + 1]] for i, v in enumerate(g.vertex_ids)}
    want = {}
    for i, row in enumerate(r.rows()):
        want.setdefault(r.row_vertex(i), []).append(row)
    assert got == want
    # in-bound rows read the in CSR (-ET keys)
    cols = [("_dst", O.EDGE, 0)]
    g = sp.get_bound(-ET, parts, q, cols)
    r = st.get_bound(-ET, parts, q, cols, in_bound=True)
    assert ms(g.rows()) == ms(r.rows())


@pytest.mark.parametrize("merge", [1, 0])
def test_writes_commit_and_snapshot_view(merge):
    """three commit rounds of AddEdges + AddVertices batches with brand-new vertices, newer
    versions, identical-key rewrites and tag rows against the oracle; merge = 1: each commit
    merges (new vertices extend the numbering, tag columns rebuilt), merge = 0: full rebuilds"""
    rng = random.Random(11)
    base, vids = random_space_kv(21)
    sp = GraphSpace(PARTS)
    try:
        sp.set_option("writable", 1)
        sp.set_option("merge_commit", merge)
        sp.set_edge_schema(ET, [("weight", O.INT)])
        sp.set_tag_schema(PERSON, "person", FIELDS)
        for p, kv in base.items():
            if kv:
                sp.load_part(p, kv)
        sp.finalize()
        history = [base]
        st = fresh_oracle(history)
        starts = vids[::19]
        check_go(sp, st, starts)
        seen = set(vids)
        for rnd in range(3):
            new_vids = []
            while len(new_vids) < 30:
                v = rng.randrange(-2**62, 2**62)
                if v not in seen:
                    seen.add(v)
                    new_vids.append(v)
            batch = write_batch(rng, vids, new_vids, BASE_VER - 10 * (rnd + 1))
            for p, kv in batch.items():
                if kv:
                    sp.write_part(p, kv)
            check_go(sp, st, starts)  # not committed yet: the previous snapshot
            sp.commit()
            history.append(batch)
            st = fresh_oracle(history)
            check_go(sp, st, starts + new_vids[:5])
            check_bound(sp, st, vids + new_vids)
            vids = vids + new_vids
        assert sp.info(ET)["merge_commits"] == (3 if merge else 0)
        sp.commit()  # empty commit: same snapshot
        check_go(sp, st, starts)
        check_bound(sp, st, vids)
    finally:
        sp.close()


def test_write_requires_writable():
    base, vids = random_space_kv(4, n_vertices=50, n_edges=200)
    sp = GraphSpace(PARTS)
    try:
        sp.set_edge_schema(ET, [("weight", O.INT)])
        sp.set_tag_schema(PERSON, "person", FIELDS)
        for p, kv in base.items():
            if kv:
                sp.write_part(p, kv)  # before finalize: a load
        sp.finalize()
        p = O.part_of(vids[0], PARTS)
        with pytest.raises(NbgError) as e:
            sp.write_part(p, [(O.edge_key(p, vids[0], ET, 0, vids[1], 5), O.encode_row([1]))])
        assert e.value.code == -1002
        with pytest.raises(NbgError) as e:
            sp.commit()
        assert e.value.code == -1002
    finally:
        sp.close()


@pytest.mark.parametrize("scale", [10, 19])
def test_rmat_writes_paths_and_go(scale):
    """Writes on top of the device-generated RMAT snapshot: shortest paths and GO after commit.
    Scale 19 (8.4 M tuples) is past one launch of the capped build grids."""
    follow = 1
    sp = GraphSpace(64)
    try:
        sp.set_option("writable", 1)
        sp.set_edge_schema(follow, [("weight", O.INT)])
        sp.gen_rmat(scale, 16, 1, follow)
        sp.finalize()
        s, t = synth.pairs(scale, 16, 1, 100)
        rng = random.Random(5)
        batch = {}
        for i in range(100):  # shortcut edges between the pair endpoints
            a, b = int(s[rng.randrange(len(s))]), int(t[rng.randrange(len(t))])
            pa, pb = O.part_of(a, 64), O.part_of(b, 64)
            batch.setdefault(pa, []).append((O.edge_key(pa, a, follow, 0, b, BASE_VER - 1), O.encode_row([7])))
            batch.setdefault(pb, []).append((O.edge_key(pb, b, -follow, 0, a, BASE_VER - 1), b""))
        for p, kv in batch.items():
            sp.write_part(p, kv)
        sp.commit()
        st = O.Store(64)
        st.set_edge_schema(follow, [("weight", O.INT)], name="follow")
        st.load_rmat(scale, 16, 1, follow)
        for p, kv in batch.items():
            st.put(p, kv)
        st.finalize()
        got = sp.shortest_path(s, t, follow, 4).rows()
        r = st.shortest_path(np.asarray(s, np.int64), np.asarray(t, np.int64), follow, 4)
        want = []
        for row in r.rows():
            row = [x for x in row if x is not None]
            want.append((row[0], row[1], row[2], tuple(row[3:])))
        assert got == want
        starts = [int(x) for x in s[:8]]
        ys = [X.EdgeDst("follow"), X.AliasProp("follow", "weight")]
        for steps in (1, 2):
            rs = sp.go(starts, steps, follow, yields=ys)
            ref = st.go(starts, steps, follow, yields=[y.encode() for y in ys])
            assert ref.code == 0, ref.error
            assert ms(rs.rows()) == ms(ref.rows())
    finally:
        sp.close()


def test_write_versions_known_answer():
    """The oracle KAT of tests/test_oracle_storage.py::test_write_path_versions through the
    device write path: base load, then a write batch with a newer version (smaller low byte), an
    identical-key rewrite and a newer version whose bytes sort later (the older row stays)."""
    t0 = (2**63 - 1 - 1_700_000_000_000_000) & ~0xFF | 0x40
    t1 = t0 & ~0xFF
    src, part = 11, O.part_of(11, 4)
    base = [(O.edge_key(part, src, 7, 0, 21, t0), O.encode_row([1])),
            (O.edge_key(part, src, 7, 0, 22, t0), O.encode_row([2])),
            (O.edge_key(part, src, 7, 0, 23, t1), O.encode_row([5]))]
    writes = [(O.edge_key(part, src, 7, 0, 21, t0 - 5), O.encode_row([3])),
              (O.edge_key(part, src, 7, 0, 22, t0), O.encode_row([4])),
              (O.edge_key(part, src, 7, 0, 23, t1 - 1), O.encode_row([6]))]
    sp = GraphSpace(4)
    try:
        sp.set_option("writable", 1)
        sp.set_edge_schema(7, [("w", O.INT)])
        sp.load_part(part, base)
        sp.finalize()
        cols = [("_dst", O.EDGE, 0), ("w", O.EDGE, 0)]
        assert [tuple(r) for r in sp.get_bound(7, [part], [src], cols).rows()] == [(21, 1), (22, 2), (23, 5)]
        sp.write_part(part, writes)
        sp.commit()
        assert [tuple(r) for r in sp.get_bound(7, [part], [src], cols).rows()] == [(21, 3), (22, 4), (23, 5)]
    finally:
        sp.close()


def test_add_processors_match_oracle():
    """Host mirrors of the write operators: InsertEdgeExecutor's out/in edge pair
    (AddEdgesRequest.insert, InsertEdgeExecutor.cpp:143-162) through AddEdgesProcessor, tag rows
    through AddVerticesProcessor, one version per request; a part this space does not have comes
    back in failed_codes and the other parts are still written."""
    from nebula_amd import (AddEdgesProcessor, AddEdgesRequest, AddVerticesProcessor, AddVerticesRequest, Edge,
                            EdgeKey, Tag, Vertex)
    base, vids = random_space_kv(6)
    rng = random.Random(9)
    new_vids = [rng.randrange(-2**62, 2**62) for _ in range(20)]
    ver_e, ver_v = BASE_VER - 100, BASE_VER - 101
    edges = [(rng.choice(vids + new_vids), rng.choice(vids + new_vids), rng.randrange(3),
              O.encode_row([rng.randrange(2000)])) for _ in range(300)]
    verts = {}
    for v in new_vids + vids[:30]:
        verts.setdefault(O.part_of(v, PARTS), []).append(
            Vertex(v, [Tag(PERSON, O.encode_row([f"n{abs(v) % 7}", rng.randrange(100), 0.25]))]))
    # the oracle's view: the same puts, in the same order
    batch = {p: [] for p in range(1, PARTS + 1)}
    for s, t, rank, props in edges:
        batch[O.part_of(s, PARTS)].append((O.edge_key(O.part_of(s, PARTS), s, ET, rank, t, ver_e), props))
        batch[O.part_of(t, PARTS)].append((O.edge_key(O.part_of(t, PARTS), t, -ET, rank, s, ver_e), b""))
    for p, vs in verts.items():
        for v in vs:
            batch[p].append((O.vertex_key(p, v.id, PERSON, ver_v), v.tags[0].props))
    st = fresh_oracle([base, batch])
    sp = GraphSpace(PARTS)
    try:
        sp.set_option("writable", 1)
        sp.set_edge_schema(ET, [("weight", O.INT)])
        sp.set_tag_schema(PERSON, "person", FIELDS)
        for p, kv in base.items():
            if kv:
                sp.load_part(p, kv)
        sp.finalize()
        req = AddEdgesRequest.insert(sp, ET, edges)
        req.parts[PARTS + 3] = [Edge(EdgeKey(1, ET, 0, 2), O.encode_row([1]))]
        resp = AddEdgesProcessor.instance(sp, commit=False, version=ver_e).process(req)
        assert resp.failed_codes == [{"part_id": PARTS + 3, "code": -14}]  # E_PART_NOT_FOUND
        resp = AddVerticesProcessor.instance(sp, version=ver_v).process(AddVerticesRequest(verts))
        assert resp.failed_codes == []
        check_go(sp, st, vids[::19] + new_vids[:5])
        check_bound(sp, st, vids + new_vids)
    finally:
        sp.close()


def _with_schema_version(row: bytes, ver: int) -> bytes:
    """a RowWriter row re-headed with a 1-byte schema version (RowWriter.cpp:49-75: header bits
    5-7 = version bytes; rows of < 16 fields carry no block offsets)"""
    return bytes([row[0] | (1 << 5), ver]) + row[1:]


def test_write_batch_all_or_nothing():
    """A refused write batch leaves nothing behind (a RocksDB WriteBatch per part is atomic):
    a tag row with another schema version, or a key whose part field is not the batch's part,
    fails the whole batch, and the next commit sees only the accepted batches"""
    base, vids = random_space_kv(12, n_vertices=300, n_edges=2000)
    rng = random.Random(3)
    sp = GraphSpace(PARTS)
    try:
        sp.set_option("writable", 1)
        sp.set_edge_schema(ET, [("weight", O.INT)])
        sp.set_tag_schema(PERSON, "person", FIELDS)
        for p, kv in base.items():
            if kv:
                sp.load_part(p, kv)
        sp.finalize()
        v0 = vids[0]
        p0 = O.part_of(v0, PARTS)
        ver = BASE_VER - 50
        good_edges = [(O.edge_key(p0, v0, ET, 0, t, ver), O.encode_row([1500 + i])) for i, t in enumerate(vids[1:20])]
        bad_tag = (O.vertex_key(p0, v0, PERSON, ver), _with_schema_version(O.encode_row(["x", 1, 2.0]), 3))
        with pytest.raises(NbgError) as e:
            sp.write_part(p0, good_edges + [bad_tag])
        assert e.value.code == -1003
        wrong_part = (O.edge_key(p0 % PARTS + 1, v0, ET, 0, vids[5], ver), O.encode_row([7]))
        with pytest.raises(NbgError) as e:
            sp.write_part(p0, good_edges[:3] + [wrong_part])
        assert e.value.code == -14
        # an accepted batch re-writing some of the refused keys with other values
        accepted = [(k, O.encode_row([99])) for k, _ in good_edges[::2]]
        sp.write_part(p0, accepted)
        sp.commit()
        st = fresh_oracle([base, {p0: accepted}])
        check_go(sp, st, vids[::17] + [v0])
        check_bound(sp, st, vids)
        sp.commit()  # a second commit of the same log: identical snapshot
        check_go(sp, st, vids[::17] + [v0])
    finally:
        sp.close()


def edge_batch(rng, vids, ver, n=800, in_keys=True):
    """edge writes between existing vertices only: new edges, newer versions of existing ones
    (bytewise order decides which version a scan reads first), identical-key rewrites;
    in_keys=False writes the out-edge keys alone (the in CSR stays as committed)"""
    part = lambda v: O.part_of(v, PARTS)  # noqa: E731
    batch = {p: [] for p in range(1, PARTS + 1)}
    for _ in range(n):
        s, t = rng.choice(vids), rng.choice(vids)
        kind = rng.random()
        v = BASE_VER if kind < 0.25 else (ver if kind < 0.8 else ver - 3)
        w = rng.randrange(1000, 2000)
        batch[part(s)].append((O.edge_key(part(s), s, ET, 0, t, v), O.encode_row([w])))
        if in_keys:
            batch[part(t)].append((O.edge_key(part(t), t, -ET, 0, s, v), b""))
    return batch


@pytest.mark.parametrize("merge", [1, 0])
def test_merge_commit_matches_full_rebuild_and_oracle(merge):
    """a commit whose batch adds no vertex and no tag row merges the sorted batch into the
    committed key order (merge_commits counts it); results equal the full rebuild's and the
    oracle's, including getBound's firstLoop rows over older versions"""
    rng = random.Random(29)
    base, vids = random_space_kv(33)
    sp = GraphSpace(PARTS)
    try:
        sp.set_option("writable", 1)
        sp.set_option("merge_commit", merge)
        sp.set_edge_schema(ET, [("weight", O.INT)])
        sp.set_tag_schema(PERSON, "person", FIELDS)
        for p, kv in base.items():
            if kv:
                sp.load_part(p, kv)
        sp.finalize()
        history = [base]
        starts = vids[::17]
        for rnd in range(3):
            batch = edge_batch(rng, vids, BASE_VER - 7 * (rnd + 1), in_keys=rnd != 1)
            for p, kv in batch.items():
                if kv:
                    sp.write_part(p, kv)
            sp.commit()
            history.append(batch)
            st = fresh_oracle(history)
            check_go(sp, st, starts)
            check_bound(sp, st, vids)
            # firstLoop: a filter that rejects the first version reads an older one
            q = vids[::5]
            parts = [O.part_of(v, PARTS) for v in q]
            cols = [("_dst", O.EDGE, 0), ("weight", O.EDGE, 0)]
            f = X.AliasProp("e", "weight") < 1500
            g = sp.get_bound(ET, parts, q, cols, filter=f)
            r = st.get_bound(ET, parts, q, cols, filt=f.encode())
            assert ms(g.rows()) == ms(r.rows())
        info = sp.info(ET)
        assert info["commits"] == 3
        assert info["merge_commits"] == (3 if merge else 0)
        # a batch with a new vertex takes the full rebuild
        v_new = 4242424242
        p = O.part_of(vids[0], PARTS)
        sp.write_part(p, [(O.edge_key(p, vids[0], ET, 0, v_new, BASE_VER - 50), O.encode_row([5]))])
        sp.commit()
        assert sp.info(ET)["merge_commits"] == (3 if merge else 0)
        assert v_new in set(int(x) for x in sp.go([vids[0]], 1, ET).columns[0])
    finally:
        sp.close()


def sst_files(rng, vids, new_vids, n_files=3):
    """SST-shaped ingest input (RocksEngine::ingest, RocksEngine.cpp:361-363: IngestExternalFile of
    prebuilt files): each file holds unique keys in key order -- edges with several versions of
    one (src, rank, dst), non-zero ranks, identical keys of base edges (the ingest overwrites
    them), in-edge keys, tag rows; a later file may repeat an earlier file's key (the later file
    wins, as a later put).  Returns the files as lists of (key, value) sorted by key bytes."""
    part = lambda v: O.part_of(v, PARTS)  # noqa: E731
    every = vids + new_vids
    files = []
    for f in range(n_files):
        kv = {}
        for _ in range(300):
            s, t = rng.choice(every), rng.choice(every)
            rank = rng.choice([0, 0, 0, 7, -3])
            vers = [BASE_VER] if rng.random() < 0.15 else rng.sample(range(BASE_VER - 500, BASE_VER - 100), 3)
            for ver in vers:  # several versions of the edge in one file
                w = rng.randrange(0, 3000)
                kv[O.edge_key(part(s), s, ET, rank, t, ver)] = O.encode_row([w])
                kv[O.edge_key(part(t), t, -ET, rank, s, ver)] = b""
        for v in rng.sample(every, 25):
            p = part(v)
            for ver in rng.sample(range(BASE_VER - 500, BASE_VER - 100), 2):
                kv[O.vertex_key(p, v, PERSON, ver)] = O.encode_row([f"s{f}_{abs(v) % 7}", rng.randrange(100), 0.5 * f])
        for v in new_vids:  # every new vertex gets a tag row (QUERIES read $$ props)
            p = part(v)
            kv[O.vertex_key(p, v, PERSON, BASE_VER - 50 - f)] = O.encode_row([f"n{abs(v) % 5}", f, 1.0])
        files.append(sorted(kv.items()))
    return files


@pytest.mark.parametrize("world", [1, 2])
def test_sst_ingest_after_finalize(world):
    """SST ingest mapped onto the write path: the files' pairs are read
    in key order, grouped by part (the key's first 4 bytes, NebulaKeyUtils.h:14-21) and passed to
    nbg_snapshot_write_part, then one nbg_snapshot_commit -- the same as puts of the same pairs in
    file order.  Multi-version edges, ranks, overwritten base keys, tag rows and new vertices;
    one rank and two LocalComm ranks (the commit merges on both: merge_commits)."""
    import struct

    from test_gpu_multirank import Group, union_rows
    rng = random.Random(5)
    base, vids = random_space_kv(13)
    seen = set(vids)
    new_vids = []
    while len(new_vids) < 24:
        v = rng.randrange(-2**62, 2**62)
        if v not in seen:
            seen.add(v)
            new_vids.append(v)
    files = sst_files(rng, vids, new_vids)
    # ingest order: file by file, each in key order, grouped by part
    ingest = []
    for kvs in files:
        by_part = {}
        for k, v in kvs:
            by_part.setdefault(struct.unpack("<i", k[:4])[0], []).append((k, v))
        ingest.append(by_part)
    st = fresh_oracle([base] + ingest)
    starts = vids[::11] + new_vids[:4]
    g = Group(world, parts=PARTS)
    try:
        def load(r, s):
            s.set_option("writable", 1)
            s.set_edge_schema(ET, [("weight", O.INT)])
            s.set_tag_schema(PERSON, "person", FIELDS)
            for p, kv in base.items():
                if kv and p % world == r:
                    s.load_part(p, kv)
            s.finalize()

        def ingest_all(r, s):
            for by_part in ingest:
                for p, kv in sorted(by_part.items()):
                    if p % world == r:
                        s.write_part(p, kv)
            s.commit()
        g.each(load)
        g.each(ingest_all)
        for steps, where, ys, distinct in QUERIES:
            res = g.go(starts, steps, ET, where=where, yields=ys, distinct=distinct)
            ref = st.go(starts, steps, ET, where=X.encode(where), yields=[y.encode() for y in ys], distinct=distinct)
            assert ref.code == 0, ref.error
            assert union_rows(res) == ms(ref.rows())
        if world == 1:
            check_bound(g.sp[0], st, vids + new_vids)
        assert g.each(lambda r, s: s.info(ET)["merge_commits"]) == [1] * world
    finally:
        g.close()
