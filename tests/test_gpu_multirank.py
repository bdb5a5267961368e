"""Sharded path (part % world ranks) on one GPU: N contexts of one process form an in-process
rank group (nbg_comm_init_local), so the exchange steps of the multi-GPU path -- the build-time
edge shuffle of the transposed CSR, the per-hop frontier mark exchange (top-down), the frontier
allgather (bottom-up), the global direction/emptiness sums and the DISTINCT row shuffle -- run
unchanged, with device-to-device copies in place of RCCL.  The union of the ranks' results must
equal the oracle's result (the reference's graphd merges the per-host responses,
GoExecutor.cpp:411-470 / StorageClient.inl:74-159).
"""
from collections import Counter
from concurrent.futures import ThreadPoolExecutor
import itertools

import numpy as np
import pytest

import oracle as O
from nebula_amd import GraphSpace, NbgError
from nebula_amd import expr as X

pytestmark = pytest.mark.gpu

FOLLOW = 1
SEED = 1
_keys = itertools.count(1000)


def ms(rows):
    return Counter(tuple(r) for r in rows)


class Group:
    """`world` contexts on device 0, one per rank; every call runs on all ranks in threads."""

    def __init__(self, world, parts=64):
        key = next(_keys)
        self.world = world
        self.sp = [GraphSpace(parts, device=0, rank=r, world_size=world) for r in range(world)]
        for s in self.sp:
            s.comm_init_local(key)
        self.pool = ThreadPoolExecutor(max_workers=world)

    def each(self, fn):
        futs = [self.pool.submit(fn, r, s) for r, s in enumerate(self.sp)]
        out, err = [], None
        for f in futs:
            try:
                out.append(f.result(timeout=300))
            except Exception as e:  # collect, so every rank has finished before raising
                out.append(None)
                err = err or e
        if err:
            raise err
        return out

    def go(self, *a, **k):
        return self.each(lambda r, s: s.go(*a, **k))

    def close(self):
        for s in self.sp:
            s.close()
        self.pool.shutdown()


def union_rows(results):
    c = Counter()
    for g in results:
        c.update(tuple(r) for r in g.rows())
    return c


def seeds_from(scale, n, seed=7):
    s, _, _ = O.rmat_edges(scale, 16, SEED)
    rng = np.random.default_rng(seed)
    return [int(x) for x in s[rng.integers(0, len(s), n)]]


@pytest.fixture(scope="module")
def oracle12():
    st = O.Store(64)
    st.set_edge_schema(FOLLOW, [("weight", O.INT)], name="follow")
    st.load_rmat(12, 16, SEED, FOLLOW)
    return st


@pytest.fixture(scope="module", params=[2, 3])
def rmat_group(request):
    g = Group(request.param)
    for s in g.sp:
        s.set_edge_schema(FOLLOW, [("weight", O.INT)])
    g.each(lambda r, s: s.gen_rmat(12, 16, SEED, FOLLOW))
    g.each(lambda r, s: s.finalize())
    yield g
    g.close()


def test_shard_sizes_cover_graph(rmat_group, oracle12):
    infos = rmat_group.each(lambda r, s: s.info(FOLLOW))
    one = GraphSpace(64)
    one.set_edge_schema(FOLLOW, [("weight", O.INT)])
    one.gen_rmat(12, 16, SEED, FOLLOW)
    one.finalize()
    i1 = one.info(FOLLOW)
    one.close()
    assert all(i["num_vertices"] == i1["num_vertices"] for i in infos)
    assert sum(i["local_vertices"] for i in infos) == i1["num_vertices"]
    assert sum(i["local_out_edges"] for i in infos) == i1["local_out_edges"]
    assert sum(i["local_in_edges"] for i in infos) == i1["local_in_edges"]


def test_comm_info_reports_group(rmat_group):
    """nbg_comm_info: the rank count the transport itself formed (LocalComm here; RCCL's
    ncclCommCount on a multi-GPU launch, reported by bench.py's comm.communicator)"""
    infos = rmat_group.each(lambda r, s: s.comm_info())
    assert all(i == {"ranks": len(rmat_group.sp), "transport": "local"} for i in infos)
    one = GraphSpace(64)
    assert one.comm_info() == {"ranks": 1, "transport": "none"}
    one.close()


@pytest.mark.parametrize("force", [0, 1, -1])
def test_sharded_go_distinct_dst(rmat_group, oracle12, force):
    g = rmat_group
    g.each(lambda r, s: s.set_option("bu_force", force))
    try:
        starts = seeds_from(12, 64)
        w = X.AliasProp("follow", "weight") > 499
        y = [X.EdgeDst("follow")]
        for steps in (1, 2, 3):
            res = g.go(starts, steps, FOLLOW, where=w, yields=y, distinct=True)
            ref = oracle12.go(starts, steps, FOLLOW, where=w.encode(), yields=[y[0].encode()], distinct=True)
            got = np.sort(np.concatenate([x.columns[0] for x in res]))
            assert np.array_equal(got, np.sort(ref.int_col(0)))
            assert len(np.unique(got)) == len(got)  # each vertex reported by its owner only
            assert sum(x.edges_scanned for x in res) == ref.edges_scanned
        t = g.each(lambda r, s: s.last_timing())
        if force == 1:
            assert all(x["bu_steps"] > 0 for x in t)
        if force == -1:
            assert all(x["bu_steps"] == 0 for x in t)
    finally:
        g.each(lambda r, s: s.set_option("bu_force", 0))


@pytest.mark.parametrize("force", [1, -1])
def test_sharded_go_rows_and_yields(rmat_group, oracle12, force):
    g = rmat_group
    g.each(lambda r, s: s.set_option("bu_force", force))
    try:
        starts = seeds_from(12, 24, seed=3)
        for steps in (1, 2, 3):
            res = g.go(starts, steps, FOLLOW)
            ref = oracle12.go(starts, steps, FOLLOW)
            assert union_rows(res) == ms(ref.rows())
            assert sum(x.edges_scanned for x in res) == ref.edges_scanned
        w2 = (X.AliasProp("follow", "weight") % 3).eq(1) & (X.EdgeSrc("follow") > 0)
        y2 = [X.EdgeSrc("follow"), X.EdgeDst("follow"), X.AliasProp("follow", "weight") * 2]
        res = g.go(starts, 2, FOLLOW, where=w2, yields=y2)
        ref = oracle12.go(starts, 2, FOLLOW, where=w2.encode(), yields=[y.encode() for y in y2])
        assert union_rows(res) == ms(ref.rows())
    finally:
        g.each(lambda r, s: s.set_option("bu_force", 0))


def test_sharded_distinct_rows_shuffle(rmat_group, oracle12):
    """DISTINCT over computed columns: equal rows made on different ranks meet on one rank"""
    g = rmat_group
    starts = seeds_from(12, 32, seed=11)
    y = [X.AliasProp("follow", "weight") % 7, X.AliasProp("follow", "weight") > 500]
    for steps in (1, 3):
        res = g.go(starts, steps, FOLLOW, yields=y, distinct=True)
        ref = oracle12.go(starts, steps, FOLLOW, yields=[v.encode() for v in y], distinct=True)
        u = union_rows(res)
        assert u == ms(ref.rows())
        assert all(n == 1 for n in u.values())


def test_sharded_eval_error_fails_every_rank(rmat_group):
    g = rmat_group
    starts = seeds_from(12, 8)
    bad = X.AliasProp("follow", "weight") / 0 > 1  # division by zero -> E_EVAL on some row
    errs = []

    def run(r, s):
        try:
            s.go(starts, 2, FOLLOW, where=bad)
        except NbgError as e:
            errs.append(e.code)

    g.each(run)
    assert len(errs) == g.world
    # the group is still consistent afterwards
    res = g.go(starts, 2, FOLLOW)
    assert sum(x.n_rows for x in res) > 0


def test_sharded_empty_frontier(rmat_group):
    g = rmat_group
    res = g.go([123456789123], 3, FOLLOW)  # not a vertex: empty result on every rank
    assert all(x.n_rows == 0 for x in res)
    res = g.go([], 2, FOLLOW, distinct=True)
    assert all(x.n_rows == 0 for x in res)


def test_sharded_kv_ingest(oracle12):
    """KV parts loaded on their owner rank (part % world) give the oracle's results"""
    g = Group(2)
    try:
        for s in g.sp:
            s.set_edge_schema(FOLLOW, [("weight", O.INT)])

        def load(r, s):
            for p in range(1, 65):
                if p % 2 == r:
                    s.load_part(p, oracle12.dump_part(p))

        g.each(load)
        g.each(lambda r, s: s.finalize())
        starts = seeds_from(12, 32, seed=5)
        w = X.AliasProp("follow", "weight") > 250
        y = [X.EdgeDst("follow"), X.AliasProp("follow", "weight")]
        for steps in (1, 3):
            res = g.go(starts, steps, FOLLOW, where=w, yields=y)
            ref = oracle12.go(starts, steps, FOLLOW, where=w.encode(), yields=[v.encode() for v in y])
            assert union_rows(res) == ms(ref.rows())
        # getBound: each rank serves its own parts, reports the others as failed
        parts = [O.part_of(v, 64) for v in starts]
        cols = [("_dst", O.EDGE, 0), ("weight", O.EDGE, 0)]
        bound = g.each(lambda r, s: s.get_bound(FOLLOW, parts, starts, cols))
        ref = oracle12.get_bound(FOLLOW, parts, starts, cols)
        assert union_rows(bound) == ms(ref.rows())
    finally:
        g.close()


def test_sharded_shortest_path(rmat_group, oracle12):
    """FIND SHORTEST PATH with world > 1: pairs sharded i % world over the ranks, each answered
    against the allgathered replica of the out / in CSRs; the union of the ranks' rows (and their
    canonical paths) equals the oracle's"""
    from nebula_amd import synth
    g = rmat_group
    s, t = synth.pairs(12, 16, SEED, 120, pick_seed=3)
    src = np.concatenate([s, [s[0], -5]]).astype(np.int64)
    dst = np.concatenate([t, [s[0], t[0]]]).astype(np.int64)
    res = g.each(lambda r, sp: sp.shortest_path(src, dst, FOLLOW, 6))
    got = Counter()
    for r, pr in enumerate(res):
        rows = pr.rows()
        assert len(rows) == len(range(r, len(src), g.world))
        got.update(rows)
    want = Counter()
    for row in oracle12.shortest_path(src, dst, FOLLOW, 6).rows():
        row = [x for x in row if x is not None]
        want[(row[0], row[1], row[2], tuple(row[3:]))] += 1
    assert got == want


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_tag_props(world):
    """$^ / $$ tag props with sharded ownership: each rank decodes the vertex keys of its own
    parts and the tag columns are replicated by owner slice, so $$ props of dsts owned by
    another rank resolve (the reference's fetchVertexProps asks the dst's host)."""
    import test_gpu_tags as T
    parts, vids = T.random_space_kv(3)
    fields = [("name", O.STRING), ("score", O.INT), ("wt", O.DOUBLE)]
    st = O.Store(T.PARTS)
    st.set_edge_schema(T.ET, [("weight", O.INT)], name="e")
    st.set_tag_schema(T.PERSON, fields, name="person")
    for p, kv in parts.items():
        if kv:
            st.put(p, kv)
    st.finalize()
    g = Group(world, parts=T.PARTS)
    try:
        def load(r, s):
            s.set_edge_schema(T.ET, [("weight", O.INT)])
            s.set_tag_schema(T.PERSON, "person", fields)
            for p, kv in parts.items():
                if kv and p % world == r:
                    s.load_part(p, kv)
            s.finalize()
        g.each(load)
        for qi in (0, 1, 3):
            steps, where, ys, distinct = T.QUERIES[qi]
            starts = vids[::23]
            res = g.go(starts, steps, T.ET, where=where, yields=ys, distinct=distinct)
            ref = st.go(starts, steps, T.ET, where=X.encode(where), yields=[y.encode() for y in ys],
                        distinct=distinct)
            assert ref.code == 0, ref.error
            assert union_rows(res) == ms(ref.rows())
    finally:
        g.close()


@pytest.mark.parametrize("world,room", [(2, 10), (3, 10), (2, 0), (3, 0)])
def test_sharded_writes_commit(world, room):
    """Write path with sharded ownership: each rank takes the write batches of its
    own parts (StorageClient routes an AddEdges part to its leader); commit is collective.  A batch
    with new vertices (INSERT EDGE to unseen vids, AddEdgesProcessor.cpp:15-31) merges on every
    rank: the new vertices take gidx in their owners' growth room (grow_room_pct), the same
    numbering on every rank; without room (grow_room_pct = 0) it rebuilds fully.  Batches of
    edges and tag rows of known vertices merge on every rank (merge_commits), also when only one
    rank has writes of its own."""
    import random

    import test_gpu_tags as T
    import test_gpu_writes as W
    base, vids = T.random_space_kv(8)
    rng = random.Random(2)
    new_vids = [rng.randrange(-2**62, 2**62) for _ in range(25)]
    ends = set()
    batch = W.write_batch(rng, vids, new_vids, W.BASE_VER - 10, ends=ends)
    # vertices with an edge after batch 1 (a new vid with only a tag row has no gidx: an edge to
    # it later is a new vertex again)
    known = vids + [v for v in new_vids if v in ends]
    g = Group(world, parts=T.PARTS)
    try:
        def load(r, s):
            s.set_option("writable", 1)
            s.set_option("grow_room_pct", room)
            s.set_edge_schema(T.ET, [("weight", O.INT)])
            s.set_tag_schema(T.PERSON, "person", W.FIELDS)
            for p, kv in base.items():
                if kv and p % world == r:
                    s.load_part(p, kv)
            s.finalize()

        # round 1: every rank writes its parts; round 2: only rank 0's parts get writes, the
        # other ranks still join the collective commit
        batch2 = W.write_batch(rng, known, [], W.BASE_VER - 20)
        batch2 = {p: kv for p, kv in batch2.items() if p % world == 0}

        def write(b):
            def run(r, s):
                for p, kv in b.items():
                    if kv and p % world == r:
                        s.write_part(p, kv)
                s.commit()
            return run
        # round 3: edges only, on every rank
        batch3 = W.write_batch(rng, known, [], W.BASE_VER - 30, tags=False)
        starts = vids[::19] + new_vids[:4]

        def check(history):
            st = W.fresh_oracle(history)
            for steps, where, ys, distinct in W.QUERIES:
                res = g.go(starts, steps, T.ET, where=where, yields=ys, distinct=distinct)
                ref = st.go(starts, steps, T.ET, where=X.encode(where), yields=[y.encode() for y in ys],
                            distinct=distinct)
                assert ref.code == 0, ref.error
                assert union_rows(res) == ms(ref.rows())
            # FIND SHORTEST PATH reads the replicated CSRs, rebuilt after each commit
            src = np.array(starts[:8], dtype=np.int64)
            dst = np.array(starts[-8:], dtype=np.int64)
            got = Counter()
            for pr in g.each(lambda r, s: s.shortest_path(src, dst, T.ET, 6)):
                got.update(pr.rows())
            want = Counter()
            for row in st.shortest_path(src, dst, T.ET, 6).rows():
                row = [x for x in row if x is not None]
                want[(row[0], row[1], row[2], tuple(row[3:]))] += 1
            assert got == want

        # round 4: edges to brand-new vertices again, on every rank
        new4 = [rng.randrange(-2**62, 2**62) for _ in range(20)]
        batch4 = W.write_batch(rng, known, new4, W.BASE_VER - 40)
        g.each(load)
        g.each(write(batch))
        check([base, batch])
        g.each(write(batch2))
        check([base, batch, batch2])
        g.each(write(batch3))
        check([base, batch, batch2, batch3])
        g.each(write(batch4))
        check([base, batch, batch2, batch3, batch4])
        merges = g.each(lambda r, s: s.info(T.ET)["merge_commits"])
        # batches 1 and 4 have new vertices: merged into the growth room; without reserved room
        # only when the owners' 64-vertex padding happens to hold them, else rebuilt
        assert len(set(merges)) == 1
        assert merges[0] == 4 if room else 2 <= merges[0] <= 4
        nv = g.each(lambda r, s: s.info(T.ET)["num_vertices"])
        assert len(set(nv)) == 1
    finally:
        g.close()


@pytest.mark.parametrize("world", [2])
def test_sharded_write_misrouted_key_refused(world):
    """a write batch carrying a key of a vertex another rank owns is refused at write time on the
    writing rank (E_PART_NOT_FOUND), nothing is appended, and the collective commit still runs on
    every rank with the accepted batches (no rank fails inside the commit's collectives)"""
    import test_gpu_tags as T
    import test_gpu_writes as W
    base, vids = T.random_space_kv(5, n_vertices=200, n_edges=1200)
    mine = [v for v in vids if (O.part_of(v, T.PARTS) % world) == 0]
    other = [v for v in vids if (O.part_of(v, T.PARTS) % world) == 1]
    p0 = O.part_of(mine[0], T.PARTS)
    ver = W.BASE_VER - 30
    bad = [(O.edge_key(p0, other[0], T.ET, 0, mine[1], ver), O.encode_row([5]))]  # src owned by rank 1
    good = [(O.edge_key(p0, mine[0], T.ET, 0, mine[2], ver), O.encode_row([6]))]
    g = Group(world, parts=T.PARTS)
    codes = {}
    try:
        def load(r, s):
            s.set_option("writable", 1)
            s.set_edge_schema(T.ET, [("weight", O.INT)])
            s.set_tag_schema(T.PERSON, "person", W.FIELDS)
            for p, kv in base.items():
                if kv and p % world == r:
                    s.load_part(p, kv)
            s.finalize()

        def write(r, s):
            if r == 0:
                try:
                    s.write_part(p0, good + bad)
                except NbgError as e:
                    codes[r] = e.code
                s.write_part(p0, good)
            s.commit()
        g.each(load)
        g.each(write)
        assert codes == {0: -14}
        st = W.fresh_oracle([base, {p0: good}])
        starts = vids[::13] + [mine[0]]
        for steps, where, ys, distinct in W.QUERIES:
            res = g.go(starts, steps, T.ET, where=where, yields=ys, distinct=distinct)
            ref = st.go(starts, steps, T.ET, where=X.encode(where), yields=[y.encode() for y in ys],
                        distinct=distinct)
            assert ref.code == 0, ref.error
            assert union_rows(res) == ms(ref.rows())
    finally:
        g.close()


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("steps", [2, 3])
def test_sharded_multistep_input(world, steps):
    """$- / $var props with STEPS > 1 across ranks (GoExecutor.h:174-193's VertexBackTracker):
    each rank's top-down hop takes the smallest root over its own in-edges, the owners take the
    minimum over all ranks (exchange_roots) -- the oracle's deterministic rule (DESIGN.md
    divergence 6), many starts sharing descendants"""
    from nebula_amd import synth
    scale = 11
    st = O.Store(16)
    st.set_edge_schema(1, [("weight", O.INT)], name="e")
    st.load_rmat(scale, 8, 3, 1)
    g = Group(world, parts=16)
    try:
        for s in g.sp:
            s.set_edge_schema(1, [("weight", O.INT)])
        g.each(lambda r, s: s.gen_rmat(scale, 8, 3, 1))
        g.each(lambda r, s: s.finalize())
        starts = list(synth.seeds(scale, 8, 3, 24))
        inputs = [("n", O.INT, [int(i * 7 % 11) for i in range(len(starts))])]
        ys = [X.InputProp("n"), X.AliasProp("e", "weight"), X.EdgeDst("e")]
        for w in (None, X.InputProp("n") > 4, (X.InputProp("n") + X.AliasProp("e", "weight")) > 600):
            for distinct in (False, True):
                res = g.go(starts, steps, 1, where=w, yields=ys, distinct=distinct, inputs=inputs)
                ref = st.go(starts, steps, 1, where=X.encode(w), yields=[y.encode() for y in ys],
                            distinct=distinct, inputs=inputs)
                assert ref.code == 0, ref.error
                assert union_rows(res) == ms(ref.rows())
                assert sum(x.n_rows for x in res) > 0
    finally:
        g.close()
