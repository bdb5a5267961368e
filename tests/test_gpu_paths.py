"""GPU parity of FIND SHORTEST PATH against the oracle.

The reference has no implementation (src/graph/FindExecutor.cpp:20-22), so the oracle
(oracle/refcpu.cpp ora_shortest_path: backward BFS from dst over the in-edge keys + greedy
smallest-vid walk from src) is the definition; no reference fixture pins it ("parity unpinned"
in DESIGN.md), and tests/test_oracle_paths_independent.py pins the oracle to an independent
restatement (scipy BFS over the raw edge list).  Hop counts and whole paths must match bit-exactly.
"""
import numpy as np
import pytest

import fixtures as F
import oracle as O
from nebula_amd import FindPathExecutor, GraphSpace, NbgError, synth

pytestmark = pytest.mark.gpu

FOLLOW = 1


def oracle_paths(st, src, dst, et, max_steps):
    r = st.shortest_path(np.asarray(src, np.int64), np.asarray(dst, np.int64), et, max_steps)
    out = []
    for row in r.rows():
        row = [x for x in row if x is not None]
        out.append((row[0], row[1], row[2], tuple(row[3:])))
    return out


@pytest.fixture(scope="module", params=[10, 13])
def rmat(request):
    scale = request.param
    sp = GraphSpace(64)
    sp.set_edge_schema(FOLLOW, [("weight", 2)])
    sp.gen_rmat(scale, 16, 1, FOLLOW)
    sp.finalize()
    st = O.Store(64)
    st.set_edge_schema(FOLLOW, [("weight", O.INT)], name="follow")
    st.load_rmat(scale, 16, 1, FOLLOW)
    yield scale, sp, st
    sp.close()


def edge_case_pairs(scale):
    s, t = synth.pairs(scale, 16, 1, 8, pick_seed=3)
    nb_s, nb_t = synth.edges(scale, 1, np.arange(4, dtype=np.uint64))  # direct edges: 1 hop
    src = list(s) + list(nb_s) + [s[0], -5, s[1], -7, t[2]]
    dst = list(t) + list(nb_t) + [s[0], t[0], -9, -7, t[2]]
    return np.array(src, np.int64), np.array(dst, np.int64)


@pytest.mark.parametrize("max_steps", [1, 2, 3, 6])
def test_rmat_pairs_vs_oracle(rmat, max_steps):
    scale, sp, st = rmat
    s, t = synth.pairs(scale, 16, 1, 200)
    es, et_ = edge_case_pairs(scale)
    src = np.concatenate([s, es])
    dst = np.concatenate([t, et_])
    got = sp.shortest_path(src, dst, FOLLOW, max_steps).rows()
    want = oracle_paths(st, src, dst, FOLLOW, max_steps)
    assert got == want
    if max_steps >= 6:
        assert sum(1 for r in got if r[2] >= 3) >= 5  # the set exercises multi-level meets


def test_rmat_batches_equal_single_launch(rmat):
    scale, sp, st = rmat
    s, t = synth.pairs(scale, 16, 1, 150, pick_seed=5)
    one = sp.shortest_path(s, t, FOLLOW, 8).rows()
    sp.set_option("sp_batch", 7)  # 22 batches of 7 pairs; distance bytes reset between batches
    try:
        many = sp.shortest_path(s, t, FOLLOW, 8).rows()
    finally:
        sp.set_option("sp_batch", 1024)
    assert one == many
    assert one == oracle_paths(st, s, t, FOLLOW, 8)


def test_repeated_calls_are_clean(rmat):
    # the distance arrays persist across calls: a second identical call must not see stale bytes
    scale, sp, st = rmat
    s, t = synth.pairs(scale, 16, 1, 64, pick_seed=9)
    a = sp.shortest_path(s, t, FOLLOW, 5).rows()
    b = sp.shortest_path(s, t, FOLLOW, 5).rows()
    c = sp.shortest_path(t, s, FOLLOW, 5).rows()
    assert a == b
    assert c == oracle_paths(st, t, s, FOLLOW, 5)


def test_duplicate_pairs_and_empty(rmat):
    scale, sp, st = rmat
    s, t = synth.pairs(scale, 16, 1, 4, pick_seed=13)
    src = np.concatenate([s, s, s])
    dst = np.concatenate([t, t, t])
    got = sp.shortest_path(src, dst, FOLLOW, 6).rows()
    assert got == oracle_paths(st, src, dst, FOLLOW, 6)
    empty = sp.shortest_path(np.zeros(0, np.int64), np.zeros(0, np.int64), FOLLOW, 4)
    assert empty.rows() == []


def test_paths_are_edges_and_shortest(rmat):
    # size-independent properties: every path step is an out-edge, length = hops
    scale, sp, st = rmat
    s, t = synth.pairs(scale, 16, 1, 64, pick_seed=21)
    res = sp.shortest_path(s, t, FOLLOW, 8)
    for (a, b, h, path) in res.rows():
        if h < 0:
            assert path == ()
            continue
        assert len(path) == h + 1 and path[0] == a and path[-1] == b
        for u, v in zip(path, path[1:]):
            nbrs = sp.go([u], 1, FOLLOW).columns[0]
            assert v in set(int(x) for x in nbrs)


def test_bad_arguments(rmat):
    scale, sp, st = rmat
    with pytest.raises(NbgError):
        sp.shortest_path([1], [2], FOLLOW, 300)
    with pytest.raises(NbgError):
        sp.shortest_path([1], [2], 99, 3)
    with pytest.raises(NbgError):
        sp.shortest_path([1], [2], -FOLLOW, 3)


def test_nba_like_paths():
    sp = GraphSpace(1)
    for et, (name, fields) in F.NBA_EDGE_SCHEMAS.items():
        sp.set_edge_schema(et, fields)
    parts, vid = F.nba_kv()
    for p, kv in parts.items():
        sp.load_part(p, kv)
    sp.finalize()
    st, _ = F.nba_oracle_store()
    names = sorted(vid)
    froms = [vid[n] for n in names[:12]]
    tos = [vid[n] for n in names[-12:]] + [vid["Tim Duncan"], vid["Tony Parker"]]
    got = FindPathExecutor(sp, froms, tos, F.NBA_LIKE, upto=5).execute().rows()
    src = np.repeat(np.array(froms, np.int64), len(tos))
    dst = np.tile(np.array(tos, np.int64), len(froms))
    want = oracle_paths(st, src, dst, F.NBA_LIKE, 5)
    assert got == want
    assert any(r[2] >= 2 for r in got)
    sp.close()


def test_list_overflow_recovery():
    # host-driven path (sp_dev = 0): tiny list bounds force every overflow path: frontier lists and
    # meet lists rebuilt from the distance bytes, the claim arena replaced by a full reset of the
    # batch's bytes
    scale = 12
    sp = GraphSpace(64)
    sp.set_edge_schema(FOLLOW, [("weight", 2)])
    sp.gen_rmat(scale, 16, 1, FOLLOW)
    sp.finalize()
    st = O.Store(64)
    st.set_edge_schema(FOLLOW, [("weight", O.INT)], name="follow")
    st.load_rmat(scale, 16, 1, FOLLOW)
    sp.set_option("sp_list_soft", 1)
    sp.set_option("sp_dev", 0)
    s, t = synth.pairs(scale, 16, 1, 300, pick_seed=17)
    got = sp.shortest_path(s, t, FOLLOW, 7).rows()
    assert got == oracle_paths(st, s, t, FOLLOW, 7)
    again = sp.shortest_path(t, s, FOLLOW, 7).rows()  # bytes were reset after the overflowed batch
    assert again == oracle_paths(st, t, s, FOLLOW, 7)
    sp.close()


@pytest.mark.parametrize("probe", [0, 1])
def test_meet_probe_on_and_off_match_oracle(rmat, probe):
    """the early-exit meet probe (pairs one edge short of meeting skip the expansion) and the
    plain level-by-level expansion give the oracle's hop counts and canonical paths (the
    vertex-major distance layout, sp_vmajor, lost and was removed in round 6)"""
    scale, sp, st = rmat
    sp.set_option("sp_probe", probe)
    sp.set_option("sp_dev", int(probe == 1))
    try:
        s, t = synth.pairs(scale, 16, 1, 300, pick_seed=17)
        es, et_ = edge_case_pairs(scale)
        src, dst = np.concatenate([s, es]), np.concatenate([t, et_])
        for max_steps in (2, 8):
            got = sp.shortest_path(src, dst, FOLLOW, max_steps).rows()
            assert got == oracle_paths(st, src, dst, FOLLOW, max_steps)
    finally:
        sp.set_option("sp_dev", 1)
        sp.set_option("sp_probe", 1)


@pytest.mark.parametrize("dev,ilv", [(1, 1), (1, 0), (0, 1), (0, 0)])
def test_distance_layouts_match_oracle(rmat, dev, ilv):
    """the distance bytes interleaved by side (sp_ilv: one 2-byte load reads both sides of a vertex)
    or in two separate halves, device-driven or host-driven: the oracle's paths; the layout
    switched between calls leaves the bytes clean (all unseen)"""
    scale, sp, st = rmat
    s, t = synth.pairs(scale, 16, 1, 300, pick_seed=31)
    es, et_ = edge_case_pairs(scale)
    src, dst = np.concatenate([s, es]), np.concatenate([t, et_])
    try:
        for lay in (ilv, 1 - ilv, ilv):
            sp.set_option("sp_dev", dev)
            sp.set_option("sp_ilv", lay)
            for max_steps in (2, 8):
                got = sp.shortest_path(src, dst, FOLLOW, max_steps).rows()
                assert got == oracle_paths(st, src, dst, FOLLOW, max_steps), (lay, max_steps)
            if dev:
                assert sp.last_timing()["spec_hops"] >= 1  # the batches ran device-driven
    finally:
        sp.set_option("sp_dev", 1)
        sp.set_option("sp_ilv", 1)


@pytest.mark.parametrize("begin_x", [1, 0])
def test_first_iteration_tables_from_batch_start(rmat, begin_x):
    """iteration 1's X table, chunk ranges and carried roots built by the batch start kernel
    (sp_dv_begin_x, default) or by k_dv_select from the depth-0 lists: the oracle's paths, with
    roots of degree 0, src == dst and unknown vids among the pairs"""
    scale, sp, st = rmat
    s, t = synth.pairs(scale, 16, 1, 300, pick_seed=41)
    es, et_ = edge_case_pairs(scale)
    src, dst = np.concatenate([s, es]), np.concatenate([t, et_])
    sp.set_option("sp_dv_begin_x", begin_x)
    try:
        for max_steps in (1, 3, 8):
            got = sp.shortest_path(src, dst, FOLLOW, max_steps).rows()
            assert got == oracle_paths(st, src, dst, FOLLOW, max_steps), max_steps
            assert sp.last_timing()["spec_hops"] >= 1
    finally:
        sp.unset_option("sp_dv_begin_x")


@pytest.mark.parametrize("push,walk_wg,sweep_src", [(0, 0, 0), (1, 0, 0), (1, 1, 0), (0, 0, 1), (1, 0, 1)])
def test_sweep_direction_and_walk_variants(rmat, push, walk_wg, sweep_src):
    """the sweep's per-pair push/pull choice (forced off: pull only), the workgroup-per-pair walk
    and the sweep that runs down to src all give the oracle's paths"""
    scale, sp, st = rmat
    sp.set_option("sp_sweep_push", push)
    sp.set_option("sp_walk_wg", walk_wg)
    sp.set_option("sp_sweep_src", sweep_src)
    sp.set_option("sp_dev", 0)
    try:
        s, t = synth.pairs(scale, 16, 1, 300, pick_seed=23)
        es, et_ = edge_case_pairs(scale)
        src, dst = np.concatenate([s, es]), np.concatenate([t, et_])
        for max_steps in (3, 8):
            got = sp.shortest_path(src, dst, FOLLOW, max_steps).rows()
            assert got == oracle_paths(st, src, dst, FOLLOW, max_steps)
        hops = sp.last_timing()["hops"]
        assert any(h["mode"] == "sp-sweep" for h in hops) or scale < 11
    finally:
        sp.set_option("sp_dev", 1)
        sp.set_option("sp_sweep_push", 1)
        sp.set_option("sp_walk_wg", 0)
        sp.set_option("sp_sweep_src", 0)


@pytest.mark.parametrize("chunks,lvbits,push", [(1, 1, 1), (1, 1, 0), (0, 1, 1), (1, 0, 1), (0, 0, 0)])
def test_sweep_kernels_and_level_filter(rmat, chunks, lvbits, push):
    """the chunked sweep (k_sp_sweep, one wave per 1024 entries of a row) and the edge-balanced
    tile sweep (k_sp_expand, sweep mode), with and without the per-side level bitmaps that filter
    the sweep / probe / walk distance reads, in pull-only and push/pull mode: the oracle's paths"""
    scale, sp, st = rmat
    sp.set_option("sp_sweep_chunks", chunks)
    sp.set_option("sp_lvbits", lvbits)
    sp.set_option("sp_sweep_push", push)
    sp.set_option("sp_dev", 0)
    try:
        s, t = synth.pairs(scale, 16, 1, 300, pick_seed=29)
        es, et_ = edge_case_pairs(scale)
        src, dst = np.concatenate([s, es]), np.concatenate([t, et_])
        for max_steps in (3, 8):
            got = sp.shortest_path(src, dst, FOLLOW, max_steps).rows()
            assert got == oracle_paths(st, src, dst, FOLLOW, max_steps)
    finally:
        sp.set_option("sp_dev", 1)
        sp.set_option("sp_sweep_chunks", 1)
        sp.set_option("sp_lvbits", 1)
        sp.set_option("sp_sweep_push", 1)


@pytest.mark.parametrize("dev", [1, 0])
@pytest.mark.parametrize("pf,gf,occ,batch", [(1, 24, 1, 1024), (0, 24, 1, 1024), (1, 0, 1, 1024), (0, 0, 8, 1024),
                                             (1, 10, 1, 1024), (1, 24, 8, 7)])
def test_device_driven_batches(rmat, dev, pf, gf, occ, batch):
    """the device-driven batch (k_dv_*: one fixed launch chain per batch, counters published by
    the step kernels' last block) with the pair filters (sp_pf), the global level filter (sp_gf_log2,
    2^10 bits: saturated, every test reaches the byte) and neither, against the host-driven path and
    the oracle; nbg_timing.spec_hops counts the batches that ran device-driven"""
    scale, sp, st = rmat
    s, t = synth.pairs(scale, 16, 1, 200, pick_seed=17)
    es, et_ = edge_case_pairs(scale)
    src = np.concatenate([s, es])
    dst = np.concatenate([t, et_])
    opts = (("sp_dev", dev), ("sp_pf", pf), ("sp_gf_log2", gf), ("sp_dv_occ", occ), ("sp_batch", batch))
    for k, v in opts:
        sp.set_option(k, v)
    try:
        for max_steps in (3, 8):
            got = sp.shortest_path(src, dst, FOLLOW, max_steps).rows()
            tm = sp.last_timing()
            again = sp.shortest_path(src, dst, FOLLOW, max_steps).rows()
            assert got == again
            assert got == oracle_paths(st, src, dst, FOLLOW, max_steps)
            nbatch = -(-len(src) // batch)
            assert tm["spec_hops"] == (nbatch if dev else 0), tm["spec_hops"]
            if dev and batch >= len(src):
                # one wait per BFS iteration (published by its step kernel) + the batch's results
                assert tm["host_waits"] <= tm["steps_run"] + 2, (tm["host_waits"], tm["steps_run"])
    finally:
        for k, _ in opts:
            sp.unset_option(k)


@pytest.mark.parametrize("cap,grid", [(64, 0), (300, 0), (2000, 0), (300, 8192), (2000, 8192)])
def test_device_driven_overflow_falls_back(cap, grid):
    """sp_dv_list bounds every list of the device-driven batch: an overflow (BFS lists, meets,
    sweep lists, chunk tables, arena) restores the clean state and re-runs the batch host-driven;
    results stay the oracle's and later calls see clean distance bytes and filters.  grid: scan
    grids of 8192 blocks, far past the resident grid, so expansion blocks start after a list
    has overflowed (they skip their chunks but must still hand the meet probe's claims to the
    arena the abort resets distance bytes from)"""
    scale = 12
    sp = GraphSpace(64)
    sp.set_edge_schema(FOLLOW, [("weight", 2)])
    sp.gen_rmat(scale, 16, 1, FOLLOW)
    sp.finalize()
    st = O.Store(64)
    st.set_edge_schema(FOLLOW, [("weight", O.INT)], name="follow")
    st.load_rmat(scale, 16, 1, FOLLOW)
    try:
        s, t = synth.pairs(scale, 16, 1, 300, pick_seed=17)
        sp.set_option("sp_dv_list", cap)
        sp.set_option("sp_batch", 100)
        if grid:
            sp.set_option("sp_dv_grid", grid)
        got = sp.shortest_path(s, t, FOLLOW, 7).rows()
        fell_back = 3 - sp.last_timing()["spec_hops"]
        assert got == oracle_paths(st, s, t, FOLLOW, 7)
        again = sp.shortest_path(t, s, FOLLOW, 7).rows()
        assert again == oracle_paths(st, t, s, FOLLOW, 7)
        if cap == 64:
            assert fell_back == 3
        sp.unset_option("sp_dv_list")
        sp.unset_option("sp_dv_grid")
        clean = sp.shortest_path(s, t, FOLLOW, 7).rows()  # device-driven again, clean state
        assert sp.last_timing()["spec_hops"] == 3
        assert clean == got
    finally:
        sp.close()
