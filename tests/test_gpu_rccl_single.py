"""The RCCL transport on one GPU: a one-rank RCCL communicator (option comm_single before
nbg_comm_init) makes the context run the sharded algorithm -- owner slices, the hop-1 mark
all-to-all, the frontier allgathers carrying the gate counters, the device all-reduces, the
DISTINCT row shuffle and the shortest-path replica allgathers -- with every exchange issued to
RCCL, the rank's own slice sent to itself with ncclSend / ncclRecv.  Every multi-rank GPU test
uses the in-process LocalComm transport (two RCCL ranks on one device are refused by
ncclCommInitRank), so this is where the RCCL calls themselves execute behind the device gates.

The reference exchange replaced: StorageClient::collectResponse's per-host scatter / gather
(src/storage/client/StorageClient.inl:74-159).  Results must equal the committed digests of the
one-GPU path (tests/golden/rmat_digests.json, made by the oracle)."""
import hashlib

import numpy as np
import pytest

import oracle as O
from nebula_amd import GraphSpace, NbgError
from nebula_amd import expr as X
from nebula_amd import synth
from test_gpu_scale import GOLD, check_gold

pytestmark = pytest.mark.gpu

FOLLOW = 1
W499 = X.AliasProp("follow", "weight") > 499


def single_rank_space(scale, **opts):
    sp = GraphSpace(64)
    for k, v in opts.items():
        sp.set_option(k, v)
    sp.set_option("comm_single", 1)
    sp.comm_init(GraphSpace.comm_unique_id())
    assert sp.comm_info() == {"ranks": 1, "transport": "rccl"}
    sp.set_edge_schema(FOLLOW, [("weight", O.INT)])
    sp.gen_rmat(scale, 16, 1, FOLLOW)
    sp.finalize()
    return sp


def paths_digest(r):
    h = hashlib.sha256(np.asarray(r.hops, dtype="<i8").tobytes())
    for p in r.paths:
        h.update(np.asarray(p, dtype="<i8").tobytes())
    return h.hexdigest()


@pytest.fixture(scope="module")
def rccl20():
    sp = single_rank_space(20)
    yield sp
    sp.close()


@pytest.mark.parametrize("force,piggy,rep1", [(0, 1, 1), (0, 1, 0), (0, 0, 0), (1, 1, 1), (-1, 1, 1)])
def test_c3_query_rmat20_through_rccl(rccl20, force, piggy, rep1):
    """configs[2]'s query at RMAT-20 through the one-rank RCCL communicator, every direction
    mode; the first hop over the out-CSR replica (go_rep1, one collective a query) or computed by
    the owners (marks all-to-all), with the gate counters riding on the frontier allgathers or
    summed by all-reduces"""
    sp = rccl20
    sp.set_option("bu_force", force)
    sp.set_option("comm_piggy", piggy)
    sp.set_option("go_rep1", rep1)
    try:
        for _ in range(2):  # the first query also gathers the snapshot's degree statistics
            r = sp.go(synth.seeds(20, 16, 1, 64), 3, FOLLOW, where=W499, yields=[X.EdgeDst("follow")],
                      distinct=True)
            check_gold("go3_where499_distinct_s20", np.sort(r.columns[0]), r.edges_scanned)
        t = sp.last_timing()
        assert t["comm_calls"] > 0, t
        if force == 0:
            assert t["host_waits"] <= 2 and t["spec_hops"] >= 2, (t["host_waits"], t["spec_hops"])
            if piggy:
                assert t["comm_calls"] == (1 if rep1 else 3), t["comm_calls"]
        print(f"force {force} piggy {piggy}: {t['comm_calls']} collectives, {t['comm_ms']:.3f} ms "
              f"({t['comm_ms'] / t['comm_calls'] * 1e3:.1f} us each), device {t['total_ms']:.3f} ms")
    finally:
        sp.unset_option("bu_force")
        sp.unset_option("comm_piggy")
        sp.unset_option("go_rep1")


def test_plain_rows_and_row_shuffle_rmat20(rccl20):
    """top-down hops (mark all-to-all each hop) with plain rows, and DISTINCT over two columns
    (rows shuffled to rank hash(row) % world through RCCL) against a context without a
    communicator"""
    sp = rccl20
    starts = synth.seeds(20, 16, 1, 16)
    ref = GraphSpace(64)
    try:
        ref.set_edge_schema(FOLLOW, [("weight", O.INT)])
        ref.gen_rmat(20, 16, 1, FOLLOW)
        ref.finalize()
        sp.set_option("bu_force", -1)
        a = sp.go(starts, 2, FOLLOW)
        b = ref.go(starts, 2, FOLLOW)
        assert np.array_equal(np.sort(a.columns[0]), np.sort(b.columns[0]))
        assert a.edges_scanned == b.edges_scanned
        assert sp.last_timing()["comm_calls"] > 0
        sp.unset_option("bu_force")
        ys = [X.EdgeSrc("follow"), X.AliasProp("follow", "weight")]
        a = sp.go(starts, 2, FOLLOW, where=W499, yields=ys, distinct=True)
        b = ref.go(starts, 2, FOLLOW, where=W499, yields=ys, distinct=True)
        ka = sorted(zip(a.columns[0].tolist(), a.columns[1].tolist()))
        kb = sorted(zip(b.columns[0].tolist(), b.columns[1].tolist()))
        assert ka == kb and len(ka) == len(set(ka))
    finally:
        sp.unset_option("bu_force")
        ref.close()


def test_c4_paths_rmat18_through_rccl():
    """configs[3]'s shape (1024 pairs) on RMAT-18: the replicated CSRs are assembled by RCCL
    allgathers; device-driven and host-driven batches against the committed digest"""
    sp = single_rank_space(18)
    try:
        s, t = synth.pairs(18, 16, 1, 1024)
        for dev in (1, 0):
            sp.set_option("sp_dev", dev)
            r = sp.shortest_path(s, t, FOLLOW, 8)
            assert paths_digest(r) == GOLD["paths1024_s18"]["sha256"], dev
        sp.unset_option("sp_dev")
        # GO on the same communicator after the replicas exist
        r = sp.go(synth.seeds(18, 16, 1, 64), 3, FOLLOW, where=W499, yields=[X.EdgeDst("follow")], distinct=True)
        check_gold("go3_where499_distinct_s18", np.sort(r.columns[0]), r.edges_scanned)
    finally:
        sp.close()


def test_comm_single_after_build_is_refused():
    """the sharded layout is chosen at build time: a one-rank communicator formed after the
    snapshot exists is refused (NBG_E_STATE), and the context keeps working unsharded"""
    sp = GraphSpace(64)
    try:
        sp.set_edge_schema(FOLLOW, [("weight", O.INT)])
        sp.gen_rmat(10, 16, 1, FOLLOW)
        sp.finalize()
        sp.set_option("comm_single", 1)
        with pytest.raises(NbgError):
            sp.comm_init(GraphSpace.comm_unique_id())
        assert sp.comm_info()["transport"] == "none"
        r = sp.go(synth.seeds(10, 16, 1, 16), 2, FOLLOW)
        assert r.n_rows > 0
    finally:
        sp.close()


def test_rmat26_c3_and_c4_through_rccl():
    """configs[2] and configs[3] at their size through the one-rank RCCL communicator: the
    replica allgathers move the 4.2 GB RMAT-26 column array through ncclSend / ncclRecv (in
    pieces of comm_chunk_mb), and both digests must hold"""
    sp = single_rank_space(26)
    try:
        r = sp.go(synth.seeds(26, 16, 1, 64), 3, FOLLOW, where=W499, yields=[X.EdgeDst("follow")], distinct=True)
        check_gold("go3_where499_distinct_s26", np.sort(r.columns[0]), r.edges_scanned)
        r = None
        s, t = synth.pairs(26, 16, 1, 1024)
        p = sp.shortest_path(s, t, FOLLOW, 8)
        assert paths_digest(p) == GOLD["paths1024_s26"]["sha256"]
    finally:
        sp.close()
