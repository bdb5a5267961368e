"""The sharded path with 4 and 8 ranks (configs[2] / configs[3] name an 8-GPU partition) at
RMAT-18/20, on one GPU: N contexts of one process form an in-process rank group
(nbg_comm_init_local, device-to-device copies in place of RCCL), vertices owned by part % N
(pickHosts, CreateSpaceProcessor.cpp:77-90; StorageClient.cpp:238-243).  The union of the ranks'
results must equal the single-GPU results the committed digests pin (tests/golden/
rmat_digests.json, made by the oracle): the reference's graphd merges the per-host responses
(StorageClient.inl:74-159)."""
import hashlib

import numpy as np
import pytest

import oracle as O
from nebula_amd import expr as X
from nebula_amd import synth
from test_gpu_multirank import Group
from test_gpu_scale import GOLD, check_gold

pytestmark = pytest.mark.gpu

FOLLOW = 1
W499 = X.AliasProp("follow", "weight") > 499


def rmat_group(world, scale):
    g = Group(world)
    for s in g.sp:
        s.set_edge_schema(FOLLOW, [("weight", O.INT)])
    g.each(lambda r, s: s.gen_rmat(scale, 16, 1, FOLLOW))
    g.each(lambda r, s: s.finalize())
    return g


@pytest.fixture(scope="module", params=[4, 8])
def group18(request):
    g = rmat_group(request.param, 18)
    yield g
    g.close()


@pytest.mark.parametrize("force", [0, 1, -1])
def test_bench_query_rmat20_sharded(force):
    """configs[2]'s query at RMAT-20 on 4 and 8 ranks, every direction mode: the union of the
    ranks' DISTINCT _dst rows is the oracle's (digest), each vertex reported by its owner once"""
    for world in (4, 8):
        g = rmat_group(world, 20)
        try:
            g.each(lambda r, s: s.set_option("bu_force", force))
            res = g.go(synth.seeds(20, 16, 1, 64), 3, FOLLOW, where=W499, yields=[X.EdgeDst("follow")],
                       distinct=True)
            col = np.sort(np.concatenate([x.columns[0] for x in res]))
            assert len(np.unique(col)) == len(col)
            check_gold("go3_where499_distinct_s20", col, sum(x.edges_scanned for x in res))
            t = g.each(lambda r, s: s.last_timing())
            if force == 1:
                assert all(x["bu_steps"] > 0 for x in t)
            if force == -1:
                assert all(x["bu_steps"] == 0 for x in t)
            if force == 0:
                # the sharded query runs from its start frontier to the result behind device
                # gates fed by stream-ordered reductions: one counter fetch, then the result's
                # copy to the host (GoExecutor.cpp:334-399's per-step round trips are gone).  The
                # first query also gathers the snapshot's degree statistics once: the second
                res = g.go(synth.seeds(20, 16, 1, 64), 3, FOLLOW, where=W499, yields=[X.EdgeDst("follow")],
                           distinct=True)
                col = np.sort(np.concatenate([x.columns[0] for x in res]))
                check_gold("go3_where499_distinct_s20", col, sum(x.edges_scanned for x in res))
                t = g.each(lambda r, s: s.last_timing())
                assert all(x["host_waits"] <= 2 and x["spec_hops"] >= 2 for x in t), \
                    [(x["host_waits"], x["spec_hops"]) for x in t]
                # every rank ran the whole first hop over the out-CSR replica (go_rep1): the
                # second hop's frontier allgather is the query's one collective
                assert all(x["comm_calls"] == 1 for x in t), [x["comm_calls"] for x in t]
                # the owner-computed first hop: marks all-to-all + two frontier allgathers
                g.each(lambda r, s: s.set_option("go_rep1", 0))
                res = g.go(synth.seeds(20, 16, 1, 64), 3, FOLLOW, where=W499, yields=[X.EdgeDst("follow")],
                           distinct=True)
                col = np.sort(np.concatenate([x.columns[0] for x in res]))
                check_gold("go3_where499_distinct_s20", col, sum(x.edges_scanned for x in res))
                t = g.each(lambda r, s: s.last_timing())
                assert all(x["comm_calls"] == 3 for x in t), [x["comm_calls"] for x in t]
                # the gates' counts summed by all-reduces instead of riding on the frontier
                # exchanges (comm_piggy = 0): same rows
                g.each(lambda r, s: s.set_option("comm_piggy", 0))
                res = g.go(synth.seeds(20, 16, 1, 64), 3, FOLLOW, where=W499, yields=[X.EdgeDst("follow")],
                           distinct=True)
                col = np.sort(np.concatenate([x.columns[0] for x in res]))
                check_gold("go3_where499_distinct_s20", col, sum(x.edges_scanned for x in res))
        finally:
            g.close()


def test_plain_rows_rmat18_sharded(group18):
    """configs[1]'s shape (GO 3 STEPS, YIELD _dst rows) at RMAT-18: the rows of all ranks"""
    res = group18.go(synth.seeds(18, 16, 1, 64), 3, FOLLOW)
    col = np.sort(np.concatenate([x.columns[0] for x in res]))
    check_gold("go3_plain_s18", col, sum(x.edges_scanned for x in res))


def test_paths1024_rmat18_sharded(group18):
    """configs[3] (1024 pairs FIND SHORTEST PATH) at RMAT-18: pair i answered by rank i % N;
    re-ordered into pair order, hops and paths hash to the committed digest"""
    g = group18
    s, t = synth.pairs(18, 16, 1, 1024)
    res = g.each(lambda r, sp: sp.shortest_path(s, t, FOLLOW, 8))
    hops = np.zeros(len(s), dtype=np.int64)
    paths = [None] * len(s)
    for r, pr in enumerate(res):
        idx = np.arange(r, len(s), g.world)
        assert len(pr.hops) == len(idx)
        assert np.array_equal(pr.src, s[idx]) and np.array_equal(pr.dst, t[idx])
        hops[idx] = pr.hops
        for k, i in enumerate(idx):
            paths[i] = pr.paths[k]
    h = hashlib.sha256(np.asarray(hops, dtype="<i8").tobytes())
    for p in paths:
        h.update(np.asarray(p, dtype="<i8").tobytes())
    assert h.hexdigest() == GOLD["paths1024_s18"]["sha256"]
