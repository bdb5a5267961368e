"""Capacity options shrunk until the engine takes its overflow / fallback paths, each once, against
the oracle (the round-5 overrun of a hand-sized workspace showed only at 8
in-process ranks).  Every hand-sized workspace is carved through a checked Carve (engine.h), so a
layout that outgrew its block fails the call instead of writing a neighbour's memory; these
tests drive the paths whose sizes depend on the options:

* sp_mem_mb: the distance-byte budget sets the batch size (many small batches);
* sp_dv_list: the device-driven batch's list capacity (overflow -> clean state, host-driven rerun);
* sp_list_soft: the host-driven lists' soft capacity (they grow between launches);
* sp_dv_grid: scan grids far past the resident grid (late blocks see an overflow flag);
* query_pool_gb / host_pool_gb = 0: no block cache (every temporary and result freshly allocated).

A second call after each shrunk one checks that the state left behind is clean."""
import numpy as np
import pytest

import oracle as O
from nebula_amd import GraphSpace, synth
from nebula_amd import expr as X
from test_gpu_paths import edge_case_pairs, oracle_paths

pytestmark = pytest.mark.gpu

FOLLOW = 1
SCALE = 12


@pytest.fixture(scope="module")
def space():
    sp = GraphSpace(64)
    sp.set_edge_schema(FOLLOW, [("weight", 2)])
    sp.gen_rmat(SCALE, 16, 1, FOLLOW)
    sp.finalize()
    st = O.Store(64)
    st.set_edge_schema(FOLLOW, [("weight", O.INT)], name="follow")
    st.load_rmat(SCALE, 16, 1, FOLLOW)
    yield sp, st
    sp.close()


CASES = [
    {"sp_mem_mb": 1},
    {"sp_dv_list": 64},
    {"sp_dv_list": 500, "sp_dv_grid": 8192},
    {"sp_dev": 0, "sp_list_soft": 1},
    {"query_pool_gb": 0, "host_pool_gb": 0},
    {"sp_mem_mb": 1, "sp_dv_list": 200, "query_pool_gb": 0},
]


@pytest.mark.parametrize("opts", CASES, ids=lambda o: ",".join(f"{k}={v}" for k, v in o.items()))
def test_shortest_path_capacities(space, opts):
    sp, st = space
    s, t = synth.pairs(SCALE, 16, 1, 300, pick_seed=19)
    es, et_ = edge_case_pairs(SCALE)
    src, dst = np.concatenate([s, es]), np.concatenate([t, et_])
    want = oracle_paths(st, src, dst, FOLLOW, 6)
    try:
        for k, v in opts.items():
            sp.set_option(k, v)
        assert sp.shortest_path(src, dst, FOLLOW, 6).rows() == want
        assert sp.shortest_path(dst, src, FOLLOW, 6).rows() == oracle_paths(st, dst, src, FOLLOW, 6)
    finally:
        for k in opts:
            sp.unset_option(k)
    # defaults again: device-driven batches on the state the shrunk calls left
    assert sp.shortest_path(src, dst, FOLLOW, 6).rows() == want
    assert sp.last_timing()["spec_hops"] >= 1


@pytest.mark.parametrize("opts", [{"query_pool_gb": 0, "host_pool_gb": 0}, {"host_pool_gb": 0},
                                  {"sum_shards": 1}, {"compact_grid": 7}])
def test_go_capacities(space, opts):
    """GO without the block caches, with dense block sums, and with a 7-block compaction grid"""
    sp, st = space
    starts = synth.seeds(SCALE, 16, 1, 32)
    w = X.AliasProp("follow", "weight") > 499
    want = np.sort(st.go(starts, 3, FOLLOW, where=w.encode(), yields=[X.EdgeDst("follow").encode()],
                         distinct=True).int_col(0))
    want2 = np.sort(st.go(starts, 2, FOLLOW).int_col(0))
    try:
        for k, v in opts.items():
            sp.set_option(k, v)
        for _ in range(2):
            g = sp.go(starts, 3, FOLLOW, where=w, yields=[X.EdgeDst("follow")], distinct=True)
            assert np.array_equal(np.sort(g.columns[0]), want)
            assert np.array_equal(np.sort(sp.go(starts, 2, FOLLOW).columns[0]), want2)
    finally:
        for k in opts:
            sp.unset_option(k)
