"""GO N STEPS on the RMAT graph restated independently of both oracles (CPU).

The index-space oracle (oracle/rmat_graph.cpp) is the checker of the RMAT-18..26 GPU tests; it is
pinned to the KV-store oracle (a restatement of QueryBaseProcessor / GoExecutor over the
reference's key and row bytes) at RMAT-10..16 by test_oracle_rmat_graph.py.  This test adds a
third, independent restatement from the raw RMAT edge list with numpy set operations: a
frontier is the set of dsts of the previous frontier's out-edges (identical keys collapse: one
edge per (src, dst) at rank 0, whose weight is a function of the pair; hop 1 scans the starts
with their multiplicity unless DISTINCT), the final step keeps the edges whose weight passes the
WHERE and yields their dsts (DISTINCT: as a set; plain: one row per edge).  Reference semantics: GoExecutor.cpp:334-431 (step loop, next frontier = dst set),
585-782 (final WHERE / YIELD / DISTINCT).
"""
import numpy as np
import pytest

import oracle as O
from nebula_amd import synth

SEED = 1


def go_numpy(scale, starts, steps, where_gt=None, distinct=False):
    s, d, w = O.rmat_edges(scale, 16, SEED)
    key = np.unique(np.stack([s, d, w], axis=1), axis=0)  # identical (src, dst) keys collapse
    s, d, w = key[:, 0], key[:, 1], key[:, 2]
    order = np.argsort(s, kind="stable")
    s, d, w = s[order], d[order], w[order]
    # hop 1 scans the starts as given, deduplicated only under DISTINCT (GoExecutor
    # sends the FROM list as is; DISTINCT makes the multiplicity invisible)
    front = np.asarray(starts, np.int64)
    if distinct:
        front = np.unique(front)
    scanned = 0
    for k in range(steps):
        lo, hi = np.searchsorted(s, front, "left"), np.searchsorted(s, front, "right")
        sel = np.concatenate([np.arange(a, b) for a, b in zip(lo, hi)]) if len(front) else np.zeros(0, np.int64)
        sel = sel.astype(np.int64)
        scanned += len(sel)
        if k < steps - 1:
            front = np.unique(d[sel])
        else:
            if where_gt is not None:
                sel = sel[w[sel] > where_gt]
            rows = d[sel]
            return (np.unique(rows) if distinct else np.sort(rows)), scanned
    return np.zeros(0, np.int64), scanned


@pytest.mark.parametrize("scale,steps,where_gt,distinct", [
    (10, 3, 499, True), (12, 3, 499, True), (14, 3, 499, True),
    (12, 2, None, False), (13, 3, None, True), (11, 1, 250, False)])
def test_index_oracle_go_matches_numpy(scale, steps, where_gt, distinct):
    g = O.RmatGraph(scale, 16, SEED)
    starts = synth.seeds(scale, 16, SEED, 64)
    got, scanned = g.go(starts, steps, where_gt=where_gt, distinct=distinct)
    want, want_scanned = go_numpy(scale, starts, steps, where_gt, distinct)
    assert np.array_equal(np.sort(got), want)
    assert len(want) > 0
    # edges scanned: the frontiers' out-degrees summed over the hops (SURVEY 8d's TEPS numerator)
    assert scanned == want_scanned, (scanned, want_scanned)
