"""bench.py's parity digests (CPU): the sorted SHA-256 and the order-free msum it prints for the
timed query must be the ones tests/golden/make_rmat_digests.py commits (oracle.digest /
oracle.msum / ora_rmat_graph_go_msum)."""
import sys
from pathlib import Path

import numpy as np

import oracle as O
from nebula_amd import synth

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import bench  # noqa: E402


def test_bench_digests_match_oracle():
    g = O.RmatGraph(14, 16, 1, threads=4)
    starts = synth.seeds(14, 16, 1, 16)
    rows, _ = g.go(starts, 2)
    shuffled = np.random.default_rng(0).permutation(rows)
    assert bench.O_digest(shuffled) == O.digest(rows)
    assert bench.msum(shuffled, chunk=1000) == O.msum(rows)
    assert bench.msum(shuffled) == g.go_msum(starts, 2)[0]
