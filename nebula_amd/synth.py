"""Synthetic RMAT definition (host side, numpy) -- used to pick query seeds and for docs.

The device generator (nebula_amd/csrc/snapshot.hip, k_gen_rmat) and the oracle
(oracle/refcpu.cpp, rmatEdge) implement the same arithmetic; tests check all three agree.

sample i of E = edge_factor << scale:
    for level pairs l = 0, 2, 4, ...:  h = splitmix64(seed ^ H1*(i+1) ^ H2*(l+1))
        the high / low 32-bit halves pick the quadrant for levels l / l+1 against
        (A, A+B, A+B+C) * 2^32 with Graph500 (A, B, C, D) = (0.57, 0.19, 0.19, 0.05)
    vid(idx) = bijective 63-bit mix of idx; weight(src, dst) = splitmix64(src ^ rotl(dst, 32) ^ seed) % 1000
"""
from __future__ import annotations

import numpy as np

M64 = (1 << 64) - 1
M63 = (1 << 63) - 1
TA, TAB, TABC = 2448131358, 3264175144, 4080218931
H1, H2 = 0xD6E8FEB86659FD93, 0xA0761D6478BD642F


def _u(x):
    return np.asarray(x, dtype=np.uint64)


def splitmix64(x):
    with np.errstate(over="ignore"):
        x = _u(x) + np.uint64(0x9E3779B97F4A7C15)
        x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return x ^ (x >> np.uint64(31))


def vid(idx, seed: int):
    with np.errstate(over="ignore"):
        m = np.uint64(M63)
        smix = splitmix64(np.uint64(seed)) & m
        x = (_u(idx) + smix) & m
        x ^= x >> np.uint64(29)
        x = (x * np.uint64(0xBF58476D1CE4E5B9)) & m
        x ^= x >> np.uint64(32)
        x = (x * np.uint64(0x94D049BB133111EB)) & m
        x ^= x >> np.uint64(29)
        return x.astype(np.int64)


def edges(scale: int, seed: int, idx):
    """(src_vid, dst_vid) of RMAT samples `idx` (any subset of [0, ef << scale))."""
    i = _u(idx)
    u = np.zeros_like(i)
    v = np.zeros_like(i)
    with np.errstate(over="ignore"):
        for lvl in range(0, scale, 2):
            h = splitmix64(np.uint64(seed) ^ (np.uint64(H1) * (i + np.uint64(1))) ^ np.uint64((H2 * (lvl + 1)) & M64))
            for half, active in ((h >> np.uint64(32), True), (h & np.uint64(0xFFFFFFFF), lvl + 1 < scale)):
                if not active:
                    continue
                r = half
                bu = (r >= np.uint64(TAB)).astype(np.uint64)
                bv = (((r >= np.uint64(TA)) & (r < np.uint64(TAB))) | (r >= np.uint64(TABC))).astype(np.uint64)
                u = (u << np.uint64(1)) | bu
                v = (v << np.uint64(1)) | bv
    return vid(u, seed), vid(v, seed)


def seeds(scale: int, edge_factor: int, graph_seed: int, n: int, pick_seed: int = 7):
    """n query seeds: sources of uniformly drawn edge samples (so out-degree >= 1)."""
    rng = np.random.default_rng(pick_seed)
    idx = rng.integers(0, edge_factor << scale, n, dtype=np.uint64)
    s, _ = edges(scale, graph_seed, idx)
    return s


def pairs(scale: int, edge_factor: int, graph_seed: int, n: int, pick_seed: int = 11):
    rng = np.random.default_rng(pick_seed)
    a = rng.integers(0, edge_factor << scale, n, dtype=np.uint64)
    b = rng.integers(0, edge_factor << scale, n, dtype=np.uint64)
    return edges(scale, graph_seed, a)[0], edges(scale, graph_seed, b)[1]


def hub_candidates(scale: int, graph_seed: int):
    """vids of the RMAT indices with at most one 1-bit (0 and 2^k): the expected out-degree of
    index u is E * 0.76^(zero bits) * 0.24^(one bits), so the highest-degree vertices are, with
    overwhelming probability, among these scale + 1 candidates.  C5's "top-8 degree" seeds are
    the 8 of them with the largest out-degree in the built snapshot."""
    idx = np.array([0] + [1 << k for k in range(scale)], dtype=np.uint64)
    return vid(idx, graph_seed)
