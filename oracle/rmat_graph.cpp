// oracle/rmat_graph.cpp -- TEST INFRASTRUCTURE ONLY (see refcpu.h).
//
// Second restatement of the GO / FIND SHORTEST PATH semantics, for parity at the configured
// sizes (RMAT-20..26) where the KV-store restatement in refcpu.cpp does not fit in host memory
// or time.  It works on the synthetic RMAT graph directly, in RMAT index space:
//
//   * the graph is the set of distinct (u, v) samples of rmat_def.h (the KV store's view after
//     the multi-edge collapse P4: duplicate samples write the identical key, last write wins,
//     and the weight depends only on (src, dst), so every duplicate carries the same row);
//   * GO N STEPS (GoExecutor.cpp:334-431, 669-782): hop 1 scans the start list as given
//     (duplicates rescan, GoExecutor.cpp:98-104 dedups only under DISTINCT), every later hop
//     scans the SET of dsts of the previous hop (getDstIdsFromResp, GoExecutor.cpp:407-431);
//     the final hop emits one row per (frontier vertex, edge) passing WHERE (P13); DISTINCT over
//     the single _dst column is the set of such dsts (P16);
//   * edges_scanned = rows the storage returned over all hops (what ora_go counts);
//   * FIND SHORTEST PATH (definition owned by the build): backward BFS to dst
//     over the in-edges until src is labelled, then the greedy smallest-vid walk, exactly as
//     ora_shortest_path in refcpu.cpp.
//
// tests/test_oracle_rmat_graph.py checks it against refcpu.cpp's faithful restatement at
// RMAT-12/14 (same rows, same edges_scanned, same paths); at the configured sizes it produces
// the committed digests (tests/golden/make_rmat_digests.py).
#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <thread>
#include <unordered_map>
#include <vector>

#include "refcpu.h"
#include "rmat_def.h"

using namespace refcpu;

struct ora_rmat_graph {
  int32_t scale = 0;
  uint64_t seed = 0;
  int64_t n = 0;                      // 2^scale index space
  std::vector<uint64_t> row_ptr;      // out CSR over idx
  std::vector<uint32_t> col;          // dst idx, ascending within a row
  std::vector<uint64_t> rrow_ptr;     // in CSR (built on the first shortest-path call)
  std::vector<uint32_t> rcol;
  std::vector<uint8_t> present;       // idx appears in some sample (is a vertex)
};

namespace {

template <typename F>
void parallel_for(int64_t n, int threads, F f) {
  if (threads <= 1 || n < 2) {
    f(0, n, 0);
    return;
  }
  std::vector<std::thread> ts;
  for (int t = 0; t < threads; t++) {
    const int64_t lo = n * t / threads, hi = n * (t + 1) / threads;
    ts.emplace_back([=, &f] { f(lo, hi, t); });
  }
  for (auto& t : ts) t.join();
}

// distinct (key >> shift, key & mask) pairs -> CSR over the high part; keys bucketed by the top
// bits of the high part, each bucket sorted and deduplicated by its own thread
void build_csr(int32_t scale, uint64_t E, int threads, bool reverse, uint64_t seed,
               std::vector<uint64_t>& row_ptr, std::vector<uint32_t>& col) {
  const int B = scale < 12 ? scale : 12;  // 4096 buckets of the row index
  const int64_t NB = int64_t(1) << B;
  const int shift_b = scale - B;
  const uint64_t lowmask = (uint64_t(1) << scale) - 1;
  auto key_of = [&](uint64_t i) {
    uint64_t u, v;
    rmatEdge(seed, scale, i, u, v);
    return reverse ? (v << scale) | u : (u << scale) | v;
  };
  std::vector<uint64_t> hist(size_t(threads) * size_t(NB), 0);
  parallel_for(int64_t(E), threads, [&](int64_t lo, int64_t hi, int t) {
    uint64_t* h = hist.data() + size_t(t) * size_t(NB);
    for (int64_t i = lo; i < hi; i++) h[key_of(uint64_t(i)) >> scale >> shift_b]++;
  });
  std::vector<uint64_t> boff(size_t(NB) + 1, 0), toff(size_t(threads) * size_t(NB));
  {
    uint64_t run = 0;
    for (int64_t b = 0; b < NB; b++) {
      boff[size_t(b)] = run;
      for (int t = 0; t < threads; t++) {
        toff[size_t(t) * size_t(NB) + size_t(b)] = run;
        run += hist[size_t(t) * size_t(NB) + size_t(b)];
      }
    }
    boff[size_t(NB)] = run;
  }
  // buckets are processed in groups of at most max_group_keys samples (one generator pass per
  // group), so the key buffer stays far below the 8 B x E of a single pass at RMAT-28
  uint64_t max_group_keys = uint64_t(1) << 30;
  if (const char* e = getenv("ORA_RMAT_GROUP_KEYS")) max_group_keys = std::max<uint64_t>(strtoull(e, nullptr, 10), 1);
  const int64_t n = int64_t(1) << scale;
  row_ptr.assign(size_t(n) + 1, 0);
  col.resize(E);  // upper bound; trimmed to the unique count at the end (capacity stays)
  std::vector<uint64_t> keys;
  std::vector<uint64_t> uniq(size_t(NB), 0);
  uint64_t pos_all = 0;
  for (int64_t g0 = 0; g0 < NB;) {
    int64_t g1 = g0 + 1;
    while (g1 < NB && boff[size_t(g1) + 1] - boff[size_t(g0)] <= max_group_keys) g1++;
    const uint64_t gbase = boff[size_t(g0)], gsize = boff[size_t(g1)] - gbase;
    keys.resize(gsize);
    parallel_for(int64_t(E), threads, [&](int64_t lo, int64_t hi, int t) {
      std::vector<uint64_t> o(size_t(g1 - g0));
      for (int64_t b = g0; b < g1; b++) o[size_t(b - g0)] = toff[size_t(t) * size_t(NB) + size_t(b)] - gbase;
      for (int64_t i = lo; i < hi; i++) {
        const uint64_t k = key_of(uint64_t(i));
        const int64_t b = int64_t(k >> scale >> shift_b);
        if (b >= g0 && b < g1) keys[o[size_t(b - g0)]++] = k;
      }
    });
    std::atomic<int64_t> next{g0};
    parallel_for(threads, threads, [&](int64_t, int64_t, int) {
      for (int64_t b; (b = next++) < g1;) {
        uint64_t* a = keys.data() + (boff[size_t(b)] - gbase);
        uint64_t* e = keys.data() + (boff[size_t(b) + 1] - gbase);
        std::sort(a, e);
        uniq[size_t(b)] = uint64_t(std::unique(a, e) - a);
      }
    });
    std::vector<uint64_t> uoff(size_t(g1 - g0) + 1, pos_all);
    for (int64_t b = g0; b < g1; b++) uoff[size_t(b - g0) + 1] = uoff[size_t(b - g0)] + uniq[size_t(b)];
    next = g0;
    parallel_for(threads, threads, [&](int64_t, int64_t, int) {
      for (int64_t b; (b = next++) < g1;) {
        const uint64_t* a = keys.data() + (boff[size_t(b)] - gbase);
        uint64_t pos = uoff[size_t(b - g0)];
        const int64_t r0 = b << shift_b, r1 = (b + 1) << shift_b;
        uint64_t j = 0;
        for (int64_t r = r0; r < r1; r++) {
          row_ptr[size_t(r)] = pos;
          while (j < uniq[size_t(b)] && (a[j] >> scale) == uint64_t(r)) col[pos++] = uint32_t(a[j++] & lowmask);
        }
      }
    });
    pos_all = uoff[size_t(g1 - g0)];
    g0 = g1;
  }
  std::vector<uint64_t>().swap(keys);
  col.resize(pos_all);
  std::vector<uint64_t> uoff(size_t(NB) + 1, 0);
  uoff[size_t(NB)] = pos_all;
  row_ptr[size_t(n)] = uoff[size_t(NB)];
}

}  // namespace

extern "C" {

ora_rmat_graph* ora_rmat_graph_new(int32_t scale, int32_t ef, uint64_t seed, int32_t threads) {
  if (scale < 1 || scale > 30 || ef < 1) return nullptr;
  auto* g = new ora_rmat_graph();
  g->scale = scale;
  g->seed = seed;
  g->n = int64_t(1) << scale;
  if (threads < 1) threads = 1;
  const uint64_t E = uint64_t(ef) << scale;
  build_csr(scale, E, threads, false, seed, g->row_ptr, g->col);
  // a vertex = an idx that is the src or dst of some sample (the snapshot's vertex set)
  g->present.assign(size_t(g->n), 0);
  parallel_for(g->n, threads, [&](int64_t lo, int64_t hi, int) {
    for (int64_t u = lo; u < hi; u++) {
      if (g->row_ptr[size_t(u) + 1] > g->row_ptr[size_t(u)])
        __atomic_store_n(&g->present[size_t(u)], uint8_t(1), __ATOMIC_RELAXED);
      for (uint64_t e = g->row_ptr[size_t(u)]; e < g->row_ptr[size_t(u) + 1]; e++)
        __atomic_store_n(&g->present[g->col[e]], uint8_t(1), __ATOMIC_RELAXED);
    }
  });
  return g;
}

void ora_rmat_graph_free(ora_rmat_graph* g) { delete g; }

void ora_rmat_graph_info(const ora_rmat_graph* g, int64_t* n_vertices, int64_t* n_edges) {
  int64_t nv = 0;
  for (uint8_t p : g->present) nv += p;
  *n_vertices = nv;
  *n_edges = int64_t(g->col.size());
}

int64_t ora_rmat_graph_out_degree(const ora_rmat_graph* g, int64_t idx) {
  if (idx < 0 || idx >= g->n) return -1;
  return int64_t(g->row_ptr[size_t(idx) + 1] - g->row_ptr[size_t(idx)]);
}

void ora_free(void* p) { free(p); }

// vid -> idx for a few vids: one pass over the index space (rmatVid is a bijection on 63 bits)
static std::vector<int64_t> idx_of(const ora_rmat_graph* g, const int64_t* vids, size_t n, int threads) {
  std::unordered_map<int64_t, std::vector<size_t>> want;
  for (size_t i = 0; i < n; i++) want[vids[i]].push_back(i);
  std::vector<int64_t> out(n, -1);
  std::mutex mu;
  parallel_for(g->n, threads, [&](int64_t lo, int64_t hi, int) {
    for (int64_t u = lo; u < hi; u++) {
      auto it = want.find(rmatVid(uint64_t(u), g->seed));
      if (it == want.end()) continue;
      std::lock_guard<std::mutex> lk(mu);
      for (size_t i : it->second) out[i] = g->present[size_t(u)] ? u : -1;
    }
  });
  return out;
}

}  // extern "C"

// the final hop's frontier (index space) of GO steps FROM starts, and the rows scanned over all hops
static std::vector<int64_t> go_frontier(const ora_rmat_graph* g, const int64_t* starts, size_t n_starts, int32_t steps,
                                        int32_t distinct, int32_t threads, uint64_t& scanned_out,
                                        std::vector<uint8_t>& mark) {
  std::vector<int64_t> idx = idx_of(g, starts, n_starts, threads);
  // hop-1 scan list: the starts as given, deduplicated only under DISTINCT (P14)
  std::vector<int64_t> F;
  if (distinct) {
    std::vector<uint8_t> seen(size_t(g->n), 0);
    for (int64_t u : idx)
      if (u >= 0 && !seen[size_t(u)]) {
        seen[size_t(u)] = 1;
        F.push_back(u);
      }
  } else {
    for (int64_t u : idx)
      if (u >= 0) F.push_back(u);
  }
  mark.assign(size_t(g->n), 0);
  uint64_t scanned = 0;
  for (int32_t step = 1; step <= steps && !F.empty(); step++) {
    for (int64_t u : F) scanned += g->row_ptr[size_t(u) + 1] - g->row_ptr[size_t(u)];
    if (step == steps) break;
    std::fill(mark.begin(), mark.end(), uint8_t(0));
    parallel_for(int64_t(F.size()), threads, [&](int64_t lo, int64_t hi, int) {
      for (int64_t i = lo; i < hi; i++) {
        const int64_t u = F[size_t(i)];
        for (uint64_t e = g->row_ptr[size_t(u)]; e < g->row_ptr[size_t(u) + 1]; e++)
          __atomic_store_n(&mark[g->col[e]], uint8_t(1), __ATOMIC_RELAXED);
      }
    });
    F.clear();
    for (int64_t v = 0; v < g->n; v++)
      if (mark[size_t(v)]) F.push_back(v);
  }
  scanned_out = scanned;
  return F;
}

extern "C" {

// GO steps FROM starts OVER the RMAT edge type [WHERE weight <op> k] YIELD _dst [DISTINCT].
// has_where: 0 no WHERE, else the relational operator of RelationalExpression (Expressions.cpp:
// 891-933, INT operands): 1 >, 2 >=, 3 <, 4 <=, 5 ==, 6 !=.
// Writes the result vids sorted ascending into *out (malloc'd, ora_free) and returns their count.
int64_t ora_rmat_graph_go(const ora_rmat_graph* g, const int64_t* starts, size_t n_starts, int32_t steps,
                          int32_t has_where, int64_t where_k, int32_t distinct, int32_t threads,
                          int64_t** out, uint64_t* edges_scanned) {
  if (threads < 1) threads = 1;
  *out = nullptr;
  *edges_scanned = 0;
  std::vector<uint8_t> mark;
  uint64_t scanned = 0;
  std::vector<int64_t> F = go_frontier(g, starts, n_starts, steps, distinct, threads, scanned, mark);
  *edges_scanned = scanned;
  if (F.empty()) return 0;
  // final hop: rows (u, v) passing WHERE; YIELD _dst
  auto pass = [&](int64_t su, int64_t dv) {
    if (!has_where) return true;
    const int64_t w = rmatWeight(su, dv, g->seed);
    switch (has_where) {
      case 1: return w > where_k;
      case 2: return w >= where_k;
      case 3: return w < where_k;
      case 4: return w <= where_k;
      case 5: return w == where_k;
      default: return w != where_k;
    }
  };
  std::vector<int64_t> res;
  if (distinct) {
    std::fill(mark.begin(), mark.end(), uint8_t(0));
    parallel_for(int64_t(F.size()), threads, [&](int64_t lo, int64_t hi, int) {
      for (int64_t i = lo; i < hi; i++) {
        const int64_t u = F[size_t(i)];
        const int64_t su = rmatVid(uint64_t(u), g->seed);
        for (uint64_t e = g->row_ptr[size_t(u)]; e < g->row_ptr[size_t(u) + 1]; e++) {
          const uint32_t v = g->col[e];
          if (!mark[v] && pass(su, rmatVid(v, g->seed))) __atomic_store_n(&mark[v], uint8_t(1), __ATOMIC_RELAXED);
        }
      }
    });
    for (int64_t v = 0; v < g->n; v++)
      if (mark[size_t(v)]) res.push_back(rmatVid(uint64_t(v), g->seed));
  } else {
    std::vector<std::vector<int64_t>> part(static_cast<size_t>(threads));
    parallel_for(int64_t(F.size()), threads, [&](int64_t lo, int64_t hi, int t) {
      auto& r = part[size_t(t)];
      for (int64_t i = lo; i < hi; i++) {
        const int64_t u = F[size_t(i)];
        const int64_t su = rmatVid(uint64_t(u), g->seed);
        for (uint64_t e = g->row_ptr[size_t(u)]; e < g->row_ptr[size_t(u) + 1]; e++) {
          const int64_t dv = rmatVid(g->col[e], g->seed);
          if (pass(su, dv)) r.push_back(dv);
        }
      }
    });
    size_t tot = 0;
    for (auto& p : part) tot += p.size();
    res.reserve(tot);
    for (auto& p : part) {
      res.insert(res.end(), p.begin(), p.end());
      std::vector<int64_t>().swap(p);
    }
  }
  std::sort(res.begin(), res.end());
  *out = static_cast<int64_t*>(malloc(sizeof(int64_t) * (res.size() ? res.size() : 1)));
  if (!res.empty()) memcpy(*out, res.data(), sizeof(int64_t) * res.size());
  return int64_t(res.size());
}

// Order-independent digest of a plain GO's final rows (YIELD _dst, no WHERE / DISTINCT), for
// result sets too large to sort (configs[4]: billions of rows): out[0] = rows, out[1] = sum of
// splitmix64(dst vid) mod 2^64, out[2] = xor of the same; *edges_scanned as ora_rmat_graph_go.
void ora_rmat_graph_go_msum(const ora_rmat_graph* g, const int64_t* starts, size_t n_starts, int32_t steps,
                            int32_t threads, uint64_t* out, uint64_t* edges_scanned) {
  if (threads < 1) threads = 1;
  std::vector<uint8_t> mark;
  uint64_t scanned = 0;
  std::vector<int64_t> F = go_frontier(g, starts, n_starts, steps, 0, threads, scanned, mark);
  *edges_scanned = scanned;
  std::vector<uint64_t> cnt(size_t(threads), 0), sum(size_t(threads), 0), x(size_t(threads), 0);
  parallel_for(int64_t(F.size()), threads, [&](int64_t lo, int64_t hi, int t) {
    uint64_t c = 0, sm = 0, xr = 0;
    for (int64_t i = lo; i < hi; i++) {
      const int64_t u = F[size_t(i)];
      for (uint64_t e = g->row_ptr[size_t(u)]; e < g->row_ptr[size_t(u) + 1]; e++) {
        const uint64_t h = splitmix64(uint64_t(rmatVid(g->col[e], g->seed)));
        c++;
        sm += h;
        xr ^= h;
      }
    }
    cnt[size_t(t)] = c;
    sum[size_t(t)] = sm;
    x[size_t(t)] = xr;
  });
  out[0] = out[1] = out[2] = 0;
  for (int t = 0; t < threads; t++) {
    out[0] += cnt[size_t(t)];
    out[1] += sum[size_t(t)];
    out[2] ^= x[size_t(t)];
  }
}

// FIND SHORTEST PATH for n pairs (definition: ora_shortest_path in refcpu.cpp).  hops[i] = -1
// when dst is not reached within max_steps; the path of pair i is
// path_vids[path_off[i] .. path_off[i+1]) (malloc'd into *path_vids, ora_free).
void ora_rmat_graph_shortest_path(ora_rmat_graph* g, const int64_t* src, const int64_t* dst, size_t n,
                                  int32_t max_steps, int32_t threads, int64_t* hops, int64_t* path_off,
                                  int64_t** path_vids) {
  if (threads < 1) threads = 1;
  // the reverse CSR (the -type in-edge keys, P5): transpose of the deduplicated out CSR
  if (g->rrow_ptr.size() != size_t(g->n) + 1 || g->rcol.size() != g->col.size()) {
    g->rrow_ptr.assign(size_t(g->n) + 1, 0);
    for (uint32_t v : g->col) g->rrow_ptr[size_t(v) + 1]++;
    for (int64_t v = 0; v < g->n; v++) g->rrow_ptr[size_t(v) + 1] += g->rrow_ptr[size_t(v)];
    g->rcol.resize(g->col.size());
    std::vector<uint64_t> fill(g->rrow_ptr.begin(), g->rrow_ptr.end() - 1);
    for (int64_t u = 0; u < g->n; u++)
      for (uint64_t e = g->row_ptr[size_t(u)]; e < g->row_ptr[size_t(u) + 1]; e++)
        g->rcol[fill[g->col[e]]++] = uint32_t(u);
  }
  std::vector<int64_t> si = idx_of(g, src, n, threads), ti = idx_of(g, dst, n, threads);
  std::vector<std::vector<int64_t>> paths(n);
  std::atomic<size_t> next{0};
  parallel_for(threads, threads, [&](int64_t, int64_t, int) {
    std::vector<int32_t> dt(size_t(g->n), -1);
    std::vector<int64_t> touched, fr, nx;
    for (size_t p; (p = next++) < n;) {
      hops[p] = -1;
      const int64_t s = si[p], t = ti[p];
      // a vid that is no vertex has no keys: only src == dst (same vid) gives a path
      if (src[p] == dst[p]) {
        hops[p] = 0;
        paths[p] = {src[p]};
        continue;
      }
      if (s < 0 || t < 0) continue;
      touched.clear();
      fr.assign(1, t);
      dt[size_t(t)] = 0;
      touched.push_back(t);
      for (int32_t lvl = 1; lvl <= max_steps && !fr.empty() && dt[size_t(s)] < 0; lvl++) {
        nx.clear();
        for (int64_t v : fr)
          for (uint64_t e = g->rrow_ptr[size_t(v)]; e < g->rrow_ptr[size_t(v) + 1]; e++) {
            const uint32_t u = g->rcol[e];
            if (dt[u] < 0) {
              dt[u] = lvl;
              touched.push_back(u);
              nx.push_back(u);
            }
          }
        fr.swap(nx);
      }
      const int32_t L = dt[size_t(s)];
      if (L >= 0) {
        hops[p] = L;
        std::vector<int64_t> path{src[p]};
        int64_t v = s;
        for (int32_t k = L; k > 0; k--) {
          int64_t best = -1, bestv = 0;
          for (uint64_t e = g->row_ptr[size_t(v)]; e < g->row_ptr[size_t(v) + 1]; e++) {
            const uint32_t w = g->col[e];
            if (dt[w] != k - 1) continue;
            const int64_t wv = rmatVid(w, g->seed);
            if (best < 0 || wv < bestv) {
              best = w;
              bestv = wv;
            }
          }
          v = best;
          path.push_back(bestv);
        }
        paths[p] = std::move(path);
      }
      for (int64_t x : touched) dt[size_t(x)] = -1;
    }
  });
  size_t tot = 0;
  path_off[0] = 0;
  for (size_t p = 0; p < n; p++) {
    tot += paths[p].size();
    path_off[p + 1] = int64_t(tot);
  }
  *path_vids = static_cast<int64_t*>(malloc(sizeof(int64_t) * (tot ? tot : 1)));
  for (size_t p = 0; p < n; p++)
    if (!paths[p].empty()) memcpy(*path_vids + path_off[p], paths[p].data(), sizeof(int64_t) * paths[p].size());
}

}  // extern "C"
