// engine.h -- internal types of the MI355X neighbour-expansion engine.
//
// Layout in HBM (per context = one space on one GPU, rank r of G):
//   vertex map   vid_of[n_global] int64 (replicated), vid->gidx open-addressing hash table,
//                owner ranges base[G+1]: gidx in [base[r], base[r+1]) are owned by rank r.
//   per edge type t:
//     out CSR    row_ptr[n_local+1] int64, col[nnz] int32 (global dst index), rank[nnz] int64
//                (absent when every rank is 0), SoA prop columns (INT narrowed to 1/2/4/8 B).
//     in  CSR    same shape for the -t in-edges (no props), used by FIND SHORTEST PATH.
//   Rows inside a CSR row follow the reference's bytewise key order (rank, dst LE bytes),
//   i.e. the order RocksEngine::prefix iterates (RocksEngine.cpp:191-200).
#pragma once
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdint>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/nebula_amd.h"

namespace nbg {

struct Error : std::runtime_error {
  int32_t code;
  Error(int32_t c, const std::string& m) : std::runtime_error(m), code(c) {}
};

#define NBG_HIP(x)                                                                        \
  do {                                                                                    \
    hipError_t e_ = (x);                                                                  \
    if (e_ != hipSuccess)                                                                 \
      throw ::nbg::Error(NBG_E_DEVICE, std::string(#x) + ": " + hipGetErrorString(e_));   \
  } while (0)

// Device buffer (RAII).  Never resized inside a launch sequence that a caller may capture.
// Per-context cache of device blocks used while a query runs: queries allocate and drop many
// temporaries, and hipFree synchronises the whole device, so blocks freed during a query go
// back to the context's pool and are reused by later queries on the same stream (stream order
// makes the reuse safe).  Blocks allocated outside a query scope (the snapshot) use
// hipMalloc/hipFree directly.
struct BufPool;
void pool_register(BufPool* p, bool add);
size_t pool_trim_all();  // every live pool's cache back to the driver (an out-of-memory retry)
struct BufPool {
  std::mutex mu;
  std::multimap<size_t, void*> blocks;
  size_t cached = 0;
  size_t limit = size_t(16) << 30;
  BufPool() { pool_register(this, true); }
  ~BufPool() {
    pool_register(this, false);
    for (auto& b : blocks) (void)hipFree(b.second);
  }
  void* get(size_t want, size_t& got) {
    std::lock_guard<std::mutex> lk(mu);
    auto it = blocks.lower_bound(want);
    if (it == blocks.end() || it->first > 2 * want + (size_t(1) << 20)) return nullptr;
    got = it->first;
    void* p = it->second;
    blocks.erase(it);
    cached -= got;
    return p;
  }
  void put(void* p, size_t cap) {
    {
      std::lock_guard<std::mutex> lk(mu);
      if (cached + cap <= limit) {
        blocks.emplace(cap, p);
        cached += cap;
        return;
      }
    }
    (void)hipFree(p);
  }
  // hand every cached block back to the driver (a failed hipMalloc retries after this)
  size_t trim() {
    std::lock_guard<std::mutex> lk(mu);
    const size_t freed = cached;
    for (auto& b : blocks) (void)hipFree(b.second);
    blocks.clear();
    cached = 0;
    return freed;
  }
};
extern thread_local std::shared_ptr<BufPool> tl_pool;  // set for the duration of a query

// Pinned host blocks for results copied back to the host.  A device->host copy into pageable
// memory goes through the driver's bounce buffer (r04k: the 173 MB of C3's DISTINCT vids took
// 64 ms, ~2.7 GB/s); into pinned memory it runs at the link's rate.  hipHostMalloc of a large
// block is itself slow, so a context caches the blocks its released results hand back.
// Cap (set per query, host_pool_cap): option host_pool_gb, else 1/16 of the host's RAM shared
// among the contexts on the device, at most 8 GiB (eight in-process LocalComm ranks on a 1.5 TB
// host: 8 GiB each; on a 64 GiB host: 512 MiB each).  Trimmed when the context is destroyed.
struct HostPool {
  std::mutex mu;
  std::multimap<size_t, void*> blocks;
  size_t cached = 0;
  size_t limit = size_t(8) << 30;
  ~HostPool() { trim(); }
  void trim() {
    std::lock_guard<std::mutex> lk(mu);
    for (auto& b : blocks) (void)hipHostFree(b.second);
    blocks.clear();
    cached = 0;
  }
  void* get(size_t want, size_t& got) {
    std::lock_guard<std::mutex> lk(mu);
    auto it = blocks.lower_bound(want);
    if (it == blocks.end() || it->first > 2 * want + (size_t(1) << 20)) return nullptr;
    got = it->first;
    void* p = it->second;
    blocks.erase(it);
    cached -= got;
    return p;
  }
  void put(void* p, size_t cap) {
    {
      std::lock_guard<std::mutex> lk(mu);
      if (cached + cap <= limit) {
        blocks.emplace(cap, p);
        cached += cap;
        return;
      }
    }
    (void)hipHostFree(p);
  }
};
struct HostBuf {
  void* p = nullptr;
  size_t bytes = 0;
  std::shared_ptr<HostPool> pool;
  HostBuf() = default;
  HostBuf(const HostBuf&) = delete;
  HostBuf& operator=(const HostBuf&) = delete;
  HostBuf(HostBuf&& o) noexcept : p(o.p), bytes(o.bytes), pool(std::move(o.pool)) {
    o.p = nullptr;
    o.bytes = 0;
  }
  HostBuf& operator=(HostBuf&& o) noexcept {
    if (this != &o) {
      release();
      p = o.p;
      bytes = o.bytes;
      pool = std::move(o.pool);
      o.p = nullptr;
      o.bytes = 0;
    }
    return *this;
  }
  ~HostBuf() { release(); }
  void release() {
    if (!p) return;
    if (pool) pool->put(p, bytes);
    else (void)hipHostFree(p);
    p = nullptr;
    bytes = 0;
    pool.reset();
  }
  void alloc(const std::shared_ptr<HostPool>& pl, size_t b) {
    if (p || b == 0) throw std::logic_error("HostBuf::alloc");
    size_t got = 0;
    if (pl && (p = pl->get(b, got))) {
      bytes = got;
      pool = pl;
      return;
    }
    if (hipHostMalloc(&p, b, hipHostMallocDefault) != hipSuccess) {
      p = nullptr;
      throw Error(NBG_E_NOMEM, "hipHostMalloc(" + std::to_string(b) + ") failed");
    }
    bytes = b;
    pool = pl;
  }
};
// host time spent in hipMalloc / hipFree of DevBufs (the build's phase trace reports it)
struct AllocClock {
  std::atomic<int64_t> alloc_ns{0}, free_ns{0}, allocs{0};
};
extern AllocClock g_alloc_clock;
inline int64_t mono_ns() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
  std::shared_ptr<BufPool> pool;
  DevBuf() = default;
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
  DevBuf(DevBuf&& o) noexcept : p(o.p), bytes(o.bytes), pool(std::move(o.pool)) {
    o.p = nullptr;
    o.bytes = 0;
  }
  DevBuf& operator=(DevBuf&& o) noexcept {
    if (this != &o) {
      release();
      p = o.p;
      bytes = o.bytes;
      pool = std::move(o.pool);
      o.p = nullptr;
      o.bytes = 0;
    }
    return *this;
  }
  ~DevBuf() { release(); }
  void release() {
    if (p) {
      if (pool) {
        pool->put(p, bytes);
      } else {
        const int64_t t0 = mono_ns();
        (void)hipFree(p);
        g_alloc_clock.free_ns += mono_ns() - t0;
      }
    }
    p = nullptr;
    bytes = 0;
    pool.reset();
  }
  // pooled blocks of 64 MiB and up are rounded up to 1/16 steps of their power of two, so a
  // buffer that grows by a write batch still fits the block its predecessor left in the cache
  static size_t pool_round(size_t b) {
    if (b < (size_t(64) << 20)) return b;
    size_t p2 = size_t(1) << (63 - __builtin_clzll(b));
    const size_t step = p2 / 16;
    return (b + step - 1) / step * step;
  }
  void alloc(size_t b) {
    release();
    if (b == 0) return;
    if (tl_pool) b = pool_round(b);
    if (tl_pool) {
      size_t got = 0;
      if (void* q = tl_pool->get(b, got)) {
        p = q;
        bytes = got;
        pool = tl_pool;
        return;
      }
    }
    const int64_t t0 = mono_ns();
    hipError_t e = hipMalloc(&p, b);
    if (e == hipErrorOutOfMemory && pool_trim_all() > 0) {
      (void)hipGetLastError();
      e = hipMalloc(&p, b);
    }
    g_alloc_clock.alloc_ns += mono_ns() - t0;
    g_alloc_clock.allocs++;
    if (e != hipSuccess) {
      p = nullptr;
      throw Error(NBG_E_NOMEM, "hipMalloc(" + std::to_string(b) + ") failed: " + hipGetErrorString(e));
    }
    bytes = b;
    pool = tl_pool;
  }
  void ensure(size_t b) {  // grow-only workspace
    if (b > bytes) alloc(b + b / 4);
  }
  template <typename T>
  T* as() const { return static_cast<T*>(p); }
};

// Carves consecutive pieces (each rounded up to `align` bytes) out of one workspace block and
// throws before a piece would pass the block's end: a hand-sized layout that drifted from its
// allocation fails the call instead of overrunning a neighbour (round 5: the device-driven
// batch's per-pair block was carved past its end at 8 in-process ranks)
struct Carve {
  char* q;
  char* const end;
  const char* what;
  size_t align;
  Carve(const DevBuf& b, const char* w, size_t a = 64)
      : q(static_cast<char*>(b.p)), end(static_cast<char*>(b.p) + b.bytes), what(w), align(a) {}
  template <typename T>
  T* take(size_t bytes) {
    char* r = q;
    const size_t step = (bytes + align - 1) / align * align;
    if (size_t(end - q) < step) throw Error(NBG_E_UNKNOWN, std::string(what) + ": workspace layout exceeds its block");
    q += step;
    return reinterpret_cast<T*>(r);
  }
};

// RAII: route DevBuf allocations of the current thread through the context's pool
struct PoolScope {
  std::shared_ptr<BufPool> prev;
  explicit PoolScope(const std::shared_ptr<BufPool>& p) : prev(tl_pool) { tl_pool = p; }
  ~PoolScope() { tl_pool = prev; }
};

struct Field {
  std::string name;
  int32_t type;
};

// One property column of a CSR (SoA).  INT columns are stored at the narrowest width that
// holds [minv, maxv]; reads sign-extend back to int64, so values are bit-identical.
struct PropCol {
  std::string name;
  int32_t type = 0;    // NBG_T_*
  int32_t width = 8;   // bytes per element in `data`
  DevBuf data;
  DevBuf present;      // uint8 per edge; empty = all present
  DevBuf str_off;      // int64 [nnz+1] for STRING
  DevBuf str_bytes;
  int64_t minv = 0, maxv = 0;
};

struct Csr {
  int64_t n_rows = 0;
  int64_t nnz = 0;
  DevBuf row_ptr;   // int64 [n_rows+1]
  DevBuf col;       // int32 [nnz] global vertex index of the other end
  DevBuf col_vid;   // int64 [nnz] vid of the other end (out CSR; rows path), or empty
  DevBuf rank;      // int64 [nnz] or empty (all zero)
  DevBuf row_part;  // int32 [n_rows]: the part holding the row's keys
  DevBuf row_ok;    // uint8 [n_rows] row_part == hash part; empty when all rows follow the rule
  std::vector<PropCol> props;
  DevBuf prop_table;  // device copy of the column descriptors (built on first query)
  // Older versions (multi-version data only): the tuples that are not the bytewise-first
  // version of their (src, rank, dst) group, in key order.  collectEdgeProps reads them until
  // its first emit (the firstLoop rule, QueryBaseProcessor.inl:349-402), so a push-down filter
  // can return an older version of a row's first passing group.  ov_edge = the group's edge
  // index (nondecreasing); ov_props: one column per schema field (INT-like as int64 bits).
  int64_t ov_n = 0;
  DevBuf ov_edge;
  std::vector<PropCol> ov_props;
  DevBuf ov_prop_table;
  size_t bytes() const {
    size_t b = row_ptr.bytes + col.bytes + col_vid.bytes + rank.bytes + row_part.bytes + row_ok.bytes + ov_edge.bytes;
    for (auto& p : props) b += p.data.bytes + p.present.bytes + p.str_off.bytes + p.str_bytes.bytes;
    for (auto& p : ov_props) b += p.data.bytes + p.present.bytes + p.str_off.bytes + p.str_bytes.bytes;
    return b;
  }
};

// Decoded edge tuples (the KV decode stage output, before CSR build).
struct Staging {
  int64_t n = 0;
  DevBuf src, dst, rank, ver;          // int64 each; rank/ver may stay empty (constant)
  DevBuf part;                         // int32 part of the key (empty: hash rule)
  DevBuf seq;                          // int64 load sequence number of the KV pair (write order)
  bool rank_const = true, ver_const = true;
  int64_t rank_value = 0, ver_value = 0;
  std::vector<DevBuf> props;           // int64 bits per field (double bits for DOUBLE/FLOAT)
  std::vector<DevBuf> present;         // uint8 per field (empty = all present)
  std::vector<DevBuf> str_len;         // STRING: int64 length; `props` holds heap offsets
  size_t cap = 0;
};

struct EdgeSpace {
  int32_t type = 0;
  int32_t schema_ver = 0;
  std::vector<Field> fields;
  Staging out_stage, in_stage;
  Csr out, in;
  // world > 1: replicas of every rank's out / in CSR over the whole gidx space (built on the
  // first FIND SHORTEST PATH, which shards its pairs over the ranks; the out replica alone and
  // rep_odeg, its out-degrees with row_ok applied, on the first GO whose first hop every rank
  // runs whole: ensure_rep_out)
  Csr rep_out, rep_in;
  bool has_rep = false, has_rep_out = false;
  DevBuf rep_odeg;  // u32 [n_global]
  // Transpose of the out CSR for bottom-up steps: row = owned dst, col = global src index,
  // props = copies of the INT-like out props in transpose order, t_eid = out-edge index.
  Csr tr;
  DevBuf t_eid;   // uint32 [nnz] (single rank only)
  bool has_tr = false;
  bool has_t_eid = false;
  int64_t out_nnz_global = -1;  // sum of out.nnz over ranks (direction heuristic)
  // streamed RMAT (one rank, graphs past the tuple stage's 2^32 cap): gen_rmat only records the
  // generator's parameters and finalize builds the CSRs bucket by bucket from regenerated samples
  // writable snapshots: the sorted tuple order of the last build per direction (0 out, 1 in):
  // tuple permutation, (src_local << 32 | byterank(dst)) keys and dst gidx by tuple index.  A
  // commit without new vertices merges its sorted batch into it instead of re-sorting every tuple
  struct Order {
    DevBuf perm, skey, dstg;
    int64_t n = 0;
  };
  Order ord[2];
  bool rmat_stream = false;
  int32_t rmat_scale = 0, rmat_ef = 0;
  uint64_t rmat_seed = 0;
  DevBuf odeg;                     // uint32 [owned rows]: out-degree, 0 where row_ok == 0
                                   // (padded with 0 to whole 128-row tiles)
  int64_t max_odeg = -1;           // largest owned out-degree (-1: unknown)
  int64_t max_odeg_global = -1;    // largest out-degree over all ranks (with out_nnz_global)
  // prefix sums of the kTopDeg largest out-degrees over all ranks (top_deg[k] = sum of the k
  // largest): bounds the start frontier's out-degree sum of a GO from k starts (with
  // out_nnz_global; empty: unknown)
  std::vector<int64_t> top_deg;
  int64_t bu_in_tiles = 0;         // 128-row tiles up to the last row with an in-edge (final hop)
  int64_t bu_both_tiles = 0;       // ... with an in-edge and an out-edge (non-final hops)
  DevBuf odeg8;                    // uint8 [owned rows, padded as odeg]: min(out-degree, 255); 255 =
                                   // read odeg (the non-final bottom-up pass streams 1 B per row)
  // quad slab (bottom-up first pass): the first 4 entries of every transposed row, row-major in
  // two halves (slots 0-1 -> pair_col[0], slots 2-3 -> pair_col[1], 2 x int32 per row, -1 past
  // the row's end, padded to whole 128-row tiles)
  DevBuf pair_col[2];
  // quantised predicate packing (bottom-up hops): the words of pair_col and tcol_q carry the
  // source gidx in their low q_gbits bits and, above it, q_bits bits of the bucket of transposed
  // prop q_field's value: bucket(v) = (v - q_min) * 2^q_bits / q_range (monotone), so a
  // compare against a constant is decided from the bucket except in the one bucket holding the
  // constant.  q_field < 0: words unpacked (plain gidx).  tcol_q: tr.col packed the same way.
  int32_t q_field = -1, q_gbits = 0, q_bits = 0;
  int64_t q_min = 0;
  uint64_t q_range = 1;
  DevBuf tcol_q;
  // rest records (bottom-up rest pass): one 64-byte line per transposed row below brec_rows (the
  // rows a bottom-up hop can leave pending): words 0-1 the row's start in tr (bits 0-47) and
  // min(in-degree, 65535) (bits 48-63), words 2-15 its first kRecEntries entries as in tcol_q /
  // tr.col (-1 past the row).  A pending row then costs one line instead of a row_ptr line and
  // one or two column lines.
  DevBuf brec;
  int64_t brec_rows = 0;
};
constexpr int kRecEntries = 14;

// Vertex tag props: per tag, one row per vertex = the bytewise-first version under
// the vertex key prefix (part, vid, tag) of the vid's own part -- what collectVertexProps reads
// (QueryBaseProcessor.inl:309-333).  Columns span the whole gidx space so $^ (src) and $$ (dst)
// props are one indexed load; `present` = the vertex has the row and the field decoded.
struct TagSpace {
  int32_t id = 0;
  int32_t schema_ver = 0;
  std::string name;
  std::vector<Field> fields;
  Staging stage;              // src = vid, ver, part, rank = load sequence number (write order)
  int64_t committed_n = 0;    // stage.n at the last finalize / commit (merge-commit eligibility)
  std::vector<PropCol> cols;  // per field, [n_global]; data int64 bits, present uint8:
                              // 0 none, 1 row of the vid's own part, 2 row of a foreign part only
  DevBuf part;                // int32 [n_global]: the part the vertex's row came from
};
// flat (tag, prop) table the expression compiler resolves $^.tag.prop / $$.tag.prop against
struct TagFieldRef {
  std::string tag, prop;
  int32_t type;
};

struct Timing {
  double total_ms = 0, expand_ms = 0;
  int64_t expand_launches = 0;
  uint64_t edges_scanned = 0, expand_bytes = 0;
  int32_t steps_run = 0;
  int32_t bu_steps = 0;
  double comm_ms = 0;
  uint64_t comm_bytes = 0;
  int32_t n_hops = 0;
  nbg_hop_stat hops[NBG_MAX_HOP_STATS] = {};
  int32_t host_waits = 0;  // engine-level host waits on the device (fetches, stream syncs)
  int32_t spec_hops = 0;   // hops that ran behind a device gate
  int32_t launches = 0;    // kernel launches of the device-driven shortest-path batches
  int32_t comm_calls = 0;  // collectives issued through the communicator (comm.cpp)
  uint64_t hop_bytes_mark = 0;  // expand_bytes at the previous hop record
  // kernel_ms < 0: the hop is one kernel (its time and bytes are the hop's; a top-down hop's
  // time is filled in later by timing_resolve)
  void hop(int32_t mode, bool final_hop, double ms, const unsigned long long* c6, double kernel_ms = -1,
           uint64_t kernel_bytes = 0) {
    const uint64_t b = expand_bytes - hop_bytes_mark;
    hop_bytes_mark = expand_bytes;
    if (n_hops >= NBG_MAX_HOP_STATS) return;
    nbg_hop_stat& h = hops[n_hops++];
    h.mode = mode;
    h.final_hop = final_hop ? 1 : 0;
    h.ms = ms;
    h.bytes = b;
    for (int i = 0; i < 8; i++) h.c[i] = c6 ? c6[i] : 0;
    h.kernel_ms = kernel_ms < 0 ? ms : kernel_ms;
    h.kernel_bytes = kernel_ms < 0 ? b : kernel_bytes;
  }
  // rocprof names of the last hop's kernels: the dominant one first, then the others ("; ")
  void name_last_hop(const std::string& k0, const std::string& k1 = "", const char* k2 = nullptr) {
    if (n_hops == 0 || n_hops > NBG_MAX_HOP_STATS) return;
    std::string s = k0;
    if (!k1.empty()) s += "; " + k1;
    if (k2) s += std::string("; ") + k2;
    nbg_hop_stat& h = hops[n_hops - 1];
    snprintf(h.kernels, sizeof h.kernels, "%s", s.c_str());
  }
};

constexpr size_t kHostStageBytes = size_t(1) << 20;

struct Ctx {
  int32_t device = 0, num_parts = 1, rank = 0, world = 1;
  // the sharded algorithm runs (owner slices, exchanges through the communicator): world > 1, or
  // one rank with a real one-rank RCCL communicator (option comm_single before nbg_comm_init), so
  // the RCCL entry points run on a one-GPU box exactly as they do at world > 1
  bool sharded = false;
  hipStream_t stream = nullptr;
  std::mutex mu;
  std::string last_error;
  void* comm = nullptr;  // ncclComm_t

  // vertex map
  bool finalized = false;
  int64_t n_global = 0;          // size of the gidx space (owner ranges padded to 64)
  int64_t n_vertices = 0;        // vertices in the snapshot
  std::vector<int64_t> base;     // G+1
  std::vector<int64_t> counts;   // vertices per rank
  DevBuf vid_of;                 // int64 [n_global]
  DevBuf brank;                  // writable: bytewise rank of every gidx's vid (merge commits)
  DevBuf ht_keys, ht_vals;       // int64 / int32 [ht_cap]
  int64_t ht_cap = 0;
  bool ht_has_min = false;       // INT64_MIN vid present (the empty-slot sentinel)
  int32_t ht_min_gidx = -1;
  DevBuf heap;                   // device copy of all loaded value blobs (STRING props)
  size_t heap_used = 0;
  std::map<int32_t, EdgeSpace> edges;
  std::map<int32_t, TagSpace> tags;
  int64_t load_seq = 0;               // KV pairs loaded so far (write order across parts)
  std::vector<TagFieldRef> tag_refs;  // flat (tag, prop) table, tag-id order then field order
  DevBuf tag_table;                   // device descriptors of tag_refs' columns (first query)
  double build_seconds = 0;
  // write path: with option writable=1 finalize builds the CSRs without consuming
  // the decoded tuples and the value heap (the stages are the write log);
  // nbg_snapshot_write_part decodes later write batches behind them and nbg_snapshot_commit
  // rebuilds the CSRs from the stages.  Queries read the last commit.
  bool has_log = false;
  bool pending_writes = false;
  int64_t commits = 0;
  int64_t merge_commits = 0;

  // workspaces for queries
  DevBuf ws_map;       // uint8 [n_global] visited / next-set bytemap
  DevBuf ws_map2;
  DevBuf ws_front[2];  // int32 frontier lists
  DevBuf ws_off;       // int64 [n+1] degree scan
  DevBuf ws_tmp;       // scan temp
  DevBuf ws_rows;      // final rows (int32 src idx, int64 edge)
  DevBuf ws_counters;  // small device counters
  DevBuf ws_bits_send, ws_bits_recv;
  DevBuf ws_bits_glob;  // world > 1: allgathered frontier bitmap / per-owner mark bitmap
  DevBuf ws_bits_xchg;  // world > 1: received mark segments [world][owned/32]
  DevBuf ws_bits_rep1;  // world > 1: the hop-1 frontier over the whole gidx space (go_rep1)
  DevBuf ws_piggy;      // world > 1: every rank's (n, e) counters per speculated hop
  DevBuf ws_starts;
  DevBuf ws_partials;  // per-block partial sums of the aggregated kernels
  DevBuf ws_pend;      // deferred bottom-up rows: pending bits + compacted list
  // FIND SHORTEST PATH distance bytes [side][pair][owned row], kept 0xFF between calls, and
  // its tuple lists (kept across calls; allocated outside the query pool)
  DevBuf sp_dist[2];
  size_t sp_dist_bytes = 0;
  bool sp_dirty = false;
  struct SpWork {
    DevBuf live[2], live_next[2], arena, meet, sweep[2], X, Xdeg, Xoff, state, cnt, vids, gidx, plist;
    DevBuf tile_rows;  // k_sp_expand: X entry of each tile's first slot
    DevBuf lvbits;     // per side and depth, the vertices some pair of the batch holds there
    int64_t cap_live[2] = {0, 0}, cap_next[2] = {0, 0}, cap_arena = 0, cap_meet = 0, cap_sweep[2] = {0, 0};
    int64_t cap_x = 0, cap_state = 0, cap_plist = 0;
    // device-driven batches (paths.hip, option sp_dev): fixed-capacity lists, chunk tables, the
    // per-pair arrays, the pair and global level filters and the counter blocks
    DevBuf dv_cnt, dv_live[4], dv_arena, dv_meet, dv_sw[2], dv_X, dv_Xcb, dv_chx, dv_slot, dv_wchx, dv_pair, dv_path,
        dv_pf, dv_gf;
    int64_t dv_B = 0, dv_cap = 0, dv_cap_ch = 0, dv_cap_wch = 0, dv_gf_log2 = -1;
    bool dv_pf_on = false;
    bool dv_clean = false;  // filter words and counters all zero
    // per direction (0 out, 1 in): min(degree, 65535) of every row of the CSR the last call used,
    // rebuilt when that CSR changed (row_ptr block, rows or commit count differ)
    DevBuf deg16[2];
    const void* deg16_rp[2] = {nullptr, nullptr};
    int64_t deg16_rows[2] = {-1, -1}, deg16_commits[2] = {-1, -1};
  } sp;
  // coherent pinned host block of the device-driven batches: publish slots, the pairs, results
  void* sp_host = nullptr;
  size_t sp_host_bytes = 0;
  Timing timing;
  hipEvent_t ev[8] = {};
  DevBuf ws_tile_rows;  // k_expand: frontier entry of each tile's first slot
  std::string bu_kernel_name, bu_rest_name;  // rocprof names of the last bottom-up launch
  bool bu_rest_rec = false;                  // ... whose rest pass read the rest records
  uint64_t bu_od_bytes = 0;                  // ... out-degree bytes its first pass read (non-final hop)
  // deferred kernel timing: event pairs recorded around expansion launches and read once the
  // query's stream has drained, so timing never makes the host wait on a launch
  struct PendingTime {
    size_t a, b;
    int32_t hop;   // Timing::hops index the time belongs to (-1: none)
    int32_t kind;  // 0: expand_ms + the hop's ms (+ kernel_ms of a top-down hop), 1: kernel_ms only, 2: comm_ms
  };
  bool hop_timing = true;  // option hop_timing: event pairs around the hops' kernels (0: none)
  bool total_pending = false;  // ev[1] recorded, total_ms not read yet (resolve_total)
  std::vector<hipEvent_t> tev;
  size_t tev_used = 0;
  std::vector<PendingTime> tpend;
  // query temporaries and results (results return their blocks when released).  Capped by
  // option query_pool_gb: a plain-rows result of RMAT-28 GO 2 STEPS is 21 GB, and re-allocating
  // it per query stalled one hipMalloc in ~9 for 5.7 s (r03 HIP API trace)
  std::shared_ptr<BufPool> pool = std::make_shared<BufPool>();
  std::shared_ptr<HostPool> host_pool = std::make_shared<HostPool>();  // pinned result blocks
  // snapshot build / commit temporaries: freed blocks stay with the process (a fresh multi-GB
  // hipMalloc costs up to seconds: r03a trace), so the phases of a build and later commits of a
  // writable snapshot reuse them.  Trimmed after a read-only build.
  std::shared_ptr<BufPool> build_pool = std::make_shared<BufPool>();
  unsigned long long* host_counters = nullptr;  // pinned, coherent, 256 entries
  // counters published by k_publish: host_counters + a sequence word the host spins on (a
  // hipStreamSynchronize round trip costs ~19 us on this stack, tools/launch_gap)
  unsigned long long* host_seq = nullptr;  // pinned, coherent
  uint64_t pub_seq = 0;
  void* host_stage = nullptr;                   // pinned, kHostStageBytes (query inputs)
  int64_t* starts_host = nullptr;               // pinned, coherent: a GO's small start set (k_starts_small)
  size_t host_stage_used = 0;
  // async host->device copy of a query input through the pinned stage when it fits (the stage
  // is reset at every query start; the stream drains before a query returns)
  void h2d(void* dst, const void* src, size_t bytes) {
    if (host_stage && host_stage_used + bytes <= kHostStageBytes) {
      uint8_t* p = static_cast<uint8_t*>(host_stage) + host_stage_used;
      memcpy(p, src, bytes);
      host_stage_used += (bytes + 255) & ~size_t(255);
      NBG_HIP(hipMemcpyAsync(dst, p, bytes, hipMemcpyHostToDevice, stream));
    } else {
      NBG_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, stream));
    }
  }
  std::map<std::string, int64_t> options;
  size_t hbm_total = 0;  // the device's memory (hipMemGetInfo at create)

  int64_t owned_lo() const { return base.empty() ? 0 : base[size_t(rank)]; }
  int64_t owned_hi() const { return base.empty() ? n_global : base[size_t(rank) + 1]; }
  int64_t opt(const std::string& k, int64_t d) const {
    auto it = options.find(k);
    return it == options.end() ? d : it->second;
  }
};

// live contexts per device (nbg_ctx_create / nbg_ctx_destroy): in-process rank groups put
// several contexts on one GPU, and each caches query blocks of its own
int ctx_count_on_device(int device);
// the cap of the context's pinned result cache (HostPool)
size_t host_ram_bytes();
inline void host_pool_cap(Ctx& c) {
  const int64_t gb = c.opt("host_pool_gb", -1);
  size_t cap = size_t(8) << 30;
  if (gb >= 0) {
    cap = size_t(gb) << 30;
  } else if (const size_t ram = host_ram_bytes()) {
    cap = std::min(cap, ram / 16 / size_t(std::max(1, ctx_count_on_device(c.device))));
  }
  std::lock_guard<std::mutex> lk(c.host_pool->mu);
  c.host_pool->limit = cap;
}
// the context's query block cache.  Cap: option query_pool_gb, else a quarter of the device's
// HBM shared among the contexts on it, at most 64 GiB (one MI355X context: 64 GiB; eight
// LocalComm ranks on one GPU: 8.9 GiB each), so the cache never holds what RCCL or the driver
// allocate outside DevBuf (those never trigger its trim)
inline std::shared_ptr<BufPool>& query_pool(Ctx& c) {
  const int64_t gb = c.opt("query_pool_gb", -1);
  size_t cap = size_t(64) << 30;
  if (gb >= 0) {
    cap = size_t(gb) << 30;
  } else if (c.hbm_total) {
    cap = std::min(cap, c.hbm_total / 4 / size_t(std::max(1, ctx_count_on_device(c.device))));
  }
  c.pool->limit = cap;
  return c.pool;
}

// ---- helpers implemented in the .hip files -------------------------------------------------
// snapshot.hip
void snapshot_load_part(Ctx& c, int32_t part, const uint8_t* kb, const uint64_t* koff,
                        const uint8_t* vb, const uint64_t* voff, size_t n);
void snapshot_gen_rmat(Ctx& c, int32_t scale, int32_t ef, uint64_t seed, int32_t et);
void snapshot_finalize(Ctx& c);
void snapshot_write_part(Ctx& c, int32_t part, const uint8_t* kb, const uint64_t* koff,
                         const uint8_t* vb, const uint64_t* voff, size_t n);
void snapshot_commit(Ctx& c);
void lookup_gidx(Ctx& c, const int64_t* d_vids, int32_t* d_gidx, int64_t n);
// the device counters d[0, n) (n <= 256) into pinned host h[0, n) once every launch before has
// finished on the context's stream (a one-block publish kernel + a host spin, traverse.hip)
// `before` (optional): an event recorded just ahead of the publish kernel
// shards > 1: d is a sharded counter block (word i = sum of d[i + s * kShardStride], s < shards)
void fetch_counters(Ctx& c, const unsigned long long* d, int n, unsigned long long* h, hipEvent_t before = nullptr,
                    int shards = 1);
// sharded block sums (traverse.hip block_add_sums): shard s of counter word i at i + s * kShardStride
constexpr size_t kShardStride = 256;
constexpr int kSumShards = 8;
// one host wait (counted in Timing::host_waits) until the device publishes `seq` in `word`
void wait_host_word(Ctx& c, const unsigned long long* word, uint64_t seq);
// a query's total_ms (ev[0] -> ev[1]) once asked for (go_run records ev[1] without waiting)
void resolve_total(Ctx& c);
// traverse.hip
int32_t go_run(Ctx& c, const nbg_go_spec& spec, nbg_rows* out);
// the out CSR replica and its out-degrees (collective: every rank calls it at the same point)
void ensure_rep_out(Ctx& c, EdgeSpace& es);
int32_t get_bound_run(Ctx& c, int32_t et, const int32_t* parts, const int64_t* vids, size_t n,
                      const uint8_t* filter, size_t flen, const nbg_prop_def* cols, size_t ncols,
                      nbg_rows* out, const int32_t* stats = nullptr);
int32_t shortest_path_run(Ctx& c, int32_t et, const int64_t* src, const int64_t* dst, size_t n,
                          int32_t max_steps, nbg_rows* out);
void timing_reset(Ctx& c);
void timing_resolve(Ctx& c);
// comm.cpp
void comm_alltoallv_bytes(Ctx& c, const void* send, const size_t* send_bytes, const size_t* send_off,
                          void* recv, const size_t* recv_bytes, const size_t* recv_off);
void comm_allgather_bytes(Ctx& c, const void* send, size_t bytes_each, void* recv);
void comm_allreduce_sum_i64(Ctx& c, int64_t* d_vals, size_t n);
void comm_allgatherv2_bytes(Ctx& c, const void* send, size_t send_bytes, void* recv, const size_t* recv_bytes,
                            const size_t* recv_off, const void* send2, size_t bytes2, void* recv2);
void comm_allgatherv_bytes(Ctx& c, const void* send, size_t send_bytes, void* recv, const size_t* recv_bytes,
                           const size_t* recv_off);
void comm_init_local(Ctx& c, int64_t key);
void comm_info(const Ctx& c, int32_t* ranks, int32_t* transport);
void comm_destroy(Ctx& c);

inline double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
inline int owner_of_part(int32_t part, int32_t world) { return int(part % world); }
inline int32_t part_of_vid(int64_t vid, int32_t parts) {
  return int32_t(uint64_t(vid) % uint64_t(parts) + 1);
}

}  // namespace nbg
