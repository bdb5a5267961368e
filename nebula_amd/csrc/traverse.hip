// traverse.hip -- the neighbour-expansion hot path on MI355X (gfx950).
//
// Replaces, for a whole frontier at once:
//   * QueryBaseProcessor::collectEdgeProps prefix scan + filter (QueryBaseProcessor.inl:335-405)
//     -> k_expand: edge-balanced tiles over the frontier's CSR rows;
//   * GoExecutor::getDstIdsFromResp unordered_set (GoExecutor.cpp:407-431)
//     -> byte-map marks (plain stores, no atomics) + k_compact (ballot/prefix compaction);
//   * processFinalResult WHERE / YIELD / DISTINCT (GoExecutor.cpp:585-782)
//     -> predicate fused into k_expand, k_materialize for YIELD, byte-map or hash DISTINCT.
//
// Load balance (power-law degrees): the frontier's degrees are prefix-summed; each 256-thread
// workgroup takes a fixed tile of 2048 consecutive edges of that flattened space, stages the
// (<= 2048) frontier entries covering it in LDS, and each lane finds its edge's owner by a
// binary search in LDS.  Consecutive lanes read consecutive adjacency entries, so the col /
// prop loads of a tile are coalesced whatever the degree distribution (a supernode simply
// spans many tiles).
#include <chrono>
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_reduce.hpp>
#include <rocprim/device/device_scan.hpp>
#include <rocprim/device/device_select.hpp>
#include <rocprim/iterator/counting_iterator.hpp>
#include <rocprim/iterator/transform_iterator.hpp>

#include <algorithm>
#include <cmath>
#include <unordered_map>
#include <thread>
#include <initializer_list>

#include "device_common.h"
#include "engine.h"
#include "program.h"
#include "rows.h"

namespace nbg {

int32_t compile_expr(const uint8_t* buf, size_t len, const std::vector<Field>& fields, bool graphd,
                     bool out_bound, Program* out, std::string* msg,
                     const std::vector<TagFieldRef>* tags = nullptr, const std::vector<Field>* inputs = nullptr);
Program program_dst();
FastPred classify_pred(const Program& p, const std::vector<Field>& fields);

constexpr int kThreads = 256;
constexpr int kItems = 8;
constexpr int kTile = kThreads * kItems;

static int grid_cap(int64_t n, int block = 256, int cap = 256 * 16) {
  int64_t g = (n + block - 1) / block;
  return int(std::max<int64_t>(1, std::min<int64_t>(g, cap)));
}

// ------------------------------------------------------------------------------------------
// device value model (boost::variant<int64,double,bool,string> + error)
// ------------------------------------------------------------------------------------------
struct Val {
  int64_t b;
  int32_t t;
  int32_t len;
};

struct PropDev {
  int32_t type;
  int32_t width;
  const void* data;
  const uint8_t* present;
  const int64_t* str_off;
  const uint8_t* str_bytes;
  const int32_t* part;  // tag columns: the part of each vertex's row (TagSpace::part)
};
struct EvalEnv {
  const PropDev* props;  // device table, one entry per schema field (Csr::prop_table)
  int32_t nprops;
  int32_t etype;
  const int64_t* vid_of;
  const int32_t* col;
  const int64_t* rank;
  const PropDev* tprops;  // tag columns over the gidx space (Ctx::tag_refs order), or null
  // $- / $var input table: open-addressing index src gidx -> its last input row, and columns
  const int32_t* in_keys;
  const int32_t* in_rows;
  uint32_t in_mask;
  const PropDev* iprops;
  // STEPS > 1: root start (vid rank) of every final-frontier vertex and rank -> start gidx
  const int32_t* in_root;
  const int32_t* in_root_tab;
  // storage (getBound) filters: a $^ tag row is visible when it sits in the request's part,
  // which for an edge row is the part of the row's keys (Csr::row_part, local row = src - lo)
  int32_t storage;
  int64_t lo;
  const int32_t* row_part;
};
__device__ inline uint32_t gidx_hash(int32_t g) { return uint32_t(g) * 2654435761u; }
// row of the input table whose FROM vid is gidx g (-1: none)
__device__ inline int32_t input_row(const EvalEnv& env, int32_t g) {
  uint32_t h = gidx_hash(g) & env.in_mask;
  for (uint32_t probe = 0; probe <= env.in_mask; probe++) {
    const int32_t k = env.in_keys[h];
    if (k == g) return env.in_rows[h];
    if (k < 0) return -1;
    h = (h + 1) & env.in_mask;
  }
  return -1;
}

__device__ inline int64_t load_int(const void* data, int width, int64_t i) {
  switch (width) {
    case 1: return int64_t(static_cast<const int8_t*>(data)[i]);
    case 2: return int64_t(static_cast<const int16_t*>(data)[i]);
    case 4: return int64_t(static_cast<const int32_t*>(data)[i]);
    default: return static_cast<const int64_t*>(data)[i];
  }
}

// compile-time width variant (W = 0: runtime width)
template <int W>
__device__ inline int64_t load_w(const void* data, int width, int64_t i) {
  if (W == 1) return int64_t(static_cast<const int8_t*>(data)[i]);
  if (W == 2) return int64_t(static_cast<const int16_t*>(data)[i]);
  if (W == 4) return int64_t(static_cast<const int32_t*>(data)[i]);
  if (W == 8) return static_cast<const int64_t*>(data)[i];
  return load_int(data, width, i);
}

__device__ inline Val load_prop(const PropDev& p, int64_t ge) {
  Val v;
  v.len = 0;
  if (p.present && !p.present[ge]) {
    v.t = VT_ERR;
    v.b = 0;
    return v;
  }
  switch (p.type) {
    case NBG_T_DOUBLE:
    case NBG_T_FLOAT:
      v.t = VT_DOUBLE;
      v.b = static_cast<const int64_t*>(p.data)[ge];
      break;
    case NBG_T_BOOL:
      v.t = VT_BOOL;
      v.b = load_int(p.data, p.width, ge) != 0;
      break;
    case NBG_T_STRING: {
      int64_t o = p.str_off[ge];
      v.t = VT_STR;
      v.b = int64_t(reinterpret_cast<uintptr_t>(p.str_bytes + o));
      v.len = int32_t(p.str_off[ge + 1] - o);
      break;
    }
    default:
      v.t = VT_INT;
      v.b = load_int(p.data, p.width, ge);
  }
  return v;
}

__device__ inline double as_d(const Val& v) { return v.t == VT_INT ? double(v.b) : __longlong_as_double(v.b); }
__device__ inline bool as_bool(const Val& v) {
  switch (v.t) {
    case VT_INT: return v.b != 0;
    case VT_DOUBLE: return __longlong_as_double(v.b) != 0.0;
    case VT_BOOL: return v.b != 0;
    default: return v.len == 0;  // string -> empty() (Expressions.h:172-173)
  }
}
__device__ inline int str_cmp(const Val& a, const Val& b) {
  const uint8_t* x = reinterpret_cast<const uint8_t*>(uintptr_t(a.b));
  const uint8_t* y = reinterpret_cast<const uint8_t*>(uintptr_t(b.b));
  int n = a.len < b.len ? a.len : b.len;
  for (int i = 0; i < n; i++)
    if (x[i] != y[i]) return x[i] < y[i] ? -1 : 1;
  return a.len == b.len ? 0 : (a.len < b.len ? -1 : 1);
}
// boost::variant operator< : index first, then value
__device__ inline bool v_lt(const Val& a, const Val& b) {
  if (a.t != b.t) return a.t < b.t;
  switch (a.t) {
    case VT_INT: return a.b < b.b;
    case VT_DOUBLE: return __longlong_as_double(a.b) < __longlong_as_double(b.b);
    case VT_BOOL: return a.b < b.b;
    default: return str_cmp(a, b) < 0;
  }
}
__device__ inline bool v_eq(const Val& a, const Val& b) {
  if (a.t != b.t) return false;
  switch (a.t) {
    case VT_INT:
    case VT_BOOL: return a.b == b.b;
    case VT_DOUBLE: return __longlong_as_double(a.b) == __longlong_as_double(b.b);
    default: return str_cmp(a, b) == 0;
  }
}
__device__ inline Val mk(int32_t t, int64_t b) {
  Val v;
  v.t = t;
  v.b = b;
  v.len = 0;
  return v;
}
__device__ inline Val mkd(double d) { return mk(VT_DOUBLE, __double_as_longlong(d)); }

__device__ Val eval_program(const Program* __restrict__ P, const EvalEnv& env, int64_t ge, int32_t src_g,
                            int32_t dst_g) {
  Val st[kMaxStack];
  int sp = 0;
  const int n = P->n;
  for (int pc = 0; pc < n; pc++) {
    Ins in = P->ins[pc];
    switch (in.op) {
      case P_CONST: {
        Val v;
        v.t = P->ctype[in.arg];
        v.b = P->cbits[in.arg];
        v.len = P->clen[in.arg];
        if (v.t == VT_STR) v.b = int64_t(reinterpret_cast<uintptr_t>(P->cstr + P->cbits[in.arg]));
        st[sp++] = v;
        break;
      }
      case P_PROP: st[sp++] = load_prop(env.props[in.arg], ge); break;
      case P_DST: st[sp++] = mk(VT_INT, env.vid_of[dst_g]); break;
      case P_SRC: st[sp++] = mk(VT_INT, env.vid_of[src_g]); break;
      case P_RANK: st[sp++] = mk(VT_INT, env.rank ? env.rank[ge] : 0); break;
      case P_TYPE: st[sp++] = mk(VT_INT, env.etype); break;
      case P_SRCTAG:
      case P_DSTTAG: {
        // only a row of the vertex's own part is visible to GO (presence byte 1; 2 = a row that
        // only a getBound naming its foreign part reads)
        const PropDev& tp = env.tprops[in.arg];
        const int32_t g = in.op == P_SRCTAG ? src_g : dst_g;
        const bool vis = env.storage ? tp.present[g] != 0 && tp.part[g] == env.row_part[src_g - env.lo]
                                     : tp.present[g] == 1;
        st[sp++] = vis ? load_prop(tp, g) : mk(VT_ERR, 0);
        break;
      }
      case P_INPUT: {
        int32_t g0 = src_g;
        if (env.in_root) {  // multi-step: the input row of the vertex's root start
          const int32_t r = env.in_root[src_g];
          g0 = r == INT32_MAX ? -1 : env.in_root_tab[r];
        }
        const int32_t row = g0 < 0 ? -1 : input_row(env, g0);
        st[sp++] = row < 0 ? mk(VT_ERR, 0) : load_prop(env.iprops[in.arg], row);
        break;
      }
      case P_UNARY: {
        Val& a = st[sp - 1];
        if (a.t == VT_ERR) break;
        if (in.sub == 0) break;  // PLUS
        if (in.sub == 1) {       // NEGATE
          if (a.t == VT_INT) a.b = int64_t(0ull - uint64_t(a.b));
          else if (a.t == VT_DOUBLE) a.b = __double_as_longlong(-__longlong_as_double(a.b));
          else a.t = VT_ERR;
        } else {
          a = mk(VT_BOOL, !as_bool(a));
        }
        break;
      }
      case P_ARITH: {
        Val r = st[--sp];
        Val l = st[sp - 1];
        Val o;
        if (l.t == VT_ERR) o = l;
        else if (r.t == VT_ERR) o = r;
        else {
          bool ar = (l.t == VT_INT || l.t == VT_DOUBLE) && (r.t == VT_INT || r.t == VT_DOUBLE);
          bool dbl = l.t == VT_DOUBLE || r.t == VT_DOUBLE;
          o = mk(VT_ERR, 0);
          switch (in.sub) {
            case 0:
              if (ar) o = dbl ? mkd(as_d(l) + as_d(r)) : mk(VT_INT, int64_t(uint64_t(l.b) + uint64_t(r.b)));
              break;
            case 1:
              if (ar) o = dbl ? mkd(as_d(l) - as_d(r)) : mk(VT_INT, int64_t(uint64_t(l.b) - uint64_t(r.b)));
              break;
            case 2:
              if (ar) o = dbl ? mkd(as_d(l) * as_d(r)) : mk(VT_INT, int64_t(uint64_t(l.b) * uint64_t(r.b)));
              break;
            case 3:
              if (ar) {
                if (dbl) o = mkd(as_d(l) / as_d(r));
                else if (r.b == 0) o = mk(VT_ERR, 0);
                else if (r.b == -1) o = mk(VT_INT, int64_t(0ull - uint64_t(l.b)));
                else o = mk(VT_INT, l.b / r.b);
              }
              break;
            default:
              if (l.t == VT_INT && r.t == VT_INT) {
                if (r.b == 0) o = mk(VT_ERR, 0);
                else if (r.b == -1) o = mk(VT_INT, 0);
                else o = mk(VT_INT, l.b % r.b);
              }
          }
        }
        st[sp - 1] = o;
        break;
      }
      case P_REL: {
        Val r = st[--sp];
        Val l = st[sp - 1];
        Val o;
        if (l.t == VT_ERR) o = l;
        else if (r.t == VT_ERR) o = r;
        else {
          bool res;
          bool mixed = (l.t == VT_INT || l.t == VT_DOUBLE) && (r.t == VT_INT || r.t == VT_DOUBLE) &&
                       (l.t == VT_DOUBLE || r.t == VT_DOUBLE);
          switch (in.sub) {
            case 0: res = v_lt(l, r); break;
            case 1: res = !v_lt(r, l); break;
            case 2: res = v_lt(r, l); break;
            case 3: res = !v_lt(l, r); break;
            case 4: res = mixed ? fabs(as_d(l) - as_d(r)) < 1e-8 : v_eq(l, r); break;
            default: res = mixed ? !(fabs(as_d(l) - as_d(r)) < 1e-8) : !v_eq(l, r); break;
          }
          o = mk(VT_BOOL, res);
        }
        st[sp - 1] = o;
        break;
      }
      case P_LOGIC: {
        Val r = st[--sp];
        Val l = st[sp - 1];
        Val o;
        if (l.t == VT_ERR) o = l;
        else if (r.t == VT_ERR) o = r;
        else if (in.sub == 0) o = mk(VT_BOOL, as_bool(l) ? as_bool(r) : false);
        else o = mk(VT_BOOL, as_bool(l) ? true : as_bool(r));
        st[sp - 1] = o;
        break;
      }
    }
  }
  return st[0];
}

// ------------------------------------------------------------------------------------------
// expansion
// ------------------------------------------------------------------------------------------
enum ExpMode : int { EXP_MARK = 0, EXP_ROWS = 1, EXP_FLAGS = 2 };
enum PredKind : int { PK_NONE = 0, PK_FAST = 1, PK_VM = 2 };

struct ExpandArgs {
  const int32_t* F;
  int64_t nF;
  const int64_t* off;      // exclusive degree scan, off[nF] = total edges
  const int64_t* row_ptr;
  const int32_t* col;
  int64_t lo;              // gidx of local row 0
  uint8_t* map;            // EXP_MARK
  int32_t* rows_src;       // EXP_ROWS: local row index
  int64_t* rows_edge;      //           global edge index into the CSR
  unsigned long long* rows_cnt;
  uint8_t* flags;          // EXP_FLAGS: one byte per flattened edge slot
  unsigned long long* err; // eval errors (GO semantics)
  int32_t storage;         // 1: eval error keeps the edge (QueryBaseProcessor.inl:391-396)
  int32_t mark_check;      // read the byte before storing it
  int64_t* out_vid;        // EXP_ROWS fused YIELD _dst: write vid_of[dst] instead of (src, edge)
  const int64_t* vid_of;
  const int64_t* col_vid;  // per-edge dst vid (Csr::col_vid) or null: vid_of[col[e]]
  const int32_t* tile_row; // [ntiles + 1]: frontier entry holding the first slot of each tile
                           // (k_tile_rows), or null: binary search of off[]
  // multi-step $- / $var (VertexBackTracker, GoExecutor.h:174-193): root start of every marked
  // dst = the smallest (by vid rank) root of its in-edges' srcs this hop, or null
  const int32_t* root_cur;
  int32_t* root_next;
};
struct FastArgs {
  const void* data;
  const uint8_t* present;
  int32_t width;
  int32_t op;
  int64_t k;
};

__host__ __device__ inline bool fast_cmp(int op, int64_t a, int64_t k) {
  switch (op) {
    case 0: return a < k;
    case 1: return a <= k;
    case 2: return a > k;
    case 3: return a >= k;
    case 4: return a == k;
    default: return a != k;
  }
}

// Quantised predicate on packed bottom-up words (EdgeSpace::q_*): the low gbits bits are the
// source gidx, the bits above the bucket of the predicate column's value.  The compare decides
// every bucket below ulo (`below`: 1 pass, 0 fail) and above uhi (`above`); buckets in
// [ulo, uhi] hold the constant and need the exact value (-1).  Host-built per query
// (make_qargs); all scalars, so the test is two compares, no table loads.  Unpacked words:
// gmask all ones, ulo 0, uhi INT_MAX (every word undecided).
struct QArgs {
  uint32_t gmask = 0xffffffffu;
  int32_t gbits = 0;
  int32_t ulo = 0, uhi = INT32_MAX;
  int32_t below = -1, above = -1;
};
// The kernels' copy of QArgs in scalar registers.  Read through the by-value kernel argument,
// q_test's select between `below` and `above` compiled to a per-lane select of two kernarg
// addresses and a vector load, i.e. one dependent load and a vmcnt(0) wait per slot word.
__device__ inline QArgs q_sgpr(const QArgs& a) {
  QArgs r;
  r.gmask = __builtin_amdgcn_readfirstlane(a.gmask);
  r.gbits = __builtin_amdgcn_readfirstlane(a.gbits);
  r.ulo = __builtin_amdgcn_readfirstlane(a.ulo);
  r.uhi = __builtin_amdgcn_readfirstlane(a.uhi);
  r.below = __builtin_amdgcn_readfirstlane(a.below);
  r.above = __builtin_amdgcn_readfirstlane(a.above);
  return r;
}
__device__ inline int32_t q_gidx(int32_t s, const QArgs& q) { return s & int32_t(q.gmask); }
// 1 pass, 0 fail, -1 undecided (load the value)
__device__ inline int q_test(int32_t s, const QArgs& q) {
  const int32_t b = int32_t(uint32_t(s) >> q.gbits);
  int r = -1;
  r = b > q.uhi ? q.above : r;
  r = b < q.ulo ? q.below : r;
  return r;
}

// raw buffer resource over p (gfx9 word 3; bounds left to the caller): loads through it are
// buffer instructions, which the compiler never merges with LDS reads into a flat load
__device__ inline __amdgpu_buffer_rsrc_t raw_rsrc(const void* p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, 0x7fffffff, 0x00020000);
}

template <int MODE, int PK>
__global__ __launch_bounds__(kThreads) void k_expand(ExpandArgs a, FastArgs fp, const Program* __restrict__ prog,
                                                     EvalEnv env) {
  __shared__ int32_t s_off[kTile + 1];  // off[k] - e0 (fits: tile-relative)
  __shared__ int64_t s_rs[kTile];       // row_ptr[F[k]] - off[k]
  __shared__ int32_t s_src[kTile];      // F[k]
  __shared__ int32_t s_scan[kThreads / 64];
  int32_t* s_own = s_off;               // after the owner map is built: owner k of tile slot j
  __shared__ int64_t s_hdr[2];
  __shared__ uint32_t s_wsum[kThreads / 64];
  __shared__ unsigned long long s_base;
  const int64_t nF = a.nF;
  const int64_t E = a.off[nF];
  const int64_t ntiles = (E + kTile - 1) / kTile;
  for (int64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const int64_t e0 = t * kTile;
    const int64_t e1 = min(e0 + int64_t(kTile), E);
    if (threadIdx.x == 0 && a.tile_row) {
      int64_t i0, cnt;
      tile_entries(a.tile_row, a.off, nF, t, e1, E, i0, cnt);
      s_hdr[0] = i0;
      s_hdr[1] = cnt;
    } else if (threadIdx.x == 0) {
      // i0 = last k with off[k] <= e0 ; i1 = last k with off[k] <= e1 - 1
      int64_t lo = 0, hi = nF;  // off[lo] <= e0 < off[hi] invariant (off[0] = 0, off[nF] = E)
      while (hi - lo > 1) {
        int64_t mid = (lo + hi) >> 1;
        if (a.off[mid] <= e0) lo = mid; else hi = mid;
      }
      int64_t i0 = lo;
      lo = i0;
      hi = nF;
      while (hi - lo > 1) {
        int64_t mid = (lo + hi) >> 1;
        if (a.off[mid] <= e1 - 1) lo = mid; else hi = mid;
      }
      s_hdr[0] = i0;
      s_hdr[1] = lo - i0 + 1;
    }
    __syncthreads();
    const int64_t i0 = s_hdr[0];
    const int64_t cnt64 = s_hdr[1];
    // a run of zero-degree frontier entries can put more than kTile entries under one tile:
    // such a tile searches off[] in global memory instead of staging it in LDS
    const bool big = cnt64 > kTile;
    const int cnt = big ? 0 : int(cnt64);
    for (int k = threadIdx.x; k <= cnt && !big; k += kThreads) {
      int64_t o = a.off[i0 + k];
      s_off[k] = int32_t(min(o - e0, int64_t(kTile + 1)));
      if (k < cnt) {
        int32_t f = a.F[i0 + k];
        s_src[k] = f;
        s_rs[k] = a.row_ptr[f] - o;
      }
    }
    __syncthreads();
    if (!big) tile_owner_map<kTile, kThreads>(s_off, cnt, s_scan);
    // owner of tile slot j: its frontier row and (row_ptr - off) so that ge = rsk + e
    auto locate = [&](int j, int32_t& srck, int64_t& rsk) {
      const int64_t e = e0 + j;
      if (!big) {
        const int lo = s_own[j];
        srck = s_src[lo];
        rsk = s_rs[lo];
      } else {
        int64_t lo = i0, hi = i0 + cnt64;  // off[lo] <= e < off[hi]
        while (hi - lo > 1) {
          const int64_t mid = (lo + hi) >> 1;
          if (a.off[mid] <= e) lo = mid; else hi = mid;
        }
        srck = a.F[lo];
        rsk = a.row_ptr[srck] - a.off[lo];
      }
    };
    if constexpr (MODE == EXP_ROWS && PK == PK_NONE) {
      if (a.out_vid && a.col_vid && !big) {
        // plain dst-vid copy: all kItems loads of this thread in flight before the stores
        int64_t v[kItems];
#pragma unroll
        for (int r = 0; r < kItems; r++) {
          const int j = threadIdx.x + r * kThreads;
          v[r] = e0 + j < e1 ? __builtin_nontemporal_load(a.col_vid + s_rs[s_own[j]] + e0 + j) : 0;
        }
#pragma unroll
        for (int r = 0; r < kItems; r++) {
          const int64_t e = e0 + threadIdx.x + r * kThreads;
          if (e < e1) __builtin_nontemporal_store(v[r], a.out_vid + e);
        }
        __syncthreads();
        continue;
      }
    }
    if constexpr (MODE == EXP_MARK && PK == PK_NONE) {
      if (!a.mark_check && !a.root_next && !big) {
        // unfiltered marking: the thread's kItems col loads in flight before its byte stores
        int32_t d[kItems];
#pragma unroll
        for (int r = 0; r < kItems; r++) {
          const int j = threadIdx.x + r * kThreads;
          d[r] = e0 + j < e1 ? a.col[s_rs[s_own[j]] + e0 + j] : -1;
        }
#pragma unroll
        for (int r = 0; r < kItems; r++)
          if (d[r] >= 0) a.map[d[r]] = 1;
        __syncthreads();
        continue;
      }
    }
    uint32_t pm = 0;  // ROWS: items of this thread that pass
#pragma unroll 2
    for (int r = 0; r < kItems; r++) {
      const int j = threadIdx.x + r * kThreads;
      const int64_t e = e0 + j;
      const bool valid = e < e1;
      int32_t srck = 0;
      int64_t rsk = 0;
      if (valid) locate(j, srck, rsk);
      const int64_t ge = valid ? rsk + e : 0;
      bool pass = valid;
      int32_t d = 0;
      if (valid && (MODE != EXP_FLAGS || PK == PK_VM)) d = a.col[ge];
      if (PK == PK_FAST && valid) {
        if (fp.present && !fp.present[ge]) {
          if (a.storage) pass = true;
          else {
            atomicAdd(a.err, 1ull);
            pass = false;
          }
        } else {
          pass = fast_cmp(fp.op, load_int(fp.data, fp.width, ge), fp.k);
        }
      } else if (PK == PK_VM && valid) {
        Val v = eval_program(prog, env, ge, int32_t(a.lo) + srck, d);
        if (v.t == VT_ERR) {
          if (a.storage) pass = true;
          else {
            atomicAdd(a.err, 1ull);
            pass = false;
          }
        } else {
          pass = as_bool(v);
        }
      }
      if (MODE == EXP_ROWS && PK == PK_NONE && a.out_vid) {
        // every edge is a row: the row of flattened edge e is row e (no append, no atomics)
        if (valid) a.out_vid[e] = a.col_vid ? a.col_vid[ge] : a.vid_of[a.col[ge]];
      } else if (MODE == EXP_MARK) {
        if (pass) {
          if (a.mark_check) {
            if (a.map[d] == 0) a.map[d] = 1;
          } else {
            a.map[d] = 1;
          }
          if (a.root_next) atomicMin(a.root_next + d, a.root_cur[a.lo + srck]);
        }
      } else if (MODE == EXP_ROWS) {
        if (pass) pm |= 1u << r;
      } else {
        if (valid) a.flags[e] = pass;
      }
    }
    if (MODE == EXP_ROWS && !(PK == PK_NONE && a.out_vid)) {
      // block-aggregated append: one returning atomic per tile (a single counter serialises at
      // ~90 appends / us, so a per-wave append made row output the bottleneck)
      const uint32_t c0 = __popc(pm);
      const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
      uint32_t incl = c0;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(incl, o);
        if (lane >= o) incl += y;
      }
      if (lane == 63) s_wsum[wv] = incl;
      __syncthreads();
      if (threadIdx.x == 0) {
        uint32_t tot = 0;
        for (int w = 0; w < kThreads / 64; w++) {
          const uint32_t x = s_wsum[w];
          s_wsum[w] = tot;
          tot += x;
        }
        s_base = tot ? atomicAdd(a.rows_cnt, (unsigned long long)tot) : 0ull;
      }
      __syncthreads();
      unsigned long long pos = s_base + s_wsum[wv] + (incl - c0);
      while (pm) {
        const int r = __ffs(pm) - 1;
        pm &= pm - 1;
        const int j = threadIdx.x + r * kThreads;
        int32_t srck;
        int64_t rsk;
        locate(j, srck, rsk);
        if (a.out_vid) {
          const int64_t ge = rsk + e0 + j;
          a.out_vid[pos] = a.col_vid ? a.col_vid[ge] : a.vid_of[a.col[ge]];
        } else {
          a.rows_src[pos] = srck;
          a.rows_edge[pos] = rsk + e0 + j;
        }
        pos++;
      }
    }
    __syncthreads();
  }
}

// wave-wide exclusive prefix sum of a per-lane count
__device__ inline uint32_t wave_excl_scan(uint32_t x, uint32_t& total) {
  const int lane = threadIdx.x & 63;
  uint32_t v = x;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    uint32_t y = __shfl_up(v, o);
    if (lane >= o) v += y;
  }
  total = __shfl(v, 63);
  return v - x;
}

__device__ inline unsigned long long wave_sum_u64(unsigned long long x) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o);
  return x;
}

// ---- block-level aggregation helpers (one atomic per block or none: a single global counter
// serialises at ~88 returning atomics/us on MI355X, MI355X_MICROARCH "dequeue") ----------------
constexpr int kAggBlocks = 8192;  // max grid of the aggregated kernels (partials are [block][kSlots])
constexpr int kSlots = 8;
constexpr int kRestMax = 2;  // bu_rest_scan: max 64- / 16-entry chunks of a rest loaded per step

__device__ inline uint32_t block_excl_scan_u32(uint32_t x, uint32_t& total, uint32_t* lds) {
  uint32_t wt;
  uint32_t pre = wave_excl_scan(x, wt);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) lds[w] = wt;
  __syncthreads();
  uint32_t off = 0, tot = 0;
  for (int i = 0; i < int(blockDim.x >> 6); i++) {
    if (i < w) off += lds[i];
    tot += lds[i];
  }
  __syncthreads();
  total = tot;
  return pre + off;
}
__device__ inline void block_store_partials(const unsigned long long* v, int k, unsigned long long* lds,
                                            unsigned long long* partials) {
  const int w = threadIdx.x >> 6;
  const int nw = int(blockDim.x >> 6);
  for (int i = 0; i < k; i++) {
    unsigned long long s = wave_sum_u64(v[i]);
    if ((threadIdx.x & 63) == 0) lds[i * 16 + w] = s;
  }
  __syncthreads();
  if (threadIdx.x < unsigned(kSlots)) {
    unsigned long long s = 0;
    if (threadIdx.x < unsigned(k))
      for (int j = 0; j < nw; j++) s += lds[threadIdx.x * 16 + j];
    partials[size_t(threadIdx.x) * kAggBlocks + blockIdx.x] = s;  // slot-major: coalesced reduce
  }
}
// the block's sums straight into out[0, k) with no-return atomics (option bu_atomic_sums: the
// bottom-up passes then need no k_reduce_partials launch; out starts at zero).
// shards > 1: block b adds into shard b % shards, kShardStride words further per shard, and every
// reader folds the shards (gate_open, k_publish): the adds of one address serialise at the memory
// side (~10 ns each), so 512 blocks ending together added ~4 us to a kernel and 1024 ~10 us
// (tools/atomic_tail, profiles/r12c_atomic_tail.jsonl); with 8 shards ~0.
__device__ inline void block_add_sums(const unsigned long long* v, int k, unsigned long long* lds,
                                      unsigned long long* out, int shards = 1) {
  if (shards > 1) out += size_t(blockIdx.x % unsigned(shards)) * kShardStride;
  const int w = threadIdx.x >> 6;
  const int nw = int(blockDim.x >> 6);
  for (int i = 0; i < k; i++) {
    unsigned long long s = wave_sum_u64(v[i]);
    if ((threadIdx.x & 63) == 0) lds[i * 16 + w] = s;
  }
  __syncthreads();
  if (threadIdx.x < unsigned(k)) {
    unsigned long long s = 0;
    for (int j = 0; j < nw; j++) s += lds[threadIdx.x * 16 + j];
    if (s) __hip_atomic_fetch_add(out + threadIdx.x, s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}
// sums the [kSlots][kAggBlocks] partials into out[0..kSlots) (one block of 1024 threads; all
// kSlots loads of an iteration are independent, so the block has 8 loads in flight per lane
// instead of one dependent chain per slot)
// gate (speculative hops, go_run): when *gate == 0 the kernel does nothing
__global__ __launch_bounds__(1024) void k_reduce_partials(const unsigned long long* partials, int nblocks,
                                                          unsigned long long* out,
                                                          const unsigned long long* gate = nullptr) {
  if (gate && *gate == 0ull) return;
  __shared__ unsigned long long s[kSlots][16];
  unsigned long long a[kSlots];
#pragma unroll
  for (int k = 0; k < kSlots; k++) a[k] = 0;
  for (int b = threadIdx.x; b < nblocks; b += blockDim.x) {
#pragma unroll
    for (int k = 0; k < kSlots; k++) a[k] += partials[size_t(k) * kAggBlocks + b];
  }
  const int w = threadIdx.x >> 6, nw = int(blockDim.x >> 6);
#pragma unroll
  for (int k = 0; k < kSlots; k++) {
    unsigned long long v = wave_sum_u64(a[k]);
    if ((threadIdx.x & 63) == 0) s[k][w] = v;
  }
  __syncthreads();
  if (threadIdx.x < unsigned(kSlots)) {
    unsigned long long v = 0;
    for (int j = 0; j < nw; j++) v += s[threadIdx.x][j];
    out[threadIdx.x] = v;
  }
}

// The rests of a tile's rows: rows still pending after their slab slots scan [rb, re) of their
// transposed row.  Long rests (> kLongRest entries) are scanned by the whole wave, 64 entries a
// step; short ones by 16-lane groups, four rows at a time, so the tile's latency chain is paid
// once per four pending rows instead of once per row.  Both stop at the row's first hit.
template <int PK, int W, int R, typename InFront>
__device__ inline void bu_rest_scan(const bool (&pend)[R], bool (&found)[R], const int64_t (&rb)[R],
                                    const int64_t (&re)[R], const int32_t* __restrict__ tcol, const FastArgs& fp,
                                    int ru, uint32_t (&acc)[6], InFront in_front, const QArgs& q) {
  // entry test: frontier probe + predicate; a packed word settles the predicate from its bucket
  // before the probe, else the value is read after a probe hit
  auto entry = [&](int32_t raw, int64_t ex) -> bool {
    const int32_t g = q_gidx(raw, q);
    if (PK != PK_FAST) return in_front(g);
    const int t = q_test(raw, q);
    if (t == 0) return false;
    if (!in_front(g)) return false;
    if (t == 1) return true;
    acc[5]++;
    return fast_cmp(fp.op, load_w<W>(fp.data, fp.width, ex), fp.k);
  };
  const int lane = threadIdx.x & 63;
  constexpr int kLongRest = 256, GL = 16, NG = 64 / GL;
  unsigned long long pml[R], pms[R];
#pragma unroll
  for (int j = 0; j < R; j++) {
    const bool lng = pend[j] && re[j] - rb[j] > kLongRest;
    pml[j] = __ballot(lng);
    pms[j] = __ballot(pend[j] && !lng);
  }
#pragma unroll
  for (int j = 0; j < R; j++) {
    unsigned long long pm = pml[j];
    while (pm) {
      const int src = __ffsll((long long)pm) - 1;
      pm &= pm - 1;
      const int64_t b = __shfl((long long)rb[j], src), e = __shfl((long long)re[j], src);
      acc[3] += lane == 0;
      bool f = false;
      for (int64_t x = b; x < e && !f; x += 64 * ru) {
        int32_t sr[kRestMax];
#pragma unroll
        for (int u = 0; u < kRestMax; u++) {
          const int64_t ex = x + u * 64 + lane;
          sr[u] = (u < ru && ex < e) ? tcol[ex] : -1;
        }
        bool h = false;
#pragma unroll
        for (int u = 0; u < kRestMax; u++) {
          const int64_t ex = x + u * 64 + lane;
          if (sr[u] < 0) continue;
          acc[4]++;
          if (entry(sr[u], ex)) h = true;
        }
        f = __ballot(h) != 0;
      }
      if (lane == src) found[j] = f;
    }
  }
  {
    const int grp = lane / GL, gl = lane % GL;
    for (;;) {
      int my_j = -1, my_src = 0, taken = 0;
#pragma unroll
      for (int j = 0; j < R; j++) {
        while (pms[j] && taken < NG) {
          const int sidx = __ffsll((long long)pms[j]) - 1;
          if (taken == grp) {
            my_j = j;
            my_src = sidx;
          }
          pms[j] &= pms[j] - 1;
          taken++;
        }
      }
      if (taken == 0) break;
      int64_t b = 0, e = 0;
#pragma unroll
      for (int j = 0; j < R; j++) {
        const int64_t bj = __shfl((long long)rb[j], my_src), ej = __shfl((long long)re[j], my_src);
        if (my_j == j) {
          b = bj;
          e = ej;
        }
      }
      acc[3] += gl == 0 && my_j >= 0;
      bool f = false;
      for (int64_t x = b;; x += GL * ru) {
        const bool act = !f && x < e;
        if (__ballot(act) == 0) break;
        bool h = false;
        if (act) {
          int32_t sr[kRestMax];
#pragma unroll
          for (int u = 0; u < kRestMax; u++) {
            const int64_t ex = x + u * GL + gl;
            sr[u] = (u < ru && ex < e) ? tcol[ex] : -1;
          }
#pragma unroll
          for (int u = 0; u < kRestMax; u++) {
            const int64_t ex = x + u * GL + gl;
            if (sr[u] < 0) continue;
            acc[4]++;
            if (entry(sr[u], ex)) h = true;
          }
        }
        const unsigned long long hb = __ballot(h);
        if (act && ((hb >> (grp * GL)) & ((1ull << GL) - 1ull))) f = true;
      }
#pragma unroll
      for (int g = 0; g < NG; g++) {
        const int sj = __shfl(my_j, g * GL), ss = __shfl(my_src, g * GL);
        const int fg = __shfl(int(f), g * GL);
#pragma unroll
        for (int j = 0; j < R; j++)
          if (sj == j && lane == ss) found[j] = fg != 0;
      }
    }
  }
}

// Bottom-up hop (direction-optimising BFS, Beamer et al.): every owned vertex d looks for an
// in-neighbour (transposed CSR) in the frontier bitmap whose edge passes the predicate, and is
// in the next frontier iff it finds one -- the set getDstIdsFromResp builds
// (GoExecutor.cpp:407-431), with no random writes: the frontier bitmap is read-only and each
// wave writes only its own words.  Two passes: k_bu_lean over the quad slab (the first 4
// hub-first in-neighbours of every transposed row, two 8-byte halves per row), then
// k_bu_rest_lean over the rows it left pending.
// The first pass's instruction stream is cut to what the hop needs (round 2: a general slab
// kernel with per-slot branches and bounds checks was issue-bound at ~2.2 TB/s with no probes):
//  * the slab halves and the out-degrees are padded to whole 128-row tiles at build (pad slots
//    -1, degree 0), so the tile loads carry no bounds checks and no branches;
//  * a lane owns rows l and l + 64 of a 128-row tile (8-byte loads per half), so the two ballots
//    are the tile's two 64-row frontier words as they are;
//  * U tiles per iteration: every slab load of the U tiles is issued, then every probe, then the
//    bit tests (sched_barrier keeps the scheduler from pulling the consumers up to the loads,
//    which put a vmcnt(0) wait behind every probe);
//  * every probe is a buffer load whose offset is out of bounds for a non-candidate slot (the
//    hardware returns 0: no branch);
//  * a non-final hop (PK_NONE) reads the second half only for rows still pending after the
//    first (almost none: hub-first slot 0 is nearly always in a dense frontier), and only the
//    tiles below es.bu_both_tiles (the last row with an in- and an out-edge: one rank numbers
//    such vertices first, snapshot k_class_key); the tiles past it get zero words;
//  * the final hop (PK_FAST) decides each slot by two scalar compares of its packed bucket
//    (QArgs); a frontier hit in an undecided bucket and rows with more than 4 entries are left
//    pending for k_bu_rest_lean (rest_from 0).  A predicate on a column that is not the packed
//    one makes every bucket undecided: the first pass then only clears rows with no frontier
//    in-neighbour among their slots, and the rest pass reads the values.
// Outputs: next-frontier and pending words; partials [0] found, [1] their out-degree sum,
// [2] slab words read, [3] pending rows.
// HUB: the block keeps the first cw words of the bitmap (the highest-out-degree vertices) in LDS
// and answers candidates there from it; the global probe of such a slot is out of bounds.
// Partials [6] / [7]: candidate probes sent to L2 / answered from LDS.
// Speculative hops (go_run): the first pass of a gated hop evaluates the host's direction rule
// itself on the previous hop's device counters -- open iff the previous hop ran (pg), its next
// frontier is non-empty (*n > 0) and its out-degree sum reaches the threshold (*e >= thr) -- and
// block 0 publishes the answer at `gate` for the hop's later kernels and the host (a separate
// one-thread k_gate launch cost ~4.6 us a hop).  e == nullptr: not gated.
// Several ranks (all != nullptr): the previous hop's (n, e) of every rank arrived with this
// hop's frontier allgather (all[2r], all[2r + 1]); the gate sums them and block 0 also publishes
// the sums at gate[2], gate[3] (the host's global counts of the previous hop).
struct GateIn {
  const unsigned long long* e = nullptr;
  const unsigned long long* n = nullptr;
  const unsigned long long* pg = nullptr;
  unsigned long long thr = 0;
  const unsigned long long* all = nullptr;
  int world = 1;
  int shards = 1;  // e / n are sharded block sums (block_add_sums): their shards are summed
};
__device__ inline bool gate_open(const GateIn& gi, unsigned long long* gate) {
  // (plain loads: agent-scope ones at every block's start cost the C3 query 0.405 -> 0.415 ms)
  if (gi.e == nullptr && gi.all == nullptr) return gate == nullptr || *gate != 0ull;
  unsigned long long n, e;
  if (gi.all) {
    n = e = 0ull;
    for (int r = 0; r < gi.world; r++) n += gi.all[2 * r], e += gi.all[2 * r + 1];
  } else {
    n = e = 0ull;
    for (int s = 0; s < gi.shards; s++) n += gi.n[size_t(s) * kShardStride], e += gi.e[size_t(s) * kShardStride];
  }
  const bool open = (gi.pg == nullptr || *gi.pg != 0ull) && n > 0ull && e >= gi.thr;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    __hip_atomic_store(gate, open ? 1ull : 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (gi.all) {
      __hip_atomic_store(gate + 2, n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(gate + 3, e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  return open;
}

template <int PK, int U, int HUB, int STATS, int NT = 0, int SKIP = 0>
__global__ __launch_bounds__(1024, 8) void k_bu_lean(const uint2* __restrict__ lo, const uint2* __restrict__ hi,
                                                     int64_t ntiles, int64_t work_tiles,
                                                     const uint32_t* __restrict__ fbits, uint32_t fb_bytes,
                                                     unsigned long long* __restrict__ nbits,
                                                     unsigned long long* __restrict__ pbits,
                                                     const uint32_t* __restrict__ odeg, QArgs q_arg,
                                                     unsigned long long* __restrict__ partials, int cw,
                                                     const uint8_t* __restrict__ odeg8,
                                                     unsigned long long* gate, GateIn gi, int atomic_sums) {
  if (!gate_open(gi, gate)) return;  // a speculative hop that the direction choice did not take
  __shared__ unsigned long long lds[kSlots * 16];
  extern __shared__ uint32_t s_fb[];  // [0, cw): the bitmap's hub words; [cw]: a zero word
  if (HUB) hub_fill(s_fb, fbits, cw, true);
  const QArgs q = q_sgpr(q_arg);
  constexpr bool FINAL = PK == PK_FAST;
  constexpr int NS = FINAL ? 4 : 2;  // slots probed per row in the first round
  // out-of-bounds reads of the bitmap return 0: a non-candidate's probe, and an empty slot
  // (-1: its gidx bits are all ones, past every vertex, as the build guarantees)
  const __amdgpu_buffer_rsrc_t fb_rs =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t*>(fbits), 0, int(fb_bytes), 0x00020000);
  const uint32_t gmask = q.gmask, ucw = uint32_t(cw);
  const int lane = threadIdx.x & 63;
  const int64_t wave = (int64_t(blockIdx.x) * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = (int64_t(gridDim.x) * blockDim.x) >> 6;
  uint32_t nglob = 0, nhub = 0;
  unsigned long long nfound = 0, npend = 0, nwords = 0;  // wave-uniform
  unsigned long long odsum = 0;
  // One slot word: its probe (global byte offset, out of bounds unless an L2 candidate; LDS
  // index, cw -- the zero word -- unless a hub candidate) and, final hop, its bucket's answer
  // (bit k of `pm` pass, of `um` undecided).  A failing bucket is no candidate; an undecided
  // one is probed too, so only a frontier hit there leaves the row pending.
  auto prep = [&](uint32_t sw, int k, uint32_t& goff, uint32_t& lidx, uint32_t& pm, uint32_t& um) {
    const uint32_t wi = (sw & gmask) >> 5;
    bool cand = true;
    if (FINAL) {
      const int st = q_test(int32_t(sw), q);  // below / above may be -1 (undecided) too
      const bool und = st < 0, pass = st > 0;
      cand = st != 0;
      pm |= pass ? 1u << k : 0u;
      um |= und ? 1u << k : 0u;
    }
    const bool hub = HUB && wi < ucw;
    goff = cand && !hub ? wi * 4u : 0xfffffff0u;
    lidx = cand && hub ? wi : ucw;
    if (STATS) {  // (diagnostic instantiation: the counters' masks cost the hot loop registers)
      nglob += cand && !hub;
      nhub += cand && hub;
    }
  };
  auto bit = [](uint32_t w, uint32_t sw) -> uint32_t { return __builtin_amdgcn_ubfe(w, sw & 31u, 1u); };
  // (a 16-byte-lane layout, lane l holding rows 2l and 2l + 1, measured 104.7 us against 91.6)
  auto row_of = [&](int64_t t, int h) -> int64_t { return t * 128 + lane + 64 * h; };
  for (int64_t t0 = wave * U; t0 < work_tiles; t0 += nwaves * U) {
    uint2 a[U][2], b[U][2];
    uint32_t od[U][2];
    bool v[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      v[u] = t0 + u < work_tiles;
      const int64_t r = (v[u] ? t0 + u : t0) * 128 + lane;  // a past-the-end tile re-reads t0 (discarded)
#pragma unroll
      for (int h = 0; h < 2; h++) {
        if (NT) {  // the slab and degrees are read once per hop: keep L2 for the bitmap probes
          const uint64_t x = __builtin_nontemporal_load(reinterpret_cast<const uint64_t*>(lo + r + 64 * h));
          a[u][h] = make_uint2(uint32_t(x), uint32_t(x >> 32));
          if (FINAL) {
            const uint64_t y = __builtin_nontemporal_load(reinterpret_cast<const uint64_t*>(hi + r + 64 * h));
            b[u][h] = make_uint2(uint32_t(y), uint32_t(y >> 32));
          }
          // 1 B per row; 255 stands for a larger degree, read from odeg where a row is found
          od[u][h] = FINAL ? 1u : uint32_t(__builtin_nontemporal_load(odeg8 + r + 64 * h));
        } else {
          a[u][h] = lo[r + 64 * h];
          if (FINAL) b[u][h] = hi[r + 64 * h];
          od[u][h] = FINAL ? 1u : odeg[r + 64 * h];
        }
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    uint32_t goff[U][2][NS], lidx[U][2][NS], pm[U][2], um[U][2];
#pragma unroll
    for (int u = 0; u < U; u++)
#pragma unroll
      for (int h = 0; h < 2; h++) {
        pm[u][h] = um[u][h] = 0u;
        prep(a[u][h].x, 0, goff[u][h][0], lidx[u][h][0], pm[u][h], um[u][h]);
        prep(a[u][h].y, 1, goff[u][h][1], lidx[u][h][1], pm[u][h], um[u][h]);
        if (FINAL) {
          prep(b[u][h].x, 2, goff[u][h][2], lidx[u][h][2], pm[u][h], um[u][h]);
          prep(b[u][h].y, 3, goff[u][h][3], lidx[u][h][3], pm[u][h], um[u][h]);
        }
      }
    // probes: the LDS reads first (answered in ~100 cycles), then the L2 ones, each into a
    // register of its own, OR-ed afterwards (one of the two is always 0)
    // SKIP: a probe instruction only when some lane of the wave has a candidate for it (most
    // slot registers of a tile need few or no L2 probes: the hub copy answers the hub sources)
    uint32_t lw[U][2][NS], gw[U][2][NS];
    if (HUB) {
#pragma unroll
      for (int u = 0; u < U; u++)
#pragma unroll
        for (int h = 0; h < 2; h++)
#pragma unroll
          for (int k = 0; k < NS; k++) {
            if (SKIP) {
              lw[u][h][k] = 0u;
              if (__ballot(lidx[u][h][k] != ucw)) lw[u][h][k] = s_fb[lidx[u][h][k]];
            } else {
              lw[u][h][k] = s_fb[lidx[u][h][k]];
            }
          }
    }
    // SKIP bit 1 (non-final hops): rows already found through a hub word, and rows without
    // out-edges (they cannot extend the next frontier), send no L2 probe
    bool noprobe[U][2];
#pragma unroll
    for (int u = 0; u < U; u++)
#pragma unroll
      for (int h = 0; h < 2; h++) {
        noprobe[u][h] = false;
        if ((SKIP & 2) && HUB && !FINAL) {
          const uint32_t sw[2] = {a[u][h].x, a[u][h].y};
          bool hf = false;
#pragma unroll
          for (int k = 0; k < NS; k++) hf = hf || bit(lw[u][h][k], sw[k]) != 0u;
          noprobe[u][h] = hf || od[u][h] == 0u;
        }
      }
#pragma unroll
    for (int u = 0; u < U; u++)
#pragma unroll
      for (int h = 0; h < 2; h++)
#pragma unroll
        for (int k = 0; k < NS; k++) {
          if (SKIP) {
            gw[u][h][k] = 0u;
            const uint32_t go = noprobe[u][h] ? 0xfffffff0u : goff[u][h][k];
            if (__ballot(go != 0xfffffff0u)) gw[u][h][k] = __builtin_amdgcn_raw_buffer_load_b32(fb_rs, go, 0, 0);
          } else {
            gw[u][h][k] = __builtin_amdgcn_raw_buffer_load_b32(fb_rs, goff[u][h][k], 0, 0);
          }
        }
    __builtin_amdgcn_sched_barrier(0);
    bool f[U][2], pend[U][2];
#pragma unroll
    for (int u = 0; u < U; u++) {
#pragma unroll
      for (int h = 0; h < 2; h++) {
        const uint32_t sw[4] = {a[u][h].x, a[u][h].y, b[u][h].x, b[u][h].y};
        uint32_t hm = 0u;
#pragma unroll
        for (int k = 0; k < NS; k++) hm |= bit(HUB ? (lw[u][h][k] | gw[u][h][k]) : gw[u][h][k], sw[k]) << k;
        if (FINAL) {
          f[u][h] = (hm & pm[u][h]) != 0u;
          // not found: pending when a frontier hit sits in an undecided bucket, or the row has
          // a fifth entry (slot 3 present)
          pend[u][h] = v[u] && !f[u][h] && (b[u][h].y != 0xffffffffu || (hm & um[u][h]) != 0u);
        } else {
          f[u][h] = hm != 0u && od[u][h] > 0;
          // rows with a third slot to test: live, not found, slot 1 present
          pend[u][h] = v[u] && hm == 0u && od[u][h] > 0 && a[u][h].y != 0xffffffffu;
        }
      }
      nwords += v[u] ? (FINAL ? 8u : 4u) * 64u : 0u;  // every lane's two rows
    }
    if (!FINAL) {
      // second half, lazily: only lanes with a pending row load it (rarely any at all)
      bool anyp = false;
#pragma unroll
      for (int u = 0; u < U; u++) anyp = anyp || pend[u][0] || pend[u][1];
      const unsigned long long anyb = __ballot(anyp);
      if (anyb) {
#pragma unroll
        for (int u = 0; u < U; u++)
#pragma unroll
          for (int h = 0; h < 2; h++) {
            b[u][h] = make_uint2(0xffffffffu, 0xffffffffu);
            if (pend[u][h]) b[u][h] = hi[row_of(t0 + u, h)];
          }
        uint64_t pc = 0;  // rows reading the second half: 2 words each
#pragma unroll
        for (int u = 0; u < U; u++) pc += uint64_t(__popcll(__ballot(pend[u][0])) + __popcll(__ballot(pend[u][1])));
        nwords += 2 * pc;
        uint32_t g2[U][2][2], l2[U][2][2];
#pragma unroll
        for (int u = 0; u < U; u++)
#pragma unroll
          for (int h = 0; h < 2; h++) {
            uint32_t d0 = 0u, d1 = 0u;
            prep(b[u][h].x, 0, g2[u][h][0], l2[u][h][0], d0, d1);
            prep(b[u][h].y, 1, g2[u][h][1], l2[u][h][1], d0, d1);
          }
        uint32_t lv[U][2][2], gv[U][2][2];
        if (HUB) {
#pragma unroll
          for (int u = 0; u < U; u++)
#pragma unroll
            for (int h = 0; h < 2; h++)
#pragma unroll
              for (int k = 0; k < 2; k++) lv[u][h][k] = s_fb[l2[u][h][k]];
        }
#pragma unroll
        for (int u = 0; u < U; u++)
#pragma unroll
          for (int h = 0; h < 2; h++)
#pragma unroll
            for (int k = 0; k < 2; k++) gv[u][h][k] = __builtin_amdgcn_raw_buffer_load_b32(fb_rs, g2[u][h][k], 0, 0);
#pragma unroll
        for (int u = 0; u < U; u++)
#pragma unroll
          for (int h = 0; h < 2; h++) {
            const uint32_t w0 = HUB ? (lv[u][h][0] | gv[u][h][0]) : gv[u][h][0];
            const uint32_t w1 = HUB ? (lv[u][h][1] | gv[u][h][1]) : gv[u][h][1];
            const bool g = (bit(w0, b[u][h].x) | bit(w1, b[u][h].y)) != 0u;
            f[u][h] = f[u][h] || (pend[u][h] && g);
            // still pending: not found in the second half and a fifth entry may exist
            pend[u][h] = pend[u][h] && !g && b[u][h].y != 0xffffffffu;
          }
      } else {
#pragma unroll
        for (int u = 0; u < U; u++) pend[u][0] = pend[u][1] = false;
      }
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
      if (!v[u]) continue;  // wave-uniform
      const int64_t t = t0 + u;
      unsigned long long f0 = __ballot(f[u][0]), f1 = __ballot(f[u][1]);
      unsigned long long p0 = __ballot(pend[u][0]), p1 = __ballot(pend[u][1]);
      if (SKIP & 4) {  // one store: lane 0 the tile's two next-frontier words, lane 1 the pending ones
        if (lane < 2) {
          typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));
          u64x2 vv;
          vv.x = lane ? p0 : f0;
          vv.y = lane ? p1 : f1;
          *reinterpret_cast<u64x2*>((lane ? pbits : nbits) + 2 * t) = vv;
        }
      } else if (lane < 2) {
        nbits[2 * t + lane] = lane ? f1 : f0;
        pbits[2 * t + lane] = lane ? p1 : p0;
      }
      nfound += uint64_t(__popcll(f0) + __popcll(f1));
      npend += uint64_t(__popcll(p0) + __popcll(p1));
      if (!FINAL) {
#pragma unroll
        for (int h = 0; h < 2; h++) {
          uint32_t d = f[u][h] ? od[u][h] : 0u;
          if (NT && d == 255u) d = odeg[row_of(t, h)];  // odeg8 saturates at 255
          odsum += uint64_t(d);
        }
      }
    }
  }
  // tiles past the live rows (non-final hops): nothing can be found there
  for (int64_t t = work_tiles + wave; t < ntiles; t += nwaves)
    if (lane < 2) {
      nbits[2 * t + lane] = 0ull;
      pbits[2 * t + lane] = 0ull;
    }
  // wave-uniform counters enter the block sums once, from lane 0
  if (lane != 0) nfound = npend = nwords = 0;
  unsigned long long acc64[8] = {nfound, odsum, nwords, npend, 0, 0, nglob, nhub};
  if (atomic_sums) block_add_sums(acc64, 8, lds, partials, atomic_sums);
  else block_store_partials(acc64, 8, lds, partials);
}

// Final-hop first pass with the bucket tests as unsigned range checks on the raw slot word
// (k_bu_lean's select chain cost ~19 vector instructions per slot; the r04d PMC pass showed its
// waves busy issuing, 225 VALU per 128-row tile, the HBM stream at 4 TB/s).  FinArgs, host-built
// per query (fin_args): a word is a candidate iff (w - clo) <= cr, it passes iff
// ((w - plo) <= pr) != pinv (the bucket field sits above the gidx bits, so bucket ranges are
// word ranges; the -1 pad word is either no candidate or probes past the bitmap).  A candidate's
// probe byte offset is (w >> 3) & bmask, a non-candidate's kNoProbe; the global probe reads
// through a resource based cw words into the bitmap (hub words wrap out of bounds: the hardware
// returns 0), the LDS probe reads min(offset, 4 cw) (the zero word past the hub copy).
struct FinArgs {
  uint32_t clo = 0, cr = 0xffffffffu, plo = 0, pr = 0xffffffffu;
  uint32_t pinv = 0, bmask = 0xfffffffcu;
};
constexpr uint32_t kNoProbe = 0x0ffffff0u;
// CLS 1: the candidates are every word from clo up and the passing ones every word from plo up
// (pinv 0): the "greater than" compares, the benchmark's.  A non-candidate's offset then comes
// from the sign of w - clo (all ones: past the bitmap and clamped to the zero word) instead of
// a compare and a select, and the pass test is one compare.
// NT: non-temporal slab loads (the slab is read once per hop; the bitmap the probes hit stays
// in L2): 158 -> 148 us at C3.  Measured without gain (r04f/r04g): the next tile's slab loads
// issued behind the current tile's probes, an interleaved 16-byte slab (one load per row), two
// tiles per wave; with no probes at all the slab alone streams at 4.7 TB/s in this loop.
// Round 4 (r06h: 124.9 -> 105.8 us at C3): a probe instruction is issued only when some lane of
// the wave has an L2 candidate in that slot; one 16-byte store of the tile's next / pending
// words; rows a hub word already found send no L2 probe.  Measured without gain and removed
// (r06e-r06h): contiguous tile ranges per wave, the same skip for the LDS reads, 16-byte lanes
// (rows 2l and 2l + 1 per lane), the tile's L2 probes packed into the fewest lanes through an
// LDS scratch.  Round 5, removed in round 6: the 3-slot slab (12 B a row, slot 2 flagging a fourth
// entry in bit 31): this pass 106.9 -> 90.5 us but the rest pass 43 -> 74 us, the query 0.413 ->
// 0.425 ms (r10e).
template <int CLS, int NT>
__global__ __launch_bounds__(1024, 8) void k_bu_fin(const uint2* __restrict__ lo, const uint2* __restrict__ hi,
                                                    int64_t ntiles, int64_t work_tiles,
                                                    const uint32_t* __restrict__ fbits,
                                                    unsigned long long* __restrict__ nbits,
                                                    unsigned long long* __restrict__ pbits, FinArgs fa_arg,
                                                    unsigned long long* __restrict__ partials, int cw,
                                                    uint32_t fb_rest, unsigned long long* gate, GateIn gi,
                                                    int atomic_sums) {
  if (!gate_open(gi, gate)) return;  // a speculative hop that the direction choice did not take
  // dynamic LDS only, so the hub copy starts at address 0 and a probe's LDS address is its
  // clamped byte offset as it is: [0, cw) the bitmap's hub words, [cw] a zero word, then the
  // block's partials scratch
  extern __shared__ uint32_t s_fb[];
  unsigned long long* lds = reinterpret_cast<unsigned long long*>(s_fb + ((cw + 2) & ~1));
  hub_fill(s_fb, fbits, cw, true);
  const uint32_t clo = __builtin_amdgcn_readfirstlane(fa_arg.clo), cr = __builtin_amdgcn_readfirstlane(fa_arg.cr);
  const uint32_t plo = __builtin_amdgcn_readfirstlane(fa_arg.plo), pr = __builtin_amdgcn_readfirstlane(fa_arg.pr);
  const bool pinv = __builtin_amdgcn_readfirstlane(fa_arg.pinv) != 0;
  const uint32_t bmask = __builtin_amdgcn_readfirstlane(fa_arg.bmask);
  const uint32_t cw4 = __builtin_amdgcn_readfirstlane(uint32_t(cw) * 4u);
  // global probes: the bitmap from word cw on (fb_rest bytes); offsets below it (hub words) wrap
  // past the end
  const __amdgpu_buffer_rsrc_t fb_rs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint32_t*>(fbits + cw), 0, int(__builtin_amdgcn_readfirstlane(fb_rest)), 0x00020000);
  // the hub copy is the kernel's only LDS (dynamic, no static arrays), at LDS address 0: a
  // probe's address is its clamped byte offset (a pointer form cost an add per probe)
  typedef const __attribute__((address_space(3))) uint32_t* lds_u32p;
  const int lane = threadIdx.x & 63;
  const int64_t wave = (int64_t(blockIdx.x) * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = (int64_t(gridDim.x) * blockDim.x) >> 6;
  unsigned long long nfound = 0, npend = 0, nwords = 0;  // wave-uniform
  auto ld8 = [&](const uint2* p) -> uint2 {
    if (!NT) return *p;
    const uint64_t x = __builtin_nontemporal_load(reinterpret_cast<const uint64_t*>(p));
    return make_uint2(uint32_t(x), uint32_t(x >> 32));
  };
  constexpr int NS = 4;  // slots per row
  auto load = [&](int64_t t, uint32_t (&sw)[2][4]) {
    const int64_t r = t * 128 + lane;
#pragma unroll
    for (int h = 0; h < 2; h++) {
      const uint2 a = ld8(lo + r + 64 * h);
      sw[h][0] = a.x, sw[h][1] = a.y;
      const uint2 b = ld8(hi + r + 64 * h);
      sw[h][2] = b.x, sw[h][3] = b.y;
    }
  };
  const uint32_t rest_b = __builtin_amdgcn_readfirstlane(fb_rest);
  for (int64_t t = wave; t < work_tiles; t += nwaves) {
    uint32_t sw[2][4];
    load(t, sw);
    __builtin_amdgcn_sched_barrier(0);
    uint32_t ob[2][4];
#pragma unroll
    for (int h = 0; h < 2; h++)
#pragma unroll
      for (int k = 0; k < NS; k++) {
        const uint32_t w = sw[h][k];
        if (CLS == 1)
          ob[h][k] = ((w >> 3) & bmask) | uint32_t(int32_t(w - clo) >> 31);
        else
          ob[h][k] = w - clo <= cr ? (w >> 3) & bmask : kNoProbe;
      }
    uint32_t lw[2][4], gw[2][4];
#pragma unroll
    for (int h = 0; h < 2; h++)
#pragma unroll
      for (int k = 0; k < NS; k++) lw[h][k] = *(lds_u32p)(size_t(min(ob[h][k], cw4)));
    // rows already found through a hub word send no L2 probe (most found rows have a hub
    // in-neighbour in the frontier: their slots' L2 probes were wasted instructions)
    bool hubf[2] = {false, false};
#pragma unroll
    for (int h = 0; h < 2; h++)
#pragma unroll
      for (int k = 0; k < NS; k++) {
        const uint32_t w = sw[h][k];
        const bool pass = CLS == 1 ? w >= plo : (w - plo <= pr) != pinv;
        hubf[h] = hubf[h] || (__builtin_amdgcn_ubfe(lw[h][k], w, 1u) != 0u && pass);
      }
    // a probe instruction only when some lane of the wave has an L2 candidate in that slot
#pragma unroll
    for (int h = 0; h < 2; h++)
#pragma unroll
      for (int k = 0; k < NS; k++) {
        gw[h][k] = 0u;
        if (__ballot(ob[h][k] - cw4 < rest_b && !hubf[h]))
          gw[h][k] = __builtin_amdgcn_raw_buffer_load_b32(fb_rs, hubf[h] ? 0xfffffff0u : ob[h][k] - cw4, 0, 0);
      }
    __builtin_amdgcn_sched_barrier(0);
    bool f[2], pend[2];
#pragma unroll
    for (int h = 0; h < 2; h++) {
      bool fh = false, ah = false;
#pragma unroll
      for (int k = 0; k < NS; k++) {
        const uint32_t w = sw[h][k];
        const bool hit = __builtin_amdgcn_ubfe(lw[h][k] | gw[h][k], w, 1u) != 0u;
        const bool pass = CLS == 1 ? w >= plo : (w - plo <= pr) != pinv;
        fh = fh || (hit && pass);
        ah = ah || hit;
      }
      f[h] = fh;
      // pending: no passing hit, and a hit (then in an undecided bucket) or a fifth entry
      // (slot 3 set)
      pend[h] = !fh && (ah || sw[h][3] != 0xffffffffu);
    }
    unsigned long long f0 = __ballot(f[0]), f1 = __ballot(f[1]);
    unsigned long long p0 = __ballot(pend[0]), p1 = __ballot(pend[1]);
    // one store instruction: lane 0 the two next-frontier words, lane 1 the two pending words
    if (lane < 2) {
      typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));
      u64x2 v;
      v.x = lane ? p0 : f0;
      v.y = lane ? p1 : f1;
      *reinterpret_cast<u64x2*>((lane ? pbits : nbits) + 2 * t) = v;
    }
    nfound += uint64_t(__popcll(f0) + __popcll(f1));
    npend += uint64_t(__popcll(p0) + __popcll(p1));
    nwords += uint64_t(2 * NS) * 64u;
  }
  // tiles past the last row with an in-edge: nothing to find
  for (int64_t t = work_tiles + wave; t < ntiles; t += nwaves)
    if (lane < 2) {
      nbits[2 * t + lane] = 0ull;
      pbits[2 * t + lane] = 0ull;
    }
  if (lane != 0) nfound = npend = nwords = 0;
  unsigned long long acc64[8] = {nfound, 0, nwords, npend, 0, 0, 0, 0};
  if (atomic_sums) block_add_sums(acc64, 8, lds, partials, atomic_sums);
  else block_store_partials(acc64, 8, lds, partials);
}

// Second pass of a bottom-up hop: the rows k_bu_lean left pending.  A wave owns 64 pending-bit
// words spread over the row range (one per lane, nwaves apart, so every wave samples the dense
// hub end and the sparse tail alike) and ranks their pending rows (wave prefix sum of the words'
// popcounts); 64 pending rows at a time, a lane scans its row's entries [row_ptr + rest_from,
// row_ptr + 1) in aligned 8-entry chunks (two 16-byte loads): all chunk loads issued, then all
// probes (buffer loads out of bounds for non-candidates, LDS for hub words), then the tests, as
// in k_bu_lean; a value is read only for a frontier hit in an undecided bucket.  After `steps`
// chunks the rows still pending (long in-edge lists) go to bu_rest_scan (whole wave / 16-lane
// groups).  Found rows OR into the wave's 64 next-frontier words in LDS, merged into nbits by
// the owning lanes (one writer per word).  Partials [0] found, [1] their out-degree sum, [3] rows
// scanned by bu_rest_scan (counted by the first pass), [4] entries read, [5] values read.
constexpr int kLeanChunk = 8;
// The 8 entries [a, a + 8) of a transposed row's chunk, a a multiple of 4: two 16-byte loads
// (one vector-memory instruction per 4 entries instead of one per entry -- the divergent
// per-entry gathers, 64 distinct lines per instruction, held the rest passes at the L1's
// per-line rate); the second only when the row continues past a + 4.  The columns are padded
// so the first load may run past the last row.
__device__ inline void load_chunk8(const int32_t* __restrict__ tcol, int64_t a, int64_t re, bool act,
                                   int32_t (&sv)[kLeanChunk]) {
  int4 x = make_int4(-1, -1, -1, -1), y = x;
  if (act) x = *reinterpret_cast<const int4*>(tcol + a);
  if (act && a + 4 < re) y = *reinterpret_cast<const int4*>(tcol + a + 4);
  sv[0] = x.x, sv[1] = x.y, sv[2] = x.z, sv[3] = x.w;
  sv[4] = y.x, sv[5] = y.y, sv[6] = y.z, sv[7] = y.w;
}
// REC: a pending row's start, in-degree and first kRecEntries entries come from its rest record
// (EdgeSpace::brec, one 64-byte line); rows longer than that continue in tcol from there.
template <int PK, int W, int HUB, int REC>
__global__ __launch_bounds__(1024, 4) void k_bu_rest_lean(const unsigned long long* __restrict__ pbits, int64_t n,
                                                          const int64_t* __restrict__ trp,
                                                          const int32_t* __restrict__ tcol,
                                                          const uint32_t* __restrict__ fbits, uint32_t fb_bytes,
                                                          unsigned long long* nbits,
                                                          const uint32_t* __restrict__ odeg, FastArgs fp, QArgs q_arg,
                                                          unsigned long long* partials, int cw, int ru, int rest_from,
                                                          int steps, unsigned long long* dbg,
                                                          const unsigned long long* __restrict__ gate,
                                                          const uint4* __restrict__ rec, int atomic_sums) {
  if (gate && *gate == 0ull) return;
  const QArgs q = q_sgpr(q_arg);
  __shared__ unsigned long long lds[kSlots * 16];
  __shared__ unsigned long long s_found[16][64];
  extern __shared__ uint32_t s_fb[];
  const unsigned long long t_in = wall_clock64();
  if (HUB) hub_fill(s_fb, fbits, cw, false);
  const unsigned long long t_hub = wall_clock64();
  uint32_t d_rows = 0, d_batches = 0, d_steps = 0, d_scan = 0;
  unsigned long long t_scan = 0;
  const __amdgpu_buffer_rsrc_t fb_rs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint32_t*>(fbits), 0, int(__builtin_amdgcn_readfirstlane(fb_bytes)), 0x00020000);
  auto in_front = [&](int32_t g) -> bool {
    const int32_t wi = g >> 5;
    uint32_t w;
    if (HUB && wi < cw) w = s_fb[wi];
    else w = __builtin_amdgcn_raw_buffer_load_b32(fb_rs, wi * 4, 0, 0);
    return (w >> (g & 31)) & 1u;
  };
  uint32_t acc[6] = {0, 0, 0, 0, 0, 0};
  unsigned long long odsum = 0;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t nwords = (n + 63) / 64;
  const int64_t wave = (int64_t(blockIdx.x) * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = (int64_t(gridDim.x) * blockDim.x) >> 6;
  // a wave's 64 words are spread over the whole row range (word base + l * nwaves + wave for
  // lane l): the pending rows are dense among the hub rows at the low end, and a wave of 64
  // consecutive words there held 5-6 batches while most waves had one (r04h: 57 vs 12 us)
  for (int64_t cbase = 0; cbase + wave < nwords; cbase += nwaves * 64) {
    const int64_t myw = cbase + int64_t(lane) * nwaves + wave;
    const unsigned long long pw = myw < nwords ? pbits[myw] : 0ull;
    s_found[wv][lane] = 0ull;
    uint32_t total;
    const uint32_t pre = wave_excl_scan(uint32_t(__popcll(pw)), total);
    for (uint32_t k0 = 0; k0 < total; k0 += 64) {
      // the (k0 + lane)-th pending row of the chunk: its word (binary search over the lanes'
      // exclusive prefix sums) and the matching set bit of that word
      const uint32_t p = k0 + uint32_t(lane);
      bool pend[1] = {p < total}, found[1] = {false};
      int64_t rb[1] = {0}, re[1] = {0};
      int wsel = 0;
#pragma unroll
      for (int st = 32; st > 0; st >>= 1) {
        const uint32_t pv = __shfl(pre, wsel + st);
        if (wsel + st < 64 && pv <= p) wsel += st;
      }
      const unsigned long long wbits = __shfl((long long)pw, wsel);
      const uint32_t kk = p - __shfl(pre, wsel);  // the kk-th set bit of wbits
      int bit = 0;
#pragma unroll
      for (int st = 32; st > 0; st >>= 1)
        if (uint32_t(__popcll(wbits & ((1ull << (bit + st)) - 1ull))) <= kk) bit += st;
      const int32_t r = int32_t((cbase + int64_t(wsel) * nwaves + wave) * 64 + bit);
      // the entries [base, base + 8) (those in [lo_e, hi_e) are valid): bitmap probes, then the
      // tests; a frontier hit in the constant's bucket reads its value.  Wave-uniform call.
      auto test_chunk = [&](const int32_t(&sv)[kLeanChunk], int64_t base, int64_t lo_e, int64_t hi_e, bool act,
                            bool count) __attribute__((always_inline)) -> bool {
        uint32_t w[kLeanChunk];
        int tq[kLeanChunk];
#pragma unroll
        for (int k = 0; k < kLeanChunk; k++) {
          const bool valid = act && base + k >= lo_e && base + k < hi_e;
          if (count) acc[4] += valid;  // column entries (a record's are in its line)
          tq[k] = PK == PK_FAST ? q_test(sv[k], q) : 1;
          const bool cand = valid && tq[k] != 0;
          const int32_t wi = q_gidx(sv[k], q) >> 5;
          const bool hub = HUB && wi < cw;
          const uint32_t gw = __builtin_amdgcn_raw_buffer_load_b32(fb_rs, cand && !hub ? uint32_t(wi) * 4u : 0xfffffff0u,
                                                                   0, 0);
          if (HUB) {
            const uint32_t lw = s_fb[cand && hub ? wi : 0];
            w[k] = cand && hub ? lw : gw;
          } else {
            w[k] = gw;
          }
        }
        __builtin_amdgcn_sched_barrier(0);
        bool h = false, need = false;
        uint32_t und = 0;
#pragma unroll
        for (int k = 0; k < kLeanChunk; k++) {
          const bool inf = (w[k] >> (uint32_t(sv[k]) & 31u)) & 1u;
          h = h || (inf && tq[k] > 0);
          if (PK == PK_FAST && inf && tq[k] < 0) {
            und |= 1u << k;
            need = true;
          }
        }
        if (PK == PK_FAST && __ballot(need && !h)) {
          // frontier hits in the constant's bucket: the exact value decides
          if (!h) {
#pragma unroll
            for (int k = 0; k < kLeanChunk; k++)
              if ((und >> k) & 1u) {
                acc[5]++;
                h = h || fast_cmp(fp.op, load_w<W>(fp.data, fp.width, base + k), fp.k);
              }
          }
        }
        return h;
      };
      int64_t r0 = 0;  // the row's first entry to test; chunks start at the aligned a <= r0
      if (REC) {
        // the rest record: entries [0, 8) and [8, kRecEntries), then tcol past kRecEntries
        uint4 x0 = make_uint4(0u, 0u, 0u, 0u), x1 = x0, x2 = x0, x3 = x0;
        if (pend[0]) {
          const uint4* rp = rec + size_t(r) * 4;
          x0 = rp[0], x1 = rp[1], x2 = rp[2], x3 = rp[3];
        }
        const int64_t start = int64_t(x0.x) | (int64_t(x0.y & 0xffffu) << 32);
        const uint32_t deg = x0.y >> 16;
        const int64_t rend = start + int64_t(deg < uint32_t(kRecEntries) ? deg : uint32_t(kRecEntries));
        r0 = start + rest_from;
        const int32_t sa[kLeanChunk] = {int32_t(x0.z), int32_t(x0.w), int32_t(x1.x), int32_t(x1.y),
                                        int32_t(x1.z), int32_t(x1.w), int32_t(x2.x), int32_t(x2.y)};
        bool h = test_chunk(sa, start, r0, rend, pend[0], false);
        if (__ballot(pend[0] && !h && deg > 8u)) {
          const int32_t sb[kLeanChunk] = {int32_t(x2.z), int32_t(x2.w), int32_t(x3.x), int32_t(x3.y),
                                          int32_t(x3.z), int32_t(x3.w), -1, -1};
          h = test_chunk(sb, start + 8, r0, rend, pend[0] && !h, false) || h;
        }
        if (h) found[0] = true;
        pend[0] = pend[0] && !h && deg > uint32_t(kRecEntries);
        if (pend[0]) {
          re[0] = deg < 65535u ? start + deg : trp[r + 1];
          r0 = start + kRecEntries;
          rb[0] = r0 & ~int64_t(3);
        }
      } else if (pend[0]) {
        r0 = trp[r] + rest_from;
        re[0] = trp[r + 1];
        rb[0] = r0 & ~int64_t(3);
        pend[0] = r0 < re[0];
      }
      d_batches++;
      d_rows += p < total;
      for (int step = 0; step < steps; step++) {
        if (__ballot(pend[0]) == 0) break;
        d_steps++;
        int32_t sv[kLeanChunk];
        load_chunk8(tcol, rb[0], re[0], pend[0], sv);
        __builtin_amdgcn_sched_barrier(0);
        const bool h = test_chunk(sv, rb[0], r0, re[0], pend[0], true);
        if (h) found[0] = true;
        rb[0] += kLeanChunk;
        pend[0] = pend[0] && !h && rb[0] < re[0];
      }
      const uint32_t a3 = acc[3];
      const unsigned long long ts0 = wall_clock64();
      bu_rest_scan<PK, W, 1>(pend, found, rb, re, tcol, fp, ru, acc, in_front, q);
      t_scan += wall_clock64() - ts0;
      d_scan += acc[3] - a3;
      acc[3] = a3;  // the pending rows were counted by the first pass
      if (found[0]) {
        atomicOr(&s_found[wv][wsel], 1ull << (r & 63));
        acc[0]++;
        if (odeg) odsum += odeg[r];
      }
    }
    __builtin_amdgcn_wave_barrier();
    const unsigned long long fw = s_found[wv][lane];
    if (fw) nbits[myw] |= fw;
    __builtin_amdgcn_wave_barrier();
  }
  if (dbg) {  // diagnostics: per wave timestamps (wall_clock64) and work
    const unsigned long long t_out = wall_clock64();
    uint32_t tr = d_rows, te = acc[4];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) tr += __shfl_xor(tr, o), te += __shfl_xor(te, o);
    if (lane == 0) {
      unsigned long long* d = dbg + wave * 8;
      d[0] = t_in, d[1] = t_hub, d[2] = t_out, d[3] = tr, d[4] = d_batches << 16 | d_steps, d[5] = d_scan, d[6] = te,
      d[7] = t_scan;
    }
  }
  unsigned long long acc64[6] = {acc[0], odsum, acc[2], acc[3], acc[4], acc[5]};
  if (atomic_sums) block_add_sums(acc64, 6, lds, partials, atomic_sums);
  else block_store_partials(acc64, 6, lds, partials);
}

// bitmap -> compacted list.  mode 0: local rows (a top-down hop's frontier; the bitmaps this
// reads already exclude rows without out-edges); mode 1: vids of every set vertex (the DISTINCT
// _dst output).  A tile of 4096 words (131072 vertices) per block-iteration: the words and their
// exclusive offsets go to LDS, one returning atomic reserves the tile's output range, then each
// wave expands two words per step with one lane per bit, so consecutive set bits write
// consecutive output slots (coalesced stores, coalesced vid_of reads).
template <int MODE, int U = 4, int NT = 0>
__global__ __launch_bounds__(1024) void k_bits_compact(const uint32_t* __restrict__ bits, int64_t n, int64_t lo,
                                                       const int64_t* __restrict__ vid_of, void* out,
                                                       unsigned long long* n_out,
                                                       const unsigned long long* gate = nullptr) {
  if (gate && *gate == 0ull) return;
  // one word per thread: a 1024-thread block owns 1024 words (32 K vertices) per iteration, so
  // a 32.8 M-vertex bitmap is ~1000 blocks (4096-word tiles gave ~250: one block per CU, half
  // the resident waves this latency-bound gather needs); one counter atomic per tile
  constexpr int kTileWords = 1024;
  __shared__ uint32_t sw[kTileWords];
  __shared__ uint32_t so[kTileWords];
  __shared__ uint32_t lds[16];
  __shared__ unsigned long long s_base;
  const int64_t nwords = (n + 31) / 32;
  const int64_t ntiles = (nwords + kTileWords - 1) / kTileWords;
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  for (int64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const int64_t w0 = t * kTileWords + int64_t(threadIdx.x);
    uint32_t x = w0 < nwords ? bits[w0] : 0u;
    // bits at or past n (a bitmap's unused tail may hold stale bits) are never listed
    if ((w0 + 1) * 32 > n && w0 < nwords) x &= (1u << uint32_t(n - w0 * 32)) - 1u;
    uint32_t total;
    const uint32_t pre = block_excl_scan_u32(__popc(x), total, lds);
    // the tile's output range: the returning atomic (serialised with every other tile's on the
    // one counter) is issued here and read only after the first step's vid_of loads are out, so
    // its wait overlaps them instead of preceding every load of the tile
    unsigned long long my_base = 0;
    if (threadIdx.x == 0 && total) my_base = atomicAdd(n_out, (unsigned long long)total);
    sw[threadIdx.x] = x;
    so[threadIdx.x] = pre;
    __syncthreads();
    if (total) {  // block-uniform
      // U word pairs per step: the step's U vid_of loads are issued before any of its stores,
      // so each lane keeps U HBM requests in flight instead of one load -> store chain per pair
      unsigned long long base = 0;
      const int half = lane >> 5, bit = lane & 31;
      const int per_wave = kTileWords / int(blockDim.x >> 6);
      for (int j = wv * per_wave; j < (wv + 1) * per_wave; j += 2 * U) {
        bool has[U];
        uint32_t rel[U];
        int64_t val[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
          const int wi = j + 2 * u + half;
          const uint32_t xw = sw[wi];
          has[u] = (xw >> bit) & 1u;
          rel[u] = so[wi] + __popc(xw & ((1u << bit) - 1u));
          const int64_t v = (t * kTileWords + wi) * 32 + bit;
          val[u] = v;
          if (MODE == 1 && has[u]) val[u] = NT ? __builtin_nontemporal_load(vid_of + lo + v) : vid_of[lo + v];
        }
        if (j == wv * per_wave) {  // every wave's first step (same trip count in every wave)
          if (threadIdx.x == 0) s_base = my_base;
          __syncthreads();
          base = s_base;
        }
#pragma unroll
        for (int u = 0; u < U; u++) {
          if (!has[u]) continue;
          if (MODE == 0) static_cast<int32_t*>(out)[base + rel[u]] = int32_t(val[u]);
          else if (NT) __builtin_nontemporal_store(val[u], static_cast<int64_t*>(out) + base + rel[u]);
          else static_cast<int64_t*>(out)[base + rel[u]] = val[u];
        }
      }
    }
    __syncthreads();
  }
}

// deg[i] = outdeg(F[i]); deg[nF] = 0
__global__ void k_degrees(const int32_t* F, int64_t nF, const int64_t* row_ptr, int64_t* deg) {
  for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i <= nF; i += int64_t(gridDim.x) * blockDim.x) {
    if (i == nF) {
      deg[i] = 0;
    } else {
      int32_t f = F[i];
      deg[i] = row_ptr[f + 1] - row_ptr[f];
    }
  }
}

// Compact the owned slice [lo, lo+n) of the byte-map into a frontier list of local indices,
// clearing it.  require_deg: drop vertices without out-edges (they cannot produce rows).
// n_set counts every set byte (the reference's "starts_ non-empty" test, GoExecutor.cpp:392).
__global__ __launch_bounds__(256) void k_compact(uint8_t* map, int64_t lo, int64_t n, const int64_t* row_ptr,
                                                 const uint8_t* row_ok, int require_deg, int32_t* out,
                                                 unsigned long long* n_out, unsigned long long* partials,
                                                 uint16_t* bits, const uint32_t* __restrict__ odeg,
                                                 unsigned long long* sums = nullptr, int shards = 1,
                                                 int64_t own_lo = 0, int64_t own_hi = -1,
                                                 uint16_t* __restrict__ own_bits = nullptr, int64_t n_read = INT64_MAX) {
  // tile = 256 threads x 4 chunks of 16 bytes = 16384 vertices; one returning atomic per tile
  // (1024-thread tiles, a quarter of the atomics, measured slower: 40 -> 47 us at hop 1);
  // n_set (partials[0]), the kept out-degree sum (partials[1]) and the kept count (partials[2])
  // go to per-block partials.  out == nullptr: bitmap and counts only, no list (the list is built
  // from the bitmap later if a top-down hop needs it: the per-tile list atomics were most of
  // this kernel's time - 4096 tiles on one counter at RMAT-26).  own_lo < own_hi: the kept count
  // and out-degree sum of the vertices in [own_lo, own_hi) too (slots 3, 4: a rank's share of a
  // whole-space frontier, go_rep1; own_lo a multiple of 16), and own_bits (if set) gets that
  // range's bitmap.  n_read: past it the map is known to be zero (no dst of the hop's edge type
  // lies there: the class-ordered numbering puts the vertices without in-edges last), so those
  // chunks are not read and their bitmap words are written as zero
  __shared__ uint32_t lds[16];
  __shared__ unsigned long long lds64[kSlots * 16];
  __shared__ unsigned long long s_base;
  const int64_t nchunks = (n + 15) / 16;
  const int64_t rchunks = min(nchunks, (n_read + 15) / 16);  // chunks whose map bytes are read
  const int64_t tile = int64_t(blockDim.x) * 4;
  const int64_t ntiles = (nchunks + tile - 1) / tile;
  unsigned long long acc[5] = {0, 0, 0, 0, 0};
  const int nsum = own_lo < own_hi ? 5 : 3;
  // bitmap-only compaction (out == nullptr, the bottom-up path): the next tile's chunk loads are
  // issued with this one's (its map words stay in registers for the next round), so a block waits
  // one map latency per round of tiles, not one per tile
  const bool pre = out == nullptr;
  uint4 wn[4];
  if (pre) {
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const int64_t ch = int64_t(blockIdx.x) * tile + q * int64_t(blockDim.x) + threadIdx.x;
      wn[q] = int64_t(blockIdx.x) < ntiles && ch < rchunks ? reinterpret_cast<const uint4*>(map + lo)[ch]
                                                            : make_uint4(0, 0, 0, 0);
    }
  }
  for (int64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    uint32_t keep[4];
    uint32_t cnt = 0;
    // the tile's four chunk loads issued together (the clearing stores below would otherwise
    // order each load behind the previous chunk's store)
    uint4 wq[4];
    if (pre) {
      const int64_t tn = t + gridDim.x;
#pragma unroll
      for (int q = 0; q < 4; q++) {
        wq[q] = wn[q];
        const int64_t ch = tn * tile + q * int64_t(blockDim.x) + threadIdx.x;
        wn[q] = tn < ntiles && ch < rchunks ? reinterpret_cast<const uint4*>(map + lo)[ch] : make_uint4(0, 0, 0, 0);
      }
    } else {
#pragma unroll
      for (int q = 0; q < 4; q++) {
        const int64_t ch = t * tile + q * int64_t(blockDim.x) + threadIdx.x;
        wq[q] = ch < rchunks ? reinterpret_cast<const uint4*>(map + lo)[ch] : make_uint4(0, 0, 0, 0);
      }
    }
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const int64_t ch = t * tile + q * int64_t(blockDim.x) + threadIdx.x;
      const uint4 w = wq[q];
      const uint32_t words[4] = {w.x, w.y, w.z, w.w};
      uint32_t setmask = 0;
#pragma unroll
      for (int a = 0; a < 4; a++)
#pragma unroll
        for (int b = 0; b < 4; b++)
          if ((words[a] >> (8 * b)) & 0xff) setmask |= 1u << (a * 4 + b);
      uint32_t keepmask = setmask;
      const unsigned long long deg0 = acc[1];
      if (require_deg && setmask && odeg) {
        // out-degrees (0 where row_ok == 0) of the chunk's 16 vertices: four 16-byte loads issued
        // together, instead of a dependent row_ptr pair per set vertex (hub tiles are dense)
        uint32_t dg[16];
        if ((ch + 1) * 16 <= n) {
          const uint4* p4 = reinterpret_cast<const uint4*>(odeg + ch * 16);
#pragma unroll
          for (int a = 0; a < 4; a++) {
            const uint4 v4 = p4[a];
            dg[a * 4 + 0] = v4.x, dg[a * 4 + 1] = v4.y, dg[a * 4 + 2] = v4.z, dg[a * 4 + 3] = v4.w;
          }
        } else {
#pragma unroll
          for (int j = 0; j < 16; j++) dg[j] = ch * 16 + j < n ? odeg[ch * 16 + j] : 0u;
        }
#pragma unroll
        for (int j = 0; j < 16; j++) {
          if (!((setmask >> j) & 1u)) continue;
          if (dg[j] == 0) keepmask &= ~(1u << j);
          else acc[1] += dg[j];
        }
      } else if (require_deg && setmask) {
        for (uint32_t m = setmask; m; m &= m - 1) {
          const int j = __ffs(m) - 1;
          const int64_t v = ch * 16 + j;
          const int64_t dg = row_ptr[v + 1] - row_ptr[v];
          if (dg == 0 || (row_ok && !row_ok[v])) keepmask &= ~(1u << j);
          else acc[1] += (unsigned long long)dg;
        }
      }
      if (bits && ch < nchunks) bits[ch] = uint16_t(keepmask);  // frontier bitmap for bottom-up
      if (setmask) reinterpret_cast<uint4*>(map + lo)[ch] = make_uint4(0, 0, 0, 0);
      acc[0] += __popc(setmask);
      if (ch * 16 + lo >= own_lo && ch * 16 + lo < own_hi) {
        acc[3] += __popc(keepmask), acc[4] += acc[1] - deg0;
        if (own_bits) own_bits[ch - (own_lo - lo) / 16] = uint16_t(keepmask);
      }
      keep[q] = keepmask;
      cnt += __popc(keepmask);
    }
    acc[2] += cnt;
    if (!out) continue;  // uniform: no block barrier is skipped by part of the block
    uint32_t total;
    const uint32_t pre = block_excl_scan_u32(cnt, total, lds);
    if (threadIdx.x == 0) s_base = total ? atomicAdd(n_out, (unsigned long long)total) : 0ull;
    __syncthreads();
    unsigned long long p = s_base + pre;
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const int64_t ch = t * tile + q * int64_t(blockDim.x) + threadIdx.x;
      for (uint32_t m = keep[q]; m; m &= m - 1) out[p++] = int32_t(ch * 16 + (__ffs(m) - 1));
    }
    __syncthreads();
  }
  // sums (zeroed by the caller): the block sums added there, no k_reduce_partials launch
  if (sums) block_add_sums(acc, nsum, lds64, sums, shards);
  else block_store_partials(acc, nsum, lds64, partials);
}

// starts (gidx) -> deduplicated frontier: bitmap bits (set once, by a returning atomicOr) and
// list of the starts with out-edges; Kd[0] list length, Kd[12] vertices, Kd[13] out-degree sum
// (the counters launch_compact leaves)
__global__ void k_starts_bits(const int32_t* g, int64_t n, int64_t lo, int64_t hi, const uint32_t* odeg,
                              uint32_t* bits, int32_t* out, unsigned long long* Kd) {
  const int64_t stride = int64_t(gridDim.x) * blockDim.x;
  const int64_t rounds = (n + stride - 1) / stride;
  for (int64_t r = 0; r < rounds; r++) {
    const int64_t i = r * stride + blockIdx.x * int64_t(blockDim.x) + threadIdx.x;
    bool keep = false;
    int32_t loc = 0;
    uint32_t od = 0;
    if (i < n) {
      const int32_t x = g[i];
      if (x >= lo && x < hi) {
        loc = int32_t(x - lo);
        od = odeg[loc];
        const uint32_t bit = 1u << (loc & 31);
        keep = od && !(atomicOr(bits + (loc >> 5), bit) & bit);
      }
    }
    const int64_t s = wave_append(Kd, keep);
    if (keep) {
      out[s] = loc;
      atomicAdd(Kd + 12, 1ull);
      atomicAdd(Kd + 13, (unsigned long long)od);
    }
  }
}

// starts (gidx) -> mark owned in the byte-map (dedup path) or list them (steps == 1 path)
// One-block start frontier for a few starts (ns <= kSmallStarts, one rank), everything the
// first top-down hop needs in one launch instead of a lookup, three memsets, the bitmap dedup, a
// degree pass, a scan and a counter round trip: zero the query counters Kd[0, 256), look the
// start vids up (gidx -> g), dedup through the start words of the frontier bitmap (only those
// words are cleared: a top-down first hop never reads the rest, k_compact rewrites it all), keep
// starts with out-edges (row_ok) as the list F, write its exclusive degree scan to off[0, ns]
// (entries past the list: degree 0, row 0) and the counts: Kd[40] list length, Kd[41] its
// out-degree sum, Kd[30] the degree sum over every start with duplicates (hop-1 rows of a
// query without DISTINCT rescan duplicate starts, QueryBaseProcessor.inl:462-505).
constexpr int kSmallStarts = 4096;
__global__ __launch_bounds__(1024) void k_starts_small(const int64_t* __restrict__ vids, int32_t ns, const int64_t* keys,
                                                       const int32_t* vals, uint64_t mask, bool has_min,
                                                       int32_t min_gidx, int32_t* __restrict__ g, int64_t lo,
                                                       int64_t hi, const int64_t* __restrict__ row_ptr,
                                                       const uint8_t* __restrict__ row_ok, uint32_t* bits,
                                                       int32_t* __restrict__ F, int64_t* __restrict__ off,
                                                       unsigned long long* __restrict__ Kd,
                                                       int32_t* __restrict__ tile_row = nullptr) {
  __shared__ int32_t s_loc[kSmallStarts];
  __shared__ int64_t s_off[kSmallStarts];  // the kept starts' exclusive degree offsets
  __shared__ unsigned long long s_w[32];  // [0, 16): per-wave counts, [16, 32): per-wave degree sums
  __shared__ unsigned long long s_carry[2];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  for (int i = tid; i < int(kShardStride) * kSumShards; i += blockDim.x) Kd[i] = 0ull;  // every shard
  for (int i = tid; i < ns; i += blockDim.x) {
    const int32_t x = ht_lookup(keys, vals, mask, vids[i], has_min, min_gidx);
    g[i] = x;
    int32_t loc = -1;
    if (x >= lo && x < hi && (row_ok == nullptr || row_ok[x - lo]) && row_ptr[x - lo + 1] > row_ptr[x - lo])
      loc = int32_t(x - lo);
    s_loc[i] = loc;
    if (loc >= 0) bits[loc >> 5] = 0u;
  }
  if (tid < 2) s_carry[tid] = 0ull;
  __syncthreads();
  unsigned long long scanned = 0;  // every start's degree, duplicates included
  for (int i0 = 0; i0 < ns; i0 += blockDim.x) {
    const int i = i0 + tid;
    const int32_t loc = i < ns ? s_loc[i] : -1;
    const unsigned long long d = loc >= 0 ? (unsigned long long)(row_ptr[loc + 1] - row_ptr[loc]) : 0ull;
    scanned += d;
    bool keep = false;
    if (loc >= 0) {
      const uint32_t bit = 1u << (loc & 31);
      keep = !(atomicOr(bits + (loc >> 5), bit) & bit);
    }
    // block prefix of (kept count, kept degree): wave inclusive scans, then the wave totals
    unsigned long long kc = keep ? 1ull : 0ull, kd = keep ? d : 0ull;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const unsigned long long a = __shfl_up(kc, o), b = __shfl_up(kd, o);
      if (lane >= o) kc += a, kd += b;
    }
    if (lane == 63) s_w[wv] = kc, s_w[16 + wv] = kd;
    __syncthreads();
    unsigned long long bc = s_carry[0], bd = s_carry[1], tc = 0, td = 0;
    for (int w = 0; w < int(blockDim.x >> 6); w++) {
      const unsigned long long wc = s_w[w], wd = s_w[16 + w];
      if (w < wv) bc += wc, bd += wd;
      tc += wc, td += wd;
    }
    if (keep) {
      const unsigned long long pos = bc + kc - 1;
      F[pos] = loc;
      off[pos] = int64_t(bd + kd - d);
      s_off[pos] = int64_t(bd + kd - d);
    }
    __syncthreads();
    if (tid == 0) s_carry[0] += tc, s_carry[1] += td;
    __syncthreads();
  }
  const unsigned long long nF = s_carry[0], E = s_carry[1];
  for (int i = int(nF) + tid; i <= ns; i += blockDim.x) {
    if (i < ns) F[i] = 0;
    off[i] = int64_t(E);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) scanned += __shfl_xor(scanned, o);
  if (lane == 0) s_w[wv] = scanned;
  __syncthreads();
  if (tid == 0) {
    unsigned long long t = 0;
    for (int w = 0; w < int(blockDim.x >> 6); w++) t += s_w[w];
    Kd[40] = nF;
    Kd[41] = E;
    Kd[30] = t;
  }
  // the hop-1 expansion's tile-row table (k_tile_rows' rule) from the offsets just written: one
  // launch and its gap less before the first hop.  Tile t's row is the last kept start whose
  // range begins at or before t * kTile (every kept start has out-edges, so the ranges tile
  // [0, E)): one thread per tile, a binary search of the offsets in LDS (a thread per start
  // walked a hub seed's hundreds of tiles alone)
  if (tile_row && nF > 0) {
    const int64_t nT = (int64_t(E) + kTile - 1) / kTile;
    for (int64_t t = tid; t < nT; t += blockDim.x) {
      const int64_t e0 = t * kTile;
      int k = 0;
      for (int st = kSmallStarts / 2; st > 0; st >>= 1)
        if (k + st < int(nF) && s_off[k + st] <= e0) k += st;
      tile_row[t] = k;
    }
  }
}

__global__ void k_mark_gidx(const int32_t* g, int64_t n, int64_t lo, int64_t hi, uint8_t* map) {
  for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < n; i += int64_t(gridDim.x) * blockDim.x) {
    int32_t x = g[i];
    if (x >= lo && x < hi) map[x] = 1;
  }
}
__global__ void k_list_starts(const int32_t* g, int64_t n, int64_t lo, int64_t hi, const int64_t* row_ptr,
                              const uint8_t* row_ok, int32_t* out, unsigned long long* n_out) {
  // order-preserving is not required (multiset results); wave-aggregated append
  int64_t stride = int64_t(gridDim.x) * blockDim.x;
  int64_t rounds = (n + stride - 1) / stride;
  for (int64_t r = 0; r < rounds; r++) {
    int64_t i = r * stride + blockIdx.x * int64_t(blockDim.x) + threadIdx.x;
    bool keep = false;
    int32_t loc = 0;
    if (i < n) {
      int32_t x = g[i];
      if (x >= lo && x < hi) {
        loc = int32_t(x - lo);
        keep = row_ptr[loc + 1] > row_ptr[loc] && (row_ok == nullptr || row_ok[loc]);
      }
    }
    int64_t s = wave_append(n_out, keep);
    if (keep) out[s] = loc;
  }
}
// rows the hop-1 scans return for a start list WITH its duplicates: each duplicate start rescans
// its prefix (GoExecutor.cpp:98-104 dedups the starts only under DISTINCT), so the edges scanned
// (the TEPS numerator, and what the reference's storage returns) count them, while the device
// expands the deduplicated frontier (P12 makes the next frontier a set either way)
__global__ void k_starts_degree(const int32_t* g, int64_t n, int64_t lo, int64_t hi, const int64_t* row_ptr,
                                const uint8_t* row_ok, unsigned long long* sum) {
  unsigned long long acc = 0;
  for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < n; i += int64_t(gridDim.x) * blockDim.x) {
    const int32_t x = g[i];
    if (x >= lo && x < hi && (row_ok == nullptr || row_ok[x - lo])) acc += (unsigned long long)(row_ptr[x - lo + 1] - row_ptr[x - lo]);
  }
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
  if ((threadIdx.x & 63) == 0 && acc) atomicAdd(sum, acc);
}

// ---- multi-rank frontier exchange ----------------------------------------------------------
// global byte-map -> 32-bit mark words (one word per thread), clearing the map
__global__ void k_map_to_bits(uint8_t* map, int64_t n, uint32_t* bits) {
  const int64_t nw = (n + 31) / 32;
  for (int64_t w = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; w < nw; w += int64_t(gridDim.x) * blockDim.x) {
    uint4* p = reinterpret_cast<uint4*>(map + w * 32);
    uint4 a = p[0], b = p[1];
    const uint32_t x[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    uint32_t m = 0;
#pragma unroll
    for (int i = 0; i < 8; i++)
#pragma unroll
      for (int k = 0; k < 4; k++)
        if ((x[i] >> (8 * k)) & 0xff) m |= 1u << (i * 4 + k);
    bits[w] = m;
    if (m) {
      p[0] = make_uint4(0, 0, 0, 0);
      p[1] = make_uint4(0, 0, 0, 0);
    }
  }
}
// OR the [G][nw] received mark words and set the owned slice of the byte-map
__global__ void k_or_segments_to_map(const uint32_t* recv, int G, int64_t nw, uint8_t* map_lo) {
  for (int64_t w = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; w < nw; w += int64_t(gridDim.x) * blockDim.x) {
    uint32_t m = 0;
    for (int p = 0; p < G; p++) m |= recv[size_t(p) * size_t(nw) + size_t(w)];
    for (; m; m &= m - 1) map_lo[w * 32 + (__ffs(m) - 1)] = 1;
  }
}
// several ranks, a top-down hop whose next frontier goes on as a bitmap (bottom-up hops): OR the
// [G][nw] received mark words straight into the owned frontier bitmap, dropping vertices without
// out-edges, with the compaction's counts -- sums[0] vertices set, [1] kept out-degree sum,
// [2] kept vertices (k_compact's Kd[12, 15)) -- instead of writing the marks into the byte map
// and compacting it again (k_or_segments_to_map + k_compact: 6 + 29 us at RMAT-26, r12h)
__global__ __launch_bounds__(256) void k_or_segments_bits(const uint32_t* __restrict__ recv, int G, int64_t nw,
                                                          const uint32_t* __restrict__ odeg, uint32_t* bits,
                                                          unsigned long long* sums) {
  __shared__ unsigned long long lds[kSlots * 16];
  unsigned long long acc[3] = {0, 0, 0};
  for (int64_t w = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; w < nw; w += int64_t(gridDim.x) * blockDim.x) {
    uint32_t m = 0;
    for (int p = 0; p < G; p++) m |= recv[size_t(p) * size_t(nw) + size_t(w)];
    uint32_t keep = m;
    if (m) {
      // the word's 32 out-degrees as eight 16-byte loads issued together (odeg is padded to whole
      // 128-row tiles), not one dependent load per set bit (24 us at RMAT-26 one rank, r12i)
      uint32_t dg[32];
      const uint4* p4 = reinterpret_cast<const uint4*>(odeg + w * 32);
#pragma unroll
      for (int a = 0; a < 8; a++) {
        const uint4 v = p4[a];
        dg[4 * a] = v.x, dg[4 * a + 1] = v.y, dg[4 * a + 2] = v.z, dg[4 * a + 3] = v.w;
      }
#pragma unroll
      for (int j = 0; j < 32; j++) {
        const uint32_t d = (m >> j) & 1u ? dg[j] : 0u;
        if ((m >> j) & 1u && d == 0) keep &= ~(1u << j);
        acc[1] += d;
      }
    }
    bits[w] = keep;
    acc[0] += __popc(m);
    acc[2] += __popc(keep);
  }
  block_add_sums(acc, 3, lds, sums);
}
// DISTINCT over rows with several ranks: rows are shuffled to rank hash(row) % G first
__global__ void k_flag_dest(const uint32_t* dest, int64_t n, uint32_t p, uint8_t* flag) {
  for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < n; i += int64_t(gridDim.x) * blockDim.x)
    flag[i] = dest[i] == p;
}

// gidx list (local indices + lo) -> vids
__global__ void k_local_to_vid(const int32_t* loc, int64_t n, int64_t lo, const int64_t* vid_of, int64_t* out) {
  for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < n; i += int64_t(gridDim.x) * blockDim.x)
    out[i] = vid_of[lo + loc[i]];
}

// YIELD materialisation: one program per output column
struct ColOut {
  void* data;
  int32_t type;  // VT_*
  int64_t* len;  // VT_STR: byte length per row (`data` holds the device address of the bytes)
};
constexpr int kMaxYields = 16;
struct YieldArgs {
  int32_t ncols;
  ColOut cols[kMaxYields];
};
__global__ void k_materialize(const int32_t* rows_src, const int64_t* rows_edge, int64_t n, const Program* progs,
                              YieldArgs ya, EvalEnv env, int64_t lo, unsigned long long* err) {
  for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < n; i += int64_t(gridDim.x) * blockDim.x) {
    const int64_t ge = rows_edge[i];
    const int32_t sg = int32_t(lo) + rows_src[i];
    const int32_t dg = env.col[ge];
    for (int c = 0; c < ya.ncols; c++) {
      Val v = eval_program(progs + c, env, ge, sg, dg);
      if (v.t == VT_ERR || v.t != ya.cols[c].type) {
        atomicAdd(err, 1ull);
        continue;
      }
      if (v.t == VT_BOOL) static_cast<uint8_t*>(ya.cols[c].data)[i] = uint8_t(v.b != 0);
      else static_cast<int64_t*>(ya.cols[c].data)[i] = v.b;
      if (v.t == VT_STR) ya.cols[c].len[i] = v.len;
    }
  }
}
// STRING YIELD columns: (address, length) per row -> packed bytes at exclusive-scan offsets
__global__ void k_str_pack(const int64_t* addr, const int64_t* off, int64_t n, uint8_t* out) {
  for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < n; i += int64_t(gridDim.x) * blockDim.x) {
    const uint8_t* s = reinterpret_cast<const uint8_t*>(uintptr_t(addr[i]));
    const int64_t len = off[i + 1] - off[i];
    for (int64_t j = 0; j < len; j++) out[off[i] + j] = s[j];
  }
}
// fast path for YIELD e._dst (the default YIELD)
__global__ void k_yield_dst(const int64_t* rows_edge, int64_t n, const int32_t* col, const int64_t* vid_of,
                            int64_t* out) {
  for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < n; i += int64_t(gridDim.x) * blockDim.x)
    out[i] = vid_of[col[rows_edge[i]]];
}

// DISTINCT over materialised rows (GoExecutor.cpp:638-646 dedups by encoded row bytes; for the
// fixed-width VID/DOUBLE/BOOL columns the engine emits, equal bytes == equal 64-bit words).
__device__ inline uint64_t row_hash(const YieldArgs& ya, int64_t i) {
  uint64_t h = 0x12345678ull;
  for (int c = 0; c < ya.ncols; c++) {
    uint64_t w;
    if (ya.cols[c].type == VT_STR) {  // by content: equal strings may sit at different addresses
      const uint8_t* p = reinterpret_cast<const uint8_t*>(uintptr_t(static_cast<const int64_t*>(ya.cols[c].data)[i]));
      const int64_t len = ya.cols[c].len[i];
      w = 0xcbf29ce484222325ull ^ uint64_t(len);
      for (int64_t k = 0; k < len; k++) w = (w ^ p[k]) * 0x100000001b3ull;
    } else {
      w = ya.cols[c].type == VT_BOOL ? static_cast<const uint8_t*>(ya.cols[c].data)[i]
                                     : uint64_t(static_cast<const int64_t*>(ya.cols[c].data)[i]);
    }
    h = splitmix64(h ^ w);
  }
  return h;
}
__device__ inline bool row_eq(const YieldArgs& ya, int64_t i, int64_t j) {
  for (int c = 0; c < ya.ncols; c++) {
    if (ya.cols[c].type == VT_STR) {
      const int64_t li = ya.cols[c].len[i];
      if (li != ya.cols[c].len[j]) return false;
      const uint8_t* a = reinterpret_cast<const uint8_t*>(uintptr_t(static_cast<const int64_t*>(ya.cols[c].data)[i]));
      const uint8_t* b = reinterpret_cast<const uint8_t*>(uintptr_t(static_cast<const int64_t*>(ya.cols[c].data)[j]));
      for (int64_t k = 0; k < li; k++)
        if (a[k] != b[k]) return false;
    } else if (ya.cols[c].type == VT_BOOL) {
      if (static_cast<const uint8_t*>(ya.cols[c].data)[i] != static_cast<const uint8_t*>(ya.cols[c].data)[j]) return false;
    } else if (static_cast<const int64_t*>(ya.cols[c].data)[i] != static_cast<const int64_t*>(ya.cols[c].data)[j]) {
      return false;
    }
  }
  return true;
}
__global__ void k_row_dedup(YieldArgs ya, int64_t n, long long* table, uint64_t mask, uint8_t* keep) {
  for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < n; i += int64_t(gridDim.x) * blockDim.x) {
    uint64_t h = row_hash(ya, i) & mask;
    bool k = true;
    while (true) {
      long long prev = atomicCAS(reinterpret_cast<unsigned long long*>(table + h), ~0ull, (unsigned long long)i);
      if (prev == -1) break;
      if (row_eq(ya, prev, i)) {
        k = false;
        break;
      }
      h = (h + 1) & mask;
    }
    keep[i] = k;
  }
}

__global__ void k_row_dest(YieldArgs ya, int64_t n, uint32_t G, uint32_t* dest) {
  for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < n; i += int64_t(gridDim.x) * blockDim.x)
    dest[i] = uint32_t((row_hash(ya, i) >> 17) % G);
}

// input table index: gidx of starts[i] -> i, the LAST row of a vid winning
// (InterimResult::buildIndex overwrites vidToRowIndex_ row by row, InterimResult.cpp:158-160)
__global__ void k_input_index(const int32_t* sg, int64_t n, int32_t* keys, int32_t* rows, uint32_t mask) {
  for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < n; i += int64_t(gridDim.x) * blockDim.x) {
    const int32_t g = sg[i];
    if (g < 0) continue;
    uint32_t h = gidx_hash(g) & mask;
    while (true) {
      const int32_t prev = atomicCAS(keys + h, -1, g);
      if (prev == -1 || prev == g) {
        atomicMax(rows + h, int32_t(i));
        break;
      }
      h = (h + 1) & mask;
    }
  }
}

// roots of the starts: rank of the start's vid among the distinct start vids (host-computed),
// so a min over ranks is the min over root vids; tab[rank] = the start's gidx
__global__ void k_root_init(const int32_t* sg, const int32_t* srank, int64_t n, int32_t* root, int32_t* tab) {
  for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < n; i += int64_t(gridDim.x) * blockDim.x) {
    const int32_t g = sg[i];
    if (g < 0) continue;
    root[g] = srank[i];
    tab[srank[i]] = g;
  }
}

// ------------------------------------------------------------------------------------------
// host drivers
// ------------------------------------------------------------------------------------------
namespace {

EvalEnv make_env(Ctx& c, EdgeSpace& es, Csr& csr, int32_t etype) {
  EvalEnv env{};
  env.nprops = int32_t(csr.props.size());
  if (env.nprops && !csr.prop_table.p) {
    std::vector<PropDev> tab;
    for (const PropCol& p : csr.props)
      tab.push_back(PropDev{p.type, p.width, p.data.p, p.present.as<uint8_t>(), p.str_off.as<int64_t>(),
                            p.str_bytes.as<uint8_t>()});
    csr.prop_table.alloc(sizeof(PropDev) * tab.size());
    NBG_HIP(hipMemcpy(csr.prop_table.p, tab.data(), sizeof(PropDev) * tab.size(), hipMemcpyHostToDevice));
  }
  env.props = csr.prop_table.as<PropDev>();
  if (!c.tag_refs.empty() && !c.tag_table.p) {
    std::vector<PropDev> tab;
    for (auto& kv : c.tags)
      for (const PropCol& p : kv.second.cols)
        tab.push_back(PropDev{p.type, p.width, p.data.p, p.present.as<uint8_t>(), p.str_off.as<int64_t>(),
                              p.str_bytes.as<uint8_t>(), kv.second.part.as<int32_t>()});
    c.tag_table.alloc(sizeof(PropDev) * tab.size());
    NBG_HIP(hipMemcpy(c.tag_table.p, tab.data(), sizeof(PropDev) * tab.size(), hipMemcpyHostToDevice));
  }
  env.tprops = c.tag_table.as<PropDev>();
  env.etype = etype;
  env.vid_of = c.vid_of.as<int64_t>();
  env.col = csr.col.as<int32_t>();
  env.rank = csr.rank.as<int64_t>();
  return env;
}

template <typename T>
void exclusive_scan_dev(Ctx& c, const T* in, T* out, int64_t n) {
  size_t tb = 0;
  NBG_HIP(rocprim::exclusive_scan(nullptr, tb, in, out, T(0), size_t(n), rocprim::plus<T>(), c.stream));
  c.ws_tmp.ensure(tb);
  NBG_HIP(rocprim::exclusive_scan(c.ws_tmp.p, tb, in, out, T(0), size_t(n), rocprim::plus<T>(), c.stream));
}

struct Counters {
  unsigned long long* d;  // device counters
  unsigned long long* h;  // pinned host mirror (64 entries)
};

}  // namespace

// Copies n device counters into coherent host memory, then the sequence word: each thread's
// store is made visible system-wide before thread 0 publishes the sequence number.
// One wave copies the words (a lane per word, loads in flight together), and lane 0 publishes
// the sequence with one system-scope release store: one system fence (an L2 write-back) instead
// of one per word.  A single wave, so the release's wait on the wave's outstanding stores covers
// every copy.  (One thread copying every word waited on each load in turn: ~10 us more.)
__global__ void k_publish(const unsigned long long* src, int n, unsigned long long* __restrict__ dst,
                          unsigned long long* seq_slot, unsigned long long seq, int shards) {
  // shards > 1: word i is the sum of its shards src[i + s * kShardStride] (block_add_sums).  All
  // loads of a lane (<= 4 words x kSumShards shards; n <= 256) are issued before any add: one
  // round trip (a per-word shard loop had made this launch 3.6 -> 8.0 us, r12d)
  // (agent-scope loads: the words were added by other launches' atomics; a plain load may be
  // served by a stale copy -- twice this round a count came back low)
  auto ld = [&](size_t k) { return __hip_atomic_load(src + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); };
  if (shards <= 1) {
    unsigned long long x[4];  // every load issued before the stores (n <= 256: 4 words a lane)
#pragma unroll
    for (int j = 0; j < 4; j++) {
      const int i = int(threadIdx.x) + 64 * j;
      x[j] = i < n ? ld(size_t(i)) : 0ull;
    }
#pragma unroll
    for (int j = 0; j < 4; j++) {
      const int i = int(threadIdx.x) + 64 * j;
      if (i < n) dst[i] = x[j];
    }
  } else {
    unsigned long long x[4][kSumShards];
#pragma unroll
    for (int j = 0; j < 4; j++)
#pragma unroll
      for (int s = 0; s < kSumShards; s++) {
        const int i = int(threadIdx.x) + 64 * j;
        x[j][s] = i < n && s < shards ? ld(size_t(s) * kShardStride + size_t(i)) : 0ull;
      }
#pragma unroll
    for (int j = 0; j < 4; j++) {
      const int i = int(threadIdx.x) + 64 * j;
      unsigned long long v = 0;
#pragma unroll
      for (int s = 0; s < kSumShards; s++) v += x[j][s];
      if (i < n) dst[i] = v;
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_store(seq_slot, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// the device counters d[0, n) into host h[0, n) once every launch before has finished: a
// one-thread-block kernel writes them and a sequence word to coherent host memory and the host
// spins on the word (a memcpy + hipStreamSynchronize round trip cost ~19 us, tools/launch_gap);
// past 2 s without it the stream is synchronised the ordinary way, which reports a fault
void fetch_counters(Ctx& c, const unsigned long long* d, int n, unsigned long long* h, hipEvent_t before,
                    int shards) {
  if (n > 256) throw Error(NBG_E_INVALID_ARG, "fetch_counters: at most 256 words");
  if (before) NBG_HIP(hipEventRecord(before, c.stream));
  const uint64_t seq = ++c.pub_seq;
  k_publish<<<1, 64, 0, c.stream>>>(d, n, h, c.host_seq, seq, std::max(shards, 1));
  NBG_HIP(hipGetLastError());
  if (c.opt("wait_trace", 0)) fprintf(stderr, "[nbg wait] rank %d: counter fetch of %d words\n", c.rank, n);
  wait_host_word(c, c.host_seq, seq);
}

// one host wait on a word the device publishes with a system-scope release (k_publish, the
// paths kernels' last-block publications)
void wait_host_word(Ctx& c, const unsigned long long* word, uint64_t seq) {
  c.timing.host_waits++;
  // pure spin for the first ~100 us (most waits: a hop of tens of us), then yield the core
  // between polls (a long hop, or several in-process LocalComm ranks waiting at once)
  const auto t0 = std::chrono::steady_clock::now();
  for (uint32_t spin = 0;; spin++) {
    if (__atomic_load_n(word, __ATOMIC_ACQUIRE) == seq) return;
    __builtin_ia32_pause();
    if ((spin & 255u) == 255u) {
      const auto dt = std::chrono::steady_clock::now() - t0;
      if (dt > std::chrono::microseconds(100)) std::this_thread::yield();
      if (dt > std::chrono::seconds(2)) {
        NBG_HIP(hipStreamSynchronize(c.stream));  // a fault surfaces here
        if (__atomic_load_n(word, __ATOMIC_ACQUIRE) == seq) return;
        throw Error(NBG_E_DEVICE, "counter publication lost");
      }
    }
  }
}

// the query's device time (ev[0] -> ev[1]) once it is asked for: go_run does not wait for ev[1]
void resolve_total(Ctx& c) {
  if (!c.total_pending) return;
  c.total_pending = false;
  float ms = 0;
  if (hipEventSynchronize(c.ev[1]) == hipSuccess && hipEventElapsedTime(&ms, c.ev[0], c.ev[1]) == hipSuccess)
    c.timing.total_ms = ms;
}

namespace {

int64_t map_bytes(const Ctx& c) { return ((c.n_global + 63) / 64) * 64 + 64; }

void ensure_workspaces(Ctx& c, int64_t nF_cap) {
  int64_t mb = map_bytes(c);
  if (c.ws_map.bytes < size_t(mb)) {
    c.ws_map.alloc(size_t(mb));
    NBG_HIP(hipMemsetAsync(c.ws_map.p, 0, size_t(mb), c.stream));
  }
  c.ws_front[0].ensure(size_t(nF_cap + 64) * 4);
  c.ws_front[1].ensure(size_t(nF_cap + 64) * 4);
  c.ws_off.ensure(size_t(nF_cap + 2) * 8);
  // [0, 64) hop counters, [64, 256) speculative hop blocks; then shards 1 .. kSumShards - 1 of
  // every word (block_add_sums), kShardStride words apart
  c.ws_counters.ensure(kShardStride * kSumShards * 8);
  c.ws_partials.ensure(size_t(kAggBlocks) * kSlots * 8);
  c.ws_bits_send.ensure(size_t(mb / 8 + 64));
  c.ws_bits_recv.ensure(size_t(mb / 8 + 64));
  if (c.sharded) {
    c.ws_piggy.ensure(size_t(12) * size_t(c.world) * 16 + 64);  // spec hops' counters of every rank
    c.ws_bits_glob.ensure(size_t(mb / 8 + 64));
    c.ws_bits_xchg.ensure(size_t(c.world) * size_t((c.owned_hi() - c.owned_lo()) / 8) + 64);
  }
}

// ---- cross-rank helpers (no-ops with one rank) ---------------------------------------------
// a host wait of the engine on the device (Timing::host_waits counts them; waits inside the
// transport are not the engine's)
void host_sync_at(Ctx& c, int line) {
  c.timing.host_waits++;
  if (c.opt("wait_trace", 0)) fprintf(stderr, "[nbg wait] rank %d: stream sync at traverse.hip:%d\n", c.rank, line);
  NBG_HIP(hipStreamSynchronize(c.stream));
}
#define host_sync(c) host_sync_at((c), __LINE__)
size_t timing_event(Ctx& c);
// time of the exchanges between ranks: an event pair around each, read after the query (a host
// wait per collective here would serialise the stream-ordered transport)
struct CommTimer {
  Ctx& c;
  size_t a;
  explicit CommTimer(Ctx& cc) : c(cc), a(timing_event(cc)) {}
  ~CommTimer() {
    const size_t b = timing_event(c);
    if (a != ~size_t(0) && b != ~size_t(0)) c.tpend.push_back(Ctx::PendingTime{a, b, -1, 2});
  }
};

// element-wise sum of a few host counters over ranks
void allsum(Ctx& c, int64_t* v, int n, unsigned long long* dscratch) {
  if (!c.sharded) return;
  {
    CommTimer t(c);
    NBG_HIP(hipMemcpyAsync(dscratch, v, size_t(n) * 8, hipMemcpyHostToDevice, c.stream));
    comm_allreduce_sum_i64(c, reinterpret_cast<int64_t*>(dscratch), size_t(n));
    NBG_HIP(hipMemcpyAsync(v, dscratch, size_t(n) * 8, hipMemcpyDeviceToHost, c.stream));
  }
  host_sync(c);
}

// device counters summed over ranks into dst (stream-ordered: a gate kernel reads the sums)
// srcs: up to 8 counter indices of K.d; dst: n consecutive words
__global__ void k_pick_counters(const unsigned long long* K, uint64_t idx, int n, unsigned long long* dst) {
  if (threadIdx.x < unsigned(n))
    dst[threadIdx.x] = __hip_atomic_load(K + ((idx >> (8 * threadIdx.x)) & 0xffu), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
void dev_allsum(Ctx& c, const unsigned long long* K, std::initializer_list<int> idx, unsigned long long* dst) {
  uint64_t packed = 0;
  int n = 0;
  for (int i : idx) packed |= uint64_t(uint8_t(i)) << (8 * n++);
  k_pick_counters<<<1, 64, 0, c.stream>>>(K, packed, n, dst);
  NBG_HIP(hipGetLastError());
  if (!c.sharded) return;
  CommTimer t(c);
  comm_allreduce_sum_i64(c, reinterpret_cast<int64_t*>(dst), size_t(n));
}

// owned frontier bitmap -> bitmap over the whole gidx space (bottom-up hops read sources of
// every rank).  Owner ranges are padded to 64, so every segment is whole 64-bit words.
const uint32_t* global_bits(Ctx& c, const uint32_t* owned) {
  if (!c.sharded) return owned;
  CommTimer t(c);
  const size_t G = size_t(c.world);
  std::vector<size_t> rb(G), ro(G);
  for (size_t p = 0; p < G; p++) {
    rb[p] = size_t(c.base[p + 1] - c.base[p]) / 8;
    ro[p] = size_t(c.base[p]) / 8;
  }
  comm_allgatherv_bytes(c, owned, rb[size_t(c.rank)], c.ws_bits_glob.p, rb.data(), ro.data());
  c.timing.comm_bytes += uint64_t(rb[size_t(c.rank)]) * (G - 1);
  return c.ws_bits_glob.as<uint32_t>();
}

// global_bits + every rank's two counters (n, e) at cnt into all[2r, 2r + 2), one exchange
const uint32_t* global_bits_cnt(Ctx& c, const uint32_t* owned, const unsigned long long* cnt, unsigned long long* all) {
  CommTimer t(c);
  const size_t G = size_t(c.world);
  std::vector<size_t> rb(G), ro(G);
  for (size_t p = 0; p < G; p++) {
    rb[p] = size_t(c.base[p + 1] - c.base[p]) / 8;
    ro[p] = size_t(c.base[p]) / 8;
  }
  comm_allgatherv2_bytes(c, owned, rb[size_t(c.rank)], c.ws_bits_glob.p, rb.data(), ro.data(), cnt, 16, all);
  c.timing.comm_bytes += uint64_t(rb[size_t(c.rank)] + 16) * (G - 1);
  return c.ws_bits_glob.as<uint32_t>();
}

// top-down hops mark dsts of every rank in the global byte-map: ship each owner its slice as
// a bitmap and OR the received slices back into the owned range of the map
void exchange_marks(Ctx& c, uint8_t* map, uint32_t* owned_bits = nullptr, const uint32_t* odeg = nullptr,
                    unsigned long long* sums = nullptr) {
  if (!c.sharded) return;
  CommTimer t(c);
  const size_t G = size_t(c.world);
  const int64_t lo = c.owned_lo(), n_own = c.owned_hi() - lo;
  uint32_t* sb = c.ws_bits_glob.as<uint32_t>();
  uint32_t* rbuf = c.ws_bits_xchg.as<uint32_t>();
  int64_t nw = c.n_global / 32;
  k_map_to_bits<<<grid_cap(nw), 256, 0, c.stream>>>(map, c.n_global, sb);
  NBG_HIP(hipGetLastError());
  std::vector<size_t> sbytes(G), soff(G), rbytes(G), roff(G);
  for (size_t p = 0; p < G; p++) {
    sbytes[p] = size_t(c.base[p + 1] - c.base[p]) / 8;
    soff[p] = size_t(c.base[p]) / 8;
    rbytes[p] = size_t(n_own) / 8;
    roff[p] = p * size_t(n_own) / 8;
  }
  comm_alltoallv_bytes(c, sb, sbytes.data(), soff.data(), rbuf, rbytes.data(), roff.data());
  c.timing.comm_bytes += uint64_t(c.n_global - n_own) / 8;
  if (owned_bits) {  // the next frontier as the owned bitmap + its counts (no byte map, no compaction)
    const int grid = int(std::max<int64_t>(1, std::min<int64_t>((n_own / 32 + 255) / 256, 512)));
    k_or_segments_bits<<<grid, 256, 0, c.stream>>>(rbuf, int(G), n_own / 32, odeg, owned_bits, sums);
  } else {
    k_or_segments_to_map<<<grid_cap(n_own / 32), 256, 0, c.stream>>>(rbuf, int(G), n_own / 32, map + lo);
  }
  NBG_HIP(hipGetLastError());
}

__global__ void k_min_segments(const int32_t* recv, int G, int64_t n, int32_t* out) {
  for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < n; i += int64_t(gridDim.x) * blockDim.x) {
    int32_t m = INT32_MAX;
    for (int g = 0; g < G; g++) m = min(m, recv[size_t(g) * size_t(n) + size_t(i)]);
    out[i] = m;
  }
}

// world > 1, $- / $var props with STEPS > 1: every rank's top-down hop took the smallest root
// rank over ITS in-edges of each dst (one atomicMin per edge, any owner); the owner of a dst
// needs the minimum over all ranks' edges (GoExecutor.h:174-193's VertexBackTracker, under the
// deterministic rule of DESIGN.md divergence 6).  Each rank sends every owner its slice of the
// root array and takes the elementwise minimum of the slices it receives.
void exchange_roots(Ctx& c, int32_t* root_next) {
  if (!c.sharded) return;
  CommTimer t(c);
  const size_t G = size_t(c.world);
  const int64_t lo = c.owned_lo(), n_own = c.owned_hi() - lo;
  DevBuf rbuf;
  rbuf.alloc(std::max<size_t>(G * size_t(n_own) * 4, 4));
  std::vector<size_t> sbytes(G), soff(G), rbytes(G), roff(G);
  for (size_t p = 0; p < G; p++) {
    sbytes[p] = size_t(c.base[p + 1] - c.base[p]) * 4;
    soff[p] = size_t(c.base[p]) * 4;
    rbytes[p] = size_t(n_own) * 4;
    roff[p] = p * size_t(n_own) * 4;
  }
  comm_alltoallv_bytes(c, root_next, sbytes.data(), soff.data(), rbuf.p, rbytes.data(), roff.data());
  c.timing.comm_bytes += uint64_t(c.n_global - n_own) * 4;
  if (n_own)
    k_min_segments<<<grid_cap(n_own), 256, 0, c.stream>>>(rbuf.as<int32_t>(), int(G), n_own, root_next + lo);
  NBG_HIP(hipGetLastError());
}

__global__ void k_hist_dest(const uint32_t* dest, int64_t n, int G, unsigned long long* counts) {
  __shared__ unsigned int h[64];
  if (threadIdx.x < 64) h[threadIdx.x] = 0;
  __syncthreads();
  for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < n; i += int64_t(gridDim.x) * blockDim.x)
    atomicAdd(&h[dest[i]], 1u);
  __syncthreads();
  if (threadIdx.x < unsigned(G) && h[threadIdx.x]) atomicAdd(counts + threadIdx.x, (unsigned long long)h[threadIdx.x]);
}

// DISTINCT with several ranks: every row goes to rank hash(row) % G (all copies of a row meet
// on one rank), then the local dedup runs as with one rank.  Returns the received row count.
int64_t shuffle_rows(Ctx& c, YieldArgs& ya, std::vector<DevBuf>& cols, int64_t n) {
  CommTimer t(c);
  const size_t G = size_t(c.world);
  if (G > 64) throw Error(NBG_E_UNSUPPORTED, "more than 64 ranks");
  DevBuf dest, flag, cnt, dcounts;
  dest.alloc(size_t(n + 1) * 4);
  flag.alloc(size_t(n + 1));
  cnt.alloc(8);
  dcounts.alloc(G * G * 8 + 8);
  NBG_HIP(hipMemsetAsync(dcounts.p, 0, G * 8, c.stream));
  if (n) {
    k_row_dest<<<grid_cap(n), 256, 0, c.stream>>>(ya, n, uint32_t(G), dest.as<uint32_t>());
    k_hist_dest<<<grid_cap(n), 256, 0, c.stream>>>(dest.as<uint32_t>(), n, int(G), dcounts.as<unsigned long long>());
  }
  std::vector<int64_t> all(G * G);
  DevBuf dall;
  dall.alloc(G * G * 8);
  comm_allgather_bytes(c, dcounts.p, G * 8, dall.p);
  NBG_HIP(hipMemcpyAsync(all.data(), dall.p, G * G * 8, hipMemcpyDeviceToHost, c.stream));
  host_sync(c);
  const size_t me = size_t(c.rank);
  std::vector<int64_t> soff(G + 1, 0), roff(G + 1, 0);
  for (size_t p = 0; p < G; p++) {
    soff[p + 1] = soff[p] + all[me * G + p];
    roff[p + 1] = roff[p] + all[p * G + me];
  }
  const int64_t R = roff[G];
  std::vector<DevBuf> send(cols.size()), recv(cols.size());
  for (size_t cc = 0; cc < cols.size(); cc++) {
    size_t w = ya.cols[cc].type == VT_BOOL ? 1 : 8;
    send[cc].alloc(size_t(n + 1) * w);
    recv[cc].alloc(size_t(R + 1) * w);
  }
  for (size_t p = 0; p < G && n; p++) {
    if (!all[me * G + p]) continue;
    k_flag_dest<<<grid_cap(n), 256, 0, c.stream>>>(dest.as<uint32_t>(), n, uint32_t(p), flag.as<uint8_t>());
    for (size_t cc = 0; cc < cols.size(); cc++) {
      size_t tb = 0;
      if (ya.cols[cc].type == VT_BOOL) {
        uint8_t* o = send[cc].as<uint8_t>() + soff[p];
        NBG_HIP(rocprim::select(nullptr, tb, cols[cc].as<uint8_t>(), flag.as<uint8_t>(), o, cnt.as<uint64_t>(),
                                size_t(n), c.stream));
        c.ws_tmp.ensure(tb);
        NBG_HIP(rocprim::select(c.ws_tmp.p, tb, cols[cc].as<uint8_t>(), flag.as<uint8_t>(), o, cnt.as<uint64_t>(),
                                size_t(n), c.stream));
      } else {
        int64_t* o = send[cc].as<int64_t>() + soff[p];
        NBG_HIP(rocprim::select(nullptr, tb, cols[cc].as<int64_t>(), flag.as<uint8_t>(), o, cnt.as<uint64_t>(),
                                size_t(n), c.stream));
        c.ws_tmp.ensure(tb);
        NBG_HIP(rocprim::select(c.ws_tmp.p, tb, cols[cc].as<int64_t>(), flag.as<uint8_t>(), o, cnt.as<uint64_t>(),
                                size_t(n), c.stream));
      }
    }
  }
  for (size_t cc = 0; cc < cols.size(); cc++) {
    size_t w = ya.cols[cc].type == VT_BOOL ? 1 : 8;
    std::vector<size_t> sb(G), so(G), rb(G), ro(G);
    for (size_t p = 0; p < G; p++) {
      sb[p] = size_t(soff[p + 1] - soff[p]) * w;
      so[p] = size_t(soff[p]) * w;
      rb[p] = size_t(roff[p + 1] - roff[p]) * w;
      ro[p] = size_t(roff[p]) * w;
    }
    comm_alltoallv_bytes(c, send[cc].p, sb.data(), so.data(), recv[cc].p, rb.data(), ro.data());
    c.timing.comm_bytes += uint64_t(n - (soff[me + 1] - soff[me])) * w;
  }
  host_sync(c);
  for (size_t cc = 0; cc < cols.size(); cc++) {
    cols[cc] = std::move(recv[cc]);
    ya.cols[cc].data = cols[cc].p;
  }
  return R;
}

// frontier degree scan: fills c.ws_off[0..nF] and returns total edges (synchronises)
// known >= 0: the caller already has the total (from a compaction's partials): no round trip
int64_t degree_scan(Ctx& c, const int32_t* F, int64_t nF, const Csr& csr, DevBuf& degbuf, int64_t known) {
  degbuf.ensure(size_t(nF + 1) * 8);
  k_degrees<<<grid_cap(nF + 1), 256, 0, c.stream>>>(F, nF, csr.row_ptr.as<int64_t>(), degbuf.as<int64_t>());
  exclusive_scan_dev<int64_t>(c, degbuf.as<int64_t>(), c.ws_off.as<int64_t>(), nF + 1);
  if (known >= 0) return known;
  int64_t E = 0;
  NBG_HIP(hipMemcpyAsync(&E, c.ws_off.as<int64_t>() + nF, 8, hipMemcpyDeviceToHost, c.stream));
  host_sync(c);
  return E;
}

// raise a kernel's dynamic LDS limit once per process (the attribute call costs a host round
// trip: done per launch it showed up as ~10 us gaps before every bottom-up pass)
static void lds_limit(const void* kern, size_t shm) {
  static std::mutex mu;
  static std::unordered_map<const void*, size_t> done;
  std::lock_guard<std::mutex> lk(mu);
  auto it = done.find(kern);
  if (it != done.end() && it->second >= shm) return;
  NBG_HIP(hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, int(shm)));
  done[kern] = shm;
}

void launch_compact(Ctx& c, uint8_t* map, int64_t lo, int64_t n, const int64_t* row_ptr, const uint8_t* row_ok,
                    int require_deg, int32_t* out, uint16_t* bits, unsigned long long* Kd,
                    const uint32_t* odeg = nullptr, bool sums_zero = false, int shards = 1, int64_t own_lo = 0,
                    int64_t own_hi = -1, uint16_t* own_bits = nullptr, int64_t n_read = -1) {
  // counters: Kd[0] list length (atomic), Kd[12] vertices set, Kd[13] kept out-degree sum,
  // Kd[14] kept vertices (= the list length, also when out == nullptr writes no list).
  // sums_zero: Kd[12, 15) are already zero, so the blocks add into them (bu_atomic_sums)
  unsigned long long* partials = c.ws_partials.as<unsigned long long>();
  int64_t ntiles = ((n + 15) / 16 + 1023) / 1024;
  int grid = int(std::max<int64_t>(1, std::min<int64_t>(ntiles, std::min<int64_t>(kAggBlocks, c.opt("compact_grid", 1024)))));
  const bool atomic = sums_zero && c.opt("bu_atomic_sums", 1) != 0;
  k_compact<<<grid, 256, 0, c.stream>>>(map, lo, n, row_ptr, row_ok, require_deg, out, Kd, partials, bits, odeg,
                                        atomic ? Kd + 12 : nullptr, atomic ? shards : 1, own_lo, own_hi, own_bits,
                                        n_read >= 0 ? n_read : n);
  if (!atomic) k_reduce_partials<<<1, 1024, 0, c.stream>>>(partials, grid, Kd + 12);
  NBG_HIP(hipGetLastError());
}

// records a pooled timing event on the query stream; returns its pool index
constexpr size_t kNoEvent = ~size_t(0);
// an event recorded on the engine stream for deferred hop timing (kNoEvent: hop_timing off)
size_t timing_event(Ctx& c) {
  if (!c.hop_timing) return kNoEvent;
  if (c.tev_used == c.tev.size()) {
    hipEvent_t e;
    NBG_HIP(hipEventCreate(&e));
    c.tev.push_back(e);
  }
  NBG_HIP(hipEventRecord(c.tev[c.tev_used], c.stream));
  return c.tev_used++;
}

template <int MODE>
void launch_expand(Ctx& c, ExpandArgs a, int pk, const FastArgs& fp, const Program* dprog, const EvalEnv& env,
                   int64_t E, bool tile_rows_ready = false) {
  int64_t ntiles = (E + kTile - 1) / kTile;
  int grid = int(std::max<int64_t>(1, std::min<int64_t>(ntiles, int64_t(256 * 8))));
  const size_t ia = timing_event(c);
  if (tile_rows_ready) {  // k_starts_small wrote the table
    a.tile_row = c.ws_tile_rows.as<int32_t>();
  } else if (a.nF < (int64_t(1) << 31)) {
    c.ws_tile_rows.ensure(size_t(ntiles + 2) * 4);
    a.tile_row = c.ws_tile_rows.as<int32_t>();
    k_tile_rows<kTile><<<grid_cap(a.nF), 256, 0, c.stream>>>(a.off, a.nF, c.ws_tile_rows.as<int32_t>());
  }
  switch (pk) {
    case PK_NONE: k_expand<MODE, PK_NONE><<<grid, kThreads, 0, c.stream>>>(a, fp, dprog, env); break;
    case PK_FAST: k_expand<MODE, PK_FAST><<<grid, kThreads, 0, c.stream>>>(a, fp, dprog, env); break;
    default: k_expand<MODE, PK_VM><<<grid, kThreads, 0, c.stream>>>(a, fp, dprog, env); break;
  }
  NBG_HIP(hipGetLastError());
  const size_t ib = timing_event(c);
  c.tpend.push_back(Ctx::PendingTime{ia, ib, c.timing.n_hops, 0});  // read by timing_resolve
  c.timing.expand_launches++;
}

// values min + [ceil(b * range / 2^bits), ceil((b + 1) * range / 2^bits) - 1]; it passes (fails)
// when every value in it passes (fails) the compare, else the kernels read the exact value.
QArgs make_qargs(const EdgeSpace& es, int pk, int fcol, const FastArgs& fp) {
  QArgs q;
  if (es.q_field < 0) return q;
  q.gmask = (1u << es.q_gbits) - 1u;
  q.gbits = es.q_gbits;
  if (pk != PK_FAST || fcol != es.q_field) return q;  // packed words, every value read
  using u128 = unsigned __int128;
  const u128 R = es.q_range ? u128(es.q_range) : (u128(1) << 64);
  const int bits = es.q_bits, nb = 1 << bits;
  auto edge = [&](uint64_t b) -> u128 { return ((u128(b) * R) + ((u128(1) << bits) - 1)) >> bits; };  // ceil
  // per bucket: 1 pass, 0 fail, -1 undecided, 2 empty (no value lands there: either answer)
  std::vector<int> dec(size_t(nb), 2);
  for (int b = 0; b < nb; b++) {
    const u128 o0 = edge(uint64_t(b)), o1 = edge(uint64_t(b) + 1);
    if (o0 >= o1) continue;
    const int64_t lo = int64_t(uint64_t(es.q_min) + uint64_t(o0));
    const int64_t hi = int64_t(uint64_t(es.q_min) + uint64_t(o1 - 1));
    const int64_t k = fp.k;
    bool pass, fail;
    if (fp.op == 4) {  // ==
      pass = lo == k && hi == k;
      fail = k < lo || k > hi;
    } else if (fp.op == 5) {  // !=
      pass = k < lo || k > hi;
      fail = lo == k && hi == k;
    } else {  // monotone compares: both ends decide the bucket
      const bool x = fast_cmp(fp.op, lo, k), z = fast_cmp(fp.op, hi, k);
      pass = x && z;
      fail = !x && !z;
    }
    dec[size_t(b)] = pass ? 1 : fail ? 0 : -1;
  }
  // below: the first non-empty bucket's answer, up to the first bucket answering otherwise;
  // above: the last one's, down to the last bucket answering otherwise; between: undecided
  int first = 2, last = 2;
  for (int b = 0; b < nb && first == 2; b++) first = dec[size_t(b)];
  for (int b = nb - 1; b >= 0 && last == 2; b--) last = dec[size_t(b)];
  if (first == 2) return q;  // no values at all
  int ulo = nb, uhi = nb - 1;
  for (int b = 0; b < nb; b++)
    if (dec[size_t(b)] != 2 && dec[size_t(b)] != first) {
      ulo = b;
      break;
    }
  for (int b = nb - 1; b >= 0; b--)
    if (dec[size_t(b)] != 2 && dec[size_t(b)] != last) {
      uhi = b;
      break;
    }
  q.ulo = ulo;
  q.uhi = ulo == nb ? nb - 1 : uhi;
  q.below = first;
  q.above = ulo == nb ? first : last;
  return q;
}

// DISTINCT _dst output: the vids of a bitmap's set rows (8 word pairs per lane and step; r05
// sweep: 8 took the C3 final hop 266 -> 258 us against 4, removed in round 6)
static void launch_bits_vids(Ctx& c, const uint32_t* bits, int64_t rows, int64_t lo, void* out,
                             unsigned long long* n_out, const unsigned long long* gate) {
  // non-temporal vid loads and output stores (the 173 MB of C3's output no longer pass through
  // L2 as dirty lines): 0.4048 -> 0.4001 ms a C3 query, 4 A/B pairs (+ 3: 0.403 -> 0.397)
  const int grid = grid_cap((rows + 31) / 32, 1024, 4096);
  k_bits_compact<1, 8, 1><<<grid, 1024, 0, c.stream>>>(bits, rows, lo, c.vid_of.as<int64_t>(), out, n_out, gate);
}

// k_bu_fin's word ranges from a query's bucket decisions (q_test: buckets below ulo answer
// `below`, above uhi `above`, the rest are undecided).  The field above the gidx bits is the
// bucket; every decision region is a contiguous field range, so each set is one word range.
FinArgs fin_args(const QArgs& q) {
  FinArgs f;
  const int gb = q.gbits;
  f.bmask = (q.gmask >> 3) & ~3u;
  if (gb <= 0) {  // unpacked words: no buckets (every word undecided, or no predicate at all)
    f.clo = 0, f.cr = 0xffffffffu;
    const bool all_pass = q.below == 1 && q.above == 1;
    f.plo = 0, f.pr = 0xffffffffu, f.pinv = all_pass ? 0u : 1u;
    return f;
  }
  const int64_t B = (int64_t(1) << (32 - gb)) - 1;  // largest field value (the -1 pad's)
  const int64_t lo_end = std::min<int64_t>(std::max<int64_t>(q.ulo, 0), B + 1);  // [0, lo_end): below
  const int64_t u_end = std::min<int64_t>(std::max<int64_t>(q.uhi, lo_end - 1), B);  // [lo_end, u_end]: undecided
  auto word_lo = [&](int64_t a) { return uint32_t(uint64_t(a) << gb); };
  auto word_hi = [&](int64_t b) { return uint32_t(((uint64_t(b) + 1) << gb) - 1); };
  auto set_range = [&](int64_t a, int64_t b, uint32_t& lo, uint32_t& r) {  // field range [a, b], a <= b
    lo = word_lo(a);
    r = word_hi(b) - lo;
  };
  const bool c0 = q.below != 0, c2 = q.above != 0;  // below / above regions are candidates
  if (c0 && c2) set_range(0, B, f.clo, f.cr);
  else if (c0) set_range(0, u_end, f.clo, f.cr);
  else if (c2) set_range(lo_end, B, f.clo, f.cr);
  else if (lo_end <= u_end) set_range(lo_end, u_end, f.clo, f.cr);
  else f.clo = 0xffffffffu, f.cr = 0;  // no candidate but the pad word (whose probe is out of bounds)
  const bool p0 = q.below == 1 && lo_end > 0, p2 = q.above == 1 && u_end < B;
  f.pinv = 0;
  if (p0 && p2) {
    if (lo_end <= u_end) set_range(lo_end, u_end, f.plo, f.pr), f.pinv = 1;  // all but the undecided
    else f.plo = 0, f.pr = 0xffffffffu;
  } else if (p0) {
    set_range(0, lo_end - 1, f.plo, f.pr);
  } else if (p2) {
    set_range(u_end + 1, B, f.plo, f.pr);
  } else {
    f.plo = 0, f.pr = 0xffffffffu, f.pinv = 1;  // nothing passes
  }
  return f;
}

// bottom-up hop: the first pass (k_bu_lean) over the quad slab and the pending rows' rests in
// k_bu_rest_lean; counters reduced into out[0..8) (no synchronisation).  pk: PK_NONE (a
// non-final hop: odeg keeps found rows with out-edges and sums their degrees) or PK_FAST (the
// final hop's typed compare on transposed column fcol; decided from the packed buckets when fcol
// is the packed column, else every value of a frontier hit is read by the rest pass).
// hop_front: the frontier came out of a hop (not the starts), so on one rank with the
// class-ordered numbering (snapshot k_class_key) its bits lie below row bu_both_tiles * 128: a
// frontier vertex has an in-edge (it was found) and an out-edge (the hops keep only those).
// Probes past that bound are out of bounds of their buffer resource (the hardware answers 0
// without a memory access).
size_t launch_bu_lean(Ctx& c, EdgeSpace& es, const uint32_t* fb, uint32_t* nbits, const uint32_t* odeg, int pk,
                      const FastArgs& fp, int fcol, unsigned long long* out, bool hop_front,
                      unsigned long long* gate = nullptr, GateIn gi = GateIn{}, bool out_zero = false,
                      int shards = 1) {
  const Csr& tr = es.tr;
  if (pk != PK_NONE && pk != PK_FAST) throw Error(NBG_E_DEVICE, "bottom-up hop with a VM predicate");
  if (!es.pair_col[0].p) throw Error(NBG_E_DEVICE, "bottom-up hop without the quad slab");
  // the final hop (no odeg) runs the final-hop kernels; without a WHERE every bucket passes
  const bool fast = pk == PK_FAST || !odeg;
  QArgs q;
  if (pk == PK_FAST) {
    // bu_qpred = 0 (tests): ignore the buckets, every frontier hit reads its value
    q = make_qargs(es, c.opt("bu_qpred", 1) != 0 ? pk : PK_NONE, fcol, fp);
  } else {
    q = make_qargs(es, PK_NONE, -1, fp);
    if (fast) q.ulo = q.uhi = INT32_MAX, q.below = q.above = 1;
  }
  // rows pending after the slab rescan it only when a slot may be undecided (a predicate)
  const int rest_from = pk == PK_FAST ? 0 : 4;
  pk = fast ? PK_FAST : PK_NONE;
  const int64_t ntiles = (tr.n_rows + 127) / 128;
  // rows past the last one that can be found (final) or extend the next frontier (non-final)
  // get zero words without being read (exact bounds, snapshot build_transpose)
  const int64_t work = std::min(ntiles, fast ? es.bu_in_tiles : es.bu_both_tiles);
  const int64_t waves = std::max<int64_t>(1, work);
  // hub words in LDS (bu_lean_lds_kb KiB, 0 = off): 1024-thread blocks, two per CU
  const int64_t fb_words = (c.n_global + 31) / 32;
  // bu_hub_cap (tests): at most that many hub words, so small graphs exercise the L2 probes too
  const int64_t hub_cap = std::max<int64_t>(0, c.opt("bu_hub_cap", 36 * 1024));
  // (final hop 72 KiB, two blocks per CU still fit: r06g/r06h 1 % faster than 64)
  const int cw = int(std::min<int64_t>(c.opt(fast ? "bu_lean_lds_kb_final" : "bu_lean_lds_kb", fast ? 72 : 64) * 256,
                                       std::min<int64_t>({fb_words, int64_t(36 * 1024), hub_cap})));
  const int bs = cw > 0 ? 1024 : 256;
  const int grid = int(std::max<int64_t>(
      1, std::min<int64_t>((waves + bs / 64 - 1) / (bs / 64),
                           std::min<int64_t>(cw > 0 ? 512 : 2048, kAggBlocks / 2))));
  const size_t shm = size_t(cw + 1) * 4;  // + the zero word non-hub probes read
  uint32_t fb_bytes = uint32_t(fb_words * 4);
  if (hop_front && !c.sharded && es.bu_both_tiles > 0)
    fb_bytes = uint32_t(std::min<int64_t>(fb_bytes, (es.bu_both_tiles * 128 + 31) / 32 * 4));
  const int probe_stats = int(c.opt("bu_probe_stats", 0));  // partials [6] / [7]
  c.ws_pend.ensure(size_t(ntiles * 2 + 2) * 8);  // the pending bits, 2 words per tile
  unsigned long long* pbits = c.ws_pend.as<unsigned long long>();
  // option bu_atomic_sums: both passes add their block sums into `out` (zeroed first unless the
  // caller's block is known zero) and no k_reduce_partials launch follows
  // (r06j: 0.4796 -> 0.4663 ms per C3 query, the two k_reduce_partials launches gone)
  // (sharded sums, shards > 1: only into a block the caller zeroed with its shards)
  const int atomic_sums =
      c.opt("bu_atomic_sums", 1) != 0 && c.opt("bu_rest_dbg", 0) == 0 ? (out_zero ? std::max(shards, 1) : 1) : 0;
  unsigned long long* partials = atomic_sums ? out : c.ws_partials.as<unsigned long long>();
  if (atomic_sums && !out_zero) NBG_HIP(hipMemsetAsync(out, 0, 8 * 8, c.stream));
  auto* nb = reinterpret_cast<unsigned long long*>(nbits);
  const uint2* lo = es.pair_col[0].as<uint2>();
  const uint2* hi = es.pair_col[1].as<uint2>();
  const uint32_t* od = fast ? nullptr : odeg;
  auto go = [&](auto kern) {
    if (shm > 48 * 1024)
      lds_limit(reinterpret_cast<const void*>(kern), shm);
    kern<<<grid, bs, shm, c.stream>>>(lo, hi, ntiles, work, fb, fb_bytes, nb, pbits, od, q, partials, cw,
                                      es.odeg8.as<uint8_t>(), gate, gi, atomic_sums);
  };
  // sel 0 / 2: no hub copy / hub copy; 4 / 5 the counting (diagnostic) instantiations; 8 the
  // default: non-temporal slab, 1 B degrees, the probe skip and hub-first L2 probes (r06j: 100.7
  // -> 91.6 us at C3 hop 2).  Removed in round 6, each measured without gain: two tiles per
  // iteration (bu_lean_u 2), one store per tile in the non-final pass (bu_lean_skip 7), the probe
  // skip without the hub-first probes (bu_lean_skip 1).
  int sel = probe_stats ? 4 + (cw > 0 ? 1 : 0) : (cw > 0 ? 2 : 0);
  if (sel == 2 && (fast || es.odeg8.p)) sel = 8;
#define NBG_LEAN(PKV)                                \
  switch (sel) {                                     \
    case 8: go(k_bu_lean<PKV, 1, 1, 0, 1, 3>); break; \
    case 0: go(k_bu_lean<PKV, 1, 0, 0>); break;      \
    case 2: go(k_bu_lean<PKV, 1, 1, 0>); break;      \
    case 4: go(k_bu_lean<PKV, 1, 0, 1>); break;      \
    default: go(k_bu_lean<PKV, 1, 1, 1>); break;     \
  }
  const bool fin = fast && !probe_stats && c.opt("bu_fin", 1) != 0;
  char fin_nm[64] = "";
  if (fin) {
    const FinArgs fa = fin_args(q);
    // CLS 1 ("greater than"): candidates and passing words are each one upper range
    const bool cls1 = fa.pinv == 0 && fa.cr == ~fa.clo && fa.pr == ~fa.plo && fa.clo <= 0x80000000u &&
                      fa.plo <= 0x80000000u && c.opt("bu_fin_cls", 1) != 0;
    const size_t fshm = size_t((cw + 2) & ~1) * 4 + size_t(kSlots) * 16 * 8;
    const uint32_t rest = fb_bytes > uint32_t(cw) * 4u ? fb_bytes - uint32_t(cw) * 4u : 0u;
    const int nt = int(c.opt("bu_fin_nt", 1) != 0);
    auto gof = [&](auto kern) {
      if (fshm > 48 * 1024) lds_limit(reinterpret_cast<const void*>(kern), fshm);
      kern<<<grid, bs, fshm, c.stream>>>(lo, hi, ntiles, work, fb, nb, pbits, fa, partials, cw, rest, gate, gi,
                                         atomic_sums);
    };
    switch ((cls1 ? 1 : 0) | nt << 1) {
      case 0: gof(k_bu_fin<0, 0>); break;
      case 1: gof(k_bu_fin<1, 0>); break;
      case 2: gof(k_bu_fin<0, 1>); break;
      default: gof(k_bu_fin<1, 1>); break;
    }
    snprintf(fin_nm, sizeof fin_nm, "nbg::k_bu_fin<%d, %d>", cls1 ? 1 : 0, nt);
  } else if (fast) {
    NBG_LEAN(PK_FAST)
  } else {
    NBG_LEAN(PK_NONE)
  }
#undef NBG_LEAN
  NBG_HIP(hipGetLastError());
  const size_t ev_first = timing_event(c);  // end of the first pass (the hop's kernel_ms)
  const int64_t* trp = tr.row_ptr.as<int64_t>();
  const int32_t* tc = q.gbits ? es.tcol_q.as<int32_t>() : tr.col.as<int32_t>();
  const int ru = int(std::max<int64_t>(1, std::min<int64_t>(c.opt("bu_unroll", 1), kRestMax)));
  const int grid2 = 512;
  const int W = fast ? int(fp.width) : 0;
  // the rest pass probes global memory only by default: its hub copy cost each block ~6 us of
  // LDS fill (r04h/r04k sweeps: 0.637 -> 0.625 ms per C3 query without it)
  const int rcw = int(std::min<int64_t>(c.opt(fast ? "bu_rest_lds_kb_final" : "bu_rest_lds_kb", 0) * 256,
                                        std::min<int64_t>({fb_words, int64_t(36 * 1024), hub_cap})));
  const size_t rshm = size_t(std::max(rcw, 1)) * 4;
  const int rsteps = int(std::max<int64_t>(1, c.opt("bu_rest_steps", 4)));
  // diagnostics (option bu_rest_dbg): per-wave records of the rest pass appended to $NBG_DBG_FILE
  DevBuf dbg_buf;
  unsigned long long* dbg = nullptr;
  if (c.opt("bu_rest_dbg", 0)) {
    dbg_buf.alloc(size_t(grid2) * 16 * 64);
    NBG_HIP(hipMemsetAsync(dbg_buf.p, 0, size_t(grid2) * 16 * 64, c.stream));
    dbg = dbg_buf.as<unsigned long long>();
  }
  // pending bits exist only below the work tiles (the first pass zeroes the words past them)
  const int64_t rest_rows = std::min(tr.n_rows, work * 128);
  // rest records cover every row the first pass can leave pending (rows below work tiles)
  const bool use_rec = es.brec.p && es.brec_rows >= std::min(tr.n_rows, work * 128) && c.opt("bu_rec", 1) != 0;
  const uint4* rec = use_rec ? es.brec.as<uint4>() : nullptr;
  auto rest = [&](auto kern) {
    if (rshm > 48 * 1024)
      lds_limit(reinterpret_cast<const void*>(kern), rshm);
    kern<<<grid2, 1024, rshm, c.stream>>>(pbits, rest_rows, trp, tc, fb, fb_bytes, nb, odeg, fp, q,
                                          atomic_sums ? partials : partials + grid, rcw, ru, rest_from, rsteps, dbg,
                                          gate, rec, atomic_sums);
  };
#define NBG_REST(PKV, WV)                                                 \
  if (rcw > 0) {                                                          \
    if (use_rec) rest(k_bu_rest_lean<PKV, WV, 1, 1>);                     \
    else rest(k_bu_rest_lean<PKV, WV, 1, 0>);                             \
  } else {                                                                \
    if (use_rec) rest(k_bu_rest_lean<PKV, WV, 0, 1>);                     \
    else rest(k_bu_rest_lean<PKV, WV, 0, 0>);                             \
  }
  if (fast) {
    switch (W) {
      case 1: NBG_REST(PK_FAST, 1); break;
      case 2: NBG_REST(PK_FAST, 2); break;
      case 4: NBG_REST(PK_FAST, 4); break;
      default: NBG_REST(PK_FAST, 8); break;
    }
  } else {
    NBG_REST(PK_NONE, 0);
  }
#undef NBG_REST
  NBG_HIP(hipGetLastError());
  if (!atomic_sums) k_reduce_partials<<<1, 1024, 0, c.stream>>>(partials, grid + grid2, out, gate);
  NBG_HIP(hipGetLastError());
  if (dbg) {
    std::vector<unsigned long long> h(size_t(grid2) * 16 * 8);
    NBG_HIP(hipMemcpyAsync(h.data(), dbg, h.size() * 8, hipMemcpyDeviceToHost, c.stream));
    NBG_HIP(hipStreamSynchronize(c.stream));
    if (const char* fn = getenv("NBG_DBG_FILE")) {
      if (FILE* f = fopen(fn, "ab")) {
        const uint64_t hdr[2] = {uint64_t(pk), uint64_t(grid2) * 16};
        fwrite(hdr, 8, 2, f);
        fwrite(h.data(), 8, h.size(), f);
        fclose(f);
      }
    }
  }
  char nm[96];
  if (fin)
    snprintf(nm, sizeof nm, "%s", fin_nm);
  else
    snprintf(nm, sizeof nm, "nbg::k_bu_lean<%d, 1, %d, %d%s>", pk, cw > 0 ? 1 : 0, probe_stats ? 1 : 0,
             sel == 8 ? ", 1, 3" : ", 0, 0");
  c.bu_kernel_name = nm;
  // the non-final first pass reads one out-degree per row of its work tiles: 1 B (odeg8, the
  // non-temporal instantiations) or 4 B (odeg)
  if (!fast) c.bu_od_bytes = uint64_t(work) * 128u * (sel == 8 ? 1u : 4u);
  const int wn = fast ? (W == 1 || W == 2 || W == 4 ? W : 8) : 0;
  snprintf(nm, sizeof nm, "nbg::k_bu_rest_lean<%d, %d, %d, %d>", pk, wn, rcw > 0 ? 1 : 0, use_rec ? 1 : 0);
  c.bu_rest_rec = use_rec;
  c.bu_rest_name = nm;
  return ev_first;
}

// byte models of a bottom-up hop's two passes from their counters.
// First pass: 4 B per slab word read, the frontier bitmap once, the next-frontier and pending
// bits written, the out-degrees a non-final hop read (od_bytes: 1 B per work row from odeg8;
// rounds 2-4 counted 4 B for every row, 1.5x the bytes the default kernel reads).  Rest pass:
// a row_ptr pair (or a 64 B rest record) per pending row, 4 B per entry read, predicate values read.
uint64_t bu_first_bytes(const unsigned long long* h, int64_t n_rows, uint64_t od_bytes) {
  return h[2] * 4 + 3 * (uint64_t(n_rows) / 8) + od_bytes;
}
uint64_t bu_rest_bytes(const unsigned long long* h, int pred_width, bool rec) {
  return h[3] * (rec ? 64 : 16) + h[4] * 4 + h[5] * uint64_t(pred_width);
}
// algorithmic bytes of one expansion (DESIGN.md "byte model"): frontier id 4 B + row_ptr pair
// 16 B + off 8 B per frontier entry; per edge: col 4 B (+ predicate column width) + the
// output it makes (1 B map mark, or 12 B row, or 1 B flag).
uint64_t expand_bytes(int64_t nF, int64_t E, int pred_width, int mode) {
  uint64_t b = uint64_t(nF) * 28 + uint64_t(E) * (4 + uint64_t(pred_width));
  b += uint64_t(E) * (mode == EXP_ROWS ? 0 : 1);
  return b;
}

}  // namespace

// once per snapshot (collective): the out-edges summed over ranks, the largest out-degree and
// the prefix sums of the kTopDeg largest out-degrees over ranks, so that every rank takes the
// same direction decisions and a GO from a few starts knows its first hop's direction before
// it runs
constexpr int64_t kTopDeg = 4096;
void global_degree_stats(Ctx& c, EdgeSpace& es) {
  const Csr& csr = es.out;
  const size_t G = size_t(c.world);
  const int64_t n_own = c.owned_hi() - c.owned_lo();
  // this rank's kTopDeg largest out-degrees (0-padded), descending
  DevBuf top;
  top.alloc(size_t(kTopDeg) * 4 + 16);
  NBG_HIP(hipMemsetAsync(top.p, 0, size_t(kTopDeg) * 4, c.stream));
  if (es.odeg.p && n_own > 0) {
    DevBuf srt;
    srt.alloc(size_t(n_own) * 4);
    size_t tb = 0;
    NBG_HIP(rocprim::radix_sort_keys_desc(nullptr, tb, es.odeg.as<uint32_t>(), srt.as<uint32_t>(), size_t(n_own), 0, 32,
                                          c.stream));
    c.ws_tmp.ensure(tb);
    NBG_HIP(rocprim::radix_sort_keys_desc(c.ws_tmp.p, tb, es.odeg.as<uint32_t>(), srt.as<uint32_t>(), size_t(n_own), 0,
                                          32, c.stream));
    NBG_HIP(hipMemcpyAsync(top.p, srt.p, size_t(std::min(n_own, kTopDeg)) * 4, hipMemcpyDeviceToDevice, c.stream));
  }
  const size_t row = size_t(kTopDeg) * 4 + 16;  // the degrees, then (nnz, max out-degree)
  std::vector<int64_t> mine = {csr.nnz, es.max_odeg};
  NBG_HIP(hipMemcpyAsync(top.as<uint8_t>() + size_t(kTopDeg) * 4, mine.data(), 16, hipMemcpyHostToDevice, c.stream));
  std::vector<uint8_t> all(row * G);
  DevBuf da;
  da.alloc(row * G);
  comm_allgather_bytes(c, top.p, row, da.p);
  NBG_HIP(hipMemcpyAsync(all.data(), da.p, row * G, hipMemcpyDeviceToHost, c.stream));
  host_sync(c);
  int64_t nnz = 0, mx = 0;
  std::vector<uint32_t> degs;
  for (size_t r = 0; r < G; r++) {
    const uint8_t* b = all.data() + r * row;
    int64_t v[2];
    memcpy(v, b + size_t(kTopDeg) * 4, 16);
    nnz += v[0];
    mx = v[1] < 0 || mx < 0 ? -1 : std::max(mx, v[1]);
    const uint32_t* d = reinterpret_cast<const uint32_t*>(b);
    degs.insert(degs.end(), d, d + kTopDeg);
  }
  std::sort(degs.begin(), degs.end(), std::greater<uint32_t>());
  es.top_deg.assign(size_t(kTopDeg) + 1, 0);
  if (es.odeg.p)
    for (int64_t k = 0; k < kTopDeg; k++) es.top_deg[size_t(k) + 1] = es.top_deg[size_t(k)] + int64_t(degs[size_t(k)]);
  else
    es.top_deg.clear();  // no degree array: unknown
  es.out_nnz_global = nnz;
  es.max_odeg_global = mx;
}

// ------------------------------------------------------------------------------------------
// GO N STEPS
// ------------------------------------------------------------------------------------------
int32_t go_run(Ctx& c, const nbg_go_spec& s, nbg_rows* out) {
  PoolScope pool_scope(query_pool(c));
  if (!c.finalized) throw Error(NBG_E_STATE, "snapshot not finalized");
  if (s.steps < 1) throw Error(NBG_E_INVALID_ARG, "steps must be >= 1");
  if (s.edge_type <= 0) throw Error(NBG_E_INVALID_ARG, "GO ... REVERSELY is not supported (GoExecutor.cpp:203-205)");
  auto it = c.edges.find(s.edge_type);
  if (it == c.edges.end()) throw Error(NBG_E_INVALID_ARG, "edge type not in snapshot");
  EdgeSpace& es = it->second;
  Csr& csr = es.out;
  c.timing = Timing{};
  timing_reset(c);
  // per-hop event pairs (hop stats); bench.py's timed loop turns them off like a production
  // caller would, its statistics loop on
  c.hop_timing = c.opt("hop_timing", 1) != 0;
  if (c.host_stage_used) host_sync(c);  // a failed query's copies
  c.host_stage_used = 0;
  c.total_pending = false;
  // the query's device-time events too are instrumentation: with hop_timing off none is recorded
  // (an event between two launches leaves ~5.5 us between them on the device)
  const bool tot_ev = c.hop_timing;
  if (tot_ev) hipEventRecord(c.ev[0], c.stream);

  // compile WHERE / YIELD (errors are deferred to the final step, as the reference only
  // reports them when the final getNeighbors request is actually sent)
  Program where{};
  bool has_where = s.where_len > 0;
  std::string msg;
  // $- / $var input table columns (validated here, uploaded once the starts are resolved)
  std::vector<Field> in_fields;
  if (s.n_inputs) {
    if (!s.input_names || !s.input_types || !s.input_cols) throw Error(NBG_E_INVALID_ARG, "input table");
    for (size_t i = 0; i < s.n_inputs; i++) {
      const int32_t t = s.input_types[i];
      if (t != NBG_T_VID && t != NBG_T_INT && t != NBG_T_DOUBLE && t != NBG_T_BOOL && t != NBG_T_STRING)
        throw Error(NBG_E_UNSUPPORTED, "input column type");
      if (t == NBG_T_STRING && (!s.input_str_offsets || !s.input_str_offsets[i]))
        throw Error(NBG_E_INVALID_ARG, "input STRING column without offsets");
      in_fields.push_back(Field{s.input_names[i] ? s.input_names[i] : "", t});
    }
  }
  int32_t deferred = NBG_OK;
  std::string deferred_msg;
  if (has_where) {
    int32_t rc = compile_expr(s.where, s.where_len, es.fields, true, true, &where, &msg, &c.tag_refs, in_fields.empty() ? nullptr : &in_fields);
    if (rc == NBG_E_UNSUPPORTED || rc == NBG_E_INVALID_ARG) throw Error(rc, "WHERE: " + msg);
    if (rc != NBG_OK) {
      deferred = rc;
      deferred_msg = "WHERE: " + msg;
    }
  }
  std::vector<Program> yields;
  bool default_yield = s.n_yields == 0;
  if (default_yield) {
    yields.push_back(program_dst());
  } else {
    if (s.n_yields > size_t(kMaxYields)) throw Error(NBG_E_UNSUPPORTED, "too many YIELD columns");
    for (size_t i = 0; i < s.n_yields; i++) {
      Program p{};
      int32_t rc = compile_expr(s.yields[i], s.yield_lens[i], es.fields, true, true, &p, &msg, &c.tag_refs, in_fields.empty() ? nullptr : &in_fields);
      if (rc == NBG_E_UNSUPPORTED || rc == NBG_E_INVALID_ARG) throw Error(rc, "YIELD: " + msg);
      if (rc != NBG_OK && deferred == NBG_OK) {
        deferred = rc;
        deferred_msg = "YIELD: " + msg;
      }
      if (rc == NBG_OK && p.result_type == VT_STR && s.distinct && c.sharded)
        throw Error(NBG_E_UNSUPPORTED, "DISTINCT over STRING YIELD columns across ranks");
      yields.push_back(p);
    }
  }
  bool uses_input = false;
  for (int i = 0; i < where.n && has_where; i++) uses_input |= where.ins[i].op == P_INPUT;
  for (auto& p : yields)
    for (int i = 0; i < p.n; i++) uses_input |= p.ins[i].op == P_INPUT;
  const int64_t lo = c.owned_lo(), hi = c.owned_hi();
  const int64_t n_own = hi - lo;
  ensure_workspaces(c, std::max<int64_t>({n_own, int64_t(s.n_starts), 1}));
  Counters K{c.ws_counters.as<unsigned long long>(), c.host_counters};
  DevBuf degbuf;
  uint8_t* map = c.ws_map.as<uint8_t>();
  uint16_t* bits16 = c.ws_bits_send.as<uint16_t>();  // frontier bitmap written by k_compact
  const int64_t* row_ptr = csr.row_ptr.as<int64_t>();
  const bool bu_ok = es.has_tr && c.opt("bottom_up", 1) != 0;
  const int64_t bu_div = std::max<int64_t>(1, c.opt("bu_div", 4));  // bottom-up when E >= nnz / bu_div
  const int64_t bu_force = c.opt("bu_force", 0);                     // 1: always, -1: never
  const uint8_t* row_ok = csr.row_ok.as<uint8_t>();  // rows whose keys sit outside hash(vid)'s part

  // starts -> gidx
  int64_t ns = int64_t(s.n_starts);
  c.ws_starts.ensure(size_t(std::max<int64_t>(ns, 1)) * 12 + 64);
  int64_t* d_starts = c.ws_starts.as<int64_t>();
  int32_t* d_sg = reinterpret_cast<int32_t*>(d_starts + std::max<int64_t>(ns, 1));
  // a first hop that is certainly top-down (no transposed CSR, or even the ns largest
  // out-degrees sum below the bottom-up threshold) from a few starts on one rank: one launch
  // builds its frontier and degree scan (k_starts_small) and the hop runs without a round trip
  // (the expansion reads the frontier size from the scan; the counts come back with the
  // compaction's)
  if (es.out_nnz_global < 0) global_degree_stats(c, es);
  // a first hop from ns starts is certainly top-down when even the ns largest out-degrees sum
  // below the bottom-up threshold
  const int64_t deg_bound = ns < int64_t(es.top_deg.size()) ? es.top_deg[size_t(ns)]
                            : es.max_odeg_global >= 0       ? ns * es.max_odeg_global
                                                            : INT64_MAX;
  const bool td1_certain =
      !bu_ok || bu_force < 0 || (bu_force == 0 && deg_bound < es.out_nnz_global / bu_div);
  // (with several ranks each rank's k_starts_small keeps its own starts; the hop-1 marks are
  // exchanged before the compaction)
  const bool fast1 = ns > 0 && ns <= kSmallStarts && s.steps >= 2 && td1_certain && !(uses_input && s.steps > 1) &&
                     c.opt("starts_small", 1) != 0;
  // counters summed over ranks on the device (dev_allsum) land at K.d[48, 52)
  const bool multi = c.sharded;
  // one rank: the hop-1 compaction and the speculated hops add their block sums into kSumShards
  // shards (option sum_shards; block_add_sums), folded by their readers -- the gates and the
  // counter fetches below.  Shards are zero at the query start (k_starts_small / the memset);
  // clean_shards zeroes them again before any later dense use of the same words.
  const int ks = multi ? 1 : int(std::min<int64_t>(std::max<int64_t>(c.opt("sum_shards", kSumShards), 1), kSumShards));
  bool shards_dirty = false;
  auto clean_shards = [&]() {
    if (!shards_dirty) return;
    NBG_HIP(hipMemsetAsync(K.d + kShardStride, 0, kShardStride * size_t(ks - 1) * 8, c.stream));
    shards_dirty = false;
  };
  // the small-start path's one block reads the starts from coherent pinned host memory (the
  // stream's previous query finished before this one was enqueued): no copy between queries
  const int64_t* k_starts = d_starts;
  if (ns && fast1 && c.starts_host) {
    memcpy(c.starts_host, s.starts, size_t(ns) * 8);
    k_starts = c.starts_host;
  } else if (ns) {
    c.h2d(d_starts, s.starts, size_t(ns) * 8);
    if (!fast1) lookup_gidx(c, d_starts, d_sg, ns);
  }
  int cur = 0;
  int64_t E_known = -1;  // frontier out-degree sum when a compaction already produced it
  int32_t* F = c.ws_front[0].as<int32_t>();
  int64_t nF = 0;
  int64_t nset_global = ns;  // "starts_ non-empty" (GoExecutor.cpp:93-97)
  int64_t hop1_scanned = -1;  // hop-1 rows with duplicate starts rescanned (k_starts_degree)
  int64_t Eg_known = -1;      // several ranks: the start frontier's out-degree sum over ranks
  // several ranks (option go_rep1): every rank runs the whole first hop -- every start, over a
  // replica of the out CSR (ensure_rep_out, built on first use) -- into a frontier bitmap over the
  // whole gidx space, so the hop needs no mark exchange and the second hop no frontier allgather:
  // one collective a C3 query instead of three.  (The same branch on every rank: ns, the degree
  // statistics and the options are the same everywhere.)
  // the marks of a top-down hop over this edge type are its dsts: rows with an in-edge, the
  // first bu_in_tiles tiles of the owned range (class-ordered numbering); the compactions read
  // the byte map that far and write the bitmap past it as zero
  const int64_t map_bound = es.has_tr && es.bu_in_tiles > 0 ? std::min<int64_t>(n_own, es.bu_in_tiles * 128) : n_own;
  const bool rep1 = fast1 && multi && bu_ok && c.opt("compact_list", 0) == 0 && es.odeg.p && c.opt("go_rep1", 1) != 0;
  const Csr& csr1 = rep1 ? es.rep_out : csr;  // the first hop's rows
  if (rep1) {
    ensure_rep_out(c, es);
    c.ws_bits_rep1.ensure(size_t(map_bytes(c) / 8 + 64));
  }
  // the hop-1 expansion's tile-row table is written by k_starts_small (sized for the degree bound)
  const bool starts_tiles = fast1;
  const int64_t max_odeg1 = rep1 ? es.max_odeg_global : es.max_odeg;
  if (starts_tiles) {
    const int64_t eb = std::max<int64_t>(1, max_odeg1 >= 0 ? int64_t(ns) * max_odeg1 : csr1.nnz);
    c.ws_tile_rows.ensure(size_t(std::min<int64_t>(eb, csr1.nnz + 1) / kTile + 4) * 4);
  }
  if (fast1) {
    k_starts_small<<<1, 1024, 0, c.stream>>>(
        k_starts, int32_t(ns), c.ht_keys.as<int64_t>(), c.ht_vals.as<int32_t>(), uint64_t(c.ht_cap - 1), c.ht_has_min,
        c.ht_min_gidx, d_sg, rep1 ? 0 : lo, rep1 ? c.n_global : hi, csr1.row_ptr.as<int64_t>(),
        csr1.row_ok.as<uint8_t>(), rep1 ? c.ws_bits_rep1.as<uint32_t>() : reinterpret_cast<uint32_t*>(bits16), F,
        c.ws_off.as<int64_t>(), K.d, starts_tiles ? c.ws_tile_rows.as<int32_t>() : nullptr);
    NBG_HIP(hipGetLastError());
    nF = ns;  // an upper bound: the entries past the list have degree 0
  } else {
    NBG_HIP(hipMemsetAsync(K.d, 0, kShardStride * kSumShards * 8, c.stream));
  }
  if (ns && !fast1) {
    if (s.steps == 1 && !s.distinct) {
      k_list_starts<<<grid_cap(ns), 256, 0, c.stream>>>(d_sg, ns, lo, hi, row_ptr, row_ok, F, K.d);
    } else if (!c.sharded && es.odeg.p) {
      // one rank: dedup the starts through the frontier bitmap itself (a few hundred atomics)
      // instead of marking the byte map and compacting the whole vertex space
      NBG_HIP(hipMemsetAsync(bits16, 0, c.ws_bits_send.bytes, c.stream));
      k_starts_bits<<<grid_cap(ns), 256, 0, c.stream>>>(d_sg, ns, lo, hi, es.odeg.as<uint32_t>(),
                                                        reinterpret_cast<uint32_t*>(bits16), F, K.d);
      if (!s.distinct)
        k_starts_degree<<<grid_cap(ns), 256, 0, c.stream>>>(d_sg, ns, lo, hi, row_ptr, row_ok, K.d + 30);
    } else {
      k_mark_gidx<<<grid_cap(ns), 256, 0, c.stream>>>(d_sg, ns, lo, hi, map);
      launch_compact(c, map, lo, n_own, row_ptr, row_ok, 1, F, bits16, K.d, es.odeg.as<uint32_t>());
      if (!s.distinct)
        k_starts_degree<<<grid_cap(ns), 256, 0, c.stream>>>(d_sg, ns, lo, hi, row_ptr, row_ok, K.d + 30);
    }
    NBG_HIP(hipGetLastError());
    const bool counted = !(s.steps == 1 && !s.distinct);
    if (multi && counted) dev_allsum(c, K.d, {13}, K.d + 48);
    fetch_counters(c, K.d, multi && counted ? 52 : 32, K.h);
    nF = int64_t(K.h[0]);
    if (counted) {
      E_known = int64_t(K.h[13]);
      if (multi) Eg_known = int64_t(K.h[48]);
      if (!s.distinct) hop1_scanned = int64_t(K.h[30]);
    }
  }
  unsigned long long* red = K.d + 24;  // scratch of the cross-rank sums
  auto finish_empty = [&]() -> int32_t {
    auto* h = new HostRows();
    for (auto& p : yields) {
      h->types.push_back(p.result_type == VT_DOUBLE ? NBG_T_DOUBLE
                         : p.result_type == VT_BOOL ? NBG_T_BOOL
                         : p.result_type == VT_STR  ? NBG_T_STRING
                                                    : NBG_T_VID);
      h->cols.push_back(nullptr);
      h->str_off.push_back(nullptr);
    }
    fill_rows(out, h, 0, s.keep_on_device != 0);
    hipEventRecord(c.ev[1], c.stream);
    hipEventSynchronize(c.ev[1]);
    float ms = 0;
    hipEventElapsedTime(&ms, c.ev[0], c.ev[1]);
    c.timing.total_ms = ms;
    out->edges_scanned = c.timing.edges_scanned;
    return NBG_OK;
  };
  if (nset_global == 0) return finish_empty();

  ExpandArgs a{};
  a.row_ptr = row_ptr;
  a.col = csr.col.as<int32_t>();
  a.lo = lo;
  a.map = map;
  a.err = K.d + 4;
  a.storage = 0;
  a.mark_check = 0;
  FastArgs fp{};
  EvalEnv env = make_env(c, es, csr, s.edge_type);
  DevBuf in_keys, in_rows, in_tab;
  std::vector<DevBuf> in_cols;
  // STEPS > 1: graphd maps every dst of a non-final step back to a start (VertexBackTracker,
  // GoExecutor.h:174-193, GoExecutor.cpp:420-424) in RPC response order, last write winning --
  // order-dependent whenever a vertex is reached from several starts.  The build's rule
  // (DESIGN.md): each hop reads the previous hop's roots and a dst takes the smallest root vid
  // among its in-edges' srcs; it is the reference's answer whenever the root is unique.
  const bool multi_root = uses_input && s.steps > 1;
  DevBuf root_buf[2], root_tab;
  int root_cur = 0;
  if (multi_root) {
    // rank of every start's vid among the distinct start vids
    std::vector<int64_t> u(s.starts, s.starts + ns);
    std::sort(u.begin(), u.end());
    u.erase(std::unique(u.begin(), u.end()), u.end());
    std::vector<int32_t> rk(size_t(std::max<int64_t>(ns, 1)));
    for (int64_t i = 0; i < ns; i++)
      rk[size_t(i)] = int32_t(std::lower_bound(u.begin(), u.end(), s.starts[i]) - u.begin());
    DevBuf drk;
    drk.alloc(rk.size() * 4);
    NBG_HIP(hipMemcpyAsync(drk.p, rk.data(), rk.size() * 4, hipMemcpyHostToDevice, c.stream));
    for (auto& b : root_buf) {
      b.alloc(size_t(c.n_global + 1) * 4);
      NBG_HIP(hipMemsetAsync(b.p, 0x7f, size_t(c.n_global + 1) * 4, c.stream));  // > every rank
    }
    root_tab.alloc(std::max<size_t>(u.size(), 1) * 4);
    if (ns) k_root_init<<<grid_cap(ns), 256, 0, c.stream>>>(d_sg, drk.as<int32_t>(), ns, root_buf[0].as<int32_t>(),
                                                           root_tab.as<int32_t>());
    host_sync(c);  // rk is pageable host memory
  }
  if (uses_input) {
    uint32_t cap = 64;
    while (cap < uint32_t(2 * std::max<int64_t>(ns, 1))) cap <<= 1;
    in_keys.alloc(size_t(cap) * 4);
    in_rows.alloc(size_t(cap) * 4);
    NBG_HIP(hipMemsetAsync(in_keys.p, 0xff, size_t(cap) * 4, c.stream));
    NBG_HIP(hipMemsetAsync(in_rows.p, 0xff, size_t(cap) * 4, c.stream));
    if (ns) k_input_index<<<grid_cap(ns), 256, 0, c.stream>>>(d_sg, ns, in_keys.as<int32_t>(), in_rows.as<int32_t>(), cap - 1);
    NBG_HIP(hipGetLastError());
    std::vector<PropDev> tab;
    for (size_t i = 0; i < s.n_inputs; i++) {
      const int32_t t = s.input_types[i];
      const size_t w = t == NBG_T_BOOL ? 1 : 8;
      DevBuf col, off;
      PropDev pd{t, int32_t(w), nullptr, nullptr, nullptr, nullptr};
      if (t != NBG_T_STRING) {
        col.alloc(std::max<size_t>(size_t(ns) * w, 8));
        if (ns) NBG_HIP(hipMemcpyAsync(col.p, s.input_cols[i], size_t(ns) * w, hipMemcpyHostToDevice, c.stream));
        pd.data = col.p;
      } else {
        const int64_t* ho = s.input_str_offsets[i];
        off.alloc(size_t(ns + 1) * 8);
        NBG_HIP(hipMemcpyAsync(off.p, ho, size_t(ns + 1) * 8, hipMemcpyHostToDevice, c.stream));
        col.alloc(size_t(ho[ns]) + 8);
        if (ho[ns]) NBG_HIP(hipMemcpyAsync(col.p, s.input_cols[i], size_t(ho[ns]), hipMemcpyHostToDevice, c.stream));
        pd = PropDev{t, 8, nullptr, nullptr, off.as<int64_t>(), col.as<uint8_t>()};
      }
      tab.push_back(pd);
      in_cols.push_back(std::move(col));
      in_cols.push_back(std::move(off));
    }
    in_tab.alloc(sizeof(PropDev) * tab.size());
    NBG_HIP(hipMemcpyAsync(in_tab.p, tab.data(), sizeof(PropDev) * tab.size(), hipMemcpyHostToDevice, c.stream));
    host_sync(c);  // `tab` is pageable host memory
    env.in_keys = in_keys.as<int32_t>();
    env.in_rows = in_rows.as<int32_t>();
    env.in_mask = cap - 1;
    env.iprops = in_tab.as<PropDev>();
  }

  // Frontier state: a list of local rows (top-down) and/or a bitmap (bottom-up).  E = sum of
  // the frontier's out-degrees = the adjacency entries the hop scans (TEPS numerator).
  uint32_t* bitsA = c.ws_bits_send.as<uint32_t>();
  uint32_t* bitsB = c.ws_bits_recv.as<uint32_t>();
  bool have_list = true, off_ready = false;
  int64_t E = -1;
  int64_t list_n = -1;  // length of the list the bitmap will compact to, when already counted
  auto ensure_list = [&]() {
    if (have_list) return;
    cur ^= 1;
    F = c.ws_front[cur].as<int32_t>();
    NBG_HIP(hipMemsetAsync(K.d, 0, 8, c.stream));
    k_bits_compact<0><<<grid_cap((n_own + 31) / 32, 1024, 4096), 1024, 0, c.stream>>>(bitsA, n_own, lo, nullptr, F,
                                                                                     K.d);
    if (list_n >= 0) {
      nF = list_n;  // counted by the compaction that wrote the bitmap: no round trip
    } else {
      fetch_counters(c, K.d, 1, K.h);
      nF = int64_t(K.h[0]);
    }
    list_n = -1;
    have_list = true;
    off_ready = false;
  };
  auto ensure_off = [&]() {
    ensure_list();
    if (!off_ready) {
      int64_t e2 = nF ? degree_scan(c, F, nF, csr, degbuf, E_known) : 0;
      E = e2;
      E_known = e2;
      off_ready = true;
    }
  };
  // direction choice is global (every rank must take the same branch: bottom-up allgathers)
  auto want_bu = [&](int64_t eg) {  // (multi-step roots need every in-edge: top-down only)
    return eg > 0 && bu_ok && !multi_root && bu_force >= 0 && (bu_force > 0 || eg >= es.out_nnz_global / bu_div);
  };
  int64_t Eg = 0;  // frontier out-degree sum over all ranks
  // Speculative bottom-up hops (one rank).  A direction choice needs the previous hop's counters
  // on the host, one round trip per hop; instead, right after a top-down hop's compaction, the
  // remaining hops are enqueued as bottom-up hops gated on the device (GateIn: the same rule as
  // want_bu, on the same counters) before the one counter fetch.  A hop whose gate is 0 does
  // nothing (every kernel returns at once), and the host continues from there as before: the
  // direction never changes a hop's result, only its cost.  The final step is speculated only
  // as the DISTINCT _dst bottom-up hop (a predicate that cannot error, no deferred compile
  // error).  Blocks of 16 words from K.d[64]: [0, 8) the hop's counters, [8] its gate, [9] the
  // DISTINCT output count, [10, 12) found / next out-degree sum over ranks (several ranks).
  struct Spec {
    int32_t hop;  // Timing::hops index it will take
    bool final;
    std::string k0, k1;
  };
  std::vector<Spec> spec;
  DevBuf spec_vids;
  // option host_direct: a DISTINCT _dst result that goes to the host is written by the bottom-up
  // output kernel straight into pinned host memory (mapped into the device's address space), so
  // the hand-out copies nothing
  // (r06j: stores from the device reach 54.6 GB/s into pinned host memory, hipMemcpyAsync 29.7:
  // C3's 173 MB hand-out 7.4 -> 3.8 ms end to end)
  const bool host_direct = !s.keep_on_device && c.opt("host_direct", 1) != 0;
  HostBuf spec_hvids;
  auto vid_block = [&](DevBuf& d, HostBuf& hb) -> void* {
    if (host_direct) {
      host_pool_cap(c);
      hb.release();  // (a second speculation chain in one query replaces the first's block)
      hb.alloc(c.host_pool, size_t(c.n_global + 64) * 8);
      return hb.p;
    }
    d.alloc(size_t(c.n_global + 64) * 8);
    return d.p;
  };
  FastPred fpk0{};
  FastArgs fp0{};
  bool fin_spec = false;
  if (deferred == NBG_OK) {
    fpk0 = has_where ? classify_pred(where, es.fields) : FastPred{};
    if (fpk0.kind == PK_FAST) {
      const PropCol& pc = csr.props[size_t(fpk0.col)];
      fp0 = FastArgs{pc.data.p, pc.present.as<uint8_t>(), pc.width, fpk0.op, fpk0.k};
    }
    const bool ddst = s.distinct && yields.size() == 1 && yields[0].n == 1 && yields[0].ins[0].op == P_DST;
    const bool pbu = fpk0.kind == PK_NONE ||
                     (fpk0.kind == PK_FAST && fp0.present == nullptr && es.tr.props.size() > size_t(fpk0.col) &&
                      es.tr.props[size_t(fpk0.col)].data.p);
    fin_spec = ddst && pbu;
  }
  // (several ranks: each gate reads counters summed over ranks on the device, dev_allsum, and
  // every rank enqueues the same chain of collectives, so every rank takes the same branches)
  const bool spec_ok = bu_ok && !multi_root && bu_force >= 0 && c.opt("bu_spec", 1) != 0;
  const unsigned long long spec_thr =
      bu_force > 0 ? 1ull : (unsigned long long)std::max<int64_t>(1, es.out_nnz_global / bu_div);
  unsigned long long* const SPd = K.d + 64;
  // enqueue the gated hops from step `first` on; the compaction behind them left its counts at
  // (e, n) and its bitmap in bitsA; hop0 = the Timing::hops index of the first one
  // several ranks (piggy): instead of (e, n), cnt = this rank's (n, e) of the compaction behind
  // the first hop; every hop's frontier allgather carries the previous hop's (n, e) of every rank
  // to its gate (GateIn::all), one exchange per hop instead of an allgather and an all-reduce
  bool spec_blocks_used = false;
  // fb_first (several ranks, go_rep1): the first hop reads this whole-space frontier and (e, n)
  // summed over ranks already; the hops after it exchange as with cnt
  auto spec_enqueue = [&](int32_t first, const unsigned long long* e, const unsigned long long* n, int32_t hop0,
                          const unsigned long long* cnt = nullptr, const uint32_t* fb_first = nullptr) {
    spec.clear();
    if (!spec_ok) return;
    // the blocks start at zero (query start); a second chain in one query reuses them
    if (spec_blocks_used) {
      clean_shards();
      NBG_HIP(hipMemsetAsync(SPd, 0, 16 * 12 * 8, c.stream));
    }
    spec_blocks_used = true;
    if (ks > 1) shards_dirty = true;
    const uint32_t* in = bitsA;
    uint32_t* outb = bitsB;
    const unsigned long long* pg = nullptr;
    unsigned long long* last_blk = nullptr;
    for (int32_t st = first; st <= s.steps && spec.size() < 12; st++) {
      const bool fin = st == s.steps;
      if (fin && !fin_spec) break;
      unsigned long long* blk = SPd + 16 * spec.size();
      // the hop's first pass evaluates its gate (GateIn) and publishes it at blk[8]
      GateIn gi;
      gi.e = e, gi.n = n, gi.pg = pg, gi.thr = spec_thr;
      gi.shards = ks;  // (several ranks: ks = 1)
      const int32_t hop = hop0 + int32_t(spec.size());
      // several ranks: the frontier bitmaps of every rank (the exchange runs whatever the gate
      // says: every rank enqueued it)
      const uint32_t* fb;
      if (fb_first && spec.empty()) {
        fb = fb_first;
      } else if (cnt) {
        unsigned long long* all = c.ws_piggy.as<unsigned long long>() + spec.size() * size_t(c.world) * 2;
        fb = global_bits_cnt(c, in, cnt, all);
        gi.e = gi.n = nullptr;
        gi.all = all;
        gi.world = c.world;
      } else {
        fb = global_bits(c, in);
      }
      const size_t ia = timing_event(c);
      size_t ik;
      if (!fin) {
        ik = launch_bu_lean(c, es, fb, outb, es.odeg.as<uint32_t>(), PK_NONE, fp, -1, blk, true, blk + 8, gi, true, ks);
      } else {
        FastArgs tfp = fp0;
        if (fpk0.kind == PK_FAST) tfp.data = es.tr.props[size_t(fpk0.col)].data.p;
        ik = launch_bu_lean(c, es, fb, outb, nullptr, fpk0.kind, tfp, fpk0.kind == PK_FAST ? fpk0.col : -1, blk, true,
                            blk + 8, gi, true, ks);
        void* vout = vid_block(spec_vids, spec_hvids);
        launch_bits_vids(c, outb, es.tr.n_rows, lo, vout, blk + 9, blk + 8);
      }
      NBG_HIP(hipGetLastError());
      const size_t ib = timing_event(c);
      c.tpend.push_back(Ctx::PendingTime{ia, ib, hop, 0});
      c.tpend.push_back(Ctx::PendingTime{ia, ik, hop, 1});
      spec.push_back(Spec{hop, fin, c.bu_kernel_name, c.bu_rest_name});
      e = blk + 1;
      n = blk + 0;
      last_blk = fin ? nullptr : blk;
      if (cnt || fb_first) {
        cnt = blk;  // the next hop's exchange carries this hop's (n, e)
      } else if (multi && !fin) {
        dev_allsum(c, blk, {0, 1}, blk + 10);
        e = blk + 11;
        n = blk + 10;
      }
      pg = blk + 8;
      const uint32_t* t = in;
      in = outb;
      outb = const_cast<uint32_t*>(t);
    }
    // (piggy) a chain ending on a non-final hop: its global counts for the host, at blk[12, 14)
    if (cnt && last_blk) dev_allsum(c, last_blk, {0, 1}, last_blk + 12);
  };
  // several ranks: the global (n, e) of speculated hop j after the fetch -- piggy: published by
  // hop j + 1's gate (its block's [10, 12)) or, for the chain's last hop, at [12, 14); else [10, 12)
  auto spec_global = [&](size_t j, bool piggy, unsigned long long& ng, unsigned long long& eg) {
    const unsigned long long* hh = K.h + 64 + 16 * j;
    if (!piggy) {
      ng = hh[10], eg = hh[11];
    } else if (j + 1 < spec.size()) {
      ng = hh[16 + 10], eg = hh[16 + 11];
    } else {
      ng = hh[12], eg = hh[13];
    }
  };
  bool piggy_used = false;
  auto spec_words = [&](int base) { return spec.empty() ? base : 64 + 16 * int(spec.size()); };
  auto spec_final = [&]() { return !spec.empty() && spec.back().final; };
  // after the fetch: record the hops that ran, as the bottom-up branch below does; stops at the
  // first gate that was 0 (its timings dropped).  Returns the steps consumed; *fin_done when the
  // final step ran (its counters copied to fin_h)
  unsigned long long fin_h[16] = {};
  std::string fin_k0, fin_k1;
  bool fin_done = false;
  auto spec_replay = [&]() -> int32_t {
    int32_t used = 0;
    for (size_t j = 0; j < spec.size(); j++) {
      const unsigned long long* hh = K.h + 64 + 16 * j;
      if (hh[8] == 0) {
        const int32_t cut = spec[j].hop;
        c.tpend.erase(std::remove_if(c.tpend.begin(), c.tpend.end(),
                                     [cut](const Ctx::PendingTime& p) { return p.hop >= cut; }),
                      c.tpend.end());
        break;
      }
      c.timing.spec_hops++;
      if (spec[j].final) {
        std::copy(hh, hh + 16, fin_h);
        fin_k0 = spec[j].k0;
        fin_k1 = spec[j].k1;
        fin_done = true;
        break;
      }
      c.timing.steps_run++;
      c.timing.edges_scanned += uint64_t(E);
      c.timing.expand_launches++;
      c.timing.bu_steps++;
      const uint64_t kb = bu_first_bytes(hh, es.tr.n_rows, c.bu_od_bytes), hb = kb + bu_rest_bytes(hh, 0, c.bu_rest_rec);
      c.timing.expand_bytes += hb;
      c.timing.hop(1, false, 0.0, hh, 0.0, kb);
      c.timing.name_last_hop(spec[j].k0, spec[j].k1);
      std::swap(bitsA, bitsB);
      have_list = false;
      list_n = -1;
      off_ready = false;
      E = int64_t(hh[1]);
      E_known = E;
      nset_global = int64_t(hh[0]);
      Eg = E;
      if (multi) {
        unsigned long long ng, eg;
        spec_global(j, piggy_used, ng, eg);
        nset_global = int64_t(ng);
        Eg = int64_t(eg);
      }
      used++;
      if (nset_global == 0) break;  // the caller returns the empty result
    }
    spec.clear();
    return used;
  };
  if (fast1) {
    off_ready = true;  // k_starts_small wrote the scan; E is counted on the device
  } else {
    ensure_off();
    Eg = E;
    if (Eg_known >= 0) Eg = Eg_known;
    else allsum(c, &Eg, 1, red);
  }
  for (int32_t step = 1; step < s.steps; step++) {
    c.timing.steps_run++;
    clean_shards();  // (the speculated hops' sums were fetched: dense counters from here on)
    if (fast1 && step == 1) {
      // the first hop top-down from k_starts_small's list (nF = ns bounds it), compaction, then
      // one round trip for the start counts and the next frontier's together
      a.F = F;
      a.nF = nF;
      a.off = c.ws_off.as<int64_t>();
      const int64_t e_bound = std::max<int64_t>(1, max_odeg1 >= 0 ? ns * max_odeg1 : csr1.nnz);
      ExpandArgs a1 = a;
      if (rep1) a1.row_ptr = csr1.row_ptr.as<int64_t>(), a1.col = csr1.col.as<int32_t>(), a1.lo = 0;
      launch_expand<EXP_MARK>(c, a1, PK_NONE, fp, nullptr, env, std::min<int64_t>(e_bound, csr1.nnz + 1), starts_tiles);
      cur ^= 1;
      F = c.ws_front[cur].as<int32_t>();
      const bool lazy = bu_ok && c.opt("compact_list", 0) == 0;
      // (K.d[0, 256) are zero: k_starts_small cleared the counters)
      if (rep1) {
        // the whole-space frontier and its counts (the same on every rank), plus this rank's share
        // (K.d[15, 17)) and its owned slice in bitsA (for a host-chosen top-down hop 2).  (Block
        // partials + a reduce launch instead of the block atomics measured the same: 0.4255 vs
        // 0.4243 ms a one-rank RCCL query, profiles/r13b_*)
        launch_compact(c, map, 0, c.n_global, csr1.row_ptr.as<int64_t>(), csr1.row_ok.as<uint8_t>(), 1, nullptr,
                       c.ws_bits_rep1.as<uint16_t>(), K.d, es.rep_odeg.as<uint32_t>(), true, 1, lo, hi,
                       reinterpret_cast<uint16_t*>(bitsA));
      } else if (multi && lazy && es.odeg.p) {
        // several ranks: every owner ORs the marks it receives straight into its frontier bitmap
        exchange_marks(c, map, bitsA, es.odeg.as<uint32_t>(), K.d + 12);
      } else {
        exchange_marks(c, map);  // several ranks: every owner receives the marks of its vertices
        launch_compact(c, map, lo, n_own, row_ptr, row_ok, 1, lazy ? nullptr : F, reinterpret_cast<uint16_t*>(bitsA),
                       K.d, es.odeg.as<uint32_t>(), true, ks, 0, -1, nullptr, map_bound);
        if (ks > 1) shards_dirty = true;
      }
      // several ranks: the counts over ranks -- piggy: carried by the first speculated hop's
      // frontier exchange (its gate publishes them); else found, next out-degree sum and hop-1
      // entries summed into K.d[48, 51)
      piggy_used = multi && spec_ok && (rep1 || c.opt("comm_piggy", 1) != 0);
      if (multi && !piggy_used) dev_allsum(c, K.d, {12, 13, 41}, K.d + 48);
      if (rep1)
        spec_enqueue(2, K.d + 13, K.d + 12, c.timing.n_hops + 1, nullptr, c.ws_bits_rep1.as<uint32_t>());
      else
        spec_enqueue(2, K.d + (multi ? 49 : 13), K.d + (multi ? 48 : 12), c.timing.n_hops + 1,
                     piggy_used ? K.d + 12 : nullptr);  // (hop 1: below)
      if (piggy_used && spec.empty()) {  // nothing speculated (steps == 2 without the final): sum here
        piggy_used = false;
        if (!rep1) dev_allsum(c, K.d, {12, 13, 41}, K.d + 48);
      }
      // (the device work ends here when the speculated final hop runs: ev[1] ahead of the fetch)
      fetch_counters(c, K.d, spec_words(multi ? 52 : 42), K.h, spec_final() && tot_ev ? c.ev[1] : nullptr, ks);
      const int64_t nF1 = int64_t(K.h[40]), E1 = int64_t(K.h[41]);
      if (!s.distinct) hop1_scanned = int64_t(K.h[30]);
      // (go_rep1: every rank ran the whole hop; rank 0 counts it, so the ranks' sum is the hop's)
      if (!rep1 || c.rank == 0) c.timing.edges_scanned += uint64_t(hop1_scanned >= 0 ? hop1_scanned : E1);
      if (E1 > 0) c.timing.expand_bytes += expand_bytes(nF1, E1, 0, EXP_MARK);
      const unsigned long long hs[8] = {(unsigned long long)nF1, (unsigned long long)E1, 0, 0, 0, 0, 0, 0};
      c.timing.hop(0, false, 0.0, hs);
      int64_t n1g = int64_t(K.h[12]), e1g = int64_t(K.h[13]), E1g = E1;
      if (rep1) {
        // (whole-space counts: already the sums over ranks)
      } else if (multi && piggy_used) {  // the first speculated hop's gate published hop 1's sums
        n1g = int64_t(K.h[64 + 10]);
        e1g = int64_t(K.h[64 + 11]);
        E1g = n1g;  // (no marks anywhere iff no start has out-edges: the empty result either way)
      } else if (multi) {
        n1g = int64_t(K.h[48]);
        e1g = int64_t(K.h[49]);
        E1g = int64_t(K.h[50]);
      }
      if (E1g == 0) return finish_empty();  // every start lacks out-edges
      nF = lazy ? 0 : int64_t(K.h[0]);
      list_n = lazy ? int64_t(K.h[rep1 ? 15 : 14]) : -1;
      E = int64_t(K.h[rep1 ? 16 : 13]);
      E_known = E;
      nset_global = n1g;
      Eg = e1g;
      have_list = !lazy;
      if (lazy) cur ^= 1;  // ensure_list flips to the list buffer again
      off_ready = false;
      if (nset_global == 0) return finish_empty();  // onEmptyInputs (GoExecutor.cpp:392-395)
      step += spec_replay();
      if (nset_global == 0) return finish_empty();
      if (fin_done) break;
      continue;
    }
    c.timing.edges_scanned += uint64_t(step == 1 && hop1_scanned >= 0 ? hop1_scanned : E);
    if (Eg == 0) return finish_empty();  // every frontier vertex lacks out-edges
    if (want_bu(Eg)) {
      // bottom-up: frontier bitmap in, next frontier bitmap out
      const Csr& tr = es.tr;
      const uint32_t* fb = global_bits(c, bitsA);
      const size_t ia = timing_event(c);
      const size_t ik = launch_bu_lean(c, es, fb, bitsB, es.odeg.as<uint32_t>(), PK_NONE, fp, -1, K.d, step > 1);
      const size_t ib = timing_event(c);
      c.tpend.push_back(Ctx::PendingTime{ia, ib, c.timing.n_hops, 0});
      c.tpend.push_back(Ctx::PendingTime{ia, ik, c.timing.n_hops, 1});
      if (multi) dev_allsum(c, K.d, {0, 1}, K.d + 48);
      fetch_counters(c, K.d, multi ? 50 : 8, K.h);
      c.timing.expand_launches++;
      c.timing.bu_steps++;
      const uint64_t kb = bu_first_bytes(K.h, tr.n_rows, c.bu_od_bytes), hb = kb + bu_rest_bytes(K.h, 0, c.bu_rest_rec);
      c.timing.expand_bytes += hb;
      c.timing.hop(1, false, 0.0, K.h, 0.0, kb);
      c.timing.name_last_hop(c.bu_kernel_name, c.bu_rest_name);
      std::swap(bitsA, bitsB);
      have_list = false;
      // one rank: the found rows the two passes counted are the new bitmap's population (every
      // found row sets one bit; pending rows are disjoint from the first pass's found rows), so
      // ensure_list needs no round trip; several ranks: the local population is read back
      list_n = multi ? -1 : int64_t(K.h[0]);
      off_ready = false;
      E = int64_t(K.h[1]);
      E_known = E;
      nset_global = multi ? int64_t(K.h[48]) : int64_t(K.h[0]);
      Eg = multi ? int64_t(K.h[49]) : E;
    } else {
      ensure_off();
      a.F = F;
      a.nF = nF;
      a.off = c.ws_off.as<int64_t>();
      const double ms0 = c.timing.expand_ms;
      if (multi_root) {
        NBG_HIP(hipMemsetAsync(root_buf[root_cur ^ 1].p, 0x7f, size_t(c.n_global + 1) * 4, c.stream));
        a.root_cur = root_buf[root_cur].as<int32_t>();
        a.root_next = root_buf[root_cur ^ 1].as<int32_t>();
      }
      if (E > 0) {
        launch_expand<EXP_MARK>(c, a, PK_NONE, fp, nullptr, env, E);
        c.timing.expand_bytes += expand_bytes(nF, E, 0, EXP_MARK);
      }
      if (multi_root) {
        exchange_roots(c, a.root_next);
        root_cur ^= 1;
        a.root_cur = nullptr;
        a.root_next = nullptr;
      }
      const unsigned long long hs[8] = {(unsigned long long)nF, (unsigned long long)E, 0, 0, 0, 0, 0, 0};
      c.timing.hop(0, false, c.timing.expand_ms - ms0, hs);
      exchange_marks(c, map);
      // next frontier = set of dsts (P12): compact, drop rows without out-edges, bitmap too
      cur ^= 1;
      F = c.ws_front[cur].as<int32_t>();
      NBG_HIP(hipMemsetAsync(K.d, 0, 32, c.stream));
      // when the next hop may go bottom-up it reads the bitmap alone: the list is left to
      // ensure_list (option compact_list = 1 always writes it here).  One rank only: this
      // bitmap is slice-relative, ensure_list's input is the bottom-up's global-indexed one
      const bool lazy = bu_ok && !multi_root && c.opt("compact_list", 0) == 0;
      launch_compact(c, map, lo, n_own, row_ptr, row_ok, 1, lazy ? nullptr : F, reinterpret_cast<uint16_t*>(bitsA),
                     K.d, es.odeg.as<uint32_t>(), false, 1, 0, -1, nullptr, map_bound);
      piggy_used = multi && lazy && spec_ok && c.opt("comm_piggy", 1) != 0;
      if (multi && !piggy_used) dev_allsum(c, K.d, {12, 13}, K.d + 48);
      if (lazy)
        spec_enqueue(step + 1, K.d + (multi ? 49 : 13), K.d + (multi ? 48 : 12), c.timing.n_hops,
                     piggy_used ? K.d + 12 : nullptr);
      if (piggy_used && spec.empty()) {
        piggy_used = false;
        dev_allsum(c, K.d, {12, 13}, K.d + 48);
      }
      fetch_counters(c, K.d, spec_words(multi ? 50 : 16), K.h, spec_final() && tot_ev ? c.ev[1] : nullptr, ks);
      nF = lazy ? 0 : int64_t(K.h[0]);
      list_n = lazy ? int64_t(K.h[14]) : -1;
      E = int64_t(K.h[13]);
      E_known = E;
      nset_global = int64_t(K.h[12]);
      Eg = E;
      if (multi) {
        nset_global = int64_t(piggy_used ? K.h[64 + 10] : K.h[48]);
        Eg = int64_t(piggy_used ? K.h[64 + 11] : K.h[49]);
      }
      have_list = !lazy;
      if (lazy) cur ^= 1;  // ensure_list flips to the list buffer again
      off_ready = false;
    }
    if (nset_global == 0) return finish_empty();  // onEmptyInputs (GoExecutor.cpp:392-395)
    if (!spec.empty()) {
      step += spec_replay();
      if (nset_global == 0) return finish_empty();
      if (fin_done) break;
    }
  }
  // ---- final step ----
  c.timing.steps_run++;
  if (!fin_done) clean_shards();
  if (multi_root) {
    env.in_root = root_buf[root_cur].as<int32_t>();
    env.in_root_tab = root_tab.as<int32_t>();
  }
  if (deferred != NBG_OK) throw Error(deferred, deferred_msg);
  FastPred fpk = has_where ? classify_pred(where, es.fields) : FastPred{};
  int pk = fpk.kind;
  if (pk == PK_FAST) {
    const PropCol& pc = csr.props[size_t(fpk.col)];
    fp = FastArgs{pc.data.p, pc.present.as<uint8_t>(), pc.width, fpk.op, fpk.k};
  }
  DevBuf dprog;
  // DISTINCT _dst reads no YIELD program (and the WHERE program only on the VM path)
  const bool lone_dst_distinct = s.distinct && yields.size() == 1 && yields[0].n == 1 && yields[0].ins[0].op == P_DST;
  if (pk == PK_VM || (!default_yield && !lone_dst_distinct)) {
    dprog.alloc(sizeof(Program) * (yields.size() + 1));
    c.h2d(dprog.p, &where, sizeof(Program));
    c.h2d(dprog.as<Program>() + 1, yields.data(), sizeof(Program) * yields.size());
  }
  int pred_w = pk == PK_FAST ? fp.width : 0;
  c.timing.edges_scanned += uint64_t(E);
  bool distinct_dst = s.distinct && yields.size() == 1 && yields[0].n == 1 && yields[0].ins[0].op == P_DST;
  auto* h = new HostRows();
  int64_t nrows = 0;
  std::vector<DevBuf> slen(yields.size());  // STRING yield columns: byte length per row
  std::map<size_t, bool> host_cols;         // columns already in pinned host memory (host_direct)
  try {
    if (distinct_dst) {
      // DISTINCT e._dst: mark surviving dsts, compact the whole vertex space (no deg filter).
      // Bottom-up only when the predicate cannot error (the reference fails the query on any
      // row's eval error, so every row must be evaluated when errors are possible).
      bool pred_bu = pk == PK_NONE || (pk == PK_FAST && fp.present == nullptr &&
                                       es.tr.props.size() > size_t(fpk.col) && es.tr.props[size_t(fpk.col)].data.p);
      bool bu = pred_bu && want_bu(Eg);
      DevBuf vids;
      HostBuf hvids;
      void* vout = nullptr;
      if (fin_done) {
        // the speculated final hop ran (spec_replay): its counters, rows and kernel names
        vids = std::move(spec_vids);
        hvids = std::move(spec_hvids);
        c.timing.expand_launches++;
        c.timing.bu_steps++;
        nrows = int64_t(fin_h[9]);
        const int pw = pk == PK_FAST ? fp.width : 0;
        const uint64_t kb = bu_first_bytes(fin_h, es.tr.n_rows, 0), hb = kb + bu_rest_bytes(fin_h, pw, c.bu_rest_rec);
        c.timing.expand_bytes += hb + uint64_t(es.tr.n_rows) / 8 + uint64_t(nrows) * 16;
        c.timing.hop(1, true, 0.0, fin_h, 0.0, kb);
        c.timing.name_last_hop(fin_k0, fin_k1, "nbg::k_bits_compact<1, 8, 1>");
      } else {
        vout = nullptr;
      }
      if (fin_done) {
      } else if (bu) {
        FastArgs tfp = fp;
        if (pk == PK_FAST) tfp.data = es.tr.props[size_t(fpk.col)].data.p;
        const Csr& tr = es.tr;
        NBG_HIP(hipMemsetAsync(K.d, 0, 8, c.stream));
        const uint32_t* fb = global_bits(c, bitsA);
        const size_t ia = timing_event(c);
        const size_t ik =
            launch_bu_lean(c, es, fb, bitsB, nullptr, pk, tfp, pk == PK_FAST ? fpk.col : -1, K.d + 8, s.steps > 1);
        vout = vid_block(vids, hvids);
        launch_bits_vids(c, bitsB, tr.n_rows, lo, vout, K.d, nullptr);
        NBG_HIP(hipGetLastError());
        const size_t ib = timing_event(c);
        c.tpend.push_back(Ctx::PendingTime{ia, ib, c.timing.n_hops, 0});
        c.tpend.push_back(Ctx::PendingTime{ia, ik, c.timing.n_hops, 1});
        fetch_counters(c, K.d, 16, K.h);
        c.timing.expand_launches++;
        c.timing.bu_steps++;
        nrows = int64_t(K.h[0]);
        const int pw = pk == PK_FAST ? tfp.width : 0;
        const uint64_t kb = bu_first_bytes(K.h + 8, tr.n_rows, 0), hb = kb + bu_rest_bytes(K.h + 8, pw, c.bu_rest_rec);
        // + the DISTINCT _dst output (k_bits_compact<1>): next bits once, vid_of read + vid written
        c.timing.expand_bytes += hb + uint64_t(tr.n_rows) / 8 + uint64_t(nrows) * 16;
        c.timing.hop(1, true, 0.0, K.h + 8, 0.0, kb);
        c.timing.name_last_hop(c.bu_kernel_name, c.bu_rest_name, "nbg::k_bits_compact<1, 8, 1>");
      } else {
        vids.alloc(size_t(c.n_global + 64) * 8);
        ensure_off();
        a.F = F;
        a.nF = nF;
        a.off = c.ws_off.as<int64_t>();
        const double ms0 = c.timing.expand_ms;
        if (E > 0) {
          launch_expand<EXP_MARK>(c, a, pk, fp, dprog.as<Program>(), env, E);
          c.timing.expand_bytes += expand_bytes(nF, E, pred_w, EXP_MARK);
        }
        const unsigned long long hs[8] = {(unsigned long long)nF, (unsigned long long)E, 0, 0, 0, 0, 0, 0};
        c.timing.hop(0, true, c.timing.expand_ms - ms0, hs);
        exchange_marks(c, map);
        DevBuf lst;
        lst.alloc(size_t(n_own + 64) * 4);
        NBG_HIP(hipMemsetAsync(K.d, 0, 16, c.stream));  // keep the eval-error counter (K.d[4])
        launch_compact(c, map, lo, n_own, row_ptr, nullptr, 0, lst.as<int32_t>(), nullptr, K.d);
        if (multi) dev_allsum(c, K.d, {4}, K.d + 48);
        fetch_counters(c, K.d, multi ? 49 : 6, K.h);
        const int64_t errs = int64_t(K.h[multi ? 48 : 4]);
        if (errs) throw Error(NBG_E_EVAL, "WHERE evaluation failed");
        nrows = int64_t(K.h[0]);
        if (nrows)
          k_local_to_vid<<<grid_cap(nrows), 256, 0, c.stream>>>(lst.as<int32_t>(), nrows, lo, c.vid_of.as<int64_t>(),
                                                               vids.as<int64_t>());
      }
      h->types.push_back(NBG_T_VID);
      if (hvids.p) {  // already on the host (host_direct)
        host_cols[h->dev.size()] = true;
        h->hpin.push_back(std::move(hvids));
      }
      h->dev.push_back(std::move(vids));
    } else {
      // rows (src, edge) passing WHERE; a lone YIELD _dst (the default) is written directly as
      // vids by the expansion (no row list, no materialisation pass)
      ensure_off();
      a.F = F;
      a.nF = nF;
      a.off = c.ws_off.as<int64_t>();
      const bool dst_only = yields.size() == 1 && yields[0].n == 1 && yields[0].ins[0].op == P_DST;
      DevBuf fused;
      int64_t* rows_edge = nullptr;
      int32_t* rows_src = nullptr;
      if (dst_only) {
        fused.alloc(size_t(E + 64) * 8);
        a.out_vid = fused.as<int64_t>();
        a.vid_of = c.vid_of.as<int64_t>();
        a.col_vid = csr.col_vid.as<int64_t>();
      } else {
        c.ws_rows.ensure(size_t(E + 64) * 12);
        rows_edge = c.ws_rows.as<int64_t>();
        rows_src = reinterpret_cast<int32_t*>(rows_edge + E + 32);
      }
      a.rows_edge = rows_edge;
      a.rows_src = rows_src;
      a.rows_cnt = K.d + 2;
      NBG_HIP(hipMemsetAsync(K.d, 0, 48, c.stream));
      const double ms0 = c.timing.expand_ms;
      if (E > 0) launch_expand<EXP_ROWS>(c, a, pk, fp, dprog.as<Program>(), env, E);
      if (multi) dev_allsum(c, K.d, {4}, K.d + 48);
      fetch_counters(c, K.d, multi ? 49 : 6, K.h);
      const int64_t errs = int64_t(K.h[multi ? 48 : 4]);
      if (errs) throw Error(NBG_E_EVAL, "WHERE evaluation failed");
      const bool direct = dst_only && pk == PK_NONE;  // every edge is a row, written at its index
      nrows = direct ? E : int64_t(K.h[2]);
      // the hop's bytes: frontier entries + per edge the col (+ predicate);
      // per row its 8 B vid write and where the vid comes from: the 8 B dst-vid column read
      // instead of col (direct rows), else an 8 B vid_of gather behind the col read (a 4 B
      // (src) + 8 B (edge) row pair without the fused _dst)
      if (E > 0) {
        if (direct && csr.col_vid.p)
          c.timing.expand_bytes += uint64_t(nF) * 28 + uint64_t(E) * 16;
        else
          c.timing.expand_bytes += expand_bytes(nF, E, pred_w, EXP_ROWS) + uint64_t(nrows) * (dst_only ? 16 : 12);
      }
      const unsigned long long hs[8] = {(unsigned long long)nF, (unsigned long long)E, uint64_t(nrows), 0, 0, 0, 0, 0};
      c.timing.hop(0, true, c.timing.expand_ms - ms0, hs);
      YieldArgs ya{};
      ya.ncols = int32_t(yields.size());
      for (auto& p : yields) {
        int32_t t = p.result_type;
        DevBuf b;
        if (dst_only) b = std::move(fused);
        else b.alloc(size_t(nrows + 1) * (t == VT_BOOL ? 1 : 8));
        const size_t k = h->types.size();
        if (t == VT_STR) slen[k].alloc(size_t(nrows + 1) * 8);
        ya.cols[k] = ColOut{b.p, t, slen[k].as<int64_t>()};
        h->types.push_back(t == VT_DOUBLE ? NBG_T_DOUBLE : t == VT_BOOL ? NBG_T_BOOL : t == VT_STR ? NBG_T_STRING : NBG_T_VID);
        h->dev.push_back(std::move(b));
      }
      if (nrows && !dst_only) {
        if (default_yield) {
          k_yield_dst<<<grid_cap(nrows), 256, 0, c.stream>>>(rows_edge, nrows, csr.col.as<int32_t>(),
                                                             c.vid_of.as<int64_t>(), h->dev[0].as<int64_t>());
        } else {
          k_materialize<<<grid_cap(nrows), 256, 0, c.stream>>>(rows_src, rows_edge, nrows, dprog.as<Program>() + 1, ya,
                                                               env, lo, K.d + 5);
        }
        NBG_HIP(hipGetLastError());
      }
      if (!dst_only) {  // (the fused _dst rows evaluate nothing: no error count to read)
        if (multi) dev_allsum(c, K.d, {5}, K.d + 48);
        fetch_counters(c, K.d, multi ? 49 : 6, K.h);
        const int64_t yerr = int64_t(K.h[multi ? 48 : 5]);
        if (yerr) throw Error(NBG_E_EVAL, "YIELD evaluation failed");
      }
      if (s.distinct && c.sharded) nrows = shuffle_rows(c, ya, h->dev, nrows);
      if (s.distinct && nrows) {
        uint64_t cap = 1024;
        while (cap < uint64_t(2 * nrows)) cap <<= 1;
        for (size_t cc = 0; cc < h->dev.size(); cc++) ya.cols[cc].data = h->dev[cc].p;
        DevBuf table, keep, idx, cnt;
        table.alloc(cap * 8);
        NBG_HIP(hipMemsetAsync(table.p, 0xff, cap * 8, c.stream));
        keep.alloc(size_t(nrows));
        k_row_dedup<<<grid_cap(nrows), 256, 0, c.stream>>>(ya, nrows, table.as<long long>(), cap - 1, keep.as<uint8_t>());
        cnt.alloc(8);
        int64_t kept = 0;
        for (size_t cc = 0; cc < h->dev.size(); cc++) {
          DevBuf nb;
          bool is_bool = ya.cols[cc].type == VT_BOOL;
          nb.alloc(size_t(nrows + 1) * (is_bool ? 1 : 8));
          size_t tb = 0;
          if (is_bool) {
            NBG_HIP(rocprim::select(nullptr, tb, h->dev[cc].as<uint8_t>(), keep.as<uint8_t>(), nb.as<uint8_t>(),
                                    cnt.as<uint64_t>(), size_t(nrows), c.stream));
            c.ws_tmp.ensure(tb);
            NBG_HIP(rocprim::select(c.ws_tmp.p, tb, h->dev[cc].as<uint8_t>(), keep.as<uint8_t>(), nb.as<uint8_t>(),
                                    cnt.as<uint64_t>(), size_t(nrows), c.stream));
          } else {
            NBG_HIP(rocprim::select(nullptr, tb, h->dev[cc].as<int64_t>(), keep.as<uint8_t>(), nb.as<int64_t>(),
                                    cnt.as<uint64_t>(), size_t(nrows), c.stream));
            c.ws_tmp.ensure(tb);
            NBG_HIP(rocprim::select(c.ws_tmp.p, tb, h->dev[cc].as<int64_t>(), keep.as<uint8_t>(), nb.as<int64_t>(),
                                    cnt.as<uint64_t>(), size_t(nrows), c.stream));
          }
          if (ya.cols[cc].type == VT_STR) {
            DevBuf nl;
            nl.alloc(size_t(nrows + 1) * 8);
            NBG_HIP(rocprim::select(nullptr, tb, slen[cc].as<int64_t>(), keep.as<uint8_t>(), nl.as<int64_t>(),
                                    cnt.as<uint64_t>(), size_t(nrows), c.stream));
            c.ws_tmp.ensure(tb);
            NBG_HIP(rocprim::select(c.ws_tmp.p, tb, slen[cc].as<int64_t>(), keep.as<uint8_t>(), nl.as<int64_t>(),
                                    cnt.as<uint64_t>(), size_t(nrows), c.stream));
            slen[cc] = std::move(nl);
          }
          uint64_t kc = 0;
          NBG_HIP(hipMemcpyAsync(&kc, cnt.p, 8, hipMemcpyDeviceToHost, c.stream));
          host_sync(c);
          kept = int64_t(kc);
          h->dev[cc] = std::move(nb);
        }
        nrows = kept;
      }
    }
  } catch (...) {
    delete h;
    throw;
  }
  // ev[1] ends the device time; not waited for here (resolve_total reads it when asked): a
  // speculated final hop recorded it ahead of its counter fetch, after which nothing was enqueued
  if (tot_ev && !fin_done) hipEventRecord(c.ev[1], c.stream);
  c.total_pending = tot_ev;
  // STRING columns: (address, length) rows -> packed bytes + n+1 offsets
  const size_t ncols_out = h->types.size();
  std::vector<int64_t> soff_dev_idx(ncols_out, -1);
  try {
    for (size_t cc = 0; cc < ncols_out; cc++) {
      if (h->types[cc] != NBG_T_STRING) continue;
      DevBuf off, bytes;
      off.alloc(size_t(nrows + 1) * 8);
      NBG_HIP(hipMemsetAsync(slen[cc].as<int64_t>() + nrows, 0, 8, c.stream));
      exclusive_scan_dev<int64_t>(c, slen[cc].as<int64_t>(), off.as<int64_t>(), nrows + 1);
      int64_t total = 0;
      NBG_HIP(hipMemcpyAsync(&total, off.as<int64_t>() + nrows, 8, hipMemcpyDeviceToHost, c.stream));
      host_sync(c);
      bytes.alloc(size_t(total) + 8);
      if (nrows && total)
        k_str_pack<<<grid_cap(nrows), 256, 0, c.stream>>>(h->dev[cc].as<int64_t>(), off.as<int64_t>(), nrows,
                                                          bytes.as<uint8_t>());
      NBG_HIP(hipGetLastError());
      h->dev[cc] = std::move(bytes);
      soff_dev_idx[cc] = int64_t(h->dev.size());
      h->dev.push_back(std::move(off));
    }
    // the result is complete before it is handed out: a host copy waits for its own copies
    // (below); device columns need the stream drained, which the counter fetch of a speculated
    // final hop already saw (nothing was enqueued after it)
    // (STRING columns and very large ones are copied with the blocking hipMemcpy, which does not
    // order behind the engine stream: drained first)
    bool drain = s.keep_on_device ? !fin_done : false;
    for (size_t cc = 0; cc < ncols_out && !s.keep_on_device; cc++) {
      const size_t w = h->types[cc] == NBG_T_BOOL ? 1 : 8;
      drain |= soff_dev_idx[cc] >= 0 ||
               size_t(nrows) * w + 8 > size_t(std::max<int64_t>(0, c.opt("host_pinned_mb", 4096))) << 20;
    }
    if (drain && hipStreamQuery(c.stream) != hipSuccess) host_sync(c);
    if (s.keep_on_device || drain) c.host_stage_used = 0;  // the query's input copies have completed
  } catch (...) {
    delete h;
    throw;
  }
  // hand the columns out (a failed pinned allocation or copy frees the rows and rethrows)
  bool on_dev = s.keep_on_device != 0;
  try {
  for (size_t cc = 0; cc < ncols_out; cc++) {
    if (soff_dev_idx[cc] >= 0) {  // STRING
      DevBuf& off = h->dev[size_t(soff_dev_idx[cc])];
      if (on_dev) {
        h->cols.push_back(h->dev[cc].p);
        h->str_off.push_back(off.as<int64_t>());
      } else {
        h->host_off.emplace_back(size_t(nrows) + 1);
        NBG_HIP(hipMemcpy(h->host_off.back().data(), off.p, size_t(nrows + 1) * 8, hipMemcpyDeviceToHost));
        const size_t total = size_t(h->host_off.back()[size_t(nrows)]);
        h->host.emplace_back(total + 8);
        if (total) NBG_HIP(hipMemcpy(h->host.back().data(), h->dev[cc].p, total, hipMemcpyDeviceToHost));
        h->cols.push_back(h->host.back().data());
        h->str_off.push_back(h->host_off.back().data());
      }
      continue;
    }
    h->str_off.push_back(nullptr);
    if (host_cols.count(cc)) {  // written into pinned host memory by the output kernel
      // the block spans the vertex space (n_global vids): a result far smaller than it is copied
      // into a right-sized pinned block, so a result the caller keeps pins about its own size (the
      // large block returns to the context's pinned cache, whose cap bounds what stays held)
      HostBuf& big = h->hpin.back();
      const size_t need = size_t(nrows) * 8 + 8;
      if (need * 4 < big.bytes && need <= (size_t(64) << 20)) {
        HostBuf small;
        small.alloc(c.host_pool, need);
        if (nrows) memcpy(small.p, big.p, size_t(nrows) * 8);
        big = std::move(small);
      }
      h->cols.push_back(h->hpin.back().p);
    } else if (on_dev) {
      h->cols.push_back(h->dev[cc].p);
    } else {
      size_t w = h->types[cc] == NBG_T_BOOL ? 1 : 8;
      const size_t bytes = size_t(nrows) * w + 8;
      if (bytes <= size_t(std::max<int64_t>(0, c.opt("host_pinned_mb", 4096))) << 20) {
        h->hpin.emplace_back();
        if (h->hpin.size() == 1) host_pool_cap(c);
        h->hpin.back().alloc(c.host_pool, bytes);
        if (nrows)
          NBG_HIP(hipMemcpyAsync(h->hpin.back().p, h->dev[cc].p, size_t(nrows) * w, hipMemcpyDeviceToHost, c.stream));
        h->cols.push_back(h->hpin.back().p);
      } else {  // very large results (RMAT-28's 21 GB of rows): pageable, through the driver
        h->host.emplace_back(bytes);
        if (nrows) NBG_HIP(hipMemcpy(h->host.back().data(), h->dev[cc].p, size_t(nrows) * w, hipMemcpyDeviceToHost));
        h->cols.push_back(h->host.back().data());
      }
    }
  }
  if (!on_dev) {
    host_sync(c);  // the pinned copies above (and with them the whole query)
    c.host_stage_used = 0;
    h->dev.clear();
  }
  } catch (...) {
    (void)hipStreamSynchronize(c.stream);  // no copy may still target a block freed here
    delete h;
    throw;
  }
  fill_rows(out, h, nrows, on_dev);
  out->edges_scanned = c.timing.edges_scanned;
  return NBG_OK;
}

void timing_reset(Ctx& c) {
  c.tev_used = 0;
  c.tpend.clear();
}
// adds the deferred expansion times to expand_ms and their hops (after the query's last sync)
void timing_resolve(Ctx& c) {
  for (const auto& p : c.tpend) {
    float ms = 0;
    if (p.a == kNoEvent || p.b == kNoEvent) continue;
    if (hipEventSynchronize(c.tev[p.b]) == hipSuccess && hipEventElapsedTime(&ms, c.tev[p.a], c.tev[p.b]) == hipSuccess) {
      const bool in_hop = p.hop >= 0 && p.hop < c.timing.n_hops && p.hop < NBG_MAX_HOP_STATS;
      if (p.kind == 1) {  // a bottom-up hop's first pass
        if (in_hop) c.timing.hops[p.hop].kernel_ms += ms;
        continue;
      }
      if (p.kind == 2) {  // an exchange between ranks
        c.timing.comm_ms += ms;
        continue;
      }
      c.timing.expand_ms += ms;
      if (in_hop) {
        c.timing.hops[p.hop].ms += ms;
        if (c.timing.hops[p.hop].mode == 0) c.timing.hops[p.hop].kernel_ms += ms;  // k_expand is the hop
      }
    }
  }
  timing_reset(c);
}

// ------------------------------------------------------------------------------------------
// getBound (QueryBoundProcessor)
// ------------------------------------------------------------------------------------------
// request entry -> local row; a (part, vid) pair whose part does not hold the vertex's keys scans
// an empty prefix in the reference, so it gets a zero-degree stand-in (-1)
__global__ void k_bound_frontier(const int32_t* parts, const int32_t* g, int64_t n, int64_t lo, int64_t hi,
                                 const int32_t* row_part, int32_t* F) {
  for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < n; i += int64_t(gridDim.x) * blockDim.x) {
    int32_t x = g[i];
    bool ok = x >= lo && x < hi && row_part[x - lo] == parts[i];
    F[i] = ok ? int32_t(x - lo) : -1;
  }
}
__global__ void k_degrees_masked(const int32_t* F, int64_t n, const int64_t* row_ptr, int64_t* deg) {
  for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i <= n; i += int64_t(gridDim.x) * blockDim.x) {
    if (i == n) deg[i] = 0;
    else deg[i] = F[i] < 0 ? 0 : row_ptr[F[i] + 1] - row_ptr[F[i]];
  }
}
// request entries with deg 0 are removed so every frontier entry covers >= 1 edge slot
__global__ void k_slot_owner(const int64_t* kept_slots, int64_t m, const int64_t* off, int64_t nF, int64_t* owner) {
  for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < m; i += int64_t(gridDim.x) * blockDim.x) {
    int64_t e = kept_slots[i];
    int64_t lo = 0, hi = nF;
    while (hi - lo > 1) {
      int64_t mid = (lo + hi) >> 1;
      if (off[mid] <= e) lo = mid; else hi = mid;
    }
    owner[i] = lo;
  }
}
struct BoundCol {
  int32_t kind;  // 0 prop, 1 _dst, 2 _src, 3 _rank, 4 _type
  int32_t prop;
  int32_t type;  // NBG_T_*
  int32_t stat;  // outBoundStats: cpp2::StatType SUM 1 / COUNT 2 / AVG 3 (0: plain getBound)
  void* out;
  int64_t* str_len;  // STRING pass 1
};
constexpr int kMaxBoundCols = 32;
struct BoundCols {
  int32_t n;
  BoundCol c[kMaxBoundCols];
};
// flattened slot -> edge index of the kept rows
__global__ void k_slot_ge(const int64_t* kept_slots, const int64_t* owner, int64_t m, const int64_t* off,
                          const int32_t* F, const int64_t* row_ptr, int64_t* ge) {
  for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < m; i += int64_t(gridDim.x) * blockDim.x) {
    const int64_t k = owner[i];
    ge[i] = row_ptr[F[k]] + (kept_slots[i] - off[k]);
  }
}
// one value of a getBound column for row i: edge ge's key props, and its props either from the
// CSR (old < 0) or from the older-version side table (row old, Csr::ov_*)
__device__ inline int64_t bound_value(const BoundCol& b, int64_t ge, int64_t old, int32_t f, int64_t lo,
                                      const EvalEnv& env, const PropDev* oprops, bool& present) {
  present = true;
  switch (b.kind) {
    case 1: return env.vid_of[env.col[ge]];
    case 2: return env.vid_of[lo + f];
    case 3: return env.rank ? env.rank[ge] : 0;
    case 4: return env.etype;
    default: {
      const PropDev& p = old < 0 ? env.props[b.prop] : oprops[b.prop];
      const int64_t x = old < 0 ? ge : old;
      if (p.present && !p.present[x]) {
        present = false;
        return INT64_MIN;
      }
      if (p.type == NBG_T_STRING) return x;
      if (p.type == NBG_T_DOUBLE || p.type == NBG_T_FLOAT) return static_cast<const int64_t*>(p.data)[x];
      return load_int(p.data, p.width, x);
    }
  }
}
__global__ void k_bound_rows(const int64_t* ge_in, const int64_t* old_in, const int64_t* owner, int64_t m,
                             const int32_t* F, int64_t lo, EvalEnv env, const PropDev* oprops, BoundCols bc) {
  for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < m; i += int64_t(gridDim.x) * blockDim.x) {
    const int64_t ge = ge_in[i];
    const int64_t old = old_in ? old_in[i] : -1;
    const int32_t f = F[owner[i]];
    for (int c = 0; c < bc.n; c++) {
      const BoundCol& b = bc.c[c];
      bool present;
      const int64_t v = bound_value(b, ge, old, f, lo, env, oprops, present);
      if (b.kind == 0) {
        const PropDev& p = old < 0 ? env.props[b.prop] : oprops[b.prop];
        if (p.type == NBG_T_STRING) {
          b.str_len[i] = present ? p.str_off[v + 1] - p.str_off[v] : -1;
          continue;
        }
      }
      if (b.type == NBG_T_BOOL) static_cast<uint8_t*>(b.out)[i] = uint8_t(v != 0);
      else static_cast<int64_t*>(b.out)[i] = v;
    }
  }
}
// outBoundStats / inBoundStats (QueryStatsProcessor.cpp:69-125, StatsCollector Collector.h:66-94):
// over the kept rows, the int64 sum (wrapping, as the reference's int64 adds) and the count of
// present values of column c.  acc[2c] = sum, acc[2c+1] = count.  Doubles only count (a double
// reaching the reference's int64-initialised sum throws, reported by the caller).
__global__ void k_bound_stats(const int64_t* ge_in, const int64_t* old_in, const int64_t* owner, int64_t m,
                              const int32_t* F, int64_t lo, EvalEnv env, const PropDev* oprops, BoundCol b,
                              unsigned long long* acc) {
  unsigned long long sum = 0, cnt = 0;
  for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < m; i += int64_t(gridDim.x) * blockDim.x) {
    const int64_t old = old_in ? old_in[i] : -1;
    bool present;
    int64_t v = bound_value(b, ge_in[i], old, F[owner[i]], lo, env, oprops, present);
    if (b.kind == 0) {
      const int32_t t = (old < 0 ? env.props[b.prop] : oprops[b.prop]).type;
      if (t == NBG_T_STRING || t == NBG_T_DOUBLE || t == NBG_T_FLOAT || t == NBG_T_BOOL) v = 0;
    }
    if (present) {
      sum += (unsigned long long)v;
      cnt++;
    }
  }
  sum = wave_sum_u64(sum);
  cnt = wave_sum_u64(cnt);
  if ((threadIdx.x & 63) == 0 && cnt) {
    atomicAdd(acc, sum);
    atomicAdd(acc + 1, cnt);
  }
}

// collectEdgeProps' firstLoop (QueryBaseProcessor.inl:349-402): until a key is emitted the scan
// does not skip a group's older versions, so when every key before it fails the filter (all
// versions of the earlier groups and the newer versions of its own group), the first older
// version that passes is emitted, ahead of the row's ordinary rows.  One thread per request
// entry (frontier entry k = local row F[k], flags of its edges at off[k]..): walks its edges in
// key order until the first kept one; per edge whose first version failed, its older versions.
// x_old[k] = the emitted older version's side-table row (-1: none), x_ge[k] = its edge.
template <int PK>
__global__ void k_first_loop(const int32_t* F, const int64_t* off, int64_t nF, const int64_t* row_ptr,
                             const uint8_t* flags, const int64_t* ov_edge, int64_t ov_n, const Program* prog,
                             EvalEnv oenv, FastArgs ofp, int64_t lo, int64_t* x_old, int64_t* x_ge) {
  for (int64_t k = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; k < nF; k += int64_t(gridDim.x) * blockDim.x) {
    x_old[k] = -1;
    const int32_t f = F[k];
    const int64_t b = row_ptr[f], e = row_ptr[f + 1];
    int64_t l = 0, h = ov_n;  // first older version at or after edge b
    while (l < h) {
      const int64_t mid = (l + h) >> 1;
      if (ov_edge[mid] < b) l = mid + 1; else h = mid;
    }
    int64_t x = b;  // edges [b, x) checked: their first versions failed
    for (int64_t o = l; o < ov_n && ov_edge[o] < e;) {
      const int64_t ge = ov_edge[o];
      bool kept = false;
      for (; x <= ge && !kept; x++) kept = flags[off[k] + (x - b)] != 0;
      if (kept) break;  // an ordinary row comes first: firstLoop ends there
      bool hit = false;
      for (; o < ov_n && ov_edge[o] == ge && !hit; o++) {
        bool pass;
        if (PK == PK_FAST) {
          pass = (ofp.present && !ofp.present[o]) ? true
                                                   : fast_cmp(ofp.op, static_cast<const int64_t*>(ofp.data)[o], ofp.k);
        } else {
          const Val v = eval_program(prog, oenv, o, int32_t(lo) + f, 0);
          pass = v.t == VT_ERR ? true : as_bool(v);  // storage: an eval error keeps the edge
        }
        if (pass) {
          x_old[k] = o;
          x_ge[k] = ge;
          hit = true;
        }
      }
      if (hit) break;
    }
  }
}
// merged row list: entry k's older-version row (if any) goes first, then its kept rows.
// cx = inclusive count of entries with an older-version row.
__global__ void k_merge_kept(const int64_t* ge, const int64_t* owner, int64_t m, const int64_t* cx, int64_t* mge,
                             int64_t* mold, int64_t* mowner) {
  for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < m; i += int64_t(gridDim.x) * blockDim.x) {
    const int64_t k = owner[i];
    const int64_t pos = i + cx[k];
    mge[pos] = ge[i];
    mold[pos] = -1;
    mowner[pos] = k;
  }
}
__global__ void k_merge_old(const int64_t* x_old, const int64_t* x_ge, int64_t nF, const int64_t* owner, int64_t m,
                            const int64_t* cx, int64_t* mge, int64_t* mold, int64_t* mowner) {
  for (int64_t k = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; k < nF; k += int64_t(gridDim.x) * blockDim.x) {
    if (x_old[k] < 0) continue;
    int64_t l = 0, h = m;  // kept rows of entries < k
    while (l < h) {
      const int64_t mid = (l + h) >> 1;
      if (owner[mid] < k) l = mid + 1; else h = mid;
    }
    const int64_t pos = l + cx[k] - 1;
    mge[pos] = x_ge[k];
    mold[pos] = x_old[k];
    mowner[pos] = k;
  }
}

__global__ void k_str_gather(const int64_t* ge, const int64_t* old, int64_t m, const int64_t* src_off,
                             const uint8_t* src_bytes, const int64_t* osrc_off, const uint8_t* osrc_bytes,
                             const int64_t* dst_off, uint8_t* dst) {
  for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < m; i += int64_t(gridDim.x) * blockDim.x) {
    int64_t len = dst_off[i + 1] - dst_off[i];
    const bool o = old && old[i] >= 0;
    const uint8_t* s = o ? osrc_bytes + osrc_off[old[i]] : src_bytes + src_off[ge[i]];
    for (int64_t j = 0; j < len; j++) dst[dst_off[i] + j] = s[j];
  }
}
__global__ void k_clamp_len(int64_t* l, int64_t m) {
  for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < m; i += int64_t(gridDim.x) * blockDim.x)
    if (l[i] < 0) l[i] = 0;
}

// tag column values of the returned vertices (gidx list): value bits, presence state, part, and
// STRING (offset, length) into the column's bytes
__global__ void k_tag_fetch(const int32_t* g, int64_t m, const int64_t* data, const uint8_t* present,
                            const int32_t* tpart, const int64_t* str_off, int64_t* val, uint8_t* state,
                            int32_t* part, int64_t* soff, int64_t* slen) {
  for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < m; i += int64_t(gridDim.x) * blockDim.x) {
    const int32_t x = g[i];
    const bool ok = x >= 0;
    val[i] = ok ? data[x] : 0;
    state[i] = ok ? present[x] : 0;
    part[i] = ok ? tpart[x] : -1;
    if (str_off) {
      soff[i] = ok ? str_off[x] : 0;
      slen[i] = ok ? str_off[x + 1] - str_off[x] : 0;
    }
  }
}
__global__ void k_bytes_gather(const int64_t* soff, const int64_t* doff, int64_t m, const uint8_t* src, uint8_t* dst) {
  for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < m; i += int64_t(gridDim.x) * blockDim.x)
    for (int64_t j = 0; j < doff[i + 1] - doff[i]; j++) dst[doff[i] + j] = src[soff[i] + j];
}

// Fills h->vertex_* for the returned vertices (h->vertex_ids, request parts vparts): a value is
// visible when the vertex's row sits in the request's part -- collectVertexProps scans
// prefix(request part, vid, tag) (QueryBaseProcessor.inl:309-333) -- else absent (the reference
// then skips the prop in the vertex row, RowWriter without it).
template <typename F>
void fetch_vertex_tags(Ctx& c, HostRows* h, const std::vector<int32_t>& vparts, F col_of, size_t ncols) {
  const int64_t nv = int64_t(h->vertex_ids.size());
  DevBuf dv, dg, val, stt, prt, soff, slen;
  const size_t cap = size_t(std::max<int64_t>(nv, 1));
  dv.alloc(cap * 8);
  dg.alloc(cap * 4);
  val.alloc(cap * 8);
  stt.alloc(cap);
  prt.alloc(cap * 4);
  soff.alloc(cap * 8);
  slen.alloc(cap * 8);
  if (nv) {
    NBG_HIP(hipMemcpyAsync(dv.p, h->vertex_ids.data(), size_t(nv) * 8, hipMemcpyHostToDevice, c.stream));
    lookup_gidx(c, dv.as<int64_t>(), dg.as<int32_t>(), nv);
  }
  for (size_t t = 0; t < ncols; t++) {
    const auto tf = col_of(t);
    const TagSpace& ts = *tf.first;
    const PropCol& pc = ts.cols[tf.second];
    const bool is_str = pc.type == NBG_T_STRING;
    std::vector<int64_t> hv(cap), hoff(cap), hlen(cap);
    std::vector<uint8_t> hs(cap);
    std::vector<int32_t> hp(cap);
    if (nv) {
      k_tag_fetch<<<grid_cap(nv), 256, 0, c.stream>>>(dg.as<int32_t>(), nv, pc.data.as<int64_t>(), pc.present.as<uint8_t>(),
                                                      ts.part.as<int32_t>(), is_str ? pc.str_off.as<int64_t>() : nullptr,
                                                      val.as<int64_t>(), stt.as<uint8_t>(), prt.as<int32_t>(),
                                                      soff.as<int64_t>(), slen.as<int64_t>());
      NBG_HIP(hipGetLastError());
      NBG_HIP(hipMemcpyAsync(hv.data(), val.p, size_t(nv) * 8, hipMemcpyDeviceToHost, c.stream));
      NBG_HIP(hipMemcpyAsync(hs.data(), stt.p, size_t(nv), hipMemcpyDeviceToHost, c.stream));
      NBG_HIP(hipMemcpyAsync(hp.data(), prt.p, size_t(nv) * 4, hipMemcpyDeviceToHost, c.stream));
      if (is_str) {
        NBG_HIP(hipMemcpyAsync(hoff.data(), soff.p, size_t(nv) * 8, hipMemcpyDeviceToHost, c.stream));
        NBG_HIP(hipMemcpyAsync(hlen.data(), slen.p, size_t(nv) * 8, hipMemcpyDeviceToHost, c.stream));
      }
      NBG_HIP(hipStreamSynchronize(c.stream));
    }
    std::vector<uint8_t> pres(cap, 0);
    for (int64_t i = 0; i < nv; i++) {
      const int32_t rp = vparts[size_t(i)];
      const bool own = hs[size_t(i)] == 1 && rp == part_of_vid(h->vertex_ids[size_t(i)], c.num_parts);
      const bool foreign = hs[size_t(i)] == 2 && rp == hp[size_t(i)];
      pres[size_t(i)] = own || foreign;
    }
    h->vertex_types.push_back(pc.type == NBG_T_FLOAT                               ? NBG_T_DOUBLE
                              : (pc.type == NBG_T_VID || pc.type == NBG_T_TIMESTAMP) ? NBG_T_INT
                                                                                     : pc.type);
    h->vertex_present.push_back(pres);
    if (is_str) {
      std::vector<int64_t> offs(size_t(nv) + 1, 0);
      for (int64_t i = 0; i < nv; i++) offs[size_t(i + 1)] = offs[size_t(i)] + (pres[size_t(i)] ? hlen[size_t(i)] : 0);
      std::vector<uint8_t> bytes(size_t(offs[size_t(nv)]) + 8);
      if (offs[size_t(nv)]) {
        DevBuf ddo, dbytes;
        ddo.alloc(size_t(nv + 1) * 8);
        dbytes.alloc(size_t(offs[size_t(nv)]) + 8);
        NBG_HIP(hipMemcpyAsync(ddo.p, offs.data(), size_t(nv + 1) * 8, hipMemcpyHostToDevice, c.stream));
        k_bytes_gather<<<grid_cap(nv), 256, 0, c.stream>>>(soff.as<int64_t>(), ddo.as<int64_t>(), nv,
                                                           pc.str_bytes.as<uint8_t>(), dbytes.as<uint8_t>());
        NBG_HIP(hipMemcpyAsync(bytes.data(), dbytes.p, size_t(offs[size_t(nv)]), hipMemcpyDeviceToHost, c.stream));
        NBG_HIP(hipStreamSynchronize(c.stream));
      }
      h->vertex_host.push_back(std::move(bytes));
      h->vertex_host_off.push_back(std::move(offs));
    } else {
      std::vector<uint8_t> raw(cap * 8);
      if (pc.type == NBG_T_BOOL) {
        for (int64_t i = 0; i < nv; i++) raw[size_t(i)] = uint8_t(hv[size_t(i)] != 0);
      } else {
        memcpy(raw.data(), hv.data(), size_t(nv) * 8);
      }
      h->vertex_host.push_back(std::move(raw));
      h->vertex_host_off.emplace_back();
    }
  }
}

int32_t get_bound_run(Ctx& c, int32_t et, const int32_t* parts, const int64_t* vids, size_t n, const uint8_t* filter,
                      size_t flen, const nbg_prop_def* cols, size_t ncols, nbg_rows* out, const int32_t* stats) {
  PoolScope pool_scope(query_pool(c));
  if (!c.finalized) throw Error(NBG_E_STATE, "snapshot not finalized");
  auto* h = new HostRows();
  auto finish = [&](int64_t nrows) {
    fill_rows(out, h, nrows, false);
    return NBG_OK;
  };
  // request-level validation -> every part of the request fails (QueryBaseProcessor.inl:470-477)
  std::vector<int32_t> req_parts;
  for (size_t i = 0; i < n; i++)
    if (std::find(req_parts.begin(), req_parts.end(), parts[i]) == req_parts.end()) req_parts.push_back(parts[i]);
  auto fail_all = [&](int32_t code) {
    for (auto p : req_parts) {
      h->failed_parts.push_back(p);
      h->failed_codes.push_back(code);
    }
    return finish(0);
  };
  bool in_bound = et < 0;
  auto it = c.edges.find(in_bound ? -et : et);
  if (it == c.edges.end()) return fail_all(NBG_E_EDGE_PROP_NOT_FOUND);
  EdgeSpace& es = it->second;
  Csr& csr = in_bound ? es.in : es.out;
  BoundCols bc{};
  // SOURCE / DEST tag props: the vertex row of each returned vertex (tagContexts_,
  // QueryBaseProcessor.inl:40-70; QueryBoundProcessor.cpp:19-31)
  struct TagReq {
    const TagSpace* ts;
    size_t field;
  };
  std::vector<TagReq> treq;
  // stats: the output columns in request order (retIndex): {0, edge column} or {1, tag column}
  std::vector<std::pair<int, int>> sorder;
  std::vector<int32_t> tstat;
  for (size_t i = 0; i < ncols; i++) {
    if (cols[i].owner != NBG_OWNER_EDGE) {
      auto tit = c.tags.find(cols[i].tag_id);
      if (tit == c.tags.end()) return fail_all(NBG_E_TAG_PROP_NOT_FOUND);
      const std::string tname = cols[i].name ? cols[i].name : "";
      size_t fi = tit->second.fields.size();
      for (size_t f = 0; f < tit->second.fields.size(); f++)
        if (tit->second.fields[f].name == tname) fi = f;
      if (fi == tit->second.fields.size()) return fail_all(NBG_E_IMPROPER_DATA_TYPE);
      if (stats) {  // validOperation over the tag prop's type (QueryBaseProcessor.inl:62-64)
        const int32_t st = stats[i];
        if (st < 1 || st > 3) {
          delete h;
          throw Error(NBG_E_INVALID_ARG, "stat type must be SUM 1, COUNT 2 or AVG 3");
        }
        const int32_t t = tit->second.fields[fi].type;
        if (st != 2 && (t == NBG_T_BOOL || t == NBG_T_STRING)) return fail_all(NBG_E_IMPROPER_DATA_TYPE);
        sorder.emplace_back(1, int(treq.size()));
        tstat.push_back(st);
      }
      treq.push_back(TagReq{&tit->second, fi});
      continue;
    }
    std::string name = cols[i].name ? cols[i].name : "";
    BoundCol b{};
    if (name == "_dst") b.kind = 1;
    else if (name == "_src") b.kind = 2;
    else if (name == "_rank") b.kind = 3;
    else if (name == "_type") b.kind = 4;
    if (b.kind) {
      b.type = NBG_T_INT;
    } else if (!in_bound) {
      int idx = -1;
      for (size_t f = 0; f < es.fields.size(); f++)
        if (es.fields[f].name == name) idx = int(f);
      if (idx < 0) return fail_all(NBG_E_IMPROPER_DATA_TYPE);
      b.kind = 0;
      b.prop = idx;
      int32_t t = es.fields[size_t(idx)].type;
      b.type = (t == NBG_T_FLOAT) ? NBG_T_DOUBLE : (t == NBG_T_VID || t == NBG_T_TIMESTAMP) ? NBG_T_INT : t;
    } else {
      continue;  // "InBound has none props, skip it!"
    }
    if (stats) {  // validOperation (QueryBaseProcessor.inl:18-35): SUM / AVG need a numeric column
      b.stat = stats[i];
      if (b.stat < 1 || b.stat > 3) {
        delete h;
        throw Error(NBG_E_INVALID_ARG, "stat type must be SUM 1, COUNT 2 or AVG 3");
      }
      if (b.stat != 2 && (b.type == NBG_T_BOOL || b.type == NBG_T_STRING)) return fail_all(NBG_E_IMPROPER_DATA_TYPE);
    }
    if (bc.n >= kMaxBoundCols) {
      delete h;
      throw Error(NBG_E_UNSUPPORTED, "too many return columns");
    }
    if (stats) sorder.emplace_back(0, bc.n);
    bc.c[bc.n++] = b;
  }
  Program fprog{};
  int pk = PK_NONE;
  FastArgs fp{};
  if (flen) {
    std::string msg;
    int32_t rc = compile_expr(filter, flen, es.fields, false, !in_bound, &fprog, &msg, &c.tag_refs);
    if (rc == NBG_E_UNSUPPORTED) {
      delete h;
      throw Error(rc, "filter: " + msg);
    }
    if (rc != NBG_OK) return fail_all(NBG_E_INVALID_FILTER);
    FastPred f = classify_pred(fprog, es.fields);
    pk = f.kind;
    if (pk == PK_FAST) {
      const PropCol& pc = csr.props[size_t(f.col)];
      fp = FastArgs{pc.data.p, pc.present.as<uint8_t>(), pc.width, f.op, f.k};
    }
  }
  int64_t N = int64_t(n);
  const int64_t lo = c.owned_lo(), hi = c.owned_hi();
  // parts not held by this rank -> E_PART_NOT_FOUND (NebulaStore::engine, BaseProcessor.inl:14-27)
  for (auto p : req_parts)
    if (p < 0 || p > c.num_parts || owner_of_part(p, c.world) != c.rank) {
      h->failed_parts.push_back(p);
      h->failed_codes.push_back(NBG_E_PART_NOT_FOUND);
    }
  DevBuf dv, dp, dg, dF, ddeg, doff;
  dv.alloc(size_t(N + 1) * 8);
  dp.alloc(size_t(N + 1) * 4);
  dg.alloc(size_t(N + 1) * 4);
  dF.alloc(size_t(N + 1) * 4);
  ddeg.alloc(size_t(N + 1) * 8);
  doff.alloc(size_t(N + 1) * 8);
  if (N) {
    NBG_HIP(hipMemcpyAsync(dv.p, vids, size_t(N) * 8, hipMemcpyHostToDevice, c.stream));
    NBG_HIP(hipMemcpyAsync(dp.p, parts, size_t(N) * 4, hipMemcpyHostToDevice, c.stream));
    lookup_gidx(c, dv.as<int64_t>(), dg.as<int32_t>(), N);
    k_bound_frontier<<<grid_cap(N), 256, 0, c.stream>>>(dp.as<int32_t>(), dg.as<int32_t>(), N, lo, hi,
                                                      csr.row_part.as<int32_t>(), dF.as<int32_t>());
  }
  k_degrees_masked<<<grid_cap(N + 1), 256, 0, c.stream>>>(dF.as<int32_t>(), N, csr.row_ptr.as<int64_t>(), ddeg.as<int64_t>());
  exclusive_scan_dev<int64_t>(c, ddeg.as<int64_t>(), doff.as<int64_t>(), N + 1);
  std::vector<int64_t> hoff(size_t(N + 1));
  NBG_HIP(hipMemcpyAsync(hoff.data(), doff.p, size_t(N + 1) * 8, hipMemcpyDeviceToHost, c.stream));
  NBG_HIP(hipStreamSynchronize(c.stream));
  int64_t E = hoff[size_t(N)];
  c.timing = Timing{};
  timing_reset(c);
  if (c.host_stage_used) NBG_HIP(hipStreamSynchronize(c.stream));  // a failed query's copies
  c.host_stage_used = 0;
  c.timing.edges_scanned = uint64_t(E);
  // compress away zero-degree request entries for the expansion (tile owner search needs deg>=1)
  std::vector<int32_t> hF(static_cast<size_t>(N));
  if (N) NBG_HIP(hipMemcpy(hF.data(), dF.p, size_t(N) * 4, hipMemcpyDeviceToHost));
  std::vector<int32_t> cF;
  std::vector<int64_t> coff, centry;
  for (int64_t i = 0; i < N; i++)
    if (hoff[size_t(i + 1)] > hoff[size_t(i)]) {
      cF.push_back(hF[size_t(i)]);
      coff.push_back(hoff[size_t(i)]);
      centry.push_back(i);
    }
  coff.push_back(E);
  int64_t nF = int64_t(cF.size());
  DevBuf dcF, dcoff, flags, slots, cnt, owner, geb;
  dcF.alloc(size_t(nF + 1) * 4);
  dcoff.alloc(size_t(nF + 1) * 8);
  if (nF) NBG_HIP(hipMemcpyAsync(dcF.p, cF.data(), size_t(nF) * 4, hipMemcpyHostToDevice, c.stream));
  NBG_HIP(hipMemcpyAsync(dcoff.p, coff.data(), size_t(nF + 1) * 8, hipMemcpyHostToDevice, c.stream));
  flags.alloc(size_t(E + 1));
  EvalEnv env = make_env(c, es, csr, in_bound ? -es.type : es.type);
  env.storage = 1;
  env.lo = c.owned_lo();
  env.row_part = csr.row_part.as<int32_t>();
  DevBuf dprog;
  dprog.alloc(sizeof(Program));
  NBG_HIP(hipMemcpyAsync(dprog.p, &fprog, sizeof(Program), hipMemcpyHostToDevice, c.stream));
  DevBuf cnts;
  cnts.alloc(64);
  NBG_HIP(hipMemsetAsync(cnts.p, 0, 64, c.stream));
  hipEventRecord(c.ev[0], c.stream);
  int64_t m = 0;
  if (E > 0) {
    ExpandArgs a{};
    a.F = dcF.as<int32_t>();
    a.nF = nF;
    a.off = dcoff.as<int64_t>();
    a.row_ptr = csr.row_ptr.as<int64_t>();
    a.col = csr.col.as<int32_t>();
    a.lo = lo;
    a.flags = flags.as<uint8_t>();
    a.err = cnts.as<unsigned long long>();
    a.storage = 1;
    launch_expand<EXP_FLAGS>(c, a, pk, fp, dprog.as<Program>(), env, E);
    c.timing.expand_bytes += expand_bytes(nF, E, pk == PK_FAST ? fp.width : 0, EXP_FLAGS);
    slots.alloc(size_t(E + 1) * 8);
    cnt.alloc(8);
    size_t tb = 0;
    auto first = rocprim::counting_iterator<int64_t>(0);
    NBG_HIP(rocprim::select(nullptr, tb, first, flags.as<uint8_t>(), slots.as<int64_t>(), cnt.as<uint64_t>(), size_t(E), c.stream));
    c.ws_tmp.ensure(tb);
    NBG_HIP(rocprim::select(c.ws_tmp.p, tb, first, flags.as<uint8_t>(), slots.as<int64_t>(), cnt.as<uint64_t>(), size_t(E), c.stream));
    uint64_t hm = 0;
    NBG_HIP(hipMemcpyAsync(&hm, cnt.p, 8, hipMemcpyDeviceToHost, c.stream));
    NBG_HIP(hipStreamSynchronize(c.stream));
    m = int64_t(hm);
  }
  owner.alloc(size_t(m + 1) * 8);
  geb.alloc(size_t(m + 1) * 8);
  if (m) {
    k_slot_owner<<<grid_cap(m), 256, 0, c.stream>>>(slots.as<int64_t>(), m, dcoff.as<int64_t>(), nF, owner.as<int64_t>());
    k_slot_ge<<<grid_cap(m), 256, 0, c.stream>>>(slots.as<int64_t>(), owner.as<int64_t>(), m, dcoff.as<int64_t>(),
                                                 dcF.as<int32_t>(), csr.row_ptr.as<int64_t>(), geb.as<int64_t>());
    NBG_HIP(hipGetLastError());
  }
  // firstLoop (multi-version data under a push-down filter): older versions emitted ahead of a
  // request entry's rows (QueryBaseProcessor.inl:349-402); the reader only exists for out-bound
  // rows with a value, so in-bound scans never evaluate the filter
  DevBuf oldb, ovtab;
  const PropDev* oprops = nullptr;
  if (flen && !in_bound && csr.ov_n > 0 && nF > 0) {
    std::vector<PropDev> tab;
    for (const PropCol& p : csr.ov_props)
      tab.push_back(PropDev{p.type, p.width, p.data.p, p.present.as<uint8_t>(), p.str_off.as<int64_t>(),
                            p.str_bytes.as<uint8_t>()});
    ovtab.alloc(sizeof(PropDev) * std::max<size_t>(tab.size(), 1));
    if (!tab.empty()) c.h2d(ovtab.p, tab.data(), sizeof(PropDev) * tab.size());
    oprops = ovtab.as<PropDev>();
    EvalEnv oenv = env;
    oenv.props = oprops;
    FastArgs ofp{};
    if (pk == PK_FAST) {
      const FastPred f = classify_pred(fprog, es.fields);
      const PropCol& oc = csr.ov_props[size_t(f.col)];
      ofp = FastArgs{oc.data.p, oc.present.as<uint8_t>(), 8, f.op, f.k};
    }
    DevBuf xo, xg, cx;
    xo.alloc(size_t(nF) * 8);
    xg.alloc(size_t(nF) * 8);
    cx.alloc(size_t(nF) * 8);
    if (pk == PK_FAST)
      k_first_loop<PK_FAST><<<grid_cap(nF), 256, 0, c.stream>>>(dcF.as<int32_t>(), dcoff.as<int64_t>(), nF,
                                                                csr.row_ptr.as<int64_t>(), flags.as<uint8_t>(),
                                                                csr.ov_edge.as<int64_t>(), csr.ov_n, dprog.as<Program>(),
                                                                oenv, ofp, lo, xo.as<int64_t>(), xg.as<int64_t>());
    else
      k_first_loop<PK_VM><<<grid_cap(nF), 256, 0, c.stream>>>(dcF.as<int32_t>(), dcoff.as<int64_t>(), nF,
                                                              csr.row_ptr.as<int64_t>(), flags.as<uint8_t>(),
                                                              csr.ov_edge.as<int64_t>(), csr.ov_n, dprog.as<Program>(),
                                                              oenv, ofp, lo, xo.as<int64_t>(), xg.as<int64_t>());
    NBG_HIP(hipGetLastError());
    auto has = rocprim::make_transform_iterator(xo.as<int64_t>(), [] __device__(int64_t v) -> int64_t { return v >= 0; });
    size_t tb = 0;
    NBG_HIP(rocprim::inclusive_scan(nullptr, tb, has, cx.as<int64_t>(), size_t(nF), rocprim::plus<int64_t>(), c.stream));
    c.ws_tmp.ensure(tb);
    NBG_HIP(rocprim::inclusive_scan(c.ws_tmp.p, tb, has, cx.as<int64_t>(), size_t(nF), rocprim::plus<int64_t>(), c.stream));
    int64_t X = 0;
    NBG_HIP(hipMemcpyAsync(&X, cx.as<int64_t>() + nF - 1, 8, hipMemcpyDeviceToHost, c.stream));
    NBG_HIP(hipStreamSynchronize(c.stream));
    if (X > 0) {
      DevBuf mge, mold, mown;
      mge.alloc(size_t(m + X + 1) * 8);
      mold.alloc(size_t(m + X + 1) * 8);
      mown.alloc(size_t(m + X + 1) * 8);
      if (m)
        k_merge_kept<<<grid_cap(m), 256, 0, c.stream>>>(geb.as<int64_t>(), owner.as<int64_t>(), m, cx.as<int64_t>(),
                                                        mge.as<int64_t>(), mold.as<int64_t>(), mown.as<int64_t>());
      k_merge_old<<<grid_cap(nF), 256, 0, c.stream>>>(xo.as<int64_t>(), xg.as<int64_t>(), nF, owner.as<int64_t>(), m,
                                                      cx.as<int64_t>(), mge.as<int64_t>(), mold.as<int64_t>(),
                                                      mown.as<int64_t>());
      NBG_HIP(hipGetLastError());
      m += X;
      geb = std::move(mge);
      owner = std::move(mown);
      oldb = std::move(mold);
    }
  }
  const int64_t* oldp = oldb.as<int64_t>();
  if (stats) {
    // one row: per column SUM (INT) / COUNT (INT) / AVG (DOUBLE), in request order (retIndex)
    DevBuf acc;
    acc.alloc(size_t(2 * bc.n + 2) * 8);
    NBG_HIP(hipMemsetAsync(acc.p, 0, size_t(2 * bc.n + 2) * 8, c.stream));
    if (m) {
      for (int i = 0; i < bc.n; i++)
        k_bound_stats<<<grid_cap(m, 256, 1024), 256, 0, c.stream>>>(geb.as<int64_t>(), oldp, owner.as<int64_t>(), m,
                                                                    dcF.as<int32_t>(), lo, env, oprops, bc.c[i],
                                                                    acc.as<unsigned long long>() + 2 * i);
      NBG_HIP(hipGetLastError());
    }
    std::vector<unsigned long long> ha(size_t(2 * bc.n + 2));
    NBG_HIP(hipMemcpyAsync(ha.data(), acc.p, ha.size() * 8, hipMemcpyDeviceToHost, c.stream));
    // SOURCE / DEST tag columns (QueryStatsProcessor::processVertex, QueryStatsProcessor.cpp:69-82):
    // every request entry of an owned part collects the newest version of its vertex row in that
    // part (collectVertexProps, QueryBaseProcessor.inl:309-333) - visible when the row sits in
    // the request's part, as for getBound's vertex columns - into the column's sum / count
    // (StatsCollector, Collector.h:66-94); entries without the row add nothing
    std::vector<int64_t> tsum(treq.size(), 0), tcnt(treq.size(), 0);
    std::vector<std::vector<int64_t>> tval(treq.size());
    std::vector<std::vector<uint8_t>> tstt(treq.size());
    std::vector<std::vector<int32_t>> tprt(treq.size());
    DevBuf tv, ts, tp;
    if (!treq.empty() && N) {
      tv.alloc(size_t(N) * 8);
      ts.alloc(size_t(N));
      tp.alloc(size_t(N) * 4);
      for (size_t t = 0; t < treq.size(); t++) {
        const TagSpace& tsp = *treq[t].ts;
        const PropCol& pc = tsp.cols[treq[t].field];
        k_tag_fetch<<<grid_cap(N), 256, 0, c.stream>>>(dg.as<int32_t>(), N, pc.data.as<int64_t>(), pc.present.as<uint8_t>(),
                                                       tsp.part.as<int32_t>(), nullptr, tv.as<int64_t>(), ts.as<uint8_t>(),
                                                       tp.as<int32_t>(), nullptr, nullptr);
        NBG_HIP(hipGetLastError());
        tval[t].resize(size_t(N));
        tstt[t].resize(size_t(N));
        tprt[t].resize(size_t(N));
        NBG_HIP(hipMemcpyAsync(tval[t].data(), tv.p, size_t(N) * 8, hipMemcpyDeviceToHost, c.stream));
        NBG_HIP(hipMemcpyAsync(tstt[t].data(), ts.p, size_t(N), hipMemcpyDeviceToHost, c.stream));
        NBG_HIP(hipMemcpyAsync(tprt[t].data(), tp.p, size_t(N) * 4, hipMemcpyDeviceToHost, c.stream));
        NBG_HIP(hipStreamSynchronize(c.stream));  // the host vectors are reused per column
      }
    }
    hipEventRecord(c.ev[1], c.stream);
    NBG_HIP(hipStreamSynchronize(c.stream));
    for (size_t t = 0; t < treq.size() && N; t++) {
      const int32_t ty = treq[t].ts->cols[treq[t].field].type;
      for (int64_t i = 0; i < N; i++) {
        const int32_t rp = parts[i];
        if (rp < 0 || rp > c.num_parts || owner_of_part(rp, c.world) != c.rank) continue;  // failed part
        const uint8_t stt = tstt[t][size_t(i)];
        const bool vis = (stt == 1 && rp == part_of_vid(vids[i], c.num_parts)) || (stt == 2 && rp == tprt[t][size_t(i)]);
        if (!vis) continue;
        tcnt[t]++;
        if (ty == NBG_T_DOUBLE || ty == NBG_T_FLOAT) {
          if (tstat[t] != 2) {
            delete h;
            throw Error(NBG_E_UNSUPPORTED, "SUM/AVG over a double prop (the reference's int64 sum throws bad_get)");
          }
        } else if (ty != NBG_T_BOOL && ty != NBG_T_STRING) {
          tsum[t] = int64_t(uint64_t(tsum[t]) + uint64_t(tval[t][size_t(i)]));
        }
      }
    }
    float sms = 0;
    hipEventElapsedTime(&sms, c.ev[0], c.ev[1]);
    c.timing.total_ms = sms;
    for (const auto& so : sorder) {
      if (so.first == 1) {
        const size_t t = size_t(so.second);
        const int32_t st = tstat[t];
        h->types.push_back(st == 3 ? NBG_T_DOUBLE : NBG_T_INT);
        h->host.emplace_back(8);
        if (st == 3) {
          const double avg = double(tsum[t]) / double(int32_t(tcnt[t]));  // count_ is int32 (CommonUtils.h:51)
          memcpy(h->host.back().data(), &avg, 8);
        } else {
          const int64_t v = st == 2 ? int64_t(int32_t(tcnt[t])) : tsum[t];
          memcpy(h->host.back().data(), &v, 8);
        }
        h->str_off.push_back(nullptr);
        continue;
      }
      const int i = so.second;
      const BoundCol& b = bc.c[i];
      const int64_t sum = int64_t(ha[size_t(2 * i)]);
      const int64_t cnt = int64_t(ha[size_t(2 * i + 1)]);
      if (b.stat != 2 && b.type == NBG_T_DOUBLE && cnt > 0) {
        delete h;
        throw Error(NBG_E_UNSUPPORTED, "SUM/AVG over a double prop (the reference's int64 sum throws bad_get)");
      }
      h->types.push_back(b.stat == 3 ? NBG_T_DOUBLE : NBG_T_INT);
      h->host.emplace_back(8);
      if (b.stat == 3) {
        const double avg = double(sum) / double(int32_t(cnt));  // count_ is int32 (CommonUtils.h:51)
        memcpy(h->host.back().data(), &avg, 8);
      } else {
        const int64_t v = b.stat == 2 ? int64_t(int32_t(cnt)) : sum;
        memcpy(h->host.back().data(), &v, 8);
      }
      h->str_off.push_back(nullptr);
    }
    for (auto& hc : h->host) h->cols.push_back(hc.data());
    out->edges_scanned = uint64_t(E);
    return finish(1);
  }
  std::vector<DevBuf> dcols(size_t(bc.n));
  std::vector<DevBuf> slen(size_t(bc.n));
  for (int i = 0; i < bc.n; i++) {
    BoundCol& b = bc.c[i];
    if (b.type == NBG_T_STRING) {
      slen[size_t(i)].alloc(size_t(m + 1) * 8);
      b.str_len = slen[size_t(i)].as<int64_t>();
    } else {
      dcols[size_t(i)].alloc(size_t(m + 1) * (b.type == NBG_T_BOOL ? 1 : 8));
      b.out = dcols[size_t(i)].p;
    }
  }
  std::vector<int64_t> howner(static_cast<size_t>(m));
  if (m) {
    k_bound_rows<<<grid_cap(m), 256, 0, c.stream>>>(geb.as<int64_t>(), oldp, owner.as<int64_t>(), m,
                                                  dcF.as<int32_t>(), lo, env, oprops, bc);
    NBG_HIP(hipGetLastError());
    NBG_HIP(hipMemcpyAsync(howner.data(), owner.p, size_t(m) * 8, hipMemcpyDeviceToHost, c.stream));
  }
  hipEventRecord(c.ev[1], c.stream);
  NBG_HIP(hipStreamSynchronize(c.stream));
  float ms = 0;
  hipEventElapsedTime(&ms, c.ev[0], c.ev[1]);
  c.timing.total_ms = ms;
  // assemble: typed columns to host; absent values (INT64_MIN marker / -1 length) stay absent
  for (int i = 0; i < bc.n; i++) {
    const BoundCol& b = bc.c[i];
    h->types.push_back(b.type);
    if (b.type == NBG_T_STRING) {
      std::vector<int64_t> lens(static_cast<size_t>(m));
      if (m) NBG_HIP(hipMemcpy(lens.data(), slen[size_t(i)].p, size_t(m) * 8, hipMemcpyDeviceToHost));
      std::vector<int64_t> offs(size_t(m) + 1, 0);
      for (int64_t r = 0; r < m; r++) offs[size_t(r + 1)] = offs[size_t(r)] + std::max<int64_t>(lens[size_t(r)], 0);
      DevBuf doffs, dbytes;
      doffs.alloc(size_t(m + 1) * 8);
      dbytes.alloc(size_t(offs[size_t(m)]) + 8);
      NBG_HIP(hipMemcpy(doffs.p, offs.data(), size_t(m + 1) * 8, hipMemcpyHostToDevice));
      const PropCol& pc = csr.props[size_t(b.prop)];
      if (m)
        k_str_gather<<<grid_cap(m), 256, 0, c.stream>>>(
            geb.as<int64_t>(), oldp, m, pc.str_off.as<int64_t>(), pc.str_bytes.as<uint8_t>(),
            oldp ? csr.ov_props[size_t(b.prop)].str_off.as<int64_t>() : nullptr,
            oldp ? csr.ov_props[size_t(b.prop)].str_bytes.as<uint8_t>() : nullptr, doffs.as<int64_t>(),
            dbytes.as<uint8_t>());
      NBG_HIP(hipStreamSynchronize(c.stream));
      h->host.emplace_back(size_t(offs[size_t(m)]) + 8);
      if (offs[size_t(m)]) NBG_HIP(hipMemcpy(h->host.back().data(), dbytes.p, size_t(offs[size_t(m)]), hipMemcpyDeviceToHost));
      h->host_off.push_back(offs);
      h->cols.push_back(h->host.back().data());
      h->str_off.push_back(h->host_off.back().data());
    } else {
      size_t w = b.type == NBG_T_BOOL ? 1 : 8;
      h->host.emplace_back(size_t(m) * w + 8);
      if (m) NBG_HIP(hipMemcpy(h->host.back().data(), dcols[size_t(i)].p, size_t(m) * w, hipMemcpyDeviceToHost));
      h->cols.push_back(h->host.back().data());
      h->str_off.push_back(nullptr);
    }
  }
  // vertices with >= 1 row, in request order (QueryBoundProcessor.cpp:61-67)
  h->row_vertex.resize(size_t(m));
  int64_t last = -1;
  for (int64_t r = 0; r < m; r++) {
    int64_t k = howner[size_t(r)];
    int64_t entry = centry[size_t(k)];
    h->row_vertex[size_t(r)] = vids[entry];
    if (k != last) {
      h->vertex_ids.push_back(vids[entry]);
      h->vertex_row_offsets.push_back(r);
      last = k;
    }
  }
  h->vertex_row_offsets.push_back(m);
  if (!treq.empty()) {
    // request part of each returned vertex (its first request entry)
    std::vector<int32_t> vparts;
    last = -1;
    for (int64_t r = 0; r < m; r++) {
      int64_t k = howner[size_t(r)];
      if (k != last) vparts.push_back(parts[centry[size_t(k)]]);
      last = k;
    }
    fetch_vertex_tags(c, h, vparts, [&](size_t t) { return std::make_pair(treq[t].ts, treq[t].field); },
                      treq.size());
  }
  fill_rows(out, h, m, false);
  out->edges_scanned = uint64_t(E);
  return NBG_OK;
}

void free_rows_impl(void* impl) { delete static_cast<HostRows*>(impl); }

}  // namespace nbg
