// paths.hip -- FIND SHORTEST PATH as batched bidirectional BFS on the GO snapshot
// (SURVEY 8a row A10).
//
// The reference has no implementation (src/graph/FindExecutor.cpp:20-22 is a stub and the
// parser has no grammar for it), so the definition is this build's (include/nebula_amd.h):
// the hop distance over out-edges of one type, and the lexicographically smallest vid sequence
// among the shortest paths.  The oracle (oracle/refcpu.cpp ora_shortest_path) states it as a
// backward BFS from dst over the -type in-edge keys followed by a greedy walk from src.
//
// Device algorithm, for a batch of B pairs at once (one context = one GPU):
//  * per side (F = forward from src over the out CSR, B = backward from dst over the in CSR),
//    pair and owned vertex, a distance byte dist[side][pair * n + row] (0xFF = unseen).  A
//    claim is a CAS on the 32-bit word holding the byte, so each (side, pair, vertex) enters
//    exactly one frontier.
//  * frontiers are lists of 64-bit tuples (side | pair | level | row) of all pairs together.
//    Every iteration each active pair expands the side whose frontier has the smaller sum of
//    (degree + 1), and ONE edge-balanced launch (the GO expansion's LDS tile scheme: 2048
//    adjacency entries per workgroup, owner found by binary search in LDS) expands the chosen
//    sides of all pairs; hubs spread over many tiles.
//  * a claim of a vertex the other side has already seen is a meet.  With depths (f, b) after
//    that expansion the distance is f + b, and the meet set is exactly the set of vertices at
//    position f of the shortest paths (any seen-by-both vertex has ds <= f, dt <= b and
//    ds + dt >= f + b, so ds = f and dt = b).
//  * path: the backward distances are extended from the meet set toward src over in-edges,
//    restricted to vertices whose forward distance completes a shortest path (the "sweep");
//    afterwards every shortest-path vertex carries its exact distance to dst, and one wave per
//    pair walks from src taking the smallest vid w among out-neighbours with
//    dist_B(w) = L - i - 1, the oracle's greedy rule.
//  * every claimed byte is recorded in an arena and reset after the batch, so the distance
//    arrays (2 * B * n bytes, HBM-sized) stay allocated and clean across calls.
#include <rocprim/device/device_scan.hpp>

#include <algorithm>
#include <array>
#include <map>
#include <mutex>
#include <unordered_map>
#include <climits>
#include <cmath>

#include "device_common.h"
#include "engine.h"
#include "rows.h"

namespace nbg {
namespace {

constexpr int kT = 256;
constexpr int kIt = 8;
constexpr int kTileE = kT * kIt;

enum : int32_t { SP_ACTIVE = 0, SP_MET = 1, SP_DONE = 2 };
// device counters (one array): live list F / B, arena, meets, X list, active pairs, overflow,
// sweep list, X edges
enum : int { C_LIVE0 = 0, C_LIVE1 = 1, C_ARENA = 2, C_MEET = 3, C_X = 4, C_ACTIVE = 5, C_OVF = 6, C_SWEEP = 7,
             C_XE = 8, C_WALKERR = 9, C_PE = 10, C_PLEN = 11, C_MAXL = 12, C_N = 16 };

__host__ __device__ inline uint64_t mk_tup(uint32_t side, uint32_t pair, uint32_t lvl, uint32_t row) {
  return (uint64_t(side) << 63) | (uint64_t(pair & 0x7FFFFFu) << 40) | (uint64_t(lvl & 0xFFu) << 32) | uint64_t(row);
}
__device__ inline uint32_t t_side(uint64_t t) { return uint32_t(t >> 63); }
__device__ inline uint32_t t_pair(uint64_t t) { return uint32_t(t >> 40) & 0x7FFFFFu; }
__device__ inline uint32_t t_lvl(uint64_t t) { return uint32_t(t >> 32) & 0xFFu; }
__device__ inline uint32_t t_row(uint64_t t) { return uint32_t(t); }

struct SpCsr {  // one direction's adjacency over the owned rows
  const int64_t* row_ptr;
  const int32_t* col;     // global gidx of the other end
  const uint8_t* row_ok;  // rows whose keys sit outside hash(vid)'s part are invisible
  // min(degree, 65535) per row, 0 where row_ok is 0 (null: off; 65535: read row_ptr): a claim's
  // degree from a 2-byte entry of an array the Infinity Cache holds (66 MB at RMAT-26) instead of
  // the 16-byte row_ptr pair of a 262 MB array (option sp_deg16)
  const uint16_t* deg16;
};

__device__ inline int64_t sp_deg(const SpCsr& g, uint32_t r) {
  if (g.deg16) {
    const uint32_t d = g.deg16[r];
    if (d != 0xFFFFu) return d;
  }
  if (g.row_ok && !g.row_ok[r]) return 0;
  return g.row_ptr[r + 1] - g.row_ptr[r];
}
__global__ void k_deg16(const int64_t* row_ptr, const uint8_t* row_ok, int64_t n, uint16_t* out) {
  for (int64_t r = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; r < n; r += int64_t(gridDim.x) * blockDim.x) {
    const int64_t d = row_ok && !row_ok[r] ? 0 : row_ptr[r + 1] - row_ptr[r];
    out[r] = uint16_t(d < 0xFFFF ? d : 0xFFFF);
  }
}

struct SpState {  // per-pair arrays, B entries each
  int32_t* state;
  int32_t* res;             // hops (-1 unreachable)
  int32_t* lvl;             // [2][B] depth of each side
  int32_t* side;            // side expanded this iteration
  int32_t* pside;           // side expanded by the iteration that just ended
  int32_t* met;             // 1: a meet this iteration; 2 + i: met in iteration i
  unsigned long long* deg;  // [2][B] frontier sum of (degree + 1)
  int32_t B;
  int32_t ilv;              // 1: the two sides' bytes of a (pair, vertex) adjacent (d1 = d0 + 1, index
                            // x 2): a claim reads its own and the other side's byte in one load
  // level filter (null: off): bit (v & lvmask) of level (side, l)'s lvw words is set when some
  // pair of the batch claimed vertex v at depth l on that side (1 <= l < kLv): a one-hash Bloom
  // filter of every pair's level-l set, at most 2^23 bits (1 MiB) a level so the level a launch
  // tests stays in an XCD's 4 MiB L2 (a full n-bit map at RMAT-26 is 4 MiB and its probes
  // went to the fabric: the chunked sweep fetched ~40 B per entry).  A test that needs
  // "dist[side][p][v] == l" first reads the bit; only a set bit reads the pair's distance byte
  // (a random line in the 2 * B * n byte arrays)
  uint32_t* lvbits;
  int64_t lvw;
  uint32_t lvmask;
};
// the per-pair arrays of SpState carved from the W.state block (sized B * 48 + 64 bytes)
static void sp_state_carve(const DevBuf& b, int64_t nb, SpState& st) {
  Carve cv(b, "shortest path: per-pair state", 4);
  st.deg = cv.take<unsigned long long>(size_t(nb) * 16);
  st.state = cv.take<int32_t>(size_t(nb) * 4);
  st.res = cv.take<int32_t>(size_t(nb) * 4);
  st.lvl = cv.take<int32_t>(size_t(nb) * 8);
  st.side = cv.take<int32_t>(size_t(nb) * 4);
  st.pside = cv.take<int32_t>(size_t(nb) * 4);
  st.met = cv.take<int32_t>(size_t(nb) * 4);
}
constexpr int kLv = 8;

__device__ inline void lv_mark(const SpState& st, uint32_t side, uint32_t l, uint32_t v) {
  if (st.lvbits && l >= 1 && l < uint32_t(kLv))
    atomicOr(st.lvbits + (int64_t(side) * kLv + l) * st.lvw + ((v & st.lvmask) >> 5), 1u << (v & 31u));
}
// false only when no pair holds v at depth l on the side
__device__ inline bool lv_maybe(const SpState& st, uint32_t side, int32_t l, uint32_t v) {
  if (!st.lvbits || l < 1 || l >= kLv) return true;
  return (st.lvbits[(int64_t(side) * kLv + l) * st.lvw + ((v & st.lvmask) >> 5)] >> (v & 31u)) & 1u;
}

// byte index of (pair p, vertex v) in a distance array.  Vertex-major keeps the bytes of all
// pairs of one vertex in one cache line run, so hub neighbourhoods expanded by many pairs share
// lines in L2 / the Infinity cache; pair-major keeps each pair's bytes contiguous.  Interleaved
// (ilv), the index doubles and side 1's array starts one byte after side 0's.
__device__ inline uint64_t didx(const SpState& st, uint32_t p, uint64_t v, int64_t n) {
  return (uint64_t(p) * uint64_t(n) + v) << st.ilv;  // pair-major (vertex-major lost: 3.84 vs 3.58 ms, r05)
}

struct SpBufs {
  uint64_t* live_next[2];
  uint64_t* arena;
  uint64_t* meet;
  uint64_t* sweep_next;
  int64_t cap_live[2], cap_arena, cap_meet, cap_sweep;
};

__device__ inline unsigned long long wsum(unsigned long long v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// wave-aggregated arr[key] += v over the lanes with act (lanes of one wave mostly share a key:
// an edge tile covers consecutive frontier entries, usually of one pair).  Wave-uniform call.
__device__ inline void wave_add_keyed(unsigned long long* arr, uint32_t key, unsigned long long v, bool act) {
  const int lane = threadIdx.x & 63;
  uint64_t m = __ballot(act);
  while (m) {
    const int leader = __ffsll((long long)m) - 1;
    const uint32_t k = uint32_t(__shfl(int(key), leader));
    const bool mine = act && key == k;
    const unsigned long long s = wsum(mine ? v : 0ull);
    if (lane == leader) atomicAdd(arr + k, s);
    m &= ~__ballot(mine);
    act = act && !mine;
  }
}

// append with a capacity guard (an overflow sets C_OVF; the host sizes lists so it never does)
__device__ inline void put(uint64_t* list, int64_t cap, unsigned long long* cnt, int which, bool pred, uint64_t v) {
  const int64_t s = wave_append(cnt + which, pred);
  if (pred) {
    if (s < cap) list[s] = v;
    else atomicOr(cnt + C_OVF, 1ull);
  }
}

// claim the unseen (0xFF) distance byte idx with val: true for exactly one caller
__device__ inline bool claim_byte(uint8_t* base, uint64_t idx, uint32_t val) {
  if (base[idx] != 0xFF) return false;  // already seen (values only leave 0xFF within a batch)
  // the aligned word holding the byte (the base itself may be odd: the interleaved side 1)
  const uintptr_t a = reinterpret_cast<uintptr_t>(base + idx);
  uint32_t* w = reinterpret_cast<uint32_t*>(a & ~uintptr_t(3));
  const uint32_t sh = uint32_t(a & 3) * 8;
  uint32_t old = *reinterpret_cast<volatile uint32_t*>(w);
  while (((old >> sh) & 0xFFu) == 0xFFu) {
    const uint32_t nw = (old & ~(0xFFu << sh)) | (val << sh);
    const uint32_t prev = atomicCAS(w, old, nw);
    if (prev == old) return true;
    old = prev;
  }
  return false;
}

// the depth of vertex v for pair p on a side (0xFF: unseen)
__device__ inline uint32_t dist_get(const SpState& st, const uint8_t* dense, uint32_t side, uint32_t p, uint32_t v,
                                    int64_t n, bool fresh = false) {
  (void)side;
  const uint8_t* a = dense + didx(st, p, v, n);
  return fresh ? uint32_t(*reinterpret_cast<volatile const uint8_t*>(a)) : uint32_t(*a);
}
// claim the unseen (p, v) on a side with depth val: true for exactly one caller
__device__ inline bool dist_claim(const SpState& st, uint8_t* dense, uint32_t side, uint32_t p, uint32_t v, int64_t n,
                                  uint32_t val) {
  (void)side;
  return claim_byte(dense, didx(st, p, v, n), val);
}

// zero the counter slots in `mask` (bit i = cnt[i]; one launch instead of a memset per slot run)
// and, when xdeg is given, the X degree sentinel xdeg[0] the scan reads past the list
// (z, zn: an extra array zeroed by the same launch -- the sweep's per-pair cost sums)
__global__ void k_cnt_zero(unsigned long long* cnt, uint32_t mask, int64_t* xdeg, unsigned long long* z = nullptr,
                           int64_t zn = 0) {
  const int i = threadIdx.x;
  if (i < 32 && ((mask >> i) & 1u)) cnt[i] = 0ull;
  if (i == 32 && xdeg) *xdeg = 0;
  for (int64_t k = i; k < zn; k += blockDim.x) z[k] = 0ull;
}

// seed both frontiers; trivial pairs (src == dst, unknown vertex, max_steps < 1) finish here
__global__ void k_sp_init(const int64_t* svid, const int64_t* tvid, const int32_t* gs, const int32_t* gt, int32_t B,
                          int32_t max_steps, int64_t n, SpState st, SpCsr gout, SpCsr gin, uint8_t* d0, uint8_t* d1,
                          SpBufs bf, unsigned long long* cnt) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;  // grid covers B rounded up to a block
  bool go = false;
  int32_t a = -1, b = -1;
  if (p < B) {
    a = gs[p];
    b = gt[p];
    st.res[p] = svid[p] == tvid[p] ? 0 : -1;
    st.lvl[p] = st.lvl[B + p] = 0;
    st.met[p] = 0;
    go = svid[p] != tvid[p] && a >= 0 && b >= 0 && max_steps >= 1;
    st.state[p] = go ? SP_ACTIVE : SP_DONE;
    st.deg[p] = st.deg[B + p] = 0;
    if (go) {
      dist_claim(st, d0, 0, uint32_t(p), uint32_t(a), n, 0);
      dist_claim(st, d1, 1, uint32_t(p), uint32_t(b), n, 0);
      st.deg[p] = (unsigned long long)sp_deg(gout, uint32_t(a)) + 1;
      st.deg[B + p] = (unsigned long long)sp_deg(gin, uint32_t(b)) + 1;
    }
  }
  const uint64_t tf = mk_tup(0, uint32_t(p), 0, uint32_t(a)), tb = mk_tup(1, uint32_t(p), 0, uint32_t(b));
  put(bf.live_next[0], bf.cap_live[0], cnt, C_LIVE0, go, tf);
  put(bf.live_next[1], bf.cap_live[1], cnt, C_LIVE1, go, tb);
  put(bf.arena, bf.cap_arena, cnt, C_ARENA, go, tf);
  put(bf.arena, bf.cap_arena, cnt, C_ARENA, go, tb);
}

// end of iteration `iter` (first = 0) and the side choice of the next one
__global__ void k_sp_step(SpState st, int32_t max_steps, int32_t first, int32_t iter, unsigned long long* cnt) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  bool active = false;
  if (p < st.B && st.state[p] == SP_ACTIVE) {
    const int B = st.B;
    if (!first) {
      const int s = st.side[p];
      st.pside[p] = s;
      st.lvl[s * B + p] += 1;
      const int32_t L = st.lvl[p] + st.lvl[B + p];
      if (st.met[p]) {
        st.res[p] = L;
        st.state[p] = SP_MET;
        st.met[p] = 2 + iter;
      } else if (st.deg[s * B + p] == 0 || L >= max_steps) {
        st.state[p] = SP_DONE;  // a side's reachable set is closed, or the step bound is hit
      }
    }
    if (st.state[p] == SP_ACTIVE) {
      const int s = st.deg[p] <= st.deg[B + p] ? 0 : 1;
      st.side[p] = s;
      st.deg[s * B + p] = 0;  // the expansion accumulates the new frontier's sum
      active = true;
    }
  }
  const int64_t slot = wave_append(cnt + C_ACTIVE, active);
  (void)slot;
}

// Rebuild a list whose appends overflowed from the distance bytes (claims are recorded in the
// bytes even when their tuple could not be stored).  One y-slice of the grid per listed pair.
//  RG_LIVE:  side s tuples at the side's new depth (pairs that expanded s)
//  RG_MEET:  vertices seen at depth f forward and b backward (pairs that met this iteration)
//  RG_SWEEP: sweep claims of step j (dist_B = b + j)
enum : int { RG_LIVE = 0, RG_MEET = 1, RG_SWEEP = 2 };
__global__ void k_sp_regen(int mode, int side, int32_t j, const int32_t* plist, int32_t np, SpState st,
                           const uint8_t* d0, const uint8_t* d1, int64_t n, uint64_t* out, int64_t cap,
                           unsigned long long* cnt, int which) {
  const int32_t B = st.B;
  for (int32_t q = blockIdx.y; q < np; q += gridDim.y) {
    const uint32_t p = uint32_t(plist[q]);
    uint32_t tv, tf = 0;
    if (mode == RG_LIVE) {
      tv = uint32_t(st.lvl[side * B + p]);
    } else if (mode == RG_MEET) {
      tv = uint32_t(st.lvl[B + p]);
      tf = uint32_t(st.lvl[p]);
    } else {
      tv = uint32_t(st.lvl[B + p] + j);
    }
    const uint8_t* rowd = (mode == RG_LIVE && side == 0) ? d0 : d1;
    const uint8_t* rowf = d0;
    const int64_t stride = int64_t(gridDim.x) * blockDim.x;
    const int64_t rounds = (n + stride - 1) / stride;
    for (int64_t r = 0; r < rounds; r++) {
      const int64_t v = r * stride + blockIdx.x * int64_t(blockDim.x) + threadIdx.x;
      bool hit = false;
      if (v < n) {
        hit = rowd[didx(st, p, uint64_t(v), n)] == tv;
        if (mode == RG_MEET) hit = hit && rowf[didx(st, p, uint64_t(v), n)] == tf;
      }
      put(out, cap, cnt, which, hit, mk_tup(mode == RG_LIVE ? uint32_t(side) : 1u, p, tv, uint32_t(v)));
    }
  }
}

// Block-wide reservation in two lists at once (256-thread blocks, block-uniform call): a thread
// asks for na slots of list A and nb of list B (each < 2^16 per block); returns its first slot
// in each.  One returning atomic per list and block: a counter takes ~90 returning atomics per us
// on one address, so the per-wave appends of a 748 K-tuple select (two lists, ~23 K atomics)
// had held it at ~75 us.
constexpr int kBlk = 256;
__device__ inline void blk_reserve2(unsigned long long* ca, unsigned long long* cb, uint32_t na, uint32_t nb,
                                    unsigned long long& oa, unsigned long long& ob) {
  __shared__ uint32_t s_w[kBlk / 64];
  __shared__ unsigned long long s_base[2];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint32_t x = na | (nb << 16);
  uint32_t v = x;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(v, o);
    if (lane >= o) v += y;
  }
  if (lane == 63) s_w[w] = v;
  __syncthreads();
  uint32_t pre = v - x, tot = 0;
#pragma unroll
  for (int i = 0; i < kBlk / 64; i++) {
    if (i < w) pre += s_w[i];
    tot += s_w[i];
  }
  if (threadIdx.x == 0) {
    s_base[0] = (tot & 0xFFFFu) ? atomicAdd(ca, (unsigned long long)(tot & 0xFFFFu)) : 0ull;
    s_base[1] = (tot >> 16) ? atomicAdd(cb, (unsigned long long)(tot >> 16)) : 0ull;
  }
  __syncthreads();
  oa = s_base[0] + (pre & 0xFFFFu);
  ob = s_base[1] + (pre >> 16);
  __syncthreads();  // s_w / s_base are reused by the next call
}

// split a live list: tuples of the side their pair expands now -> X (with degrees), the rest
// of still-active pairs -> carried into the next live list.  sweep = 1: the list holds sweep
// tuples; those of MET pairs short of src go to X.  kSelIt tuples per thread (their loads in
// flight together), one reservation per block and round.
constexpr int kSelIt = 8;
int grid_sel(int64_t n) { return int(std::max<int64_t>(1, std::min<int64_t>((n + kBlk * kSelIt - 1) / (kBlk * kSelIt), 4096))); }
__global__ __launch_bounds__(kBlk) void k_sp_select(const uint64_t* __restrict__ live, int64_t nl, int32_t sweep,
                                                    SpState st, SpCsr gout, SpCsr gin, uint64_t* X, int64_t* Xdeg,
                                                    int64_t cap_x, SpBufs bf, unsigned long long* cnt,
                                                    const int32_t* push_pair = nullptr) {
  constexpr int64_t per = int64_t(kBlk) * kSelIt;
  const int64_t rounds = (nl + per - 1) / per;
  // carried tuples: every tuple of one launch has the same side (one list per side)
  const uint32_t side = nl > 0 ? t_side(live[0]) : 0u;
  uint64_t* const carry = bf.live_next[side];
  const int64_t cap_carry = bf.cap_live[side];
  const SpCsr& g = side ? gin : gout;
  unsigned long long esum = 0;  // X's degree sum: one counter add per block at the end
  for (int64_t r = blockIdx.x; r < rounds; r += gridDim.x) {
    const int64_t i0 = r * per + threadIdx.x;
    uint64_t t[kSelIt];
    int32_t s[kSelIt];
#pragma unroll
    for (int u = 0; u < kSelIt; u++) t[u] = i0 + u * kBlk < nl ? live[i0 + u * kBlk] : ~0ull;
#pragma unroll
    for (int u = 0; u < kSelIt; u++) s[u] = t[u] != ~0ull ? st.state[t_pair(t[u])] : SP_DONE;
    uint32_t gm = 0, sm = 0;
#pragma unroll
    for (int u = 0; u < kSelIt; u++) {
      if (t[u] == ~0ull) continue;
      const uint32_t p = t_pair(t[u]);
      if (sweep) {
        // sweep = 2: stop one level short of src (the walk from src never reads dist_B(src),
        // and the in-lists of src's shortest-path out-neighbours are typically hub rows)
        if (s[u] == SP_MET && int32_t(t_lvl(t[u])) < st.res[p] - (sweep - 1) && !(push_pair && push_pair[p]))
          gm |= 1u << u;
      } else if (s[u] == SP_ACTIVE) {
        if (uint32_t(st.side[p]) == side) gm |= 1u << u;
        else sm |= 1u << u;
      }
    }
    int64_t d[kSelIt];
    unsigned long long dsum = 0;
#pragma unroll
    for (int u = 0; u < kSelIt; u++) {
      d[u] = (gm >> u) & 1u ? sp_deg(g, t_row(t[u])) : 0;
      dsum += (unsigned long long)d[u];
    }
    unsigned long long ox, oc;
    blk_reserve2(cnt + C_X, cnt + (side ? C_LIVE1 : C_LIVE0), uint32_t(__popc(gm)), uint32_t(__popc(sm)), ox, oc);
    bool ovf_x = false, ovf_c = false;
#pragma unroll
    for (int u = 0; u < kSelIt; u++) {
      if ((gm >> u) & 1u) {
        if (int64_t(ox) < cap_x) {
          X[ox] = t[u];
          Xdeg[ox] = d[u];
        } else {
          ovf_x = true;
        }
        ox++;
      } else if ((sm >> u) & 1u) {
        if (int64_t(oc) < cap_carry) carry[oc] = t[u];
        else ovf_c = true;
        oc++;
      }
    }
    if (ovf_x) atomicOr(cnt + C_OVF, 2ull);
    if (ovf_c) atomicOr(cnt + C_OVF, 1ull);
    esum += dsum;
  }
  __shared__ unsigned long long s_e[kBlk / 64];
  const unsigned long long e = wsum(esum);
  if ((threadIdx.x & 63) == 0) s_e[threadIdx.x >> 6] = e;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long bt = 0;
#pragma unroll
    for (int i = 0; i < kBlk / 64; i++) bt += s_e[i];
    if (bt) atomicAdd(cnt + C_XE, bt);
  }
}

// ---- sweep direction per pair -----------------------------------------------------------------
// A sweep step gives dist_B to the shortest-path vertices at forward depth k = f - j.  Pull scans
// the in-rows of the level above (the current sweep list); push scans the out-rows of the forward
// BFS's level-k vertices (the arena's side-0 tuples at depth k), claiming a vertex whose
// out-neighbour has dist_B = L - k - 1.  Both claim the same vertices; each pair takes the side
// with fewer adjacency entries.
__device__ inline bool sweep_pull_go(const SpState& st, uint64_t t, int32_t sweep) {
  const uint32_t p = t_pair(t);
  return st.state[p] == SP_MET && int32_t(t_lvl(t)) < st.res[p] - (sweep - 1);
}
__global__ void k_sweep_pull_cost(const uint64_t* __restrict__ live, int64_t nl, int32_t sweep, SpState st,
                                  SpCsr gin, unsigned long long* pull) {
  const int64_t stride = int64_t(gridDim.x) * blockDim.x;
  const int64_t rounds = (nl + stride - 1) / stride;
  for (int64_t r = 0; r < rounds; r++) {
    const int64_t i = r * stride + blockIdx.x * int64_t(blockDim.x) + threadIdx.x;
    bool go = false;
    uint32_t p = 0;
    unsigned long long d = 0;
    if (i < nl) {
      const uint64_t t = live[i];
      p = t_pair(t);
      go = sweep_pull_go(st, t, sweep);
      if (go) d = (unsigned long long)sp_deg(gin, t_row(t)) + 1;
    }
    wave_add_keyed(pull, p, d, go);
  }
}
// forward level-k tuples of the arena (k = f - j) of pairs still sweeping
__device__ inline bool sweep_push_tuple(const SpState& st, uint64_t t, int32_t j) {
  if (t_side(t) != 0) return false;
  const uint32_t p = t_pair(t);
  if (st.state[p] != SP_MET) return false;
  const int32_t k = st.lvl[p] - j;
  return k >= 1 && int32_t(t_lvl(t)) == k;
}
__global__ void k_sweep_push_cost(const uint64_t* __restrict__ arena, int64_t na, int32_t j, SpState st,
                                  SpCsr gout, const unsigned long long* pull, unsigned long long* push) {
  const int64_t stride = int64_t(gridDim.x) * blockDim.x;
  const int64_t rounds = (na + stride - 1) / stride;
  for (int64_t r = 0; r < rounds; r++) {
    const int64_t i = r * stride + blockIdx.x * int64_t(blockDim.x) + threadIdx.x;
    bool go = false;
    uint32_t p = 0;
    unsigned long long d = 0;
    if (i < na) {
      const uint64_t t = arena[i];
      go = sweep_push_tuple(st, t, j);
      p = t_pair(t);
      go = go && pull[p] > 0;  // pairs with nothing to pull are done sweeping
      if (go) d = (unsigned long long)sp_deg(gout, t_row(t)) + 1;
    }
    wave_add_keyed(push, p, d, go);
  }
}
// bias (option sp_push_bias, in 1/16): push when its entries are below pull's x bias / 16 (a push
// row scan stops at its first hit, so its full degree sum overstates it)
__global__ void k_sweep_choose(const unsigned long long* pull, const unsigned long long* push, int32_t B,
                               int32_t* push_pair, unsigned long long bias16) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p < B) push_pair[p] = pull[p] > 0 && push[p] * 16ull < pull[p] * bias16;
}
// X += the forward level-k tuples of push pairs (their out-rows are the step's adjacency)
__global__ void k_sweep_push_select(const uint64_t* __restrict__ arena, int64_t na, int32_t j, SpState st,
                                    SpCsr gout, const int32_t* push_pair, uint64_t* X, int64_t* Xdeg,
                                    int64_t cap_x, unsigned long long* cnt) {
  const int64_t stride = int64_t(gridDim.x) * blockDim.x;
  const int64_t rounds = (na + stride - 1) / stride;
  for (int64_t r = 0; r < rounds; r++) {
    const int64_t i = r * stride + blockIdx.x * int64_t(blockDim.x) + threadIdx.x;
    bool go = false;
    uint64_t t = 0;
    int64_t d = 0;
    if (i < na) {
      t = arena[i];
      go = sweep_push_tuple(st, t, j) && push_pair[t_pair(t)];
      if (go) d = sp_deg(gout, t_row(t));
    }
    const int64_t xs = wave_append(cnt + C_X, go);
    if (go) {
      if (xs < cap_x) {
        X[xs] = t;
        Xdeg[xs] = d;
      } else {
        atomicOr(cnt + C_OVF, 2ull);
      }
    }
    const unsigned long long e = wsum((unsigned long long)d);
    if ((threadIdx.x & 63) == 0 && e) atomicAdd(cnt + C_XE, e);
  }
}

struct SpExpand {
  const uint64_t* X;
  int64_t nX;
  const int64_t* off;  // exclusive scan of X degrees, off[nX] = E
  SpCsr g[2];          // [0] out CSR (forward), [1] in CSR (backward)
  uint8_t* dist[2];
  const int64_t* vid_of;
  int64_t n;           // owned rows (pair stride of dist)
  int64_t lo;
  int32_t sweep;
  const int32_t* tile_row;  // k_tile_rows: X entry holding each tile's first slot (null: search)
};

// One edge-balanced pass over the adjacency of every X tuple (tiles of kTileE entries).
//  sweep = 0: BFS level of the chosen side; claims append to that side's next live list (and
//             the arena), add (degree + 1) to the pair's frontier sum, and detect meets.
//  sweep = 1: backward extension restricted to shortest paths: u (in-neighbour of w, which has
//             dt = l) is on a shortest path iff ds(u) = L - l - 1; it gets dt = l + 1.
__global__ __launch_bounds__(kT) void k_sp_expand(SpExpand a, SpState st, SpBufs bf, unsigned long long* cnt) {
  __shared__ int32_t s_off[kTileE + 1];
  __shared__ int64_t s_rs[kTileE];
  __shared__ uint64_t s_tup[kTileE];
  __shared__ int64_t s_hdr[2];
  __shared__ int32_t s_scan[kT / 64];
  __shared__ uint32_t s_n[3];           // tile appends staged: side-0 claims, side-1 claims, meets
  __shared__ unsigned long long s_base[4];
  // Appends are staged per tile in LDS (claims in s_rs's words: side 0 from the front, side 1
  // from the back; meets in s_tup's) and reserved with one global atomic per list and tile: the
  // lists' returning counter atomics (one per wave, slot round and list) serialise at ~90 per us
  // on one address, which held a 748 K-claim BFS level at ~0.3 ms and the 67 K-claim sweep
  // behind a 72 M-entry scan.
  uint64_t* const stage = reinterpret_cast<uint64_t*>(s_rs);
  uint64_t* const mstage = s_tup;
  const int64_t nX = a.nX;
  const int64_t E = a.off[nX];
  const int64_t ntiles = (E + kTileE - 1) / kTileE;
  for (int64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const int64_t e0 = t * kTileE;
    const int64_t e1 = min(e0 + int64_t(kTileE), E);
    if (threadIdx.x < 3) s_n[threadIdx.x] = 0u;
    if (threadIdx.x == 0 && a.tile_row) {
      int64_t i0, cnt;
      tile_entries(a.tile_row, a.off, nX, t, e1, E, i0, cnt);
      s_hdr[0] = i0;
      s_hdr[1] = cnt;
    } else if (threadIdx.x == 0) {
      int64_t lo = 0, hi = nX;  // off[lo] <= e0 < off[hi]
      while (hi - lo > 1) {
        const int64_t mid = (lo + hi) >> 1;
        if (a.off[mid] <= e0) lo = mid; else hi = mid;
      }
      const int64_t i0 = lo;
      hi = nX;
      while (hi - lo > 1) {
        const int64_t mid = (lo + hi) >> 1;
        if (a.off[mid] <= e1 - 1) lo = mid; else hi = mid;
      }
      s_hdr[0] = i0;
      s_hdr[1] = lo - i0 + 1;
    }
    __syncthreads();
    const int64_t i0 = s_hdr[0];
    const int64_t cnt64 = s_hdr[1];
    // zero-degree X entries (dropped pairs, vertices without edges) can put more than kTileE
    // entries under one tile: such a tile searches off[] in global memory instead of LDS
    const bool big = cnt64 > kTileE;
    const int cnt_k = big ? 0 : int(cnt64);
    for (int k = threadIdx.x; k <= cnt_k && !big; k += kT) {
      const int64_t o = a.off[i0 + k];
      s_off[k] = int32_t(min(o - e0, int64_t(kTileE + 1)));
      if (k < cnt_k) {
        const uint64_t tu = a.X[i0 + k];
        s_tup[k] = tu;
        s_rs[k] = a.g[t_side(tu)].row_ptr[t_row(tu)] - o;
      }
    }
    __syncthreads();
    if (!big) tile_owner_map<kTileE, kT>(s_off, cnt_k, s_scan);  // s_off[j] = owner of slot j
    // The slots' memory reads in phases, each phase's loads of all kIt slots in flight before
    // the first is used (slot by slot, a tile waited on kIt chains of col -> res -> filter ->
    // distance byte: the latency-bound sweep ran at ~45 G entries/s): owners and column
    // entries, then the pairs' depths, then the level filter bits, then the distance bytes
    // the tests read; the claims (CAS loops) and appends follow.
    uint64_t tus[kIt];
    int64_t gi[kIt];  // column index of the slot's entry, -1: past the tile
#pragma unroll
    for (int r = 0; r < kIt; r++) {
      const int j = threadIdx.x + r * kT;
      const int64_t e = e0 + j;
      const bool valid = e < e1;
      uint64_t tu = 0;
      int64_t rsk = 0;
      if (valid && !big) {
        const int k = s_off[j];
        tu = s_tup[k];
        rsk = s_rs[k];
      } else if (valid) {
        int64_t lo = i0, hi = i0 + cnt64;  // off[lo] <= e < off[hi]
        while (hi - lo > 1) {
          const int64_t mid = (lo + hi) >> 1;
          if (a.off[mid] <= e) lo = mid; else hi = mid;
        }
        tu = a.X[lo];
        rsk = a.g[t_side(tu)].row_ptr[t_row(tu)] - a.off[lo];
      }
      tus[r] = tu;
      gi[r] = valid ? rsk + e : -1;
    }
    __syncthreads();  // s_tup / s_rs are staging buffers from here on
    uint32_t ws[kIt];
#pragma unroll
    for (int r = 0; r < kIt; r++)
      ws[r] = gi[r] >= 0 ? uint32_t(int64_t(a.g[t_side(tus[r])].col[gi[r]]) - a.lo) : 0u;
    // the depth a sweep test needs: pull, the in-neighbour's forward depth; push, the
    // out-neighbour's backward depth (both L - l - 1)
    int32_t need[kIt];
#pragma unroll
    for (int r = 0; r < kIt; r++)
      need[r] = a.sweep && gi[r] >= 0 ? st.res[t_pair(tus[r])] - int32_t(t_lvl(tus[r])) - 1 : -1;
    bool lv[kIt];
#pragma unroll
    for (int r = 0; r < kIt; r++)
      lv[r] = gi[r] >= 0 && (!a.sweep || (need[r] >= 0 && lv_maybe(st, t_side(tus[r]) ^ 1u, need[r], ws[r])));
    // the byte each test reads: BFS, the slot's own side (0xFF: unseen); sweep, the other side
    uint32_t bt[kIt];
#pragma unroll
    for (int r = 0; r < kIt; r++) {
      const uint32_t side = t_side(tus[r]), ds = a.sweep ? side ^ 1u : side;
      bt[r] = lv[r] ? dist_get(st, a.dist[ds], ds, t_pair(tus[r]), ws[r], a.n) : 0x1FFu;
    }
#pragma unroll
    for (int r = 0; r < kIt; r++) {
      const uint64_t tu = tus[r];
      const bool valid = gi[r] >= 0;
      const uint32_t side = t_side(tu), p = t_pair(tu), l = t_lvl(tu);
      const uint32_t w = ws[r];
      bool claimed = false;
      if (valid) {
        if (!a.sweep) {
          claimed = bt[r] == 0xFFu && dist_claim(st, a.dist[side], side, p, w, a.n, l + 1);
          if (claimed) lv_mark(st, side, l + 1, w);
        } else if (side == 1) {  // pull: in-neighbour w of a level-(k+1) vertex, forward depth k
          if (bt[r] == uint32_t(need[r])) {
            claimed = dist_claim(st, a.dist[1], 1, p, w, a.n, l + 1);
            if (claimed) lv_mark(st, 1, l + 1, w);
          }
        } else {  // push: the tuple's own vertex u (forward depth l) if out-neighbour w is on a path
          const uint32_t u = t_row(tu);
          if (bt[r] == uint32_t(need[r])) {
            claimed = dist_claim(st, a.dist[1], 1, p, u, a.n, uint32_t(need[r] + 1));
            if (claimed) lv_mark(st, 1, uint32_t(need[r] + 1), u);
          }
        }
      }
      // a push claim records u with dist_B = L - l; every other claim the neighbour at depth l + 1
      const bool push_t = a.sweep && side == 0;
      const uint64_t nt = push_t ? mk_tup(1, p, uint32_t(need[r] + 1), t_row(tu)) : mk_tup(side, p, l + 1, w);
      if (claimed) {  // arena + (sweep list | the side's live list); a sweep stages at the front
        if (a.sweep || side == 0) stage[atomicAdd(&s_n[0], 1u)] = nt;
        else stage[kTileE - 1 - int(atomicAdd(&s_n[1], 1u))] = nt;
      }
      if (a.sweep) continue;
      const unsigned long long dv = claimed ? (unsigned long long)sp_deg(a.g[side], w) + 1 : 0ull;
      wave_add_keyed(st.deg, side * uint32_t(st.B) + p, dv, claimed);
      bool meet = false;
      uint32_t dt = 0;
      if (claimed) {
        const uint32_t o = dist_get(st, a.dist[side ^ 1], side ^ 1u, p, w, a.n);
        if (o != 0xFFu) {
          meet = true;
          dt = side ? l + 1 : uint32_t(o);
          st.met[p] = 1;
        }
      }
      if (meet) mstage[atomicAdd(&s_n[2], 1u)] = mk_tup(1, p, dt, w);
    }
    __syncthreads();
    const uint32_t n0 = s_n[0], n1 = s_n[1], nm = s_n[2];
    if (threadIdx.x == 0) {
      s_base[0] = n0 + n1 ? atomicAdd(cnt + C_ARENA, (unsigned long long)(n0 + n1)) : 0ull;
      s_base[1] = n0 ? atomicAdd(cnt + (a.sweep ? C_SWEEP : C_LIVE0), (unsigned long long)n0) : 0ull;
      s_base[2] = n1 ? atomicAdd(cnt + C_LIVE1, (unsigned long long)n1) : 0ull;
      s_base[3] = nm ? atomicAdd(cnt + C_MEET, (unsigned long long)nm) : 0ull;
    }
    __syncthreads();
    auto store = [&](uint64_t* list, int64_t cap, unsigned long long at, uint64_t v) {
      if (int64_t(at) < cap) list[at] = v;
      else atomicOr(cnt + C_OVF, 1ull);
    };
    for (uint32_t q = threadIdx.x; q < n0 + n1; q += kT) {
      const bool front = q < n0;
      const uint64_t v = front ? stage[q] : stage[kTileE - 1 - int(q - n0)];
      store(bf.arena, bf.cap_arena, s_base[0] + q, v);
      if (front) store(a.sweep ? bf.sweep_next : bf.live_next[0], a.sweep ? bf.cap_sweep : bf.cap_live[0], s_base[1] + q, v);
      else store(bf.live_next[1], bf.cap_live[1], s_base[2] + (q - n0), v);
    }
    for (uint32_t q = threadIdx.x; q < nm; q += kT) store(bf.meet, bf.cap_meet, s_base[3] + q, mstage[q]);
    __syncthreads();
  }
}

// ---- chunked scans (meet probe, sweep) --------------------------------------------------------
// chunk_x[c] = the X entry holding chunk c (choff = exclusive scan of the entries' chunk counts):
// one coalesced pass instead of a binary search of choff (~15 dependent loads) per chunk
// slot (the meet probe): its per-chunk result slots are emptied here too (no memset launch)
__global__ void k_chunk_x(const int64_t* __restrict__ choff, int64_t nX, int32_t* __restrict__ chunk_x,
                          uint64_t* __restrict__ slot = nullptr) {
  wave_fill_ranges(
      nX, [&](int64_t i, int64_t& c0, int64_t& c1) { c0 = choff[i], c1 = choff[i + 1]; },
      [&](int64_t c, int64_t i) {
        chunk_x[c] = int32_t(i);
        if (slot) slot[c] = ~0ull;
      });
}

// One sweep step over the X tuples' adjacency, one wave per chunk of kSwCh entries (the meet
// vertices' in-rows average ~10 K entries: the edge-balanced tile scheme paid a tile header,
// an LDS owner map and four barriers per 2048 entries).  Pull (side 1, in-row of w at dt = l):
// an in-neighbour u with ds(u) = L - l - 1 gets dt = l + 1.  Push (side 0, out-row of u at
// ds = l): u gets dt = L - l once an out-neighbour has dt = L - l - 1 (the scan stops there).
// kProbeU entries per lane a step, their column loads, filter bits and distance bytes each in
// flight together.  Claims are staged per wave in LDS and appended to the arena and the next
// sweep list with one counter atomic per list and flush.
constexpr int kProbeU = 4;  // entries per lane and step of the chunked scans
constexpr int kSwCh = 1024;
constexpr int kSwStage = 256;
template <int OCC>  // waves per SIMD the register budget allows (option sp_sweep_occ: 5 or 8)
__global__ __launch_bounds__(256, OCC) void k_sp_sweep(const uint64_t* __restrict__ X, const int64_t* __restrict__ choff,
                                                  const int32_t* __restrict__ chunk_x, int64_t nX, SpCsr gout,
                                                  SpCsr gin, uint8_t* d0, uint8_t* d1, int64_t n, int64_t lo,
                                                  SpState st, SpBufs bf, unsigned long long* cnt) {
  __shared__ uint64_t s_stage[4][kSwStage];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  uint64_t* stg = s_stage[wid];
  const int64_t wave = (int64_t(blockIdx.x) * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = (int64_t(gridDim.x) * blockDim.x) >> 6;
  uint32_t ns = 0;  // wave-uniform: claims staged
  const int64_t total = choff[nX];
  auto flush = [&]() {
    if (ns == 0) return;
    __builtin_amdgcn_wave_barrier();
    unsigned long long ba = 0, bs = 0;
    if (lane == 0) {
      ba = atomicAdd(cnt + C_ARENA, (unsigned long long)ns);
      bs = atomicAdd(cnt + C_SWEEP, (unsigned long long)ns);
    }
    ba = __shfl(ba, 0);
    bs = __shfl(bs, 0);
    for (uint32_t q = uint32_t(lane); q < ns; q += 64) {
      const uint64_t v = stg[q];
      if (int64_t(ba + q) < bf.cap_arena) bf.arena[ba + q] = v;
      else atomicOr(cnt + C_OVF, 1ull);
      if (int64_t(bs + q) < bf.cap_sweep) bf.sweep_next[bs + q] = v;
      else atomicOr(cnt + C_OVF, 1ull);
    }
    __builtin_amdgcn_wave_barrier();
    ns = 0;
  };
  auto stage = [&](bool claimed, uint64_t v) {  // wave-uniform call
    const uint64_t m = __ballot(claimed);
    if (m == 0) return;
    if (ns + uint32_t(__popcll(m)) > uint32_t(kSwStage)) flush();
    if (claimed) stg[ns + uint32_t(__popcll(m & ((1ull << lane) - 1ull)))] = v;
    ns += uint32_t(__popcll(m));
  };
  for (int64_t c = wave; c < total; c += nwaves) {
    const int32_t a = chunk_x[c];
    const uint64_t t = X[a];
    const uint32_t side = t_side(t), p = t_pair(t), l = t_lvl(t), row = t_row(t);
    const int64_t* rp = side ? gin.row_ptr : gout.row_ptr;
    const int32_t* col = side ? gin.col : gout.col;
    const int64_t x0 = rp[row] + (c - choff[a]) * kSwCh;
    const int64_t x1 = min(x0 + int64_t(kSwCh), rp[row + 1]);
    const int32_t need = st.res[p] - int32_t(l) - 1;  // the other side's depth a neighbour needs
    for (int64_t x = x0; x < x1; x += 64 * kProbeU) {
      if (side == 0 && dist_get(st, d1, 1, p, row, n, true) != 0xFFu) break;  // u claimed
      uint32_t w[kProbeU];
#pragma unroll
      for (int u = 0; u < kProbeU; u++) {
        const int64_t ex = x + u * 64 + lane;
        w[u] = ex < x1 ? uint32_t(int64_t(col[ex]) - lo) : 0xFFFFFFFFu;
      }
      bool f[kProbeU];
#pragma unroll
      for (int u = 0; u < kProbeU; u++)
        f[u] = w[u] != 0xFFFFFFFFu && need >= 0 && lv_maybe(st, side ^ 1u, need, w[u]);
      uint32_t b[kProbeU];
#pragma unroll
      for (int u = 0; u < kProbeU; u++) b[u] = f[u] ? dist_get(st, side ? d0 : d1, side ^ 1u, p, w[u], n) : 0x1FFu;
      if (side == 1) {
#pragma unroll
        for (int u = 0; u < kProbeU; u++) {
          bool claimed = false;
          if (b[u] == uint32_t(need)) {
            claimed = dist_claim(st, d1, 1, p, w[u], n, l + 1);
            if (claimed) lv_mark(st, 1, l + 1, w[u]);
          }
          stage(claimed, mk_tup(1, p, l + 1, w[u]));
        }
      } else {
        bool hit = false;
#pragma unroll
        for (int u = 0; u < kProbeU; u++) hit = hit || b[u] == uint32_t(need);
        if (__ballot(hit)) {
          bool claimed = false;
          if (lane == 0) {
            claimed = dist_claim(st, d1, 1, p, row, n, uint32_t(need + 1));
            if (claimed) lv_mark(st, 1, uint32_t(need + 1), row);
          }
          stage(claimed, mk_tup(1, p, uint32_t(need + 1), row));
          break;
        }
      }
    }
  }
  // the final flush per block, not per wave: one pair of counter atomics for the block's four
  // stages (the waves of the grid end together, and their returning atomics on the two
  // counters queued behind each other at the kernel's tail)
  __shared__ uint32_t s_ns[4];
  __shared__ unsigned long long s_b[2];
  if (lane == 0) s_ns[wid] = ns;
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned long long tot = s_ns[0] + s_ns[1] + s_ns[2] + s_ns[3];
    s_b[0] = tot ? atomicAdd(cnt + C_ARENA, tot) : 0ull;
    s_b[1] = tot ? atomicAdd(cnt + C_SWEEP, tot) : 0ull;
  }
  __syncthreads();
  uint32_t pre = 0;
  for (int k = 0; k < wid; k++) pre += s_ns[k];
  const unsigned long long ba = s_b[0] + pre, bs = s_b[1] + pre;
  for (uint32_t q = uint32_t(lane); q < ns; q += 64) {
    const uint64_t v = stg[q];
    if (int64_t(ba + q) < bf.cap_arena) bf.arena[ba + q] = v;
    else atomicOr(cnt + C_OVF, 1ull);
    if (int64_t(bs + q) < bf.cap_sweep) bf.sweep_next[bs + q] = v;
    else atomicOr(cnt + C_OVF, 1ull);
  }
}

// ---- meet probe -----------------------------------------------------------------------------
// Before a pair expands its cheaper side s (frontier at depth l, the other side at depth l_o),
// probe whether the two frontiers are already one edge apart: a tuple's vertex r is a meet vertex
// of length f + b + 1 iff some neighbour of r (out-neighbour for s = 0, in-neighbour for s = 1)
// sits at depth l_o on the other side.  The probe scans each adjacency list only until its first
// hit, so pairs that meet skip the full expansion (whose cost is the whole frontier's degree sum,
// hubs included).  A failed probe leaves everything as it was: the expansion then finds no meet
// either (a meet at f + b + 1 is exactly such an edge), so detection stays complete.
constexpr int kProbeCh = 1024;  // adjacency entries per probe chunk (one wave each)

// ch[i] = number of chunks of `size` entries of X[i]; ch[nX] = 0
__global__ void k_sp_chunks_n(const int64_t* Xdeg, int64_t nX, int64_t* ch, int64_t size) {
  for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i <= nX; i += int64_t(gridDim.x) * blockDim.x)
    ch[i] = i == nX ? 0 : (Xdeg[i] + size - 1) / size;
}
// ch[i] = number of probe chunks of X[i]; ch[nX] = 0; the probe's examined-entry counter cleared
__global__ void k_sp_chunks(const int64_t* Xdeg, int64_t nX, int64_t* ch, unsigned long long* cnt) {
  if (blockIdx.x == 0 && threadIdx.x == 0) cnt[C_PE] = 0ull;
  for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i <= nX; i += int64_t(gridDim.x) * blockDim.x)
    ch[i] = i == nX ? 0 : (Xdeg[i] + kProbeCh - 1) / kProbeCh;
}

// One wave per chunk of kProbeCh entries of an X tuple, 64 entries a step, stopping at the first
// hit or once another chunk has claimed the vertex.  The winner claims r's byte on the other
// side (depth l_o + 1: the vertex is then seen by both sides, as after an expansion of the other
// side) and records that claim in slot[c] (an arena tuple); k_sp_gather_meets turns the slots into
// the meet list without a global atomic per meet.
template <int OCC>
__global__ __launch_bounds__(256, OCC) void k_sp_probe(const uint64_t* __restrict__ X, int64_t nX,
                                                  const int64_t* __restrict__ choff,
                                                  const int32_t* __restrict__ chunk_x, SpCsr g0, SpCsr g1, uint8_t* d0,
                                                  uint8_t* d1, int64_t n, int64_t lo, SpState st, uint64_t* slot,
                                                  unsigned long long* cnt) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = (int64_t(blockIdx.x) * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = (int64_t(gridDim.x) * blockDim.x) >> 6;
  const int64_t total = choff[nX];
  unsigned long long examined = 0;
  for (int64_t c = wave; c < total; c += nwaves) {
    const int64_t a = chunk_x[c];  // the tuple holding chunk c
    const uint64_t t = X[a];
    const uint32_t side = t_side(t), p = t_pair(t), row = t_row(t);
    const int64_t* rp = side ? g1.row_ptr : g0.row_ptr;
    const int32_t* col = side ? g1.col : g0.col;
    const int64_t x0 = rp[row] + (c - choff[a]) * kProbeCh;
    const int64_t x1 = min(x0 + int64_t(kProbeCh), rp[row + 1]);
    const uint32_t other = side ^ 1u;
    const uint32_t need = uint32_t(st.lvl[other * uint32_t(st.B) + p]);
    uint8_t* od = other ? d1 : d0;
    // kProbeU entries per lane a step: their column loads, then their filter bits, then their
    // distance bytes, each group in flight together (one entry per lane a step waited on three
    // dependent loads per 64 entries)
    for (int64_t x = x0; x < x1; x += 64 * kProbeU) {
      if (dist_get(st, od, other, p, row, n, true) != 0xFFu) break;
      uint32_t w[kProbeU];
#pragma unroll
      for (int u = 0; u < kProbeU; u++) {
        const int64_t ex = x + u * 64 + lane;
        w[u] = ex < x1 ? uint32_t(int64_t(col[ex]) - lo) : 0xFFFFFFFFu;
      }
      bool f[kProbeU];
#pragma unroll
      for (int u = 0; u < kProbeU; u++) f[u] = w[u] != 0xFFFFFFFFu && lv_maybe(st, other, int32_t(need), w[u]);
      bool hit = false;
#pragma unroll
      for (int u = 0; u < kProbeU; u++) {
        examined += w[u] != 0xFFFFFFFFu ? 1 : 0;
        hit = (f[u] && dist_get(st, od, other, p, w[u], n) == need) || hit;
      }
      if (__ballot(hit)) {
        if (lane == 0 && dist_claim(st, od, other, p, row, n, need + 1)) {
          lv_mark(st, other, need + 1, row);
          st.met[p] = 1;
          slot[c] = mk_tup(other, p, need + 1, row);
        }
        break;
      }
    }
  }
  // one counter atomic per block: the grid's waves (up to 16 K) end together, and one add each
  // on the same counter queued behind each other at the kernel's tail
  __shared__ unsigned long long s_ev[4];
  const unsigned long long ev = wsum(examined);
  if (lane == 0) s_ev[threadIdx.x >> 6] = ev;
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned long long bt = s_ev[0] + s_ev[1] + s_ev[2] + s_ev[3];
    if (bt) atomicAdd(cnt + C_PE, bt);
  }
}

// slots -> meet list (1, p, dt, r) + arena (the claimed byte).  Runs before k_sp_probe_end, so
// lvl still holds the depths the probe compared against.
__global__ __launch_bounds__(kBlk) void k_sp_gather_meets(const uint64_t* slot, int64_t m, SpState st, SpBufs bf,
                                                          unsigned long long* cnt, const int64_t* m_dev = nullptr) {
  if (m_dev) m = min(m, *m_dev);  // the probe's chunk count (slots past it are not emptied)
  constexpr int64_t per = int64_t(kBlk) * kSelIt;
  const int64_t rounds = (m + per - 1) / per;
  for (int64_t r = blockIdx.x; r < rounds; r += gridDim.x) {
    const int64_t i0 = r * per + threadIdx.x;
    uint64_t t[kSelIt];
    uint32_t k = 0;
#pragma unroll
    for (int u = 0; u < kSelIt; u++) {
      t[u] = i0 + u * kBlk < m ? slot[i0 + u * kBlk] : ~0ull;
      k += t[u] != ~0ull ? 1u : 0u;
    }
    unsigned long long om, oa;
    blk_reserve2(cnt + C_MEET, cnt + C_ARENA, k, k, om, oa);
    bool ovf = false;
#pragma unroll
    for (int u = 0; u < kSelIt; u++) {
      if (t[u] == ~0ull) continue;
      const uint32_t p = t_pair(t[u]);
      // claimed backward byte: r has dt = its new depth; claimed forward byte: r is on the
      // backward frontier (dt = the backward depth)
      const uint64_t mt = t_side(t[u]) ? mk_tup(1, p, t_lvl(t[u]), t_row(t[u]))
                                       : mk_tup(1, p, uint32_t(st.lvl[uint32_t(st.B) + p]), t_row(t[u]));
      if (int64_t(om) < bf.cap_meet) bf.meet[om] = mt;
      else ovf = true;
      if (int64_t(oa) < bf.cap_arena) bf.arena[oa] = t[u];
      else ovf = true;
      om++;
      oa++;
    }
    if (ovf) atomicOr(cnt + C_OVF, 1ull);
  }
}

// After a meet probe, one launch: thread i finishes pair i (i < B) as if the other side had
// expanded (its depth + 1) when the probe met, and drops X tuple i (i < nX) of a pair that met
// (degree 0: the expansion skips it).  An X tuple's pair was active when selected, so it met in
// this probe iff its met flag is set (1 before the pair's update, 2 + iter after: either order
// is seen as met).  Also clears the X degree sentinel Xdeg[nX] the expansion's scan reads.
__global__ void k_sp_probe_end(SpState st, int32_t iter, const uint64_t* X, int64_t* Xdeg, int64_t nX,
                               unsigned long long* cnt) {
  const int64_t stride = int64_t(gridDim.x) * blockDim.x;
  const int64_t m = max(int64_t(st.B), nX);
  const int64_t rounds = (m + stride - 1) / stride;
  if (blockIdx.x == 0 && threadIdx.x == 0) Xdeg[nX] = 0;
  for (int64_t r = 0; r < rounds; r++) {
    const int64_t i = r * stride + blockIdx.x * int64_t(blockDim.x) + threadIdx.x;
    if (i < st.B && st.state[i] == SP_ACTIVE && st.met[i] == 1) {
      const int B = st.B;
      const int p = int(i);
      const int adv = st.side[p] ^ 1;
      st.lvl[adv * B + p] += 1;
      st.res[p] = st.lvl[p] + st.lvl[B + p];
      st.state[p] = SP_MET;
      st.met[p] = 2 + iter;
      st.pside[p] = adv;
    }
    unsigned long long d = 0;
    if (i < nX && st.met[t_pair(X[i])] != 0) {
      d = (unsigned long long)Xdeg[i];
      Xdeg[i] = 0;
    }
    const unsigned long long sd = wsum(d);
    if ((threadIdx.x & 63) == 0 && sd) atomicAdd(cnt + C_XE, 0ull - sd);
  }
}


// one workgroup per pair that met: greedy walk from src (dist_B now exact on every shortest
// path).  Each step scans the current vertex's out-edges with the whole workgroup (hub rows on a
// path hold 10^5+ entries) and takes the smallest vid among those one step closer to dst.
constexpr int kWalkT = 512;
__global__ __launch_bounds__(kWalkT) void k_sp_walk(SpState st, const int32_t* gs, const int64_t* path_off,
                                                    int64_t* path, SpCsr gout, const uint8_t* dist_b,
                                                    const int64_t* vid_of, int64_t n, int64_t lo,
                                                    unsigned long long* cnt) {
  __shared__ int64_t s_best[kWalkT / 64], s_w[kWalkT / 64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t p = blockIdx.x;
  if (p >= st.B || st.state[p] != SP_MET) return;  // uniform over the workgroup
  const int32_t L = st.res[p];
  const int64_t o = path_off[p];
  uint32_t v = uint32_t(gs[p]);
  if (threadIdx.x == 0) path[o] = vid_of[lo + v];
  const uint8_t* db = dist_b;
  for (int32_t i = 0; i < L; i++) {
    const uint8_t need = uint8_t(L - i - 1);
    int64_t best = INT64_MAX;
    int64_t bw = -1;
    if (!(gout.row_ok && !gout.row_ok[v])) {
      const int64_t e1 = gout.row_ptr[v + 1];
      for (int64_t e = gout.row_ptr[v] + threadIdx.x; e < e1; e += kWalkT) {
        const int64_t w = int64_t(gout.col[e]) - lo;
        if (dist_get(st, db, 1, uint32_t(p), uint32_t(w), n) == need) {
          const int64_t vv = vid_of[lo + w];
          if (vv < best) {
            best = vv;
            bw = w;
          }
        }
      }
    }
#pragma unroll
    for (int sft = 32; sft > 0; sft >>= 1) {
      const int64_t ob = __shfl_xor(best, sft);
      const int64_t ow = __shfl_xor(bw, sft);
      if (ow >= 0 && (bw < 0 || ob < best)) {
        best = ob;
        bw = ow;
      }
    }
    if (lane == 0) {
      s_best[wv] = best;
      s_w[wv] = bw;
    }
    __syncthreads();
    best = INT64_MAX;
    bw = -1;
    for (int k = 0; k < kWalkT / 64; k++)
      if (s_w[k] >= 0 && (bw < 0 || s_best[k] < best)) {
        best = s_best[k];
        bw = s_w[k];
      }
    __syncthreads();
    if (bw < 0) {  // in-edge keys without the mirrored out-edge: the definition does not hold
      if (threadIdx.x == 0) atomicAdd(cnt + C_WALKERR, 1ull);
      return;
    }
    v = uint32_t(bw);
    if (threadIdx.x == 0) path[o + i + 1] = best;
  }
}

// ---- edge-balanced walk: one step of every walking pair per launch --------------------------
// Step i of pair p scans the out-row of its current vertex cur[p] for the smallest vid w with
// dist_B(w) = L - i - 1.  The rows of all pairs are one flattened range cut into kTileE-entry
// tiles (the expansion's tile-row table and LDS owner map), so a hub row on a path is spread over
// many workgroups instead of one.  The last step (need = 0) is dst itself and is never scanned.
__global__ void k_sp_walk_front(SpState st, int32_t i, const int32_t* cur, SpCsr gout, int64_t* wdeg,
                                long long* best) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p > st.B) return;
  int64_t d = 0;
  if (p < st.B) {
    best[p] = LLONG_MAX;
    if (st.state[p] == SP_MET && st.res[p] - 1 > i && cur[p] >= 0) d = sp_deg(gout, uint32_t(cur[p]));
  }
  wdeg[p] = d;  // wdeg[B] = 0: the scan's total
}

// wave-aggregated atomicMin(arr[key], v) over the lanes with act
__device__ inline void wave_min_keyed(long long* arr, uint32_t key, long long v, bool act) {
  const int lane = threadIdx.x & 63;
  uint64_t m = __ballot(act);
  while (m) {
    const int leader = __ffsll((long long)m) - 1;
    const uint32_t k = uint32_t(__shfl(int(key), leader));
    const bool mine = act && key == k;
    long long x = mine ? v : LLONG_MAX;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const long long y = __shfl_xor(x, o);
      x = y < x ? y : x;
    }
    if (lane == leader && x != LLONG_MAX) atomicMin(arr + k, x);
    m &= ~__ballot(mine);
    act = act && !mine;
  }
}

__global__ __launch_bounds__(kT) void k_sp_walk_scan(SpState st, int32_t i, const int32_t* cur, const int64_t* off,
                                                     const int32_t* tile_row, SpCsr gout, const uint8_t* dist_b,
                                                     const int64_t* vid_of, int64_t n, int64_t lo, long long* best) {
  __shared__ int32_t s_off[kTileE + 1];
  __shared__ int64_t s_rs[kTileE];
  __shared__ int32_t s_pair[kTileE];
  __shared__ int64_t s_hdr[2];
  __shared__ int32_t s_scan[kT / 64];
  const int64_t nP = st.B;
  const int64_t E = off[nP];
  const int64_t ntiles = (E + kTileE - 1) / kTileE;
  for (int64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const int64_t e0 = t * kTileE;
    const int64_t e1 = min(e0 + int64_t(kTileE), E);
    if (threadIdx.x == 0) {
      int64_t i0, cn;
      tile_entries(tile_row, off, nP, t, e1, E, i0, cn);
      s_hdr[0] = i0;
      s_hdr[1] = cn;
    }
    __syncthreads();
    const int64_t i0 = s_hdr[0];
    const int cnt_k = int(s_hdr[1]);  // <= B + 1 <= kTileE (the host caps the batch for this)
    for (int k = threadIdx.x; k <= cnt_k; k += kT) {
      const int64_t o = off[i0 + k];
      s_off[k] = int32_t(min(o - e0, int64_t(kTileE + 1)));
      if (k < cnt_k) {
        const int32_t v = cur[i0 + k];
        s_pair[k] = int32_t(i0 + k);
        s_rs[k] = (v >= 0 ? gout.row_ptr[v] : 0) - o;
      }
    }
    __syncthreads();
    tile_owner_map<kTileE, kT>(s_off, cnt_k, s_scan);
    // the slots' reads in phases, each phase's loads of all kIt slots in flight (as k_sp_expand):
    // column entries and depths, backward level filter bits, distance bytes, then the vids of hits
    uint32_t ps[kIt], ws[kIt];
    int32_t need[kIt];
#pragma unroll
    for (int r = 0; r < kIt; r++) {
      const int j = threadIdx.x + r * kT;
      const int64_t e = e0 + j;
      ps[r] = 0;
      ws[r] = 0xFFFFFFFFu;
      need[r] = -1;
      if (e < e1) {
        const int k = s_off[j];
        ps[r] = uint32_t(s_pair[k]);
        ws[r] = uint32_t(int64_t(gout.col[s_rs[k] + e]) - lo);
        need[r] = st.res[ps[r]] - i - 1;
      }
    }
    bool hit[kIt];
#pragma unroll
    for (int r = 0; r < kIt; r++) hit[r] = ws[r] != 0xFFFFFFFFu && lv_maybe(st, 1, need[r], ws[r]);
#pragma unroll
    for (int r = 0; r < kIt; r++) hit[r] = hit[r] && dist_get(st, dist_b, 1, ps[r], ws[r], n) == uint32_t(need[r]);
    long long cand[kIt];
#pragma unroll
    for (int r = 0; r < kIt; r++) cand[r] = hit[r] ? vid_of[lo + ws[r]] : LLONG_MAX;
#pragma unroll
    for (int r = 0; r < kIt; r++) wave_min_keyed(best, ps[r], cand[r], hit[r]);
    __syncthreads();
  }
}

// the step's choice: path vid and the next current vertex (vid -> gidx through the vertex hash)
__global__ void k_sp_walk_pick(SpState st, int32_t i, int32_t* cur, const long long* best, const int64_t* path_off,
                               int64_t* path, const int64_t* ht_keys, const int32_t* ht_vals, uint64_t ht_mask,
                               bool ht_has_min, int32_t ht_min_gidx, int64_t lo, unsigned long long* cnt) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= st.B || st.state[p] != SP_MET || st.res[p] - 1 <= i || cur[p] < 0) return;
  const long long b = best[p];
  if (b == LLONG_MAX) {  // in-edge keys without the mirrored out-edge: the definition does not hold
    atomicAdd(cnt + C_WALKERR, 1ull);
    cur[p] = -1;
    return;
  }
  path[path_off[p] + i + 1] = int64_t(b);
  cur[p] = ht_lookup(ht_keys, ht_vals, ht_mask, int64_t(b), ht_has_min, ht_min_gidx) - int32_t(lo);
}

// reset every claimed distance byte of the batch
__global__ void k_sp_clear(const uint64_t* arena, int64_t m, uint8_t* d0, uint8_t* d1, int64_t n, SpState st) {
  for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < m; i += int64_t(gridDim.x) * blockDim.x) {
    const uint64_t t = arena[i];
    (t_side(t) ? d1 : d0)[didx(st, t_pair(t), t_row(t), n)] = 0xFF;
  }
}

int grid_n(int64_t n, int cap = 4096) {
  return int(std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, cap)));
}

// (re)size a persistent list to hold `need` tuples, keeping its first `keep` ones.  Lists
// persist across calls, so growth (a synchronising hipFree) is rare.
void reserve(Ctx& c, DevBuf& b, int64_t& cap, int64_t need, int64_t keep) {
  if (need <= cap) return;
  const int64_t nc = std::max<int64_t>(need + need / 4, 1 << 16);
  PoolScope none(nullptr);
  DevBuf nb;
  nb.alloc(size_t(nc) * 8);
  if (keep > 0) {
    NBG_HIP(hipMemcpyAsync(nb.p, b.p, size_t(keep) * 8, hipMemcpyDeviceToDevice, c.stream));
    NBG_HIP(hipStreamSynchronize(c.stream));
  }
  b = std::move(nb);
  cap = nc;
}

// ==== device-driven batches (option sp_dev, default 1) ===========================================
// A batch as one fixed chain of launches.  Every kernel reads its list lengths and chunk counts
// from device counters, the producers fill the chunk tables through block-reserved ranges (no
// scans, no host-sized grids), and the last block of each BFS step publishes that iteration's
// counters to coherent host memory (no publish launch).  The host enqueues iteration i + 1 before
// it reads iteration i's counters, so the device never idles on a round trip inside the BFS; the
// sweep and the walk are enqueued in one go once the longest path is known.  Launches per batch:
// begin, 4 per BFS iteration (select, meet probe, expansion + the probe's meets, step), a post
// pass, 2 per sweep step, 2 per walk step, the result pass and the finish publish.  A list that
// overflows its fixed capacity makes the host restore the clean state and re-run the batch on the
// host-driven path (which grows its lists and regenerates lost appends).
//
// Level filters: a test "dist[side][p][v] == l" (meet probe, sweep, walk) first asks
//  * the pair's own filter of (side, l): 4096 bits per (side, level, pair), set at every claim; a
//    scanning wave holds its chunk's pair row in registers (8 bytes a lane) and tests an entry with
//    two cross-lane reads (ds_bpermute): no memory access;
//  * then a blocked Bloom filter over (side, level, pair, vertex) keys, 3 bits in one 32-bit word
//    (option sp_gf_log2, default 2^24 bits = 2 MiB, L2-resident);
// and only an entry that passes both reads the pair's distance byte (a random line of the 2 * B * n
// byte arrays).  The host-driven path's batch-wide level bitmaps (the union over all pairs) pass
// most entries of the large steps, and each passed entry fetched a whole line for one byte (PMC:
// sweep 5.1x, probe 6.7x their byte models).  Depth 0 is tested exactly (the pair's src / dst).
enum : int { D_ARENA = 0, D_MEET = 1, D_OVF = 2, D_WALKERR = 3, D_MAXL = 4, D_MAXF = 5, D_TICKET = 6, D_CLEAR = 7,
             D_G = 16 };
enum : int { Q_LIVE0 = 0, Q_LIVE1 = 1, Q_X = 2, Q_NCH = 3, Q_XE = 4, Q_PE = 5, Q_ACTIVE = 6, Q_CLAIMS = 7, Q_EE = 8,
             Q_W = 16 };
constexpr int kMaxQ = 32;                 // BFS iterations, sweep steps, walk steps (each)
constexpr int kSwQ = kMaxQ, kWkQ = 2 * kMaxQ, kNQ = 3 * kMaxQ;
constexpr int kDevCnt = D_G + kNQ * Q_W;  // counter words
constexpr int kCh = 1024;                 // adjacency entries per chunk (one wave)
constexpr int kPubW = 64;                 // words per host publish slot (the sequence word last)
constexpr int kDvStage = 256;             // claims staged per wave and list
constexpr int kPairLds = 4096;            // pairs per batch whose per-pair tables the selects keep in LDS
// every counter on a 128-byte line of its own (logical counter i at word i * kCS): blocks of a grid
// ending together add to a line's words one atomic at a time at the memory side (~12 ns each), so
// counters that shared a line had serialised each other's adds (round 5: 16 counters per line)
constexpr int kCS = 16;
__host__ __device__ inline unsigned long long* gcnt(unsigned long long* cnt, int i) { return cnt + size_t(i) * kCS; }
__host__ __device__ inline const unsigned long long* gcnt(const unsigned long long* cnt, int i) {
  return cnt + size_t(i) * kCS;
}
struct QBlk {  // counter block q: q[k] / q + k address its counter k
  unsigned long long* p;
  __device__ unsigned long long& operator[](int k) const { return p[size_t(k) * kCS]; }
  __device__ unsigned long long* operator+(int k) const { return p + size_t(k) * kCS; }
};
__device__ inline QBlk qblk(unsigned long long* cnt, int q) { return QBlk{gcnt(cnt, D_G + q * Q_W)}; }

struct SpFilt {
  uint32_t* pf;     // [2 * kLv][B][128] pair filters (null: off)
  uint32_t* gf;     // blocked Bloom filter words (null: off)
  uint32_t gshift;  // 64 - log2(gf words)
  int32_t B;
  int32_t diag;     // option sp_dv_diag (diagnostics): sweep bit 0 no tests, bit 1 filter tests
                    // without the byte reads (timing only, wrong results); bit 2 a walk error
                    // returns the partial result instead of failing the call
};
__device__ inline uint32_t pf_bit(uint32_t v) { return (v * 0x9E3779B1u) >> 20; }
__device__ inline uint64_t gf_hash(uint32_t sl, uint32_t p, uint32_t v) {
  uint64_t h = (uint64_t(v) * 0xD6E8FEB86659FD93ull) ^ (uint64_t(p) * 0xA0761D6478BD642Full) ^
               (uint64_t(sl + 1) * 0xE7037ED1A0B428DBull);
  h ^= h >> 31;
  return h * 0x9E3779B97F4A7C15ull;
}
__device__ inline uint32_t gf_mask(uint64_t h) {
  return (1u << (h & 31u)) | (1u << ((h >> 5) & 31u)) | (1u << ((h >> 10) & 31u));
}
__device__ inline void filt_mark(const SpFilt& f, uint32_t side, uint32_t l, uint32_t p, uint32_t v) {
  if (l < 1 || l >= uint32_t(kLv)) return;
  const uint32_t sl = side * kLv + l;
  if (f.pf) {
    uint32_t* row = f.pf + (size_t(sl) * uint32_t(f.B) + p) * 128;
    const uint32_t b = pf_bit(v);
    atomicOr(row + (b >> 5), 1u << (b & 31u));
  }
  if (f.gf) {
    const uint64_t h = gf_hash(sl, p, v);
    atomicOr(f.gf + (h >> f.gshift), gf_mask(h));
  }
}
// the global filter's mark alone (k_dv_expand gathers a chunk's pair-filter bits in LDS instead)
__device__ inline void gf_mark(const SpFilt& f, uint32_t side, uint32_t l, uint32_t p, uint32_t v) {
  if (!f.gf || l < 1 || l >= uint32_t(kLv)) return;
  const uint64_t h = gf_hash(side * kLv + l, p, v);
  atomicOr(f.gf + (h >> f.gshift), gf_mask(h));
}
// the chunk's pair row of the pair filter (side, l) in registers: lane i holds words 2i, 2i + 1
__device__ inline uint2 pf_load(const SpFilt& f, uint32_t side, int32_t l, uint32_t p, bool& on) {
  on = f.pf && l >= 1 && l < kLv;
  if (!on) return make_uint2(~0u, ~0u);
  const uint2* r = reinterpret_cast<const uint2*>(f.pf + (size_t(side * kLv + uint32_t(l)) * uint32_t(f.B) + p) * 128);
  return r[threadIdx.x & 63];
}
// bit b of the row: wave-uniform call (cross-lane reads of every lane's row words)
__device__ inline bool pf_bit_set(uint2 row, uint32_t b) {
  const uint32_t wd = b >> 5;
  const int src = int((wd >> 1) << 2);
  const uint32_t lo = uint32_t(__builtin_amdgcn_ds_bpermute(src, int(row.x)));
  const uint32_t hi = uint32_t(__builtin_amdgcn_ds_bpermute(src, int(row.y)));
  return ((((wd & 1u) ? hi : lo) >> (b & 31u)) & 1u) != 0u;
}
__device__ inline bool pf_test(uint2 row, uint32_t v) { return pf_bit_set(row, pf_bit(v)); }  // wave-uniform call
__device__ inline bool gf_test(const SpFilt& f, uint32_t side, int32_t l, uint32_t p, uint32_t v) {
  if (!f.gf || l < 1 || l >= kLv) return true;
  const uint64_t h = gf_hash(side * kLv + uint32_t(l), p, v);
  const uint32_t m = gf_mask(h);
  return (f.gf[h >> f.gshift] & m) == m;
}

// the overflow flag as the block sees it at its start (block-uniform: the kernels below end with
// block-wide reductions, and this launch may raise the flag while its blocks run)
__device__ inline bool dv_ovf_block(const unsigned long long* cnt) {
  __shared__ int s_ovf;
  if (threadIdx.x == 0) s_ovf = __hip_atomic_load(gcnt(cnt, D_OVF), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
  __syncthreads();
  return s_ovf != 0;
}

struct SpDev {
  unsigned long long* cnt;   // kDevCnt counters
  uint64_t* live[2][2];      // [iteration parity][side]
  int64_t cap_live;
  uint64_t* arena;
  int64_t cap_arena;
  uint64_t* meet;
  int64_t cap_meet;
  uint64_t* sw[2];           // sweep lists by step parity
  int64_t cap_sw;
  uint64_t* X;
  int64_t* Xcb;              // first chunk of each X entry
  int64_t cap_x;
  int32_t* chx;              // chunk -> X entry
  uint64_t* slot;            // meet probe: chunk -> the claim it made (~0: none)
  int64_t cap_ch;
  int32_t* wchx;             // walk: chunk -> pair
  int64_t cap_wch;
  int64_t* wcb;              // walk: first chunk of each pair
  int32_t* gs;               // [2B] src gidx, dst gidx
  int32_t* cur;              // walk: current vertex of each pair
  long long* best;           // walk: smallest candidate vid of each pair
  unsigned long long* pull;  // [kMaxQ][B] sweep step j's pull entries (in-degree + 1 sums)
  unsigned long long* push;  // [kMaxQ][B] forward level k's out-degree + 1 sums
  int64_t* doff;             // [B + 1] path offsets
  int32_t lg_chb, lg_chs;    // log2 entries per chunk: BFS iterations (probe / expansion), sweep steps
  int64_t* path;
  const int64_t* h_pairs;    // coherent host: [B] src vids, [B] dst vids
  int32_t* h_sr;             // coherent host: [B] state, [B] res
  int64_t* h_off;            // coherent host: [B + 1]
  int64_t* h_path;           // coherent host
};

__device__ inline void dput(uint64_t* list, int64_t cap, unsigned long long* ctr, unsigned long long* cnt, bool pred,
                            uint64_t v) {
  const int64_t s = wave_append(ctr, pred);
  if (pred) {
    if (s < cap) list[s] = v;
    else atomicOr(gcnt(cnt, D_OVF), 1ull);
  }
}

// block-wide reservation in K counters (kBlk threads, block-uniform call): thread asks n[k] slots
// of counter k, gets its first slot o[k]; one returning atomic per counter and block
template <int K>
__device__ inline void blk_reserve_n(unsigned long long* const* ctr, const uint32_t* n, unsigned long long* o) {
  __shared__ uint32_t s_w[K][kBlk / 64];
  __shared__ unsigned long long s_base[K];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t v[K];
#pragma unroll
  for (int k = 0; k < K; k++) {
    v[k] = n[k];
#pragma unroll
    for (int of = 1; of < 64; of <<= 1) {
      const uint32_t y = __shfl_up(v[k], of);
      if (lane >= of) v[k] += y;
    }
    if (lane == 63) s_w[k][w] = v[k];
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < K; k++) {
    uint32_t pre = v[k] - n[k], tot = 0;
#pragma unroll
    for (int i = 0; i < kBlk / 64; i++) {
      if (i < w) pre += s_w[k][i];
      tot += s_w[k][i];
    }
    v[k] = pre;
    if (threadIdx.x == 0) s_base[k] = tot ? atomicAdd(ctr[k], (unsigned long long)tot) : 0ull;
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < K; k++) o[k] = s_base[k] + v[k];
  __syncthreads();
}

// one add per block of a per-thread value (kBlk threads, block-uniform call)
__device__ inline void blk_add(unsigned long long* ctr, unsigned long long v) {
  __shared__ unsigned long long s_a[kBlk / 64];
  v = wsum(v);
  if ((threadIdx.x & 63) == 0) s_a[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long t = 0;
#pragma unroll
    for (int i = 0; i < kBlk / 64; i++) t += s_a[i];
    if (t) atomicAdd(ctr, t);
  }
  __syncthreads();
}

// items [c0, c0 + nc) of every lane get fill(item, val): short ranges by their lane, long ones
// (a hub row's thousands of chunks) by the whole wave.  Wave-uniform call.
template <typename Fill>
__device__ inline void wave_fill_val(int64_t c0, int64_t nc, int64_t val, Fill fill) {
  const int lane = threadIdx.x & 63;
  if (nc <= 4) {
    for (int64_t k = 0; k < nc; k++) fill(c0 + k, val);
    nc = 0;
  }
  uint64_t m = __ballot(nc > 0);
  while (m) {
    const int j = __ffsll((long long)m) - 1;
    m &= m - 1;
    const int64_t a = __shfl(c0, j), z = a + __shfl(nc, j), v = __shfl(val, j);
    for (int64_t c = a + lane; c < z; c += 64) fill(c, v);
  }
}

// Publication by the last block of a kernel: every block takes a ticket after its work; the
// last one copies the global counters and counter block q to the host slot (one wave: lane 0's
// system-scope release covers the wave's stores) and then the sequence word the host spins on.
__device__ inline void dv_publish_last(unsigned long long* cnt, int q, unsigned long long* hslot, uint64_t seq) {
  __shared__ int s_last;
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence();
    s_last = atomicAdd(gcnt(cnt, D_TICKET), 1ull) == (unsigned long long)(gridDim.x - 1);
  }
  __syncthreads();
  if (!s_last || threadIdx.x >= 64) return;
  __threadfence();
  const int i = threadIdx.x;
  if (i < D_G + Q_W) {
    const unsigned long long* src = i < D_G ? gcnt(cnt, i) : qblk(cnt, q) + (i - D_G);
    hslot[i] = __hip_atomic_load(src, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (i == 0) __hip_atomic_store(gcnt(cnt, D_TICKET), 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __builtin_amdgcn_wave_barrier();
  if (i == 0) __hip_atomic_store(hslot + kPubW - 1, (unsigned long long)seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// batch start: pairs from host memory, vid -> gidx, both frontiers seeded, the first side choice
// (trivial pairs finish here); the sweep cost sums cleared
__global__ __launch_bounds__(256) void k_dv_begin(SpDev d, SpState st, SpCsr gout, SpCsr gin, uint8_t* d0, uint8_t* d1,
                                                  int64_t n, int32_t max_steps, const int64_t* ht_keys,
                                                  const int32_t* ht_vals, uint64_t ht_mask, bool ht_has_min,
                                                  int32_t ht_min_gidx, int32_t sel1) {
  const int32_t B = st.B;
  const int64_t gt = int64_t(blockIdx.x) * blockDim.x + threadIdx.x, gn = int64_t(gridDim.x) * blockDim.x;
  int32_t s1 = 0;   // the side pair gt expands in iteration 1
  int64_t dg1 = 0;  // its root's degree there
  // pull and push adjacent, 64-byte aligned, 2 kMaxQ B words: 16-byte stores
  for (int64_t i = gt; i < int64_t(kMaxQ) * B; i += gn) reinterpret_cast<uint4*>(d.pull)[i] = make_uint4(0u, 0u, 0u, 0u);
  bool go = false;
  int32_t a = -1, b = -1;
  if (gt < B) {
    const int p = int(gt);
    const int64_t sv = d.h_pairs[p], tv = d.h_pairs[B + p];
    a = ht_lookup(ht_keys, ht_vals, ht_mask, sv, ht_has_min, ht_min_gidx);
    b = ht_lookup(ht_keys, ht_vals, ht_mask, tv, ht_has_min, ht_min_gidx);
    d.gs[p] = a;
    d.gs[B + p] = b;
    st.res[p] = sv == tv ? 0 : -1;
    st.lvl[p] = st.lvl[B + p] = 0;
    st.met[p] = 0;
    st.pside[p] = 0;
    st.side[p] = 0;
    st.deg[p] = st.deg[B + p] = 0;
    go = sv != tv && a >= 0 && b >= 0 && max_steps >= 1;
    if (go) {
      // the batch's bytes are all unseen here and no other thread writes these two: plain stores
      d0[didx(st, uint32_t(p), uint32_t(a), n)] = 0;
      d1[didx(st, uint32_t(p), uint32_t(b), n)] = 0;
      const unsigned long long df = (unsigned long long)sp_deg(gout, uint32_t(a)) + 1;
      const unsigned long long db = (unsigned long long)sp_deg(gin, uint32_t(b)) + 1;
      const int s = df <= db ? 0 : 1;
      s1 = s;
      dg1 = int64_t(s == 0 ? df : db) - 1;
      st.side[p] = s;
      st.deg[p] = s == 0 ? 0ull : df;  // the expanding side's sum restarts (the expansion adds)
      st.deg[B + p] = s == 1 ? 0ull : db;
    }
    st.state[p] = go ? SP_ACTIVE : SP_DONE;
  }
  // the batch's first writer of the lists and the arena (their counters start at 0): pair k of
  // the active ones takes slot k of both live lists and arena slots 2k, 2k + 1, so one returning
  // atomic (the active count) places all four tuples
  const uint32_t pp = uint32_t(gt);
  const QBlk q0 = qblk(d.cnt, 0);
  const int64_t k = wave_append(q0 + Q_ACTIVE, go);
  if (go) {
    if (k < d.cap_live) {
      d.live[0][0][k] = mk_tup(0, pp, 0, uint32_t(a));
      d.live[0][1][k] = mk_tup(1, pp, 0, uint32_t(b));
    }
    if (2 * k + 1 < d.cap_arena) {
      d.arena[2 * k] = mk_tup(0, pp, 0, uint32_t(a));
      d.arena[2 * k + 1] = mk_tup(1, pp, 0, uint32_t(b));
    }
    if (k >= d.cap_live || 2 * k + 1 >= d.cap_arena) atomicOr(gcnt(d.cnt, D_OVF), 1ull);
  }
  const uint64_t m = __ballot(go);
  if ((threadIdx.x & 63) == 0 && m) {
    const unsigned long long nw = (unsigned long long)__popcll(m);
    atomicAdd(q0 + Q_LIVE0, nw);
    atomicAdd(q0 + Q_LIVE1, nw);
    atomicAdd(gcnt(d.cnt, D_ARENA), 2 * nw);
  }
  if (!sel1) return;  // (grid-uniform) k_dv_select builds iteration 1's tables
  // iteration 1's tables, which k_dv_select would build from the lists above: the expanding root
  // of active pair k is X entry k with its chunk range, the other root is carried into iteration
  // 1's list of its side (one launch and its dependent chain less per batch)
  const QBlk q1 = qblk(d.cnt, 1);
  const int lane = threadIdx.x & 63;
  const int64_t nc = go ? (dg1 + (int64_t(1) << d.lg_chb) - 1) >> d.lg_chb : 0;
  int64_t inc = nc;  // inclusive wave scan of the chunk counts
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int64_t y = __shfl_up(inc, o);
    if (lane >= o) inc += y;
  }
  const int64_t wtot = __shfl(inc, 63);
  unsigned long long cb = 0;
  if (lane == 0 && wtot) cb = atomicAdd(q1 + Q_NCH, (unsigned long long)wtot);
  const int64_t ca = int64_t(__shfl(cb, 0)) + inc - nc;
  const bool fit = go && k < d.cap_x && ca + nc <= d.cap_ch;
  if (go) {
    if (fit) {
      d.X[k] = mk_tup(uint32_t(s1), pp, 0, uint32_t(s1 ? b : a));
      d.Xcb[k] = ca;
    } else {
      atomicOr(gcnt(d.cnt, D_OVF), 2ull);
    }
  }
  wave_fill_val(ca, fit ? nc : 0, k, [&](int64_t c, int64_t v) {
    d.chx[c] = int32_t(v);
    d.slot[c] = ~0ull;
  });
  const int64_t c0 = wave_append(q1 + Q_LIVE0, go && s1 == 1);  // side 0's root carried
  const int64_t c1 = wave_append(q1 + Q_LIVE1, go && s1 == 0);  // side 1's root carried
  if (go && s1 == 1) {
    if (c0 < d.cap_live) d.live[1][0][c0] = mk_tup(0, pp, 0, uint32_t(a));
    else atomicOr(gcnt(d.cnt, D_OVF), 2ull);
  }
  if (go && s1 == 0) {
    if (c1 < d.cap_live) d.live[1][1][c1] = mk_tup(1, pp, 0, uint32_t(b));
    else atomicOr(gcnt(d.cnt, D_OVF), 2ull);
  }
  unsigned long long esum = go ? (unsigned long long)dg1 : 0ull;
  esum = wsum(esum);
  if (lane == 0 && m) {
    atomicAdd(q1 + Q_X, (unsigned long long)__popcll(m));
    if (esum) atomicAdd(q1 + Q_XE, esum);
  }
}

// BFS iteration it, first launch: the live lists of iteration it - 1 -> X (tuples of the side
// their pair expands, with their chunk ranges in the chunk table) + the tuples carried into
// iteration it's lists.  kSelIt tuples per thread, one reservation per block and round.
__global__ __launch_bounds__(kBlk) void k_dv_select(SpDev d, SpState st, SpCsr gout, SpCsr gin, int32_t it) {
  const QBlk qp = qblk(d.cnt, it - 1);
  const QBlk q = qblk(d.cnt, it);
  if (qp[Q_ACTIVE] == 0) return;  // the BFS ended (a speculative iteration): nothing selected
  const int64_t n0 = min(int64_t(qp[Q_LIVE0]), d.cap_live), n1 = min(int64_t(qp[Q_LIVE1]), d.cap_live);
  const int64_t nl = n0 + n1;
  const uint64_t* in0 = d.live[(it - 1) & 1][0];
  const uint64_t* in1 = d.live[(it - 1) & 1][1];
  uint64_t* out0 = d.live[it & 1][0];
  uint64_t* out1 = d.live[it & 1][1];
  constexpr int64_t per = int64_t(kBlk) * kSelIt;
  const int64_t rounds = (nl + per - 1) / per;
  unsigned long long esum = 0;
  unsigned long long* ctr[4] = {q + Q_X, q + Q_LIVE0, q + Q_LIVE1, q + Q_NCH};
  // per pair, the side it expands (1 + side; 0: not active), in LDS: a tuple's lookup is then no
  // global load behind its own (one round trip less in the chain tuple -> pair -> degree)
  __shared__ uint8_t s_ps[kPairLds];
  if (int64_t(blockIdx.x) < rounds) {
    for (int p = threadIdx.x; p < st.B; p += blockDim.x)
      s_ps[p] = st.state[p] == SP_ACTIVE ? uint8_t(1 + st.side[p]) : uint8_t(0);
  }
  __syncthreads();
  for (int64_t r = blockIdx.x; r < rounds; r += gridDim.x) {
    const int64_t i0 = r * per + threadIdx.x;
    uint64_t t[kSelIt];
#pragma unroll
    for (int u = 0; u < kSelIt; u++) {
      const int64_t i = i0 + u * kBlk;
      t[u] = i < n0 ? in0[i] : i < nl ? in1[i - n0] : ~0ull;
    }
    uint32_t xm = 0, cm0 = 0, cm1 = 0;
#pragma unroll
    for (int u = 0; u < kSelIt; u++) {
      if (t[u] == ~0ull) continue;
      const uint32_t ps = s_ps[t_pair(t[u])];
      if (ps == 0) continue;
      const uint32_t ts = t_side(t[u]);
      if (ps - 1 == ts) xm |= 1u << u;
      else if (ts) cm1 |= 1u << u;
      else cm0 |= 1u << u;
    }
    // the degrees of the tuples that expand (a carried tuple's row is not read)
    int64_t dg[kSelIt];
#pragma unroll
    for (int u = 0; u < kSelIt; u++) dg[u] = (xm >> u) & 1u ? sp_deg(t_side(t[u]) ? gin : gout, t_row(t[u])) : 0;
    uint32_t nch = 0;
#pragma unroll
    for (int u = 0; u < kSelIt; u++) {
      if (dg[u] == 0) xm &= ~(1u << u);  // nothing to scan
      nch += uint32_t((dg[u] + (int64_t(1) << d.lg_chb) - 1) >> d.lg_chb);
      esum += (unsigned long long)dg[u];
    }
    const uint32_t nn[4] = {uint32_t(__popc(xm)), uint32_t(__popc(cm0)), uint32_t(__popc(cm1)), nch};
    unsigned long long o[4];
    blk_reserve_n<4>(ctr, nn, o);
    bool ovf = false;
#pragma unroll
    for (int u = 0; u < kSelIt; u++) {
      const bool x = (xm >> u) & 1u;
      const int64_t nc = x ? (dg[u] + (int64_t(1) << d.lg_chb) - 1) >> d.lg_chb : 0;
      const int64_t xa = int64_t(o[0]), ca = int64_t(o[3]);
      if (x) {
        if (xa < d.cap_x && ca + nc <= d.cap_ch) {
          d.X[xa] = t[u];
          d.Xcb[xa] = ca;
        } else {
          ovf = true;
        }
        o[0]++;
        o[3] += uint64_t(nc);
      }
      const bool fill = x && xa < d.cap_x && ca + nc <= d.cap_ch;
      wave_fill_val(ca, fill ? nc : 0, xa, [&](int64_t c, int64_t v) {
        d.chx[c] = int32_t(v);
        d.slot[c] = ~0ull;
      });
      if ((cm0 >> u) & 1u) {
        if (int64_t(o[1]) < d.cap_live) out0[o[1]] = t[u];
        else ovf = true;
        o[1]++;
      } else if ((cm1 >> u) & 1u) {
        if (int64_t(o[2]) < d.cap_live) out1[o[2]] = t[u];
        else ovf = true;
        o[2]++;
      }
    }
    if (ovf) atomicOr(gcnt(d.cnt, D_OVF), 2ull);
  }
  blk_add(q + Q_XE, esum);
}

// Chunk groups.  A wave takes G virtual chunks, nwaves apart (the grid-stride order: at any time
// neighbouring waves scan neighbouring chunks, often of one row), and its first G lanes load their
// descriptors together (chunk table -> tuple -> row bounds: a chain of dependent loads paid once
// per group, not once per chunk); the wave then scans the live ones one by one with the
// descriptor read from its lane into scalar registers.  G (a power of two <= 64) is the share of
// chunks per wave of the grid, so small steps still spread over every wave.
struct ChunkRec {
  uint64_t t;
  int64_t x0, x1;
  int32_t a0, a1;
};
__device__ inline int64_t rl64(int64_t v, int j) {
  const uint32_t lo = uint32_t(__builtin_amdgcn_readlane(int(uint32_t(uint64_t(v))), j));
  const uint32_t hi = uint32_t(__builtin_amdgcn_readlane(int(uint32_t(uint64_t(v) >> 32)), j));
  return int64_t((uint64_t(hi) << 32) | lo);
}
template <typename Desc, typename Body>
__device__ inline void chunk_groups(int64_t vtotal, Desc desc, Body body) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = (int64_t(blockIdx.x) * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = (int64_t(gridDim.x) * blockDim.x) >> 6;
  int lg = 0;
  while (lg < 6 && (nwaves << (lg + 1)) <= vtotal) lg++;
  for (int64_t base = wave; base < vtotal; base += nwaves << lg) {
    ChunkRec r{0, 0, 0, 0, 0};
    bool live = false;
    const int64_t mine = base + int64_t(lane) * nwaves;
    if (lane < (1 << lg) && mine < vtotal) live = desc(mine, r);
    uint64_t m = __ballot(live);
    while (m) {
      const int j = __ffsll((long long)m) - 1;
      m &= m - 1;
      ChunkRec u;
      u.t = uint64_t(rl64(int64_t(r.t), j));
      u.x0 = rl64(r.x0, j);
      u.x1 = rl64(r.x1, j);
      u.a0 = __builtin_amdgcn_readlane(r.a0, j);
      u.a1 = __builtin_amdgcn_readlane(r.a1, j);
      body(u, base + int64_t(j) * nwaves);
    }
  }
}
// one step's column entries: 64 * U from the 16-byte aligned x (lane L holds entries x + 4L .. +3
// of each 256-entry block: one 16-byte load per lane and block instead of four 4-byte ones);
// entries outside the slice [x0, x1) read as ~0.  A load stays inside the column array: it starts
// below x1, and the arrays are padded past their last entry.
template <int U = kProbeU>
__device__ inline void col_step(const int32_t* col, int64_t x, int64_t x0, int64_t x1, int64_t lo, uint32_t* w) {
  static_assert(U % 4 == 0, "whole 16-byte groups");
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int j = 0; j < U / 4; j++) {
    const int64_t e0 = x + j * 256 + 4 * lane;
    int4 v = make_int4(-1, -1, -1, -1);
    if (e0 < x1) v = *reinterpret_cast<const int4*>(col + e0);
    const int32_t vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int k = 0; k < 4; k++)
      w[4 * j + k] = e0 + k >= x0 && e0 + k < x1 ? uint32_t(int64_t(vv[k]) - lo) : 0xFFFFFFFFu;
  }
}
__device__ inline int64_t step_start(int64_t x0) { return x0 & ~int64_t(3); }

// the X chunk c's row slice [x0, x1) (2^lg_ch entries; sub-chunk s of 2^lg_sub) for its X entry a
// holding tuple t
__device__ inline bool x_chunk_at(const SpDev& d, const SpCsr& g0, const SpCsr& g1, int64_t c, int32_t a, uint64_t t,
                                  int32_t lg_ch, int32_t lg_sub, int64_t s, ChunkRec& r) {
  r.t = t;
  const SpCsr& g = t_side(r.t) ? g1 : g0;
  const uint32_t row = t_row(r.t);
  const int64_t re = g.row_ptr[row + 1];
  r.x0 = g.row_ptr[row] + ((c - d.Xcb[a]) << lg_ch) + (s << (lg_ch - lg_sub));
  r.x1 = min(r.x0 + (int64_t(1) << (lg_ch - lg_sub)), re);
  return r.x0 < r.x1;
}
__device__ inline bool x_chunk(const SpDev& d, const SpCsr& g0, const SpCsr& g1, int64_t c, int32_t lg_ch, int32_t lg_sub,
                               int64_t s, ChunkRec& r) {
  const int32_t a = d.chx[c];
  return x_chunk_at(d, g0, g1, c, a, d.X[a], lg_ch, lg_sub, s, r);
}

// BFS iteration it, meet probe: one wave per chunk of an X tuple's row, stopping at the first
// neighbour at the other side's depth (or once another chunk claimed the vertex); the winner
// claims the vertex on the other side, marks the pair (met = -1) and records the claim in its
// chunk's slot
template <int U>  // column entries per lane and step (4, 8, 16: a whole chunk in one step)
__global__ __launch_bounds__(256) void k_dv_probe(SpDev d, SpState st, SpFilt f, SpCsr g0, SpCsr g1,
                                                       uint8_t* d0, uint8_t* d1, int64_t n, int64_t lo, int32_t it) {
  if (dv_ovf_block(d.cnt)) return;  // a producer overflowed: its tables are incomplete (the host re-runs)
  const int lane = threadIdx.x & 63;
  const QBlk q = qblk(d.cnt, it);
  const int64_t total = min(int64_t(q[Q_NCH]), d.cap_ch);
  if (total == 0) return;  // nothing selected (grid-uniform)
  const uint32_t B = uint32_t(st.B);
  unsigned long long examined = 0;
  // option sp_dv_diag bit 3 (diagnostics): entries passing the pair filter, distance bytes read
  // (entries passing both filters), bytes at the wanted depth -- counters Q_W-3 .. Q_W-1
  const bool stats = (f.diag & 8) != 0;
  unsigned long long n_pf = 0, n_rd = 0, n_hit = 0;
  chunk_groups(
      total,
      [&](int64_t c, ChunkRec& r) {
        if (!x_chunk(d, g0, g1, c, d.lg_chb, 0, 0, r)) return false;
        const uint32_t o = t_side(r.t) ^ 1u, p = t_pair(r.t);
        r.a0 = st.lvl[o * B + p];  // the other side's depth
        r.a1 = d.gs[o * B + p];    // its root (depth 0)
        return true;
      },
      [&](const ChunkRec& r, int64_t c) {
        const uint32_t side = t_side(r.t), p = t_pair(r.t), row = t_row(r.t), o = side ^ 1u;
        const int32_t* col = side ? g1.col : g0.col;
        const int32_t need = r.a0;
        const uint32_t sh = uint32_t(st.ilv);
        uint8_t* const odp = (o ? d1 : d0) + ((uint64_t(p) * uint64_t(n)) << sh);  // the pair's bytes (pair-major)
        bool pf_on;
        const uint2 prow = pf_load(f, o, need, p, pf_on);
        // the next step's columns are loaded before this step's tests wait on their filter and
        // byte loads (one round trip less per step of the chain)
        uint32_t wn[U];
        col_step<U>(col, step_start(r.x0), r.x0, r.x1, lo, wn);
        for (int64_t x = step_start(r.x0); x < r.x1; x += 64 * U) {
          if (uint32_t(*reinterpret_cast<volatile const uint8_t*>(odp + (uint64_t(row) << sh))) != 0xFFu)
            break;  // another chunk claimed r
          uint32_t w[U];
#pragma unroll
          for (int u = 0; u < U; u++) w[u] = wn[u];
          if (x + 64 * U < r.x1) col_step<U>(col, x + 64 * U, r.x0, r.x1, lo, wn);
          bool hit = false;
          if (need == 0) {
#pragma unroll
            for (int u = 0; u < U; u++) hit = hit || w[u] == uint32_t(r.a1);
          } else {
            uint32_t fm = 0;
#pragma unroll
            for (int u = 0; u < U; u++) {
              const bool pv = pf_on ? pf_test(prow, w[u]) : true;
              if (stats) n_pf += (w[u] != 0xFFFFFFFFu && pv) ? 1u : 0u;
              fm |= (w[u] != 0xFFFFFFFFu && pv && gf_test(f, o, need, p, w[u])) ? 1u << u : 0u;
            }
#pragma unroll
            for (int u = 0; u < U; u++) {
              const bool h = ((fm >> u) & 1u) && uint32_t(odp[uint64_t(w[u]) << sh]) == uint32_t(need);
              if (stats) n_rd += (fm >> u) & 1u, n_hit += h ? 1u : 0u;
              hit = h || hit;
            }
          }
          examined += uint64_t(min(x + 64 * U, r.x1) - max(x, r.x0)) * (lane == 0);
          if (__ballot(hit)) {
            if (lane == 0 && claim_byte(odp, uint64_t(row) << sh, uint32_t(need + 1))) {
              filt_mark(f, o, uint32_t(need + 1), p, row);
              st.met[p] = -1;
              d.slot[c] = mk_tup(o, p, uint32_t(need + 1), row);
            }
            break;
          }
        }
      });
  blk_add(q + Q_PE, examined);
  if (stats) {
    blk_add(q + (Q_W - 3), n_pf);
    blk_add(q + (Q_W - 2), n_rd);
    blk_add(q + (Q_W - 1), n_hit);
  }
}

// stage a wave-uniform batch of claims (lanes with `claimed`) into the wave's LDS buffer, flushing
// it to the arena and `list` when full (two counter atomics per flush)
struct DvStage {
  uint64_t* buf;
  uint32_t n;  // wave-uniform
};
__device__ inline void dv_flush(DvStage& s, unsigned long long* cnt, unsigned long long* lctr, uint64_t* list,
                                int64_t cap_list, uint64_t* arena, int64_t cap_arena) {
  if (s.n == 0) return;
  const int lane = threadIdx.x & 63;
  __builtin_amdgcn_wave_barrier();
  unsigned long long ba = 0, bl = 0;
  if (lane == 0) {
    ba = atomicAdd(gcnt(cnt, D_ARENA), (unsigned long long)s.n);
    bl = atomicAdd(lctr, (unsigned long long)s.n);
  }
  ba = __shfl(ba, 0);
  bl = __shfl(bl, 0);
  bool ovf = false;
  for (uint32_t k = uint32_t(lane); k < s.n; k += 64) {
    const uint64_t v = s.buf[k];
    if (int64_t(ba + k) < cap_arena) arena[ba + k] = v;
    else ovf = true;
    if (int64_t(bl + k) < cap_list) list[bl + k] = v;
    else ovf = true;
  }
  if (ovf) atomicOr(gcnt(cnt, D_OVF), 1ull);
  __builtin_amdgcn_wave_barrier();
  s.n = 0;
}
__device__ inline void dv_stage(DvStage& s, bool claimed, uint64_t v, unsigned long long* cnt,
                                unsigned long long* lctr, uint64_t* list, int64_t cap_list, uint64_t* arena,
                                int64_t cap_arena) {
  const uint64_t m = __ballot(claimed);
  if (m == 0) return;
  const uint32_t k = uint32_t(__popcll(m));
  if (s.n + k > uint32_t(kDvStage)) dv_flush(s, cnt, lctr, list, cap_list, arena, cap_arena);
  const int lane = threadIdx.x & 63;
  if (claimed) s.buf[s.n + uint32_t(__popcll(m & ((1ull << lane) - 1ull)))] = v;
  s.n += k;
}
// the block's final stages (one per wave) appended with one pair of counter atomics for the block
// (the grid's waves end together: one atomic each queued at the kernel's tail).  Block-uniform.
__device__ inline void dv_flush_block(DvStage& s, unsigned long long* cnt, unsigned long long* lctr, uint64_t* list,
                                      int64_t cap_list, uint64_t* arena, int64_t cap_arena) {
  __shared__ uint32_t s_ns[4];
  __shared__ unsigned long long s_b[2];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) s_ns[wid] = s.n;
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned long long tot = s_ns[0] + s_ns[1] + s_ns[2] + s_ns[3];
    s_b[0] = tot ? atomicAdd(gcnt(cnt, D_ARENA), tot) : 0ull;
    s_b[1] = tot ? atomicAdd(lctr, tot) : 0ull;
  }
  __syncthreads();
  uint32_t pre = 0;
  for (int k = 0; k < wid; k++) pre += s_ns[k];
  const unsigned long long ba = s_b[0] + pre, bl = s_b[1] + pre;
  bool ovf = false;
  for (uint32_t k = uint32_t(lane); k < s.n; k += 64) {
    const uint64_t v = s.buf[k];
    if (int64_t(ba + k) < cap_arena) arena[ba + k] = v;
    else ovf = true;
    if (int64_t(bl + k) < cap_list) list[bl + k] = v;
    else ovf = true;
  }
  if (ovf) atomicOr(gcnt(cnt, D_OVF), 1ull);
  s.n = 0;
  __syncthreads();
}

// BFS iteration it, expansion: 2^lg_sub waves per chunk of the X tuples of pairs the probe did not
// finish (a BFS level's claims are CAS and atomic round trips: more waves in flight, not longer
// streams, set its pace); a claim (CAS on the pair's distance byte) sets the filters, joins the
// side's next list and the arena (staged per wave), adds (degree + 1) to the pair's frontier sum
// (one atomic per chunk: a chunk is one pair's) and is a meet when the other side has seen the
// vertex.  Then the probe's slots become meet tuples and arena entries.
template <int OCC>
__global__ __launch_bounds__(256, OCC) void k_dv_expand(SpDev d, SpState st, SpFilt f, SpCsr g0, SpCsr g1,
                                                        uint8_t* d0, uint8_t* d1, int64_t n, int64_t lo, int32_t it,
                                                        int32_t lg_sub, int32_t pf_agg) {
  __shared__ uint64_t s_stage[4][2][kDvStage];
  // per wave, the pair-filter row its current chunk fills: every claim of a chunk is one
  // (side, pair, level), so the chunk's bits are OR-ed here and leave as at most 128 word atomics
  // over one contiguous 512-byte row (option sp_dv_pf_lds, default 1) instead of one scattered
  // memory-side atomic per claim
  __shared__ uint32_t s_pf[4][128];
  // a producer overflowed: its tables are incomplete and the host re-runs the batch, so the block
  // expands nothing -- but the probe's claims still go to the arena below, which is the only
  // record the host's abort resets distance bytes from (block-uniform)
  const bool skip = dv_ovf_block(d.cnt);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int64_t wave = (int64_t(blockIdx.x) * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = (int64_t(gridDim.x) * blockDim.x) >> 6;
  const QBlk q = qblk(d.cnt, it);
  const int64_t total = min(int64_t(q[Q_NCH]), d.cap_ch);
  if (total == 0) return;  // nothing selected (grid-uniform)
  const uint32_t B = uint32_t(st.B);
  uint64_t* const out0 = d.live[it & 1][0];
  uint64_t* const out1 = d.live[it & 1][1];
  DvStage sg0{s_stage[wid][0], 0u}, sg1{s_stage[wid][1], 0u};
  unsigned long long claims = 0, entries = 0;
  // sp_dv_diag (timing only, wrong results): bit 4 no chunk is expanded, bit 5 no probe claim
  // is moved to the arena
  if (!skip && !(f.diag & 16))
  chunk_groups(
      total << lg_sub,
      [&](int64_t vc, ChunkRec& r) {
        // a pair the probe finished (met = -1) is dropped before its row bounds are loaded
        const int64_t c = vc >> lg_sub;
        const int32_t a = d.chx[c];
        const uint64_t t = d.X[a];
        if (st.met[t_pair(t)] == -1) return false;
        return x_chunk_at(d, g0, g1, c, a, t, d.lg_chb, lg_sub, vc & ((int64_t(1) << lg_sub) - 1), r);
      },
      [&](const ChunkRec& r, int64_t) {
        const uint32_t side = t_side(r.t), p = t_pair(r.t), l = t_lvl(r.t);
        const SpCsr& g = side ? g1 : g0;
        const uint32_t sh = uint32_t(st.ilv);
        uint8_t* const sdp = (side ? d1 : d0) + ((uint64_t(p) * uint64_t(n)) << sh);  // the pair's bytes (pair-major)
        const uint8_t* const odp = (side ? d0 : d1) + ((uint64_t(p) * uint64_t(n)) << sh);
        // interleaved: both sides' bytes of a vertex in one 2-byte load (the other side's bytes do
        // not change during an expansion: only the expanding side of a pair is written)
        const uint16_t* const bdp = reinterpret_cast<const uint16_t*>(d0 + ((uint64_t(p) * uint64_t(n)) << 1));
        entries += uint64_t(r.x1 - r.x0) * (lane == 0);
        unsigned long long dsum = 0;
        const bool pf_lds = pf_agg && f.pf && l + 1 < uint32_t(kLv);  // wave-uniform
        if (pf_lds) {
          s_pf[wid][lane] = 0u;
          s_pf[wid][lane + 64] = 0u;
          __builtin_amdgcn_wave_barrier();
        }
        for (int64_t x = step_start(r.x0); x < r.x1; x += 64 * kProbeU) {
          uint32_t w[kProbeU];
          col_step(g.col, x, r.x0, r.x1, lo, w);
          uint32_t bt[kProbeU], obt[kProbeU];
#pragma unroll
          for (int u = 0; u < kProbeU; u++) {
            bt[u] = 0x1FFu;
            obt[u] = 0xFFu;
            if (w[u] != 0xFFFFFFFFu) {
              if (sh) {
                const uint32_t both = bdp[w[u]];
                bt[u] = side ? both >> 8 : both & 0xFFu;
                obt[u] = side ? both & 0xFFu : both >> 8;
              } else {
                bt[u] = sdp[w[u]];
              }
            }
          }
#pragma unroll
          for (int u = 0; u < kProbeU; u++) {
            // a claim: a plain byte store (two chunks of one
            // pair reaching the same vertex in this level may both list it; the byte holds l + 1 either
            // way, and a duplicate tuple only repeats work)
            const uint64_t wi = uint64_t(w[u]) << sh;
            const bool cl = bt[u] == 0xFFu && (sdp[wi] = uint8_t(l + 1), true);
            bool meet = false;
            uint32_t dt = 0;
            if (cl) {
              if (pf_lds) {
                const uint32_t b = pf_bit(w[u]);
                atomicOr(&s_pf[wid][b >> 5], 1u << (b & 31u));
                gf_mark(f, side, l + 1, p, w[u]);
              } else {
                filt_mark(f, side, l + 1, p, w[u]);
              }
              dsum += (unsigned long long)sp_deg(g, w[u]) + 1;
              const uint32_t ob = sh ? obt[u] : uint32_t(odp[w[u]]);
              if (ob != 0xFFu) {
                meet = true;
                dt = side ? l + 1 : ob;
                st.met[p] = 1;
              }
            }
            const uint64_t cm = __ballot(cl);
            if (cm == 0) continue;
            claims += uint64_t(__popcll(cm)) * (lane == 0);
            if (side)
              dv_stage(sg1, cl, mk_tup(1, p, l + 1, w[u]), d.cnt, q + Q_LIVE1, out1, d.cap_live, d.arena, d.cap_arena);
            else
              dv_stage(sg0, cl, mk_tup(0, p, l + 1, w[u]), d.cnt, q + Q_LIVE0, out0, d.cap_live, d.arena, d.cap_arena);
            dput(d.meet, d.cap_meet, gcnt(d.cnt, D_MEET), d.cnt, meet, mk_tup(1, p, dt, w[u]));
          }
        }
        if (pf_lds) {  // the chunk's row: nonzero words OR-ed into the pair filter
          __builtin_amdgcn_wave_barrier();
          uint32_t* const row = f.pf + (size_t(side * kLv + l + 1) * uint32_t(f.B) + p) * 128;
          const uint32_t w0 = s_pf[wid][lane], w1 = s_pf[wid][lane + 64];
          if (w0) atomicOr(row + lane, w0);
          if (w1) atomicOr(row + lane + 64, w1);
        }
        dsum = wsum(dsum);
        if (lane == 0 && dsum) {
          atomicAdd(st.deg + side * B + p, dsum);
          // a forward level's (degree + 1) sum is also the sweep's push entries for that level
          if (side == 0 && l + 1 < uint32_t(kMaxQ)) atomicAdd(d.push + int64_t(l + 1) * B + p, dsum);
        }
      });
  // the probe's claims: meet tuples (the vertex at the backward depth) + arena entries
  for (int64_t c0 = wave * 64; c0 < total && !(f.diag & 32); c0 += nwaves * 64) {
    const int64_t c = c0 + lane;
    const uint64_t v = c < total ? d.slot[c] : ~0ull;
    const bool hit = v != ~0ull;
    uint64_t mt = 0;
    if (hit) {
      const uint32_t o = t_side(v), lv = t_lvl(v);
      mt = mk_tup(1, t_pair(v), o ? lv : t_lvl(d.X[d.chx[c]]), t_row(v));
    }
    if (__ballot(hit) == 0) continue;
    dput(d.arena, d.cap_arena, gcnt(d.cnt, D_ARENA), d.cnt, hit, v);
    dput(d.meet, d.cap_meet, gcnt(d.cnt, D_MEET), d.cnt, hit, mt);
  }
  if (skip || (f.diag & 64)) return;  // (diag bit 6: no final flush / sums, timing only)
  dv_flush_block(sg0, d.cnt, q + Q_LIVE0, out0, d.cap_live, d.arena, d.cap_arena);
  dv_flush_block(sg1, d.cnt, q + Q_LIVE1, out1, d.cap_live, d.arena, d.cap_arena);
  blk_add(q + Q_CLAIMS, claims);
  blk_add(q + Q_EE, entries);
}

// BFS iteration it, last launch: per pair, the end of the iteration (depth, meet, done) and the
// next side choice; the last block publishes the iteration's counters to host slot `hslot`
__global__ __launch_bounds__(256) void k_dv_step(SpDev d, SpState st, int32_t max_steps, int32_t it,
                                                 unsigned long long* hslot, uint64_t seq) {
  const int32_t B = st.B;
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  bool active = false;
  if (p < B && st.state[p] == SP_ACTIVE) {
    const int32_t m = st.met[p];
    if (m == -1) {  // the probe met: the other side advanced by one
      const int o = st.side[p] ^ 1;
      st.lvl[o * B + p] += 1;
      st.res[p] = st.lvl[p] + st.lvl[B + p];
      st.state[p] = SP_MET;
      st.met[p] = 2 + it;
      st.pside[p] = o;
    } else {
      const int s = st.side[p];
      st.pside[p] = s;
      st.lvl[s * B + p] += 1;
      const int32_t L = st.lvl[p] + st.lvl[B + p];
      if (m == 1) {
        st.res[p] = L;
        st.state[p] = SP_MET;
        st.met[p] = 2 + it;
      } else if (st.deg[s * B + p] == 0 || L >= max_steps) {
        st.state[p] = SP_DONE;
      }
    }
    if (st.state[p] == SP_MET) {
      atomicMax(gcnt(d.cnt, D_MAXL), (unsigned long long)st.res[p]);
      atomicMax(gcnt(d.cnt, D_MAXF), (unsigned long long)st.lvl[p]);
    } else if (st.state[p] == SP_ACTIVE) {
      const int s = st.deg[p] <= st.deg[B + p] ? 0 : 1;
      st.side[p] = s;
      st.deg[s * B + p] = 0;
      active = true;
    }
  }
  (void)wave_append(qblk(d.cnt, it) + Q_ACTIVE, active);
  dv_publish_last(d.cnt, it, hslot, seq);
}

// path offsets of the batch by one block: pair p's path holds L + 1 vids when it finished at
// length L (an ACTIVE pair has none); doff[B] the total
__device__ inline void dv_path_offsets(const SpState& st, int64_t nb, int64_t* doff) {
  __shared__ int64_t s_w[kBlk / 64];
  __shared__ int64_t s_carry;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (threadIdx.x == 0) s_carry = 0;
  __syncthreads();
  for (int64_t p0 = 0; p0 < nb; p0 += kBlk) {
    const int64_t p = p0 + threadIdx.x;
    int64_t len = 0;
    if (p < nb && st.state[p] != SP_ACTIVE && st.res[p] >= 0) len = st.res[p] + 1;
    int64_t v = len;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int64_t y = __shfl_up(v, o);
      if (lane >= o) v += y;
    }
    if (lane == 63) s_w[wv] = v;
    __syncthreads();
    int64_t pre = s_carry, tot = 0;
#pragma unroll
    for (int w = 0; w < kBlk / 64; w++) {
      if (w < wv) pre += s_w[w];
      tot += s_w[w];
    }
    if (p < nb) doff[p] = pre + v - len;
    __syncthreads();
    if (threadIdx.x == 0) s_carry += tot;
    __syncthreads();
  }
  if (threadIdx.x == 0) doff[nb] = s_carry;
}

// walk step i's front (block-uniform): the pick of step i - 1 (path vid, next vertex through the
// vertex hash), then the chunks of the current vertex's out-row for step i
__device__ inline void dv_walk_front(SpDev& d, const SpState& st, const SpCsr& gout, int32_t i, int64_t lo,
                                     const int64_t* ht_keys, const int32_t* ht_vals, uint64_t ht_mask,
                                     bool ht_has_min, int32_t ht_min_gidx) {
  const int32_t B = st.B;
  const QBlk q = qblk(d.cnt, kWkQ + i);
  unsigned long long* ctr[1] = {q + Q_NCH};
  const int64_t rounds = (int64_t(B) + kBlk - 1) / kBlk;
  for (int64_t r = blockIdx.x; r < rounds; r += gridDim.x) {
    const int64_t p = r * kBlk + threadIdx.x;
    int64_t dg = 0;
    if (p < B && st.state[p] == SP_MET) {
      const int32_t L = st.res[p];
      if (i == 0) {
        d.cur[p] = d.gs[p];
      } else if (L - 1 > i - 1 && d.cur[p] >= 0) {
        const long long b = d.best[p];
        if (b == LLONG_MAX) {  // in-edge keys without the mirrored out-edge: the definition does not hold
          atomicAdd(gcnt(d.cnt, D_WALKERR), 1ull);
          d.cur[p] = -1;
        } else {
          d.path[d.doff[p] + i] = int64_t(b);
          d.cur[p] = ht_lookup(ht_keys, ht_vals, ht_mask, int64_t(b), ht_has_min, ht_min_gidx) - int32_t(lo);
        }
      }
      if (L - 1 > i && d.cur[p] >= 0) dg = sp_deg(gout, uint32_t(d.cur[p]));
      d.best[p] = LLONG_MAX;
    }
    const uint32_t nc = uint32_t((dg + kCh - 1) / kCh);
    unsigned long long o[1];
    blk_reserve_n<1>(ctr, &nc, o);
    const bool ok = int64_t(o[0]) + int64_t(nc) <= d.cap_wch;
    if (nc && !ok) atomicOr(gcnt(d.cnt, D_OVF), 4ull);
    if (p < B && nc) d.wcb[p] = int64_t(o[0]);
    wave_fill_val(int64_t(o[0]), ok ? int64_t(nc) : 0, p, [&](int64_t c, int64_t v) { d.wchx[c] = int32_t(v); });
  }
}

// after the BFS: path offsets (block 0), the walk's first front and sweep step 1's pull entries
// per pair (in-rows of the meet vertices short of src).  The push entries of every forward level
// were summed by the expansions that claimed it.
__global__ __launch_bounds__(kBlk) void k_dv_post(SpDev d, SpState st, SpCsr gout, SpCsr gin, int64_t lo,
                                                  const int64_t* ht_keys, const int32_t* ht_vals, uint64_t ht_mask,
                                                  bool ht_has_min, int32_t ht_min_gidx) {
  const int32_t B = st.B;
  // the path offsets by the last block, beside the walk front the first blocks build
  if (blockIdx.x == gridDim.x - 1) dv_path_offsets(st, B, d.doff);
  dv_walk_front(d, st, gout, 0, lo, ht_keys, ht_vals, ht_mask, ht_has_min, ht_min_gidx);
  const int64_t gn = int64_t(gridDim.x) * blockDim.x;
  const int64_t nm = min(int64_t((*gcnt(d.cnt, D_MEET))), d.cap_meet);
  const int64_t rm = (nm + gn - 1) / gn;
  for (int64_t r = 0; r < rm; r++) {
    const int64_t i = r * gn + int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    bool go = false;
    uint32_t p = 0;
    unsigned long long dg = 0;
    if (i < nm) {
      const uint64_t t = d.meet[i];
      p = t_pair(t);
      go = st.state[p] == SP_MET && int32_t(t_lvl(t)) < st.res[p] - 1;
      if (go) dg = (unsigned long long)sp_deg(gin, t_row(t)) + 1;
    }
    wave_add_keyed(d.pull + B, p, dg, go);  // step 1
  }
}

// sweep step j: pull (in-rows of the level above, from the current sweep list) or push (out-rows
// of the forward level k = f - j, from the arena), per pair the side with fewer entries (option
// sp_push_bias in 1/16: push when its entries are below pull's x bias / 16)
__device__ inline bool dv_push_pair(const SpDev& d, const SpState& st, uint32_t p, int32_t j,
                                    unsigned long long bias16) {
  const int32_t B = st.B;
  const unsigned long long pl = d.pull[int64_t(j) * B + p];
  const int32_t k = st.lvl[p] - j;
  if (pl == 0 || k < 1 || k >= kMaxQ) return false;
  return d.push[int64_t(k) * B + p] * 16ull < pl * bias16;
}
__global__ __launch_bounds__(kBlk) void k_dv_sweep_select(SpDev d, SpState st, SpCsr gout, SpCsr gin, int32_t j,
                                                          unsigned long long bias16) {
  const QBlk q = qblk(d.cnt, kSwQ + j);
  const uint64_t* cur = j == 1 ? d.meet : d.sw[(j - 1) & 1];
  const int64_t ncur = j == 1 ? min(int64_t((*gcnt(d.cnt, D_MEET))), d.cap_meet)
                              : min(int64_t(qblk(d.cnt, kSwQ + j - 1)[Q_CLAIMS]), d.cap_sw);
  // per pair in LDS: res - 1 of a MET pair (0: not sweeping) and the forward level it pushes at this
  // step (0: it pulls); the arena's forward tuples are scanned only when some pair pushes (every
  // block asks every pair: a few loads per thread instead of 1 M+ arena tuples per step)
  __shared__ uint8_t s_rm1[kPairLds], s_pk[kPairLds];
  int anyp = 0;
  for (int p = threadIdx.x; p < st.B; p += blockDim.x) {
    const bool met = st.state[p] == SP_MET;
    const bool push = met && dv_push_pair(d, st, uint32_t(p), j, bias16);
    s_rm1[p] = met ? uint8_t(max(st.res[p] - 1, 0)) : uint8_t(0);
    s_pk[p] = push ? uint8_t(st.lvl[p] - j) : uint8_t(0);
    anyp |= push ? 1 : 0;
  }
  const int64_t na = __syncthreads_or(anyp) ? min(int64_t((*gcnt(d.cnt, D_ARENA))), d.cap_arena) : 0;
  const int64_t nt = ncur + na;
  constexpr int64_t per = int64_t(kBlk) * kSelIt;
  const int64_t rounds = (nt + per - 1) / per;
  unsigned long long esum = 0;
  unsigned long long* ctr[2] = {q + Q_X, q + Q_NCH};
  for (int64_t r = blockIdx.x; r < rounds; r += gridDim.x) {
    const int64_t i0 = r * per + threadIdx.x;
    uint64_t t[kSelIt];
#pragma unroll
    for (int u = 0; u < kSelIt; u++) {
      const int64_t i = i0 + u * kBlk;
      t[u] = i < ncur ? cur[i] : i < nt ? d.arena[i - ncur] : ~0ull;
    }
    uint32_t xm = 0;
    int64_t dg[kSelIt];
    uint32_t nch = 0;
#pragma unroll
    for (int u = 0; u < kSelIt; u++) {
      dg[u] = 0;
      if (t[u] == ~0ull) continue;
      const uint32_t p = t_pair(t[u]), lv = t_lvl(t[u]);
      const bool pulled = i0 + u * kBlk < ncur;
      const uint32_t rm1 = s_rm1[p], pk = s_pk[p];
      const bool go = pulled ? lv < rm1 && pk == 0 : t_side(t[u]) == 0 && pk != 0 && lv == pk;
      if (!go) continue;
      dg[u] = sp_deg(pulled ? gin : gout, t_row(t[u]));
      if (dg[u] == 0) continue;
      xm |= 1u << u;
      nch += uint32_t((dg[u] + (int64_t(1) << d.lg_chs) - 1) >> d.lg_chs);
      esum += (unsigned long long)dg[u];
    }
    const uint32_t nn[2] = {uint32_t(__popc(xm)), nch};
    unsigned long long o[2];
    blk_reserve_n<2>(ctr, nn, o);
    bool ovf = false;
#pragma unroll
    for (int u = 0; u < kSelIt; u++) {
      const bool x = (xm >> u) & 1u;
      const int64_t nc = x ? (dg[u] + (int64_t(1) << d.lg_chs) - 1) >> d.lg_chs : 0;
      const int64_t xa = int64_t(o[0]), ca = int64_t(o[1]);
      const bool fit = xa < d.cap_x && ca + nc <= d.cap_ch;
      if (x) {
        if (fit) {
          d.X[xa] = t[u];
          d.Xcb[xa] = ca;
        } else {
          ovf = true;
        }
        o[0]++;
        o[1] += uint64_t(nc);
      }
      wave_fill_val(ca, x && fit ? nc : 0, xa, [&](int64_t c, int64_t v) { d.chx[c] = int32_t(v); });
    }
    if (ovf) atomicOr(gcnt(d.cnt, D_OVF), 2ull);
  }
  blk_add(q + Q_XE, esum);
}

// sweep step j: one wave per chunk.  Pull (side 1, in-row of w at dt = l): an in-neighbour u with
// ds(u) = L - l - 1 gets dt = l + 1.  Push (side 0, out-row of u at ds = l): u gets dt = L - l
// once an out-neighbour has dt = L - l - 1 (the scan stops there).  Claims go to the arena and
// the next sweep list, and the pull entries of the claimed vertices that the next step scans are
// added to the pair's step j + 1 sum.
template <int U, int OCC = 1>  // column entries per lane and step; waves per SIMD the registers allow
__global__ __launch_bounds__(256, OCC) void k_dv_sweep(SpDev d, SpState st, SpFilt f, SpCsr gout, SpCsr gin,
                                                       uint8_t* d0, uint8_t* d1, int64_t n, int64_t lo, int32_t j) {
  __shared__ uint64_t s_stage[4][kDvStage];
  if (dv_ovf_block(d.cnt)) return;  // a producer overflowed: its tables are incomplete (the host re-runs)
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const QBlk q = qblk(d.cnt, kSwQ + j);
  const int64_t total = min(int64_t(q[Q_NCH]), d.cap_ch);
  const uint32_t B = uint32_t(st.B);
  uint64_t* out = d.sw[j & 1];
  unsigned long long* pull_next = j + 1 < kMaxQ ? d.pull + int64_t(j + 1) * B : nullptr;
  DvStage sg{s_stage[wid], 0u};
  unsigned long long entries = 0;
  chunk_groups(
      total,
      [&](int64_t c, ChunkRec& r) {
        if (!x_chunk(d, gout, gin, c, d.lg_chs, 0, 0, r)) return false;
        const uint32_t os = t_side(r.t) ^ 1u, p = t_pair(r.t);
        r.a0 = st.res[p];
        r.a1 = d.gs[os * B + p];
        return true;
      },
      [&](const ChunkRec& r, int64_t) {
        const uint32_t side = t_side(r.t), p = t_pair(r.t), l = t_lvl(r.t), row = t_row(r.t), os = side ^ 1u;
        const int32_t* col = side ? gin.col : gout.col;
        const int32_t L = r.a0;
        const int32_t need = L - int32_t(l) - 1;  // the other side's depth a neighbour needs
        const uint32_t sh = uint32_t(st.ilv);
        const uint8_t* const odp = (side ? d0 : d1) + ((uint64_t(p) * uint64_t(n)) << sh);  // the pair's bytes
        uint8_t* const d1p = d1 + ((uint64_t(p) * uint64_t(n)) << sh);
        bool pf_on;
        const uint2 prow = pf_load(f, os, need, p, pf_on);
        entries += uint64_t(r.x1 - r.x0) * (lane == 0);
        unsigned long long pc = 0;
        uint32_t wn[U];  // the next step's columns (see the probe)
        col_step<U>(col, step_start(r.x0), r.x0, r.x1, lo, wn);
        for (int64_t x = step_start(r.x0); x < r.x1; x += 64 * U) {
          if (side == 0 && *reinterpret_cast<volatile const uint8_t*>(d1p + (uint64_t(row) << sh)) != 0xFFu)
            break;  // u claimed
          uint32_t w[U];
#pragma unroll
          for (int u = 0; u < U; u++) w[u] = wn[u];
          if (x + 64 * U < r.x1) col_step<U>(col, x + 64 * U, r.x0, r.x1, lo, wn);
          uint32_t hm = 0;  // entries whose neighbour sits at depth need on the other side
          if (need == 0) {
#pragma unroll
            for (int u = 0; u < U; u++) hm |= w[u] == uint32_t(r.a1) ? 1u << u : 0u;
          } else {
            uint32_t fm = 0;
#pragma unroll
            for (int u = 0; u < U; u++) {
              const bool pv = pf_on ? pf_test(prow, w[u]) : true;
              fm |= (w[u] != 0xFFFFFFFFu && pv && gf_test(f, os, need, p, w[u])) ? 1u << u : 0u;
            }
            if (f.diag & 3) fm = (f.diag & 1) ? 0u : (__ballot(fm != 0) ? 0u : fm);
#pragma unroll
            for (int u = 0; u < U; u++)
              hm |= ((fm >> u) & 1u) && uint32_t(odp[uint64_t(w[u]) << sh]) == uint32_t(need) ? 1u << u : 0u;
          }
          if (__ballot(hm != 0) == 0) continue;
          if (side == 1) {
#pragma unroll
            for (int u = 0; u < U; u++) {
              const bool cl = ((hm >> u) & 1u) && claim_byte(d1p, uint64_t(w[u]) << sh, l + 1);
              if (cl) {
                filt_mark(f, 1, l + 1, p, w[u]);
                if (int32_t(l + 1) < L - 1) pc += (unsigned long long)sp_deg(gin, w[u]) + 1;
              }
              dv_stage(sg, cl, mk_tup(1, p, l + 1, w[u]), d.cnt, q + Q_CLAIMS, out, d.cap_sw, d.arena, d.cap_arena);
            }
          } else {
            bool cl = false;
            if (lane == 0) {
              cl = claim_byte(d1p, uint64_t(row) << sh, uint32_t(need + 1));
              if (cl) {
                filt_mark(f, 1, uint32_t(need + 1), p, row);
                if (need + 1 < L - 1) pc += (unsigned long long)sp_deg(gin, row) + 1;
              }
            }
            dv_stage(sg, cl, mk_tup(1, p, uint32_t(need + 1), row), d.cnt, q + Q_CLAIMS, out, d.cap_sw, d.arena,
                     d.cap_arena);
            break;
          }
        }
        pc = wsum(pc);
        if (lane == 0 && pc && pull_next) atomicAdd(pull_next + p, pc);
      });
  dv_flush_block(sg, d.cnt, q + Q_CLAIMS, out, d.cap_sw, d.arena, d.cap_arena);
  blk_add(q + Q_EE, entries);
}

// walk step i: one wave per chunk of a walking pair's current out-row; the smallest vid w with
// dist_B(w) = L - i - 1 (by the filters, then the byte) goes to best[p] with one atomicMin per
// chunk.  The last step is dst itself and never scanned.
__global__ __launch_bounds__(256) void k_dv_walk_scan(SpDev d, SpState st, SpFilt f, SpCsr gout, const uint8_t* d1,
                                                      const int64_t* vid_of, int64_t n, int64_t lo, int32_t i) {
  if (dv_ovf_block(d.cnt)) return;  // a producer overflowed: its tables are incomplete (the host re-runs)
  const int lane = threadIdx.x & 63;
  const QBlk q = qblk(d.cnt, kWkQ + i);
  const int64_t total = min(int64_t(q[Q_NCH]), d.cap_wch);
  unsigned long long entries = 0;
  chunk_groups(
      total,
      [&](int64_t c, ChunkRec& r) {
        const uint32_t p = uint32_t(d.wchx[c]);
        const uint32_t v = uint32_t(d.cur[p]);
        const int64_t re = gout.row_ptr[v + 1];
        r.t = p;
        r.x0 = gout.row_ptr[v] + (c - d.wcb[p]) * kCh;
        r.x1 = min(r.x0 + int64_t(kCh), re);
        r.a0 = st.res[p] - i - 1;
        return r.x0 < r.x1;
      },
      [&](const ChunkRec& r, int64_t) {
        const uint32_t p = uint32_t(r.t);
        const int32_t need = r.a0;
        entries += uint64_t(r.x1 - r.x0) * (lane == 0);
        bool pf_on;
        const uint2 prow = pf_load(f, 1, need, p, pf_on);
        const uint32_t sh = uint32_t(st.ilv);
        const uint8_t* const d1p = d1 + ((uint64_t(p) * uint64_t(n)) << sh);  // the pair's bytes (pair-major)
        long long bm = LLONG_MAX;
        // the next step's columns are loaded before this step's tests wait on their filter and
        // byte loads (one round trip less per step of the chain)
        uint32_t wn[kProbeU];
        col_step(gout.col, step_start(r.x0), r.x0, r.x1, lo, wn);
        for (int64_t x = step_start(r.x0); x < r.x1; x += 64 * kProbeU) {
          uint32_t w[kProbeU];
#pragma unroll
          for (int u = 0; u < kProbeU; u++) w[u] = wn[u];
          if (x + 64 * kProbeU < r.x1) col_step(gout.col, x + 64 * kProbeU, r.x0, r.x1, lo, wn);
          uint32_t fm = 0;
#pragma unroll
          for (int u = 0; u < kProbeU; u++) {
            const bool pv = pf_on ? pf_test(prow, w[u]) : true;
            fm |= (w[u] != 0xFFFFFFFFu && pv && gf_test(f, 1, need, p, w[u])) ? 1u << u : 0u;
          }
#pragma unroll
          for (int u = 0; u < kProbeU; u++)
            if (((fm >> u) & 1u) && uint32_t(d1p[uint64_t(w[u]) << sh]) == uint32_t(need)) {
              const long long vv = vid_of[lo + w[u]];
              bm = vv < bm ? vv : bm;
            }
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
          const long long y = __shfl_xor(bm, o);
          bm = y < bm ? y : bm;
        }
        if (lane == 0 && bm != LLONG_MAX) atomicMin(d.best + p, bm);
      });
  blk_add(q + Q_EE, entries);
}

__global__ __launch_bounds__(kBlk) void k_dv_walk_front(SpDev d, SpState st, SpCsr gout, int32_t i, int64_t lo,
                                                        const int64_t* ht_keys, const int32_t* ht_vals,
                                                        uint64_t ht_mask, bool ht_has_min, int32_t ht_min_gidx) {
  dv_walk_front(d, st, gout, i, lo, ht_keys, ht_vals, ht_mask, ht_has_min, ht_min_gidx);
}

// the batch's results: the last walk step's pick (step ilast, pairs of the longest length), then
// state, length, path offset and path of every pair into coherent host memory (the ends src and
// dst are the host's)
__global__ __launch_bounds__(256) void k_dv_out(SpDev d, SpState st, int32_t ilast) {
  const int32_t B = st.B;
  const int64_t gt = int64_t(blockIdx.x) * blockDim.x + threadIdx.x, gn = int64_t(gridDim.x) * blockDim.x;
  for (int64_t p = gt; p < B; p += gn) {
    const int32_t s = st.state[p], L = st.res[p];
    const int64_t o = d.doff[p];
    if (s == SP_MET && ilast >= 0 && L - 1 > ilast && d.cur[p] >= 0) {
      const long long b = d.best[p];
      if (b == LLONG_MAX) atomicAdd(gcnt(d.cnt, D_WALKERR), 1ull);
      else d.path[o + ilast + 1] = int64_t(b);
    }
    d.h_sr[p] = s;
    d.h_sr[B + p] = L;
    d.h_off[p] = o;
    if (p == B - 1) d.h_off[B] = d.doff[B];
    if (s != SP_ACTIVE)
      for (int32_t k = 1; k < L; k++) d.h_path[o + k] = d.path[o + k];
  }
  // the host reads these words once k_dv_finish (the next launch) publishes its sequence word:
  // every writer's stores must have left the device first (a system-scope release per wave; the
  // kernel boundary alone did not order them before the finish wave's store when several
  // contexts shared the device: stale paths at 8 in-process ranks)
  __threadfence_system();
}

// every claimed distance byte of the batch reset from the arena, and the filters zeroed whole --
// the batch's pair rows (2 kLv B x 512 B) and the global filter are a few MB of streaming stores,
// cheaper than a random store per claim (after the finish publication: the host reads the results
// while this runs; D_CLEAR holds the arena length)
__global__ __launch_bounds__(256) void k_dv_clear(SpDev d, SpState st, SpFilt f, uint8_t* d0, uint8_t* d1, int64_t n) {
  const int64_t gt = int64_t(blockIdx.x) * blockDim.x + threadIdx.x, gn = int64_t(gridDim.x) * blockDim.x;
  const int64_t pf4 = f.pf ? int64_t(2 * kLv) * st.B * 32 : 0;          // uint4 groups of the pair rows
  const int64_t gf4 = f.gf ? (int64_t(1) << (64 - f.gshift)) / 4 : 0;  // uint4 groups of the global filter
  const uint4 z = make_uint4(0u, 0u, 0u, 0u);
  for (int64_t i = gt; i < pf4; i += gn) reinterpret_cast<uint4*>(f.pf)[i] = z;
  for (int64_t i = gt; i < gf4; i += gn) reinterpret_cast<uint4*>(f.gf)[i] = z;
  const int64_t na = min(int64_t((*gcnt(d.cnt, D_CLEAR))), d.cap_arena);
  for (int64_t i = gt; i < na; i += gn) {
    const uint64_t t = d.arena[i];
    (t_side(t) ? d1 : d0)[didx(st, t_pair(t), t_row(t), n)] = 0xFF;
  }
}

// the batch's counters into coherent host memory, then cleared for the next batch: the globals
// and the blocks the batch used (BFS blocks [0, nbfs), sweep steps [1, nsw], walk steps
// [0, nwalk)); one wave, lane 0's system-scope release publishes the sequence word after the
// copies.  D_CLEAR keeps the arena length for k_dv_clear.
__global__ void k_dv_finish(unsigned long long* cnt, unsigned long long* h, unsigned long long* hseq, uint64_t seq,
                            int32_t nbfs, int32_t nsw, int32_t nwalk) {
  const unsigned long long arena = (*gcnt(cnt, D_ARENA));  // read before any lane clears it
  auto move = [&](int a, int b) {
    for (int i = a + int(threadIdx.x); i < b; i += 64) {
      h[i] = *gcnt(cnt, i);
      *gcnt(cnt, i) = i == D_CLEAR ? arena : 0ull;
    }
  };
  move(0, D_G + nbfs * Q_W);
  move(D_G + (kSwQ + 1) * Q_W, D_G + (kSwQ + 1 + nsw) * Q_W);
  move(D_G + kWkQ * Q_W, D_G + (kWkQ + nwalk) * Q_W);
  __builtin_amdgcn_wave_barrier();
  if (threadIdx.x == 0) __hip_atomic_store(hseq, (unsigned long long)seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

}  // namespace

// ---- world > 1: the pairs are independent, so they are sharded over the ranks (pair i on rank
// i % world) and every rank answers its own pairs against a replica of the whole graph's out / in
// CSRs.  The replicas are assembled once with allgathers of every rank's rows (the rows of rank r
// are the gidx range [base[r], base[r+1])); the traversal itself exchanges nothing.
// the batch's path offsets on the device (one block): pair p's path holds L + 1 vids when it met
// at length L (an ACTIVE pair has none); doff = their exclusive scan, cnt[C_PLEN] the total,
// cnt[C_MAXL] the longest L, cnt[C_WALKERR] cleared.  The host reads the two counters with one
// counter fetch instead of copying state and res back and scanning them itself.
__global__ __launch_bounds__(1024) void k_sp_path_offsets(SpState st, int64_t nb, int64_t* doff,
                                                          unsigned long long* cnt) {
  __shared__ int64_t s_w[16];
  __shared__ int32_t s_m[16];
  __shared__ int64_t s_carry;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (threadIdx.x == 0) s_carry = 0;
  int32_t mx = 0;
  __syncthreads();
  for (int64_t p0 = 0; p0 < nb; p0 += blockDim.x) {
    const int64_t p = p0 + threadIdx.x;
    int64_t len = 0;
    if (p < nb && st.state[p] != SP_ACTIVE) {
      const int32_t L = st.res[p];
      if (L >= 0) {
        len = L + 1;
        mx = max(mx, st.state[p] == SP_MET ? L : 0);
      }
    }
    int64_t v = len;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int64_t y = __shfl_up(v, o);
      if (lane >= o) v += y;
    }
    if (lane == 63) s_w[wv] = v;
    __syncthreads();
    int64_t pre = s_carry, tot = 0;
    for (int w = 0; w < int(blockDim.x >> 6); w++) {
      if (w < wv) pre += s_w[w];
      tot += s_w[w];
    }
    if (p < nb) doff[p] = pre + v - len;
    __syncthreads();
    if (threadIdx.x == 0) s_carry += tot;
    __syncthreads();
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) mx = max(mx, __shfl_xor(mx, o));
  if (lane == 0) s_m[wv] = mx;
  __syncthreads();
  if (threadIdx.x == 0) {
    int32_t m = 0;
    for (int w = 0; w < int(blockDim.x >> 6); w++) m = max(m, s_m[w]);
    doff[nb] = s_carry;
    cnt[C_PLEN] = (unsigned long long)s_carry;
    cnt[C_MAXL] = (unsigned long long)m;
    cnt[C_WALKERR] = 0ull;
  }
}

__global__ void k_add_i64(int64_t* a, int64_t n, int64_t v) {
  for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < n; i += int64_t(gridDim.x) * blockDim.x)
    a[i] += v;
}

static void replicate_csr(Ctx& c, const Csr& loc, Csr& rep) {
  const int W = c.world;
  PoolScope none(nullptr);
  DevBuf dm, dall, ok_loc, flag;
  dm.alloc(16);
  dall.alloc(size_t(W) * 16);
  int64_t mine[2] = {loc.nnz, loc.row_ok.p ? 1 : 0};
  NBG_HIP(hipMemcpyAsync(dm.p, mine, 16, hipMemcpyHostToDevice, c.stream));
  comm_allgather_bytes(c, dm.p, 16, dall.p);
  std::vector<int64_t> all(size_t(W) * 2);
  NBG_HIP(hipMemcpyAsync(all.data(), dall.p, size_t(W) * 16, hipMemcpyDeviceToHost, c.stream));
  NBG_HIP(hipStreamSynchronize(c.stream));
  std::vector<int64_t> nnz_off(size_t(W) + 1, 0);
  bool any_ok = false;
  for (int r = 0; r < W; r++) {
    nnz_off[size_t(r) + 1] = nnz_off[size_t(r)] + all[size_t(r) * 2];
    any_ok = any_ok || all[size_t(r) * 2 + 1] != 0;
  }
  const int64_t N = c.n_global;
  rep.n_rows = N;
  rep.nnz = nnz_off[size_t(W)];
  rep.col.alloc(size_t(rep.nnz + 16) * 4);
  rep.row_ptr.alloc(size_t(N + 1) * 8);
  std::vector<size_t> rb(static_cast<size_t>(W)), ro(static_cast<size_t>(W));
  for (int r = 0; r < W; r++) {
    rb[size_t(r)] = size_t(all[size_t(r) * 2]) * 4;
    ro[size_t(r)] = size_t(nnz_off[size_t(r)]) * 4;
  }
  comm_allgatherv_bytes(c, loc.col.p, size_t(loc.nnz) * 4, rep.col.p, rb.data(), ro.data());
  for (int r = 0; r < W; r++) {
    rb[size_t(r)] = size_t(c.base[size_t(r) + 1] - c.base[size_t(r)]) * 8;
    ro[size_t(r)] = size_t(c.base[size_t(r)]) * 8;
  }
  comm_allgatherv_bytes(c, loc.row_ptr.p, size_t(loc.n_rows) * 8, rep.row_ptr.p, rb.data(), ro.data());
  for (int r = 0; r < W; r++) {  // local row offsets -> offsets into the concatenated col
    const int64_t a = c.base[size_t(r)], m = c.base[size_t(r) + 1] - a;
    if (m > 0 && nnz_off[size_t(r)] > 0)
      k_add_i64<<<grid_n(m), 256, 0, c.stream>>>(rep.row_ptr.as<int64_t>() + a, m, nnz_off[size_t(r)]);
  }
  NBG_HIP(hipMemcpyAsync(rep.row_ptr.as<int64_t>() + N, &nnz_off[size_t(W)], 8, hipMemcpyHostToDevice, c.stream));
  if (any_ok) {  // rows whose keys sit outside hash(vid)'s part stay invisible on every replica
    ok_loc.alloc(size_t(loc.n_rows) + 64);
    if (loc.row_ok.p)
      NBG_HIP(hipMemcpyAsync(ok_loc.p, loc.row_ok.p, size_t(loc.n_rows), hipMemcpyDeviceToDevice, c.stream));
    else
      NBG_HIP(hipMemsetAsync(ok_loc.p, 1, size_t(loc.n_rows), c.stream));
    rep.row_ok.alloc(size_t(N) + 64);
    for (int r = 0; r < W; r++) {
      rb[size_t(r)] = size_t(c.base[size_t(r) + 1] - c.base[size_t(r)]);
      ro[size_t(r)] = size_t(c.base[size_t(r)]);
    }
    comm_allgatherv_bytes(c, ok_loc.p, size_t(loc.n_rows), rep.row_ok.p, rb.data(), ro.data());
  }
  NBG_HIP(hipGetLastError());
  NBG_HIP(hipStreamSynchronize(c.stream));
}

__global__ void k_rep_odeg(const int64_t* row_ptr, const uint8_t* row_ok, int64_t n, uint32_t* odeg) {
  for (int64_t v = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; v < n; v += int64_t(gridDim.x) * blockDim.x)
    odeg[v] = row_ok && !row_ok[v] ? 0u : uint32_t(row_ptr[v + 1] - row_ptr[v]);
}

void ensure_rep_out(Ctx& c, EdgeSpace& es) {
  if (es.has_rep_out && es.rep_odeg.p) return;
  if (!es.has_rep_out) replicate_csr(c, es.out, es.rep_out);
  es.has_rep_out = true;
  es.rep_odeg.alloc(size_t(std::max<int64_t>(c.n_global, 1)) * 4 + 64);
  k_rep_odeg<<<grid_n(c.n_global), 256, 0, c.stream>>>(es.rep_out.row_ptr.as<int64_t>(), es.rep_out.row_ok.as<uint8_t>(),
                                                      c.n_global, es.rep_odeg.as<uint32_t>());
  NBG_HIP(hipGetLastError());
}

// the grid that fills the device exactly once with blocks of `kernel` (its occupancy x CUs): a
// grid-stride scan over the chunks of a step then has no second, partial round of blocks
// (measured: 1024 blocks of the sweep 0.42 ms, its resident 1280 0.38 ms, 2048 0.43 ms)
static int cu_count() {
  static int cus = 0;
  if (cus == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        cus <= 0)
      cus = 256;
  }
  return cus;
}
static int resident_grid(const void* kernel, int block) {
  static std::mutex mu;
  static std::map<const void*, int> cache;
  std::lock_guard<std::mutex> lk(mu);
  auto it = cache.find(kernel);
  if (it != cache.end()) return it->second;
  int dev = 0, cus = 0, per = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
      hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kernel, block, 0) != hipSuccess || cus <= 0 || per <= 0)
    return cache[kernel] = 1024;
  return cache[kernel] = cus * per;
}

int32_t shortest_path_run(Ctx& c, int32_t et, const int64_t* src_all, const int64_t* dst_all, size_t npairs_all,
                          int32_t max_steps, nbg_rows* out) {
  if (!c.finalized) throw Error(NBG_E_STATE, "snapshot not finalized");
  if (et <= 0) throw Error(NBG_E_INVALID_ARG, "edge type must be > 0 (paths follow out-edges)");
  if (max_steps > 254) throw Error(NBG_E_UNSUPPORTED, "max_steps above 254");
  auto it = c.edges.find(et);
  if (it == c.edges.end()) throw Error(NBG_E_INVALID_ARG, "edge type not in snapshot");
  EdgeSpace& es = it->second;
  if (!es.out.row_ptr.p || !es.in.row_ptr.p) throw Error(NBG_E_STATE, "missing CSR");
  const Csr* cout = &es.out;
  const Csr* cin = &es.in;
  int64_t lo = c.owned_lo(), n = std::max<int64_t>(c.owned_hi() - lo, 1);
  const int64_t* src = src_all;
  const int64_t* dst = dst_all;
  size_t npairs = npairs_all;
  std::vector<int64_t> my_src, my_dst;
  if (c.sharded) {
    if (!es.has_rep) {
      if (!es.has_rep_out) replicate_csr(c, es.out, es.rep_out);
      es.has_rep_out = true;
      replicate_csr(c, es.in, es.rep_in);
      es.has_rep = true;
    }
    cout = &es.rep_out;
    cin = &es.rep_in;
    lo = 0;
    n = std::max<int64_t>(c.n_global, 1);
    for (size_t i = size_t(c.rank); i < npairs_all; i += size_t(c.world)) {
      my_src.push_back(src_all[i]);
      my_dst.push_back(dst_all[i]);
    }
    src = my_src.data();
    dst = my_dst.data();
    npairs = my_src.size();
  }

  // batch size: bounded by the distance arrays' HBM budget (2 bytes per pair and vertex)
  const int64_t budget = c.opt("sp_mem_mb", 96 * 1024) << 20;
  int64_t B = std::min<int64_t>(c.opt("sp_batch", 1024), std::max<int64_t>(1, budget / (2 * n)));
  B = std::max<int64_t>(1, std::min<int64_t>(B, std::max<int64_t>(int64_t(npairs), 1)));
  B = std::min<int64_t>(B, 0x7FFFFF);
  const size_t dist_bytes = ((size_t(B) * size_t(n) + 3) & ~size_t(3)) + 64;
  {
    // both sides' distance arrays in one block of 2 x dist_bytes: side 1 in its upper half, or
    // (option sp_ilv, default) interleaved with side 0 byte by byte.  Either layout is all 0xFF
    // between batches, so the option may change from call to call.
    PoolScope none(nullptr);  // the distance arrays live outside the query pool
    if (c.sp_dist_bytes < dist_bytes) {
      for (auto& d : c.sp_dist) d.release();
      c.sp_dist_bytes = 0;
      c.sp_dist[0].alloc(2 * dist_bytes);
      c.sp_dist_bytes = dist_bytes;
      c.sp_dirty = true;
    }
    if (c.sp_dirty) {
      NBG_HIP(hipMemsetAsync(c.sp_dist[0].p, 0xFF, 2 * c.sp_dist_bytes, c.stream));
      c.sp.dv_clean = false;  // a failed call may have left filter words and counters set too
    }
    c.sp_dirty = false;
  }
  Ctx::SpWork& W = c.sp;
  if (W.cap_state < B) {
    PoolScope none(nullptr);
    W.state.alloc(size_t(B) * 48 + 64);
    W.cnt.alloc(C_N * 8);
    W.vids.alloc(size_t(B) * 16);
    W.gidx.alloc(size_t(B) * 8);
    W.plist.alloc(size_t(B) * 4 + 64);
    W.cap_state = B;
  }
  PoolScope pool_scope(query_pool(c));
  c.timing = Timing{};
  c.tev_used = 0;
  c.hop_timing = c.opt("hop_timing", 1) != 0;  // event pairs around the scan launches (0: none)
  hipEventRecord(c.ev[0], c.stream);

  const int32_t ilv = c.opt("sp_ilv", 1) != 0 ? 1 : 0;
  uint8_t* d0 = c.sp_dist[0].as<uint8_t>();
  uint8_t* d1 = ilv ? d0 + 1 : d0 + c.sp_dist_bytes;
  auto deg16 = [&](int k, const Csr* g) -> const uint16_t* {
    if (g->n_rows <= 0) return nullptr;
    if (W.deg16_rp[k] != g->row_ptr.p || W.deg16_rows[k] != g->n_rows || W.deg16_commits[k] != c.commits) {
      PoolScope none(nullptr);  // kept across calls, outside the query pool
      W.deg16[k].alloc(size_t(g->n_rows) * 2 + 64);
      k_deg16<<<grid_n(g->n_rows), 256, 0, c.stream>>>(g->row_ptr.as<int64_t>(), g->row_ok.as<uint8_t>(), g->n_rows,
                                                       W.deg16[k].as<uint16_t>());
      NBG_HIP(hipGetLastError());
      W.deg16_rp[k] = g->row_ptr.p;
      W.deg16_rows[k] = g->n_rows;
      W.deg16_commits[k] = c.commits;
    }
    return W.deg16[k].as<uint16_t>();
  };
  SpCsr gout{cout->row_ptr.as<int64_t>(), cout->col.as<int32_t>(), cout->row_ok.as<uint8_t>(), deg16(0, cout)};
  SpCsr gin{cin->row_ptr.as<int64_t>(), cin->col.as<int32_t>(), cin->row_ok.as<uint8_t>(), deg16(1, cin)};
  const int64_t* vid_of = c.vid_of.as<int64_t>();
  unsigned long long* cnt = W.cnt.as<unsigned long long>();
  unsigned long long* hc = c.host_counters;  // pinned
  int64_t* dsv = W.vids.as<int64_t>();
  int64_t* dtv = dsv + B;
  int32_t* dgs = W.gidx.as<int32_t>();
  int32_t* dgt = dgs + B;
  const int64_t soft = std::max<int64_t>(c.opt("sp_list_soft", int64_t(16) << 20), 1024);
  const bool probe = c.opt("sp_probe", 1) != 0;

  std::vector<int64_t> hres(npairs), hoff(1, 0), hpath;
  std::vector<int32_t> hstate(static_cast<size_t>(2 * B)), hside(static_cast<size_t>(B)),
      hmet(static_cast<size_t>(B));
  // ---- device-driven batches (k_dv_*): fixed capacities sized once per context and batch size;
  // false = a list overflowed (the clean state is restored, the batch runs host-driven below)
  // (pair-major distance bytes only: the kernels address a pair's bytes from one row pointer)
  const bool dev = c.opt("sp_dev", 1) != 0 && max_steps <= kMaxQ - 2 && lo == 0 &&
                   B <= kPairLds;
  auto dv_event = [&]() -> size_t {
    if (!c.hop_timing) return ~size_t(0);
    if (c.tev_used == c.tev.size()) {
      hipEvent_t e;
      NBG_HIP(hipEventCreate(&e));
      c.tev.push_back(e);
    }
    NBG_HIP(hipEventRecord(c.tev[c.tev_used], c.stream));
    return c.tev_used++;
  };
  auto dv_ms = [&](size_t a, size_t b) -> double {
    float ms = 0;
    if (a == ~size_t(0) || b == ~size_t(0)) return 0.0;
    if (hipEventElapsedTime(&ms, c.tev[a], c.tev[b]) != hipSuccess) return 0.0;
    return ms;
  };
  // host block layout (coherent pinned): publish slots, the finish copy of every counter, the
  // pairs, then the results
  const int64_t dvB = std::max<int64_t>(W.dv_B, B);
  const size_t h_pub = 0, h_fin = h_pub + size_t(kMaxQ) * kPubW * 8, h_pairs = h_fin + size_t(kDevCnt + 64) * 8,
               h_sr = h_pairs + size_t(dvB) * 16, h_off = h_sr + ((size_t(dvB) * 8 + 63) & ~size_t(63)),
               h_path = h_off + size_t(dvB + 8) * 8, h_end = h_path + size_t(dvB) * (kMaxQ + 1) * 8;
  auto dv_pair_bytes = [](int64_t nb) {
    auto r = [](size_t b) { return (b + 63) & ~size_t(63); };
    const size_t b = size_t(nb);
    return r(b * 8) + r(b * 4) + r(b * 8) + r(b * 8) + r((b + 8) * 8) + 2 * r(b * kMaxQ * 8);
  };
  auto dv_alloc = [&]() {
    // the global filter (2^24 bits): off costs the expansions nothing but lets the pair filters'
    // false positives fetch a distance line each (sweep step 1: 3.4x its byte model, 1.1x with it)
    // below 2^5 bits: off; at least 2^7 bits otherwise (k_dv_clear zeroes the words 4 at a time)
    int64_t gf_log2 = std::min<int64_t>(std::max<int64_t>(c.opt("sp_gf_log2", 24), 0), 32);
    if (gf_log2 >= 5) gf_log2 = std::max<int64_t>(gf_log2, 7);
    const bool pf_on = c.opt("sp_pf", 1) != 0;
    const int64_t nnz = std::max(cout->nnz, cin->nnz);
    const int64_t soft_dv = std::max<int64_t>(c.opt("sp_dv_list", int64_t(8) << 20), 64);
    const int64_t cap = std::min<int64_t>(soft_dv, 2 * dvB * n + 64);
    const int64_t cap_ch = cap + nnz / 512 + 64, cap_wch = std::min<int64_t>(soft_dv, dvB * (nnz / kCh + 1)) + 64;
    if (W.dv_B >= dvB && W.dv_cap == cap && W.dv_cap_ch == cap_ch && W.dv_gf_log2 == gf_log2 && W.dv_pf_on == pf_on &&
        c.sp_host && c.sp_host_bytes >= h_end) {
      if (!W.dv_clean) {  // a failed call: every filter word and counter back to zero
        NBG_HIP(hipMemsetAsync(W.dv_cnt.p, 0, W.dv_cnt.bytes, c.stream));
        if (W.dv_pf.p) NBG_HIP(hipMemsetAsync(W.dv_pf.p, 0, W.dv_pf.bytes, c.stream));
        if (W.dv_gf.p) NBG_HIP(hipMemsetAsync(W.dv_gf.p, 0, W.dv_gf.bytes, c.stream));
        W.dv_clean = true;
      }
      return;
    }
    PoolScope none(nullptr);
    NBG_HIP(hipStreamSynchronize(c.stream));
    if (c.sp_host) (void)hipHostFree(c.sp_host);
    c.sp_host = nullptr;
    c.sp_host_bytes = 0;
    NBG_HIP(hipHostMalloc(&c.sp_host, h_end, hipHostMallocCoherent));
    memset(c.sp_host, 0, h_end);
    c.sp_host_bytes = h_end;
    W.dv_cnt = DevBuf();
    W.dv_cnt.alloc(size_t(kDevCnt) * kCS * 8);
    for (auto& b : W.dv_live) {
      b = DevBuf();
      b.alloc(size_t(cap) * 8);
    }
    for (DevBuf* b : {&W.dv_arena, &W.dv_meet, &W.dv_sw[0], &W.dv_sw[1], &W.dv_X, &W.dv_Xcb}) *b = DevBuf();
    W.dv_arena.alloc(size_t(2 * cap) * 8);
    W.dv_meet.alloc(size_t(cap) * 8);
    W.dv_sw[0].alloc(size_t(cap) * 8);
    W.dv_sw[1].alloc(size_t(cap) * 8);
    W.dv_X.alloc(size_t(cap) * 8);
    W.dv_Xcb.alloc(size_t(cap) * 8);
    for (DevBuf* b : {&W.dv_chx, &W.dv_slot, &W.dv_wchx, &W.dv_pair, &W.dv_path, &W.dv_pf, &W.dv_gf}) *b = DevBuf();
    W.dv_chx.alloc(size_t(cap_ch) * 4);
    W.dv_slot.alloc(size_t(cap_ch) * 8);
    W.dv_wchx.alloc(size_t(cap_wch) * 4);
    // per pair (the layout run_dev carves, each piece rounded up to 64 bytes): gs [2B] i32, cur [B]
    // i32, best [B] i64, wcb [B] i64, doff [B + 8] i64, pull [kMaxQ][B] u64, push [kMaxQ][B] u64
    W.dv_pair.alloc(dv_pair_bytes(dvB));
    W.dv_path.alloc(size_t(dvB) * (kMaxQ + 1) * 8);
    if (pf_on) W.dv_pf.alloc(size_t(2 * kLv) * size_t(dvB) * 512);
    if (gf_log2 >= 5) W.dv_gf.alloc(size_t(1) << (gf_log2 - 3));
    NBG_HIP(hipMemsetAsync(W.dv_cnt.p, 0, W.dv_cnt.bytes, c.stream));
    if (W.dv_pf.p) NBG_HIP(hipMemsetAsync(W.dv_pf.p, 0, W.dv_pf.bytes, c.stream));
    if (W.dv_gf.p) NBG_HIP(hipMemsetAsync(W.dv_gf.p, 0, W.dv_gf.bytes, c.stream));
    W.dv_B = dvB;
    W.dv_cap = cap;
    W.dv_cap_ch = cap_ch;
    W.dv_cap_wch = cap_wch;
    W.dv_gf_log2 = gf_log2;
    W.dv_pf_on = pf_on;
    W.dv_clean = true;
  };
  auto run_dev = [&](size_t b0, int64_t nb) -> bool {
    int32_t nl = 0;  // kernel launches of the batch (nbg_timing.launches)
    dv_alloc();
    W.dv_clean = false;  // until the batch's finish launch (or the abort below) restores it
    char* hb = static_cast<char*>(c.sp_host);
    SpState st{};
    st.B = int32_t(nb);
    sp_state_carve(W.state, nb, st);
    st.ilv = ilv;
    SpFilt f{};
    f.pf = W.dv_pf.as<uint32_t>();
    f.gf = W.dv_gf.as<uint32_t>();
    f.gshift = W.dv_gf.p ? uint32_t(64 - (W.dv_gf_log2 - 5)) : 0u;
    f.B = int32_t(nb);
    f.diag = int32_t(c.opt("sp_dv_diag", 0));
    SpDev d{};
    d.cnt = W.dv_cnt.as<unsigned long long>();
    for (int k = 0; k < 4; k++) d.live[k >> 1][k & 1] = W.dv_live[k].as<uint64_t>();
    d.cap_live = W.dv_cap;
    d.arena = W.dv_arena.as<uint64_t>();
    d.cap_arena = 2 * W.dv_cap;
    d.meet = W.dv_meet.as<uint64_t>();
    d.cap_meet = W.dv_cap;
    d.sw[0] = W.dv_sw[0].as<uint64_t>();
    d.sw[1] = W.dv_sw[1].as<uint64_t>();
    d.cap_sw = W.dv_cap;
    d.X = W.dv_X.as<uint64_t>();
    d.Xcb = W.dv_Xcb.as<int64_t>();
    d.cap_x = W.dv_cap;
    d.chx = W.dv_chx.as<int32_t>();
    d.slot = W.dv_slot.as<uint64_t>();
    d.cap_ch = W.dv_cap_ch;
    d.wchx = W.dv_wchx.as<int32_t>();
    d.cap_wch = W.dv_cap_wch;
    {
      Carve cv(W.dv_pair, "shortest path: per-pair workspace");
      d.gs = cv.take<int32_t>(size_t(nb) * 8);
      d.cur = cv.take<int32_t>(size_t(nb) * 4);
      d.best = cv.take<long long>(size_t(nb) * 8);
      d.wcb = cv.take<int64_t>(size_t(nb) * 8);
      d.doff = cv.take<int64_t>(size_t(nb + 8) * 8);
      d.pull = cv.take<unsigned long long>(size_t(nb) * kMaxQ * 8);
      d.push = cv.take<unsigned long long>(size_t(nb) * kMaxQ * 8);  // adjacent: k_dv_begin clears both in one pass
    }
    d.path = W.dv_path.as<int64_t>();
    d.lg_chb = 10;  // 1024-entry chunks
    d.lg_chs = 10;
    int64_t* hp = reinterpret_cast<int64_t*>(hb + h_pairs);
    memcpy(hp, src + b0, size_t(nb) * 8);
    memcpy(hp + nb, dst + b0, size_t(nb) * 8);
    d.h_pairs = hp;
    d.h_sr = reinterpret_cast<int32_t*>(hb + h_sr);
    d.h_off = reinterpret_cast<int64_t*>(hb + h_off);
    d.h_path = reinterpret_cast<int64_t*>(hb + h_path);
    auto pub = [&](int it) { return reinterpret_cast<unsigned long long*>(hb + h_pub) + size_t(it) * kPubW; };
    unsigned long long* fin = reinterpret_cast<unsigned long long*>(hb + h_fin);

    auto gsel = [&](const void* k) { return resident_grid(k, kBlk); };
    // scan grids: option sp_dv_grid, else each kernel's resident grid
    const int64_t grid_opt = c.opt("sp_dv_grid", 0);
    auto gsz = [&](const void* k) { return grid_opt > 0 ? int(grid_opt) : resident_grid(k, 256); };
    // the meet probe at 5 blocks per CU (its resident 8 ran the third iteration at 0.29 ms, 5: 0.22)
    auto gpr = [&](const void* k) {
      return grid_opt > 0 ? int(grid_opt) : std::min(resident_grid(k, 256), 5 * cu_count());
    };
    const int occ = int(c.opt("sp_dv_occ", 1));
    const int32_t pf_agg = 1;
    // expansion waves per BFS chunk: 256-entry sub-chunks
    const int32_t lg_sub = std::max<int32_t>(0, d.lg_chb - 8);
    const int max_it = std::min<int>(max_steps, kMaxQ - 2);
    const int64_t htm = int64_t(c.ht_cap - 1);
    const int64_t* htk = c.ht_keys.as<int64_t>();
    const int32_t* htv = c.ht_vals.as<int32_t>();
    std::vector<uint64_t> seq(size_t(kMaxQ), 0);
    std::vector<std::array<size_t, 3>> evi(size_t(kMaxQ), {~size_t(0), ~size_t(0), ~size_t(0)});
    std::vector<std::array<size_t, 2>> evs(size_t(kMaxQ), {~size_t(0), ~size_t(0)});
    std::vector<std::array<size_t, 2>> evw(size_t(kMaxQ), {~size_t(0), ~size_t(0)});

    // the state is restored from whatever the device reached: the claimed bytes from the arena
    // (wholesale when it overflowed, or `wipe`), every filter word and counter cleared; the batch
    // then runs host-driven
    auto dv_abort = [&](bool wipe) {
      NBG_HIP(hipStreamSynchronize(c.stream));
      unsigned long long na = 0;
      NBG_HIP(hipMemcpy(&na, gcnt(d.cnt, D_ARENA), 8, hipMemcpyDeviceToHost));
      if (!wipe && int64_t(na) <= d.cap_arena) {
        if (na) k_sp_clear<<<grid_n(int64_t(na)), 256, 0, c.stream>>>(d.arena, int64_t(na), d0, d1, n, st);
      } else {
        NBG_HIP(hipMemsetAsync(c.sp_dist[0].p, 0xFF, 2 * c.sp_dist_bytes, c.stream));
      }
      NBG_HIP(hipMemsetAsync(W.dv_cnt.p, 0, W.dv_cnt.bytes, c.stream));
      if (W.dv_pf.p) NBG_HIP(hipMemsetAsync(W.dv_pf.p, 0, W.dv_pf.bytes, c.stream));
      if (W.dv_gf.p) NBG_HIP(hipMemsetAsync(W.dv_gf.p, 0, W.dv_gf.bytes, c.stream));
      NBG_HIP(hipGetLastError());
      NBG_HIP(hipStreamSynchronize(c.stream));
      W.dv_clean = true;
      return false;
    };

    ++nl;
    // iteration 1's select folded into the batch start (option sp_dv_begin_x)
    const int32_t sel1 = c.opt("sp_dv_begin_x", 1) != 0 ? 1 : 0;
    k_dv_begin<<<std::max(grid_n(nb, 1 << 20), 64), 256, 0, c.stream>>>(d, st, gout, gin, d0, d1, n, max_steps, htk, htv,
                                                          uint64_t(htm), c.ht_has_min, c.ht_min_gidx, sel1);
    auto enqueue = [&](int it) {
      if (it > 1 || !sel1) {
        ++nl;
        // (at 6 / 8 waves per SIMD, 104 / 176 B spilled: C4 1.133-1.154 -> 1.176-1.197 ms, c4occ3)
        k_dv_select<<<gsel((const void*)k_dv_select), kBlk, 0, c.stream>>>(d, st, gout, gin, it);
      }
      evi[size_t(it)][0] = dv_event();
      if (probe) {
        ++nl;
        // 4 entries per lane and step (8 / 16 measured slower: 0.50 -> 0.70 ms, round 3)
        k_dv_probe<4><<<gpr((const void*)k_dv_probe<4>), 256, 0, c.stream>>>(d, st, f, gout, gin, d0, d1, n, lo, it);
      }
      evi[size_t(it)][1] = dv_event();
      ++nl;
      if (occ >= 8)
        k_dv_expand<8><<<gsz((const void*)k_dv_expand<8>), 256, 0, c.stream>>>(d, st, f, gout, gin, d0, d1, n, lo, it,
                                                                               lg_sub, pf_agg);
      else
        k_dv_expand<1><<<gsz((const void*)k_dv_expand<1>), 256, 0, c.stream>>>(d, st, f, gout, gin, d0, d1, n, lo, it,
                                                                               lg_sub, pf_agg);
      evi[size_t(it)][2] = dv_event();
      seq[size_t(it)] = ++c.pub_seq;
      ++nl;
      k_dv_step<<<grid_n(nb, 1 << 20), 256, 0, c.stream>>>(d, st, max_steps, it, pub(it), seq[size_t(it)]);
      NBG_HIP(hipGetLastError());
    };
    enqueue(1);
    int it = 1;
    for (;; it++) {
      if (it < max_it) enqueue(it + 1);  // speculative: a no-op when iteration it ends the BFS
      wait_host_word(c, pub(it) + kPubW - 1, seq[size_t(it)]);
      const unsigned long long* hs = pub(it);
      if (hs[D_OVF]) return dv_abort(false);
      if (hs[D_G + Q_ACTIVE] == 0 || it >= max_it) break;
    }
    const int64_t maxL = int64_t(pub(it)[D_MAXL]), maxF = int64_t(pub(it)[D_MAXF]);
    const int iters = it;
    ++nl;
    k_dv_post<<<int(std::max<int64_t>(1, 512)), kBlk, 0, c.stream>>>(
        d, st, gout, gin, lo, htk, htv, uint64_t(htm), c.ht_has_min, c.ht_min_gidx);
    const int nsw = int(std::min<int64_t>(std::max<int64_t>(maxF - 1, 0), kMaxQ - 2));
    const unsigned long long bias16 = (unsigned long long)std::max<int64_t>(0, 16);
    // the sweep at 6 waves per SIMD (80 VGPRs, 12 B spilled): C4 1.164 -> 1.140 ms against the
    // register-bound 5 (8: 64 VGPRs, 76 B spilled, 1.155; 8 entries per lane: 1.211; c4occ)
    const int sw_occ = int(c.opt("sp_sweep_occ", 6));
    for (int j = 1; j <= nsw; j++) {
      ++nl;
      k_dv_sweep_select<<<gsel((const void*)k_dv_sweep_select), kBlk, 0, c.stream>>>(d, st, gout, gin, j, bias16);
      evs[size_t(j)][0] = dv_event();
      ++nl;
      switch (sw_occ) {
        case 6: k_dv_sweep<4, 6><<<gsz((const void*)k_dv_sweep<4, 6>), 256, 0, c.stream>>>(d, st, f, gout, gin, d0, d1, n, lo, j); break;
        case 8: k_dv_sweep<4, 8><<<gsz((const void*)k_dv_sweep<4, 8>), 256, 0, c.stream>>>(d, st, f, gout, gin, d0, d1, n, lo, j); break;
        case 2: k_dv_sweep<8, 1><<<gsz((const void*)k_dv_sweep<8, 1>), 256, 0, c.stream>>>(d, st, f, gout, gin, d0, d1, n, lo, j); break;
        default: k_dv_sweep<4><<<gsz((const void*)k_dv_sweep<4>), 256, 0, c.stream>>>(d, st, f, gout, gin, d0, d1, n, lo, j);
      }
      evs[size_t(j)][1] = dv_event();
    }
    const int nwalk = int(std::min<int64_t>(maxL >= 2 ? maxL - 1 : 0, kMaxQ - 2));
    for (int i = 0; i < nwalk; i++) {
      if (i > 0) {
        ++nl;
        k_dv_walk_front<<<grid_n(nb, 1 << 20), kBlk, 0, c.stream>>>(d, st, gout, i, lo, htk, htv, uint64_t(htm),
                                                                   c.ht_has_min, c.ht_min_gidx);
      }
      evw[size_t(i)][0] = dv_event();
      ++nl;
      k_dv_walk_scan<<<gsz((const void*)k_dv_walk_scan), 256, 0, c.stream>>>(d, st, f, gout, d1, vid_of, n, lo, i);
      evw[size_t(i)][1] = dv_event();
    }
    ++nl;
    k_dv_out<<<grid_n(nb, 1 << 20), 256, 0, c.stream>>>(d, st, nwalk - 1);
    const uint64_t fseq = ++c.pub_seq;
    // BFS blocks written: 0 .. iters, plus the speculative iteration after the last
    const int32_t nbfs = std::min<int32_t>(iters + (iters < max_it ? 2 : 1), kMaxQ);
    ++nl;
    k_dv_finish<<<1, 64, 0, c.stream>>>(d.cnt, fin, fin + kDevCnt + 8, fseq, nbfs, nsw, nwalk);
    ++nl;
    k_dv_clear<<<gsz((const void*)k_dv_clear), 256, 0, c.stream>>>(d, st, f, d0, d1, n);
    NBG_HIP(hipGetLastError());
    wait_host_word(c, fin + kDevCnt + 8, fseq);
    W.dv_clean = true;  // the finish launch cleared the counters, the clear launch (queued) the bytes and filters
    if (fin[D_OVF]) {
      // a sweep or walk list overflowed after the BFS: the result pass reset every byte and
      // filter word the arena holds, unless the arena itself overflowed
      if (int64_t(fin[D_ARENA]) > d.cap_arena) return dv_abort(true);
      return false;
    }
    c.timing.launches += nl;
    if (fin[D_WALKERR] && !(f.diag & 4))
      throw Error(NBG_E_UNKNOWN, "shortest path: in-edge keys without mirrored out-edges on a shortest path");

    // per-launch records (modes 3 = meet probe, 2 = BFS expansion, 4 = sweep), from the copy of
    // every counter the finish launch made
    auto blkq = [&](int q) { return fin + D_G + size_t(q) * Q_W; };
    if (c.hop_timing && c.tev_used) (void)hipEventSynchronize(c.tev[c.tev_used - 1]);
    for (int i = 1; i <= iters; i++) {
      const unsigned long long* q = blkq(i);
      const unsigned long long act = blkq(i - 1)[Q_ACTIVE];
      if (act == 0) continue;
      c.timing.steps_run++;
      const double pms = dv_ms(evi[size_t(i)][0], evi[size_t(i)][1]), ems = dv_ms(evi[size_t(i)][1], evi[size_t(i)][2]);
      if (probe && q[Q_X]) {
        c.timing.expand_ms += pms;
        c.timing.expand_launches++;
        c.timing.edges_scanned += q[Q_PE];
        c.timing.expand_bytes += q[Q_X] * 24 + q[Q_PE] * 5;
        // (diag bit 3: c[2] distance bytes read, c[6] pair-filter passes, c[7] bytes at the depth)
        const unsigned long long c8[8] = {q[Q_X], q[Q_PE], q[Q_W - 2], fin[D_MEET], (unsigned long long)i, act,
                                          q[Q_W - 3], q[Q_W - 1]};
        c.timing.hop(3, false, pms, c8);
        c.timing.name_last_hop("nbg::(anonymous namespace)::k_dv_probe");
      }
      if (q[Q_EE]) {
        c.timing.expand_ms += ems;
        c.timing.expand_launches++;
        c.timing.edges_scanned += q[Q_EE];
        c.timing.expand_bytes += q[Q_X] * 32 + q[Q_EE] * 5 + q[Q_CLAIMS] * 26;
        const unsigned long long c8[8] = {q[Q_X], q[Q_EE], q[Q_CLAIMS], fin[D_MEET], (unsigned long long)i, act, 0, 0};
        c.timing.hop(2, false, ems, c8);
        c.timing.name_last_hop("nbg::(anonymous namespace)::k_dv_expand");
      }
    }
    for (int j = 1; j <= nsw; j++) {
      const unsigned long long* q = blkq(kSwQ + j);
      if (!q[Q_EE]) continue;
      const double sms = dv_ms(evs[size_t(j)][0], evs[size_t(j)][1]);
      c.timing.expand_ms += sms;
      c.timing.expand_launches++;
      c.timing.edges_scanned += q[Q_EE];
      c.timing.expand_bytes += q[Q_X] * 32 + q[Q_EE] * 6 + q[Q_CLAIMS] * 18;
      const unsigned long long c8[8] = {q[Q_X], q[Q_EE], q[Q_CLAIMS], fin[D_MEET], (unsigned long long)j, 0, 0, 0};
      c.timing.hop(4, false, sms, c8);
      c.timing.name_last_hop("nbg::(anonymous namespace)::k_dv_sweep");
    }
    // walk scans (mode 5): the out-rows of every walking pair's current vertex; not counted in
    // edges_scanned (the traversal's entries), in the scan kernels' time and bytes
    for (int i = 0; i < nwalk; i++) {
      const unsigned long long* q = blkq(kWkQ + i);
      if (!q[Q_EE]) continue;
      const double wms = dv_ms(evw[size_t(i)][0], evw[size_t(i)][1]);
      c.timing.expand_ms += wms;
      c.timing.expand_launches++;
      c.timing.expand_bytes += q[Q_NCH] * 24 + q[Q_EE] * 5;
      const unsigned long long c8[8] = {q[Q_NCH], q[Q_EE], 0, fin[D_MEET], (unsigned long long)i, 0, 0, 0};
      c.timing.hop(5, false, wms, c8);
      c.timing.name_last_hop("nbg::(anonymous namespace)::k_dv_walk_scan");
    }

    // results (the ends of each path are the host's)
    const int32_t* hsr = d.h_sr;
    const int64_t* hoffb = d.h_off;
    const int64_t plen = hoffb[nb];
    const size_t base = hpath.size();
    hpath.resize(base + size_t(plen));
    if (plen > 0) memcpy(hpath.data() + base, d.h_path, size_t(plen) * 8);
    for (int64_t p = 0; p < nb; p++) {
      const int32_t L = hsr[p] == SP_ACTIVE ? -1 : hsr[nb + p];
      hres[b0 + size_t(p)] = L;
      if (L >= 0) {
        hpath[base + size_t(hoffb[p])] = src[b0 + size_t(p)];
        if (L > 0) hpath[base + size_t(hoffb[p] + L)] = dst[b0 + size_t(p)];
      }
      hoff.push_back(hoff.back() + hoffb[p + 1] - hoffb[p]);
    }
    return true;
  };
  c.sp_dirty = true;  // until the batch's bytes are reset
  for (size_t b0 = 0; b0 < npairs; b0 += size_t(B)) {
    const int64_t nb = std::min<int64_t>(B, int64_t(npairs - b0));
    if (dev && run_dev(b0, nb)) {
      c.timing.spec_hops++;  // nbg_timing.spec_hops of a shortest-path call: batches run device-driven
      continue;
    }
    SpState st{};
    st.B = int32_t(nb);
    sp_state_carve(W.state, nb, st);
    st.ilv = ilv;
    if (c.opt("sp_lvbits", 1) != 0) {  // level filter: 2 * kLv maps, cleared per batch
      // bits per level: the power of two >= n, capped (option sp_lvbits_log2, default 23)
      const int cap = int(std::min<int64_t>(std::max<int64_t>(23, 5), 31));
      int lg = 5;
      while (lg < cap && (int64_t(1) << lg) < n) lg++;
      const int64_t lvw = (int64_t(1) << lg) / 32;
      st.lvmask = uint32_t((uint64_t(1) << lg) - 1);
      const size_t lvb = size_t(2 * kLv) * size_t(lvw) * 4;
      if (W.lvbits.bytes < lvb) {
        PoolScope none(nullptr);
        W.lvbits.alloc(lvb);
      }
      NBG_HIP(hipMemsetAsync(W.lvbits.p, 0, lvb, c.stream));
      st.lvbits = W.lvbits.as<uint32_t>();
      st.lvw = lvw;
    }
    if (c.host_stage && c.host_stage_used == 0 && size_t(nb) * 16 <= kHostStageBytes) {
      // through the pinned stage: a pageable source makes the copy wait on the host (the stage's
      // previous contents, the last batch's results, were read back before this point)
      int64_t* hs = static_cast<int64_t*>(c.host_stage);
      memcpy(hs, src + b0, size_t(nb) * 8);
      memcpy(hs + nb, dst + b0, size_t(nb) * 8);
      NBG_HIP(hipMemcpyAsync(dsv, hs, size_t(nb) * 8, hipMemcpyHostToDevice, c.stream));
      NBG_HIP(hipMemcpyAsync(dtv, hs + nb, size_t(nb) * 8, hipMemcpyHostToDevice, c.stream));
    } else {
      NBG_HIP(hipMemcpyAsync(dsv, src + b0, size_t(nb) * 8, hipMemcpyHostToDevice, c.stream));
      NBG_HIP(hipMemcpyAsync(dtv, dst + b0, size_t(nb) * 8, hipMemcpyHostToDevice, c.stream));
    }
    lookup_gidx(c, dsv, dgs, nb);
    lookup_gidx(c, dtv, dgt, nb);
    NBG_HIP(hipMemsetAsync(cnt, 0, C_N * 8, c.stream));
    for (int s = 0; s < 2; s++) reserve(c, W.live_next[s], W.cap_next[s], nb + 64, 0);
    reserve(c, W.arena, W.cap_arena, 2 * nb + 64, 0);
    reserve(c, W.meet, W.cap_meet, 4096, 0);
    SpBufs bf{};
    auto refresh = [&](DevBuf* sweep_next, int64_t cap_sweep_next) {
      bf.live_next[0] = W.live_next[0].as<uint64_t>();
      bf.live_next[1] = W.live_next[1].as<uint64_t>();
      bf.arena = W.arena.as<uint64_t>();
      bf.meet = W.meet.as<uint64_t>();
      bf.cap_live[0] = W.cap_next[0];
      bf.cap_live[1] = W.cap_next[1];
      bf.cap_arena = W.cap_arena;
      bf.cap_meet = W.cap_meet;
      bf.sweep_next = sweep_next ? sweep_next->as<uint64_t>() : nullptr;
      bf.cap_sweep = sweep_next ? cap_sweep_next : 0;
    };
    // the counters on the host (publish kernel + spin, traverse.hip: a memcpy + stream sync
    // round trip cost ~20 us per call, ~15 calls per batch)
    auto sync_counters = [&]() { fetch_counters(c, cnt, C_N, hc); };
    auto zero = [&](uint32_t mask, int64_t* xdeg = nullptr) {
      k_cnt_zero<<<1, 64, 0, c.stream>>>(cnt, mask, xdeg);
    };
    auto set_counter = [&](int which, int64_t v) {
      hc[32] = (unsigned long long)v;
      NBG_HIP(hipMemcpyAsync(cnt + which, hc + 32, 8, hipMemcpyHostToDevice, c.stream));
      NBG_HIP(hipStreamSynchronize(c.stream));
    };
    auto ensure_x = [&](int64_t need) {
      if (need + 1 > W.cap_x) {
        PoolScope none(nullptr);
        W.cap_x = std::max<int64_t>(need + need / 4 + 64, 1 << 16);
        W.X.alloc(size_t(W.cap_x) * 8);
        W.Xdeg.alloc(size_t(W.cap_x + 1) * 8);
        W.Xoff.alloc(size_t(W.cap_x + 1) * 8);
      }
    };
    auto launch_scan = [&](int64_t nX, bool sentinel_zero = false) {
      size_t tb = 0;
      if (!sentinel_zero) zero(0u, W.Xdeg.as<int64_t>() + nX);
      NBG_HIP(rocprim::exclusive_scan(nullptr, tb, W.Xdeg.as<int64_t>(), W.Xoff.as<int64_t>(), int64_t(0),
                                      size_t(nX + 1), rocprim::plus<int64_t>(), c.stream));
      c.ws_tmp.ensure(tb);
      NBG_HIP(rocprim::exclusive_scan(c.ws_tmp.p, tb, W.Xdeg.as<int64_t>(), W.Xoff.as<int64_t>(), int64_t(0),
                                      size_t(nX + 1), rocprim::plus<int64_t>(), c.stream));
    };
    auto launch_expand = [&](int64_t nX, int64_t E, int32_t sweep_mode) {
      SpExpand a{};
      a.X = W.X.as<uint64_t>();
      a.nX = nX;
      a.off = W.Xoff.as<int64_t>();
      a.g[0] = gout;
      a.g[1] = gin;
      a.dist[0] = d0;
      a.dist[1] = d1;
      a.vid_of = vid_of;
      a.n = n;
      a.lo = lo;
      a.sweep = sweep_mode;
      const int64_t tiles = (E + kTileE - 1) / kTileE;
      const int grid = int(std::max<int64_t>(1, std::min<int64_t>(tiles, 256 * 8)));
      hipEventRecord(c.ev[2], c.stream);
      a.tile_row = nullptr;
      if (nX < (int64_t(1) << 31)) {
        if (W.tile_rows.bytes < size_t(tiles + 2) * 4) {
          PoolScope none(nullptr);
          W.tile_rows.alloc(size_t(tiles + tiles / 4 + 64) * 4);
        }
        a.tile_row = W.tile_rows.as<int32_t>();
        k_tile_rows<kTileE><<<int(std::max<int64_t>(1, std::min<int64_t>((nX + 255) / 256, 4096))), 256, 0, c.stream>>>(
            a.off, nX, W.tile_rows.as<int32_t>());
      }
      k_sp_expand<<<grid, kT, 0, c.stream>>>(a, st, bf, cnt);
      NBG_HIP(hipGetLastError());
      hipEventRecord(c.ev[3], c.stream);
    };
    auto expand_time = [&]() -> double {
      float ms = 0;
      hipEventElapsedTime(&ms, c.ev[2], c.ev[3]);
      c.timing.expand_ms += ms;
      c.timing.expand_launches++;
      return ms;
    };
    // per-launch record in the hop stats: mode 2 = BFS expansion, 3 = meet probe, 4 = sweep;
    // c[] = {X tuples, adjacency entries, claims, meets (total so far), iteration, active pairs}
    unsigned long long diag[2] = {0, 0};  // (c[6], c[7] of the sweep records: unused since round 6)
    auto sp_hop = [&](int32_t mode, double ms, int64_t nX, int64_t E, int64_t claims, int64_t it, int64_t act) {
      const unsigned long long c8[8] = {(unsigned long long)nX, (unsigned long long)E, (unsigned long long)claims,
                                        hc[C_MEET], (unsigned long long)it, (unsigned long long)act, diag[0], diag[1]};
      diag[0] = diag[1] = 0;
      c.timing.hop(mode, false, ms, c8);
      c.timing.name_last_hop(mode == 3   ? "nbg::(anonymous namespace)::k_sp_probe"
                             : mode == 4 && c.opt("sp_sweep_chunks", 1) != 0 ? "nbg::(anonymous namespace)::k_sp_sweep"
                                                                             : "nbg::(anonymous namespace)::k_sp_expand");
    };
    // pairs (of this batch) matching a host predicate over (state, pside, met) -> W.plist
    auto pair_list = [&](auto pred) -> int32_t {
      NBG_HIP(hipMemcpyAsync(hstate.data(), st.state, size_t(nb) * 4, hipMemcpyDeviceToHost, c.stream));
      NBG_HIP(hipMemcpyAsync(hside.data(), st.pside, size_t(nb) * 4, hipMemcpyDeviceToHost, c.stream));
      NBG_HIP(hipMemcpyAsync(hmet.data(), st.met, size_t(nb) * 4, hipMemcpyDeviceToHost, c.stream));
      NBG_HIP(hipStreamSynchronize(c.stream));
      std::vector<int32_t> pl;
      for (int32_t p = 0; p < int32_t(nb); p++)
        if (pred(hstate[size_t(p)], hside[size_t(p)], hmet[size_t(p)])) pl.push_back(p);
      if (!pl.empty())
        NBG_HIP(hipMemcpy(W.plist.p, pl.data(), pl.size() * 4, hipMemcpyHostToDevice));
      return int32_t(pl.size());
    };
    auto regen = [&](int mode, int side, int32_t j, int32_t np, uint64_t* outl, int64_t cap, int which) {
      if (np == 0) return;
      dim3 grid(unsigned(std::min<int64_t>((n + 255) / 256, 1024)), unsigned(std::min<int32_t>(np, 65535)));
      k_sp_regen<<<grid, 256, 0, c.stream>>>(mode, side, j, W.plist.as<int32_t>(), np, st, d0, d1, n, outl, cap, cnt,
                                             which);
      NBG_HIP(hipGetLastError());
    };

    k_sp_init<<<grid_n(nb, 1 << 20), 256, 0, c.stream>>>(dsv, dtv, dgs, dgt, int32_t(nb), max_steps, n, st, gout, gin,
                                                         d0, d1, (refresh(nullptr, 0), bf), cnt);
    k_sp_step<<<grid_n(nb, 1 << 20), 256, 0, c.stream>>>(st, max_steps, 1, 0, cnt);
    NBG_HIP(hipGetLastError());
    sync_counters();
    int64_t n_live[2] = {int64_t(hc[C_LIVE0]), int64_t(hc[C_LIVE1])};
    int64_t n_arena = int64_t(hc[C_ARENA]), n_meet = 0;
    int64_t active = int64_t(hc[C_ACTIVE]);
    int64_t last_claims = 0;
    bool arena_lost = false;
    for (int s = 0; s < 2; s++) {
      std::swap(W.live[s], W.live_next[s]);
      std::swap(W.cap_live[s], W.cap_next[s]);
    }
    int32_t iter = 0;
    while (active > 0) {
      iter++;
      c.timing.steps_run++;
      // live lists -> X (expanding side) + carried tuples
      ensure_x(n_live[0] + n_live[1]);
      for (int s = 0; s < 2; s++) reserve(c, W.live_next[s], W.cap_next[s], n_live[s] + 64, 0);
      refresh(nullptr, 0);
      zero(1u << C_LIVE0 | 1u << C_LIVE1 | 1u << C_X | 1u << C_ACTIVE | 1u << C_OVF | 1u << C_XE);
      for (int s = 0; s < 2; s++)
        if (n_live[s])
          k_sp_select<<<grid_sel(n_live[s]), kBlk, 0, c.stream>>>(W.live[s].as<uint64_t>(), n_live[s], 0, st, gout, gin,
                                                                 W.X.as<uint64_t>(), W.Xdeg.as<int64_t>(), W.cap_x, bf,
                                                                 cnt);
      NBG_HIP(hipGetLastError());
      sync_counters();
      if (hc[C_OVF] & 2) throw Error(NBG_E_UNKNOWN, "shortest path: frontier list overflow");
      const int64_t nX = int64_t(hc[C_X]);
      int64_t E = int64_t(hc[C_XE]);
      const int64_t carried[2] = {int64_t(hc[C_LIVE0]), int64_t(hc[C_LIVE1])};
      // The probe's results (meets, claims, the dropped pairs' degrees) are read with the
      // iteration's last counter fetch: the expansion is sized by the pre-probe E (an upper
      // bound; it reads its own E from the scan on the device) and the lists keep room for
      // every probe claim, so no round trip separates the probe from the expansion.
      DevBuf ch, choff, slot, chx;  // live until the fetch below (stream-ordered reuse aside)
      int64_t max_chunks = 0;
      const bool probed = E > 0 && probe;
      if (probed) {
        // meet probe: pairs one edge short of meeting skip this iteration's expansion
        max_chunks = nX + E / kProbeCh + 64;
        reserve(c, W.meet, W.cap_meet, n_meet + max_chunks, n_meet);
        if (!arena_lost) reserve(c, W.arena, W.cap_arena, n_arena + max_chunks, n_arena);
        refresh(nullptr, 0);
        ch.alloc(size_t(nX + 1) * 8);
        choff.alloc(size_t(nX + 1) * 8);
        slot.alloc(size_t(max_chunks) * 8);
        k_sp_chunks<<<grid_n(nX + 1), 256, 0, c.stream>>>(W.Xdeg.as<int64_t>(), nX, ch.as<int64_t>(), cnt);
        size_t tb = 0;
        NBG_HIP(rocprim::exclusive_scan(nullptr, tb, ch.as<int64_t>(), choff.as<int64_t>(), int64_t(0),
                                        size_t(nX + 1), rocprim::plus<int64_t>(), c.stream));
        c.ws_tmp.ensure(tb);
        NBG_HIP(rocprim::exclusive_scan(c.ws_tmp.p, tb, ch.as<int64_t>(), choff.as<int64_t>(), int64_t(0),
                                        size_t(nX + 1), rocprim::plus<int64_t>(), c.stream));
        hipEventRecord(c.ev[4], c.stream);
        const int pgrid =
            int(std::max<int64_t>(1, std::min<int64_t>((max_chunks + 3) / 4, 4096)));
        chx.alloc(size_t(max_chunks) * 4);
        k_chunk_x<<<grid_n(nX), 256, 0, c.stream>>>(choff.as<int64_t>(), nX, chx.as<int32_t>(), slot.as<uint64_t>());
        k_sp_probe<1><<<pgrid, 256, 0, c.stream>>>(W.X.as<uint64_t>(), nX, choff.as<int64_t>(), chx.as<int32_t>(),
                                                     gout, gin, d0, d1, n, lo, st, slot.as<uint64_t>(), cnt);
        k_sp_gather_meets<<<grid_sel(max_chunks), kBlk, 0, c.stream>>>(slot.as<uint64_t>(), max_chunks, st, bf, cnt,
                                                                       choff.as<int64_t>() + nX);
        k_sp_probe_end<<<grid_n(std::max<int64_t>(nb, nX)), 256, 0, c.stream>>>(st, iter, W.X.as<uint64_t>(),
                                                                                W.Xdeg.as<int64_t>(), nX, cnt);
        NBG_HIP(hipGetLastError());
        hipEventRecord(c.ev[5], c.stream);
      }
      // the probe's meets and claims are at most one per chunk
      const int64_t meet_keep = n_meet + max_chunks, arena_keep = n_arena + max_chunks;
      if (E > 0) {
        // lists sized for min(every edge claims, a soft bound); an overflow is rebuilt below
        const int64_t want = std::min<int64_t>(E, std::max<int64_t>(soft, 2 * last_claims)) + 64;
        for (int s = 0; s < 2; s++) reserve(c, W.live_next[s], W.cap_next[s], carried[s] + want, carried[s]);
        if (!arena_lost)
          reserve(c, W.arena, W.cap_arena, arena_keep + want, std::min<int64_t>(arena_keep, W.cap_arena));
        reserve(c, W.meet, W.cap_meet, meet_keep + std::min<int64_t>(E, soft) + 64, std::min<int64_t>(meet_keep, W.cap_meet));
        refresh(nullptr, 0);
        launch_scan(nX, probed);  // (k_sp_probe_end cleared the sentinel)
        launch_expand(nX, E, 0);
      }
      k_sp_step<<<grid_n(nb, 1 << 20), 256, 0, c.stream>>>(st, max_steps, 0, iter, cnt);
      NBG_HIP(hipGetLastError());
      sync_counters();
      if (probed) {
        float pms = 0;
        hipEventElapsedTime(&pms, c.ev[4], c.ev[5]);
        c.timing.expand_ms += pms;
        c.timing.expand_launches++;
        c.timing.edges_scanned += hc[C_PE];
        c.timing.expand_bytes += uint64_t(nX) * 24 + hc[C_PE] * 5;
        sp_hop(3, pms, nX, int64_t(hc[C_PE]), 0, iter, active);
      }
      const bool launched = E > 0;
      E = int64_t(hc[C_XE]);  // after the probe's drops: the expansion's own E
      c.timing.edges_scanned += uint64_t(E);
      const double ems = launched && E > 0 ? expand_time() : 0.0;
      const int64_t cl = int64_t(hc[C_LIVE0] + hc[C_LIVE1]) - carried[0] - carried[1];
      last_claims = cl;
      c.timing.expand_bytes += uint64_t(nX) * 32 + uint64_t(E) * 5 + uint64_t(cl) * 26;
      if (E > 0) sp_hop(2, ems, nX, E, cl, iter, active);
      if (int64_t(hc[C_ARENA]) > W.cap_arena) arena_lost = true;  // the batch end resets every byte instead
      n_arena = std::min<int64_t>(int64_t(hc[C_ARENA]), W.cap_arena);
      bool regen_done = false;
      for (int s = 0; s < 2; s++) {
        if (int64_t(hc[C_LIVE0 + s]) <= W.cap_next[s]) continue;
        regen_done = true;
        const int64_t total = int64_t(hc[C_LIVE0 + s]);
        reserve(c, W.live_next[s], W.cap_next[s], total + 64, carried[s]);
        const int32_t np = pair_list([s](int32_t stt, int32_t ps, int32_t) { return stt == SP_ACTIVE && ps == s; });
        set_counter(C_LIVE0 + s, carried[s]);
        regen(RG_LIVE, s, 0, np, W.live_next[s].as<uint64_t>(), W.cap_next[s], C_LIVE0 + s);
      }
      if (int64_t(hc[C_MEET]) > W.cap_meet) {
        regen_done = true;
        reserve(c, W.meet, W.cap_meet, int64_t(hc[C_MEET]) + 64, n_meet);
        const int32_t tag = 2 + iter;
        const int32_t np = pair_list([tag](int32_t stt, int32_t, int32_t m) { return stt == SP_MET && m == tag; });
        set_counter(C_MEET, n_meet);
        regen(RG_MEET, 1, 0, np, W.meet.as<uint64_t>(), W.cap_meet, C_MEET);
      }
      if (regen_done) sync_counters();  // the regenerated lists' counts
      n_live[0] = int64_t(hc[C_LIVE0]);
      n_live[1] = int64_t(hc[C_LIVE1]);
      n_meet = int64_t(hc[C_MEET]);
      active = int64_t(hc[C_ACTIVE]);
      for (int s = 0; s < 2; s++) {
        std::swap(W.live[s], W.live_next[s]);
        std::swap(W.cap_live[s], W.cap_next[s]);
      }
    }

    // sweep: extend dist_B from the meet sets toward src along shortest paths only
    int64_t n_sw = n_meet;
    const int32_t sweep_mode = c.opt("sp_sweep_src", 0) ? 1 : 2;
    DevBuf* cur = &W.meet;
    int nxt = 0;
    // per pair and step: pull (in-rows of the level above) or push (out-rows of the forward
    // level, from the arena) -- needs every forward claim in the arena
    const bool push_ok = c.opt("sp_sweep_push", 1) != 0 && !arena_lost && sweep_mode == 2;
    DevBuf swc;
    unsigned long long *pullc = nullptr, *pushc = nullptr;
    int32_t* push_pair = nullptr;
    if (push_ok) {
      swc.alloc(size_t(nb) * 20 + 64);
      pullc = swc.as<unsigned long long>();
      pushc = pullc + nb;
      push_pair = reinterpret_cast<int32_t*>(pushc + nb);
    }
    for (int32_t j = 1; n_sw > 0; j++) {
      const bool push_now = push_ok && !arena_lost;  // an arena overflow mid-sweep: pull only
      ensure_x(n_sw + (push_now ? n_arena : 0));
      k_cnt_zero<<<1, 256, 0, c.stream>>>(cnt, 1u << C_X | 1u << C_ACTIVE | 1u << C_OVF | 1u << C_SWEEP | 1u << C_XE,
                                          nullptr, push_now ? pullc : nullptr, push_now ? 2 * nb : 0);
      refresh(nullptr, 0);
      if (push_now) {
        k_sweep_pull_cost<<<grid_n(n_sw), 256, 0, c.stream>>>(cur->as<uint64_t>(), n_sw, sweep_mode, st, gin, pullc);
        if (n_arena)
          k_sweep_push_cost<<<grid_n(n_arena), 256, 0, c.stream>>>(W.arena.as<uint64_t>(), n_arena, j, st, gout, pullc,
                                                                    pushc);
        k_sweep_choose<<<grid_n(nb, 1 << 20), 256, 0, c.stream>>>(
            pullc, pushc, int32_t(nb), push_pair, (unsigned long long)std::max<int64_t>(0, 16));
      }
      k_sp_select<<<grid_sel(n_sw), kBlk, 0, c.stream>>>(cur->as<uint64_t>(), n_sw, sweep_mode, st, gout, gin, W.X.as<uint64_t>(),
                                                       W.Xdeg.as<int64_t>(), W.cap_x, bf, cnt,
                                                       push_now ? push_pair : nullptr);
      if (push_now && n_arena)
        k_sweep_push_select<<<grid_n(n_arena), 256, 0, c.stream>>>(W.arena.as<uint64_t>(), n_arena, j, st, gout,
                                                                    push_pair, W.X.as<uint64_t>(),
                                                                    W.Xdeg.as<int64_t>(), W.cap_x, cnt);
      NBG_HIP(hipGetLastError());
      sync_counters();
      const int64_t nX = int64_t(hc[C_X]), E = int64_t(hc[C_XE]);
      if (nX == 0 || E == 0) break;
      c.timing.edges_scanned += uint64_t(E);
      const int64_t want = std::min<int64_t>(E, soft) + 64;
      reserve(c, W.sweep[nxt], W.cap_sweep[nxt], want, 0);
      if (!arena_lost) reserve(c, W.arena, W.cap_arena, n_arena + want, n_arena);
      refresh(&W.sweep[nxt], W.cap_sweep[nxt]);
      if (c.opt("sp_sweep_chunks", 1) != 0) {
        // chunk counts -> their scan -> chunk table -> one wave per chunk
        DevBuf ch, choff, chx;
        ch.alloc(size_t(nX + 1) * 8);
        choff.alloc(size_t(nX + 1) * 8);
        k_sp_chunks_n<<<grid_n(nX + 1), 256, 0, c.stream>>>(W.Xdeg.as<int64_t>(), nX, ch.as<int64_t>(), kSwCh);
        size_t tb = 0;
        NBG_HIP(rocprim::exclusive_scan(nullptr, tb, ch.as<int64_t>(), choff.as<int64_t>(), int64_t(0),
                                        size_t(nX + 1), rocprim::plus<int64_t>(), c.stream));
        c.ws_tmp.ensure(tb);
        NBG_HIP(rocprim::exclusive_scan(c.ws_tmp.p, tb, ch.as<int64_t>(), choff.as<int64_t>(), int64_t(0),
                                        size_t(nX + 1), rocprim::plus<int64_t>(), c.stream));
        const int64_t max_ch = nX + E / kSwCh + 1;
        chx.alloc(size_t(max_ch) * 4);
        hipEventRecord(c.ev[2], c.stream);
        k_chunk_x<<<grid_n(nX), 256, 0, c.stream>>>(choff.as<int64_t>(), nX, chx.as<int32_t>());
        const int sgrid = int(std::max<int64_t>(1, std::min<int64_t>((max_ch + 3) / 4, 8192)));
        k_sp_sweep<1><<<sgrid, 256, 0, c.stream>>>(W.X.as<uint64_t>(), choff.as<int64_t>(), chx.as<int32_t>(), nX,
                                                      gout, gin, d0, d1, n, lo, st, bf, cnt);
        NBG_HIP(hipGetLastError());
        hipEventRecord(c.ev[3], c.stream);
      } else {
        launch_scan(nX);
        launch_expand(nX, E, 1);
      }
      sync_counters();
      const double sms = expand_time();
      c.timing.expand_bytes += uint64_t(nX) * 32 + uint64_t(E) * 6 + hc[C_SWEEP] * 18;
      sp_hop(4, sms, nX, E, int64_t(hc[C_SWEEP]), j, 0);
      if (int64_t(hc[C_ARENA]) > W.cap_arena) arena_lost = true;
      n_arena = std::min<int64_t>(int64_t(hc[C_ARENA]), W.cap_arena);
      if (int64_t(hc[C_SWEEP]) > W.cap_sweep[nxt]) {
        reserve(c, W.sweep[nxt], W.cap_sweep[nxt], int64_t(hc[C_SWEEP]) + 64, 0);
        const int32_t np = pair_list([](int32_t stt, int32_t, int32_t) { return stt == SP_MET; });
        set_counter(C_SWEEP, 0);
        regen(RG_SWEEP, 1, j, np, W.sweep[nxt].as<uint64_t>(), W.cap_sweep[nxt], C_SWEEP);
        sync_counters();
      }
      n_sw = int64_t(hc[C_SWEEP]);
      cur = &W.sweep[nxt];
      nxt ^= 1;
    }

    // results + paths: the path offsets, their total and the longest path on the device (one
    // counter fetch); state, res, offsets and the walked paths come back with the batch's last
    // fetch, through the pinned stage when they fit (pageable copies and a stream synchronisation
    // here cost ~0.1 ms a batch)
    DevBuf doff, dpath, wk;  // (wk: the walk state, drained by the batch's last fetch)
    doff.alloc(size_t(nb + 1) * 8);
    k_sp_path_offsets<<<1, 1024, 0, c.stream>>>(st, nb, doff.as<int64_t>(), cnt);
    NBG_HIP(hipGetLastError());
    sync_counters();
    const int64_t plen = int64_t(hc[C_PLEN]);
    const int32_t maxL = int32_t(hc[C_MAXL]);
    if (plen > 0) {
      dpath.alloc(size_t(plen) * 8);
      if (c.opt("sp_walk_wg", 0) || nb >= kTileE) {  // a tile stages at most kTileE pair entries
        k_sp_walk<<<int(nb), kWalkT, 0, c.stream>>>(st, dgs, doff.as<int64_t>(), dpath.as<int64_t>(), gout, d1,
                                                    vid_of, n, lo, cnt);
      } else if (maxL >= 2) {
        // walk state: cur [B], best [B], degrees / offsets [B + 1], tile rows (all pairs' rows <= nnz)
        const int64_t max_tiles = (cout->nnz + kTileE - 1) / kTileE + nb + 2;
        const size_t wbytes = size_t(nb) * 4 + 64 + size_t(nb) * 8 + 64 + 2 * (size_t(nb + 1) * 8 + 64) +
                              size_t(max_tiles) * 4 + 64;
        wk.alloc(wbytes);
        Carve cv(wk, "shortest path: walk workspace");
        int32_t* dcur = cv.take<int32_t>(size_t(nb) * 4);
        long long* dbest = cv.take<long long>(size_t(nb) * 8);
        int64_t* wdeg = cv.take<int64_t>(size_t(nb + 1) * 8);
        int64_t* woff = cv.take<int64_t>(size_t(nb + 1) * 8);
        int32_t* wtr = cv.take<int32_t>(size_t(max_tiles) * 4);
        NBG_HIP(hipMemcpyAsync(dcur, dgs, size_t(nb) * 4, hipMemcpyDeviceToDevice, c.stream));
        size_t tb = 0;
        NBG_HIP(rocprim::exclusive_scan(nullptr, tb, wdeg, woff, int64_t(0), size_t(nb + 1), rocprim::plus<int64_t>(),
                                        c.stream));
        c.ws_tmp.ensure(tb);
        const int wgrid = int(std::max<int64_t>(1, std::min<int64_t>(256 * 8, max_tiles)));
        for (int32_t i = 0; i + 1 < maxL; i++) {
          k_sp_walk_front<<<grid_n(nb + 1, 1 << 20), 256, 0, c.stream>>>(st, i, dcur, gout, wdeg, dbest);
          NBG_HIP(rocprim::exclusive_scan(c.ws_tmp.p, tb, wdeg, woff, int64_t(0), size_t(nb + 1),
                                          rocprim::plus<int64_t>(), c.stream));
          k_tile_rows<kTileE><<<grid_n(nb), 256, 0, c.stream>>>(woff, nb, wtr);
          k_sp_walk_scan<<<wgrid, kT, 0, c.stream>>>(st, i, dcur, woff, wtr, gout, d1, vid_of, n, lo, dbest);
          k_sp_walk_pick<<<grid_n(nb, 1 << 20), 256, 0, c.stream>>>(
              st, i, dcur, dbest, doff.as<int64_t>(), dpath.as<int64_t>(), c.ht_keys.as<int64_t>(),
              c.ht_vals.as<int32_t>(), uint64_t(c.ht_cap - 1), c.ht_has_min, c.ht_min_gidx, lo, cnt);
          NBG_HIP(hipGetLastError());
        }
      }
      NBG_HIP(hipGetLastError());
    }
    const size_t sb = (size_t(nb) * 8 + 63) & ~size_t(63);  // state + res (adjacent in W.state)
    const size_t ob = (size_t(nb + 1) * 8 + 63) & ~size_t(63);
    const bool staged = c.host_stage && c.host_stage_used == 0 && sb + ob + size_t(plen) * 8 <= kHostStageBytes;
    std::vector<int64_t> hoff_b, hpath_b;
    int32_t* h_sr = hstate.data();  // [state nb][res nb]
    int64_t* h_off = nullptr;
    int64_t* h_path = nullptr;
    if (staged) {
      char* hs = static_cast<char*>(c.host_stage);
      h_sr = reinterpret_cast<int32_t*>(hs);
      h_off = reinterpret_cast<int64_t*>(hs + sb);
      h_path = reinterpret_cast<int64_t*>(hs + sb + ob);
    } else {
      hstate.resize(size_t(2 * nb));
      h_sr = hstate.data();
      hoff_b.resize(size_t(nb + 1));
      hpath_b.resize(size_t(std::max<int64_t>(plen, 1)));
      h_off = hoff_b.data();
      h_path = hpath_b.data();
    }
    NBG_HIP(hipMemcpyAsync(h_sr, st.state, size_t(nb) * 8, hipMemcpyDeviceToHost, c.stream));
    NBG_HIP(hipMemcpyAsync(h_off, doff.p, size_t(nb + 1) * 8, hipMemcpyDeviceToHost, c.stream));
    if (plen > 0) NBG_HIP(hipMemcpyAsync(h_path, dpath.p, size_t(plen) * 8, hipMemcpyDeviceToHost, c.stream));
    sync_counters();  // C_WALKERR is current; the staged copies above have landed (stream order)
    // pageable destinations: hipMemcpyAsync may return before such a copy completes, so the
    // stream is drained before the host reads them
    if (!staged) NBG_HIP(hipStreamSynchronize(c.stream));
    if (plen > 0 && hc[C_WALKERR])
      throw Error(NBG_E_UNKNOWN, "shortest path: in-edge keys without mirrored out-edges on a shortest path");
    const size_t base = hpath.size();
    hpath.resize(base + size_t(plen));
    if (plen > 0) memcpy(hpath.data() + base, h_path, size_t(plen) * 8);
    for (int64_t p = 0; p < nb; p++) {
      const int32_t L = h_sr[p] == SP_ACTIVE ? -1 : h_sr[nb + p];
      hres[b0 + size_t(p)] = L;
      if (L >= 0) {  // the ends: src (also the whole path of src == dst) and dst
        hpath[base + size_t(h_off[p])] = src[b0 + size_t(p)];
        if (L > 0) hpath[base + size_t(h_off[p] + L)] = dst[b0 + size_t(p)];
      }
      hoff.push_back(hoff.back() + h_off[p + 1] - h_off[p]);
    }
    // reset the batch's distance bytes
    if (arena_lost) {
      NBG_HIP(hipMemsetAsync(c.sp_dist[0].p, 0xFF, 2 * c.sp_dist_bytes, c.stream));
    } else if (n_arena) {
      k_sp_clear<<<grid_n(n_arena), 256, 0, c.stream>>>(W.arena.as<uint64_t>(), n_arena, d0, d1, n, st);
      NBG_HIP(hipGetLastError());
    }
  }
  hipEventRecord(c.ev[1], c.stream);
  NBG_HIP(hipEventSynchronize(c.ev[1]));
  c.sp_dirty = false;
  float ms = 0;
  hipEventElapsedTime(&ms, c.ev[0], c.ev[1]);
  c.timing.total_ms = ms;

  auto* h = new HostRows();
  for (int k = 0; k < 3; k++) {
    h->types.push_back(NBG_T_VID);
    h->host.emplace_back(npairs * 8 + 8);
    h->str_off.push_back(nullptr);
  }
  for (size_t i = 0; i < npairs; i++) {
    memcpy(h->host[0].data() + i * 8, src + i, 8);
    memcpy(h->host[1].data() + i * 8, dst + i, 8);
    memcpy(h->host[2].data() + i * 8, &hres[i], 8);
  }
  for (int k = 0; k < 3; k++) h->cols.push_back(h->host[size_t(k)].data());
  h->path_offsets = std::move(hoff);
  h->path_vids = std::move(hpath);
  if (h->path_vids.empty()) h->path_vids.push_back(0);  // non-null pointer for an empty result
  fill_rows(out, h, int64_t(npairs), false);
  out->edges_scanned = c.timing.edges_scanned;
  return NBG_OK;
}

}  // namespace nbg
