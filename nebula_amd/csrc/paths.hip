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
};

__device__ inline int64_t sp_deg(const SpCsr& g, uint32_t r) {
  if (g.row_ok && !g.row_ok[r]) return 0;
  return g.row_ptr[r + 1] - g.row_ptr[r];
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
  int32_t vmajor;           // distance bytes vertex-major [v][pair] (else pair-major [pair][v])
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
  // sparse distance maps (option sp_hash, null: the dense byte arrays): per side, open-addressing
  // (pair, vertex) -> depth over 64-bit words, hmask + 1 slots, sized to the batch's claims (a
  // few million per side at RMAT-26, tens of MB that stay in the Infinity Cache and in a handful
  // of TLB pages; the dense arrays are 2 * B * n bytes read at random lines)
  uint64_t* htab[2];
  uint64_t hmask;
};
constexpr int kLv = 8;

// hash map words: bits [0, 31) vertex, [31, 54) pair, [54, 62) depth; all ones = empty
constexpr uint64_t kHEmpty = ~0ull;
constexpr uint64_t kHKey = (1ull << 54) - 1;
__device__ inline uint64_t hkey(uint32_t p, uint32_t v) { return (uint64_t(p) << 31) | uint64_t(v); }
__device__ inline uint64_t hslot(uint64_t key, uint64_t mask) {
  uint64_t x = key * 0x9E3779B97F4A7C15ull;
  return (x ^ (x >> 29)) & mask;
}

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
// lines in L2 / the Infinity cache; pair-major keeps each pair's bytes contiguous.
__device__ inline uint64_t didx(const SpState& st, uint32_t p, uint64_t v, int64_t n) {
  return st.vmajor ? v * uint64_t(st.B) + p : uint64_t(p) * uint64_t(n) + v;
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
  uint32_t* w = reinterpret_cast<uint32_t*>(base + (idx & ~uint64_t(3)));
  const uint32_t sh = uint32_t(idx & 3) * 8;
  uint32_t old = *reinterpret_cast<volatile uint32_t*>(w);
  while (((old >> sh) & 0xFFu) == 0xFFu) {
    const uint32_t nw = (old & ~(0xFFu << sh)) | (val << sh);
    const uint32_t prev = atomicCAS(w, old, nw);
    if (prev == old) return true;
    old = prev;
  }
  return false;
}

// the depth of vertex v for pair p on a side (0xFF: unseen), from the dense bytes or the map
__device__ inline uint32_t dist_get(const SpState& st, const uint8_t* dense, uint32_t side, uint32_t p, uint32_t v,
                                    int64_t n, bool fresh = false) {
  if (!st.htab[0]) {
    const uint8_t* a = dense + didx(st, p, v, n);
    return fresh ? uint32_t(*reinterpret_cast<volatile const uint8_t*>(a)) : uint32_t(*a);
  }
  const uint64_t* T = st.htab[side];
  const uint64_t key = hkey(p, v);
  for (uint64_t h = hslot(key, st.hmask);; h = (h + 1) & st.hmask) {
    const uint64_t e = fresh ? __hip_atomic_load(T + h, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : T[h];
    if (e == kHEmpty) return 0xFFu;
    if ((e & kHKey) == key) return uint32_t(e >> 54) & 0xFFu;
  }
}
// claim the unseen (p, v) on a side with depth val: true for exactly one caller
__device__ inline bool dist_claim(const SpState& st, uint8_t* dense, uint32_t side, uint32_t p, uint32_t v, int64_t n,
                                  uint32_t val) {
  if (!st.htab[0]) return claim_byte(dense, didx(st, p, v, n), val);
  uint64_t* T = st.htab[side];
  const uint64_t key = hkey(p, v), word = key | (uint64_t(val & 0xFFu) << 54);
  for (uint64_t h = hslot(key, st.hmask);; h = (h + 1) & st.hmask) {
    uint64_t e = T[h];
    if (e == kHEmpty) {
      e = atomicCAS(reinterpret_cast<unsigned long long*>(T + h), (unsigned long long)kHEmpty, (unsigned long long)word);
      if (e == kHEmpty) return true;
    }
    if ((e & kHKey) == key) return false;
  }
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

// sparse maps: RG_* list rebuilds from the map words of the listed pairs (pflag[p] = 1)
__global__ void k_sp_regen_hash(int mode, int side, int32_t j, const uint8_t* pflag, SpState st, int64_t n,
                                uint64_t* out, int64_t cap, unsigned long long* cnt, int which) {
  const int32_t B = st.B;
  const uint64_t* T = st.htab[mode == RG_LIVE ? side : 1];
  const int64_t slots = int64_t(st.hmask) + 1;
  const int64_t stride = int64_t(gridDim.x) * blockDim.x;
  const int64_t rounds = (slots + stride - 1) / stride;
  for (int64_t r = 0; r < rounds; r++) {
    const int64_t i = r * stride + blockIdx.x * int64_t(blockDim.x) + threadIdx.x;
    bool hit = false;
    uint32_t p = 0, v = 0, d = 0;
    if (i < slots) {
      const uint64_t e = T[i];
      if (e != kHEmpty) {
        p = uint32_t(e >> 31) & 0x7FFFFFu;
        v = uint32_t(e & 0x7FFFFFFFu);
        d = uint32_t(e >> 54) & 0xFFu;
        if (int32_t(p) < B && pflag[p]) {
          if (mode == RG_LIVE) hit = d == uint32_t(st.lvl[side * B + p]);
          else if (mode == RG_MEET)
            hit = d == uint32_t(st.lvl[B + p]) && dist_get(st, nullptr, 0, p, v, n) == uint32_t(st.lvl[p]);
          else hit = d == uint32_t(st.lvl[B + p] + j);
        }
      }
    }
    put(out, cap, cnt, which, hit, mk_tup(mode == RG_LIVE ? uint32_t(side) : 1u, p, d, v));
  }
}
__global__ void k_set_flags(const int32_t* plist, int32_t np, uint8_t* flag) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < np) flag[plist[i]] = 1;
}
// grow a map: every word of the old table inserted into the new one (same key -> slot rule)
__global__ void k_hash_rehash(const uint64_t* old, int64_t nold, uint64_t* nt, uint64_t nmask) {
  for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < nold; i += int64_t(gridDim.x) * blockDim.x) {
    const uint64_t e = old[i];
    if (e == kHEmpty) continue;
    for (uint64_t h = hslot(e & kHKey, nmask);; h = (h + 1) & nmask)
      if (atomicCAS(reinterpret_cast<unsigned long long*>(nt + h), (unsigned long long)kHEmpty, (unsigned long long)e) ==
          kHEmpty)
        break;
  }
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
  if (c.world > 1) {
    if (!es.has_rep) {
      replicate_csr(c, es.out, es.rep_out);
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
  // option sp_hash: sparse (pair, vertex) -> depth maps sized to the claims instead of the dense
  // 2 * B * n byte arrays
  const bool hash = c.opt("sp_hash", 0) != 0;
  if (!hash) {
    PoolScope none(nullptr);  // the distance arrays live outside the query pool
    if (c.sp_dist_bytes < dist_bytes) {
      for (auto& d : c.sp_dist) d.release();
      c.sp_dist_bytes = 0;
      for (auto& d : c.sp_dist) d.alloc(dist_bytes);
      c.sp_dist_bytes = dist_bytes;
      c.sp_dirty = true;
    }
    if (c.sp_dirty)
      for (auto& d : c.sp_dist) NBG_HIP(hipMemsetAsync(d.p, 0xFF, c.sp_dist_bytes, c.stream));
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
  hipEventRecord(c.ev[0], c.stream);

  uint8_t* d0 = hash ? nullptr : c.sp_dist[0].as<uint8_t>();
  uint8_t* d1 = hash ? nullptr : c.sp_dist[1].as<uint8_t>();
  // the maps: at most half full (linear probing); grown (rehashed) before a launch whose claims
  // could pass that, from a bound on them -- the claims so far plus the launch's entries
  // (expansion), chunks (meet probe) or the claims so far again (a sweep claims only vertices the
  // forward search holds)
  auto hash_fit = [&](SpState& st, int64_t claims) {
    if (!hash) return;
    int64_t cap = std::max<int64_t>(W.hcap, int64_t(1) << std::min<int64_t>(30, std::max<int64_t>(10, c.opt("sp_hash_log2", 22))));
    while (cap < 2 * claims + 64) cap <<= 1;
    if (cap != W.hcap || !W.htab[0].p) {
      PoolScope none(nullptr);
      for (int sd = 0; sd < 2; sd++) {
        DevBuf nt;
        nt.alloc(size_t(cap) * 8);
        NBG_HIP(hipMemsetAsync(nt.p, 0xFF, size_t(cap) * 8, c.stream));
        if (W.htab[sd].p && W.hcap > 0)
          k_hash_rehash<<<grid_n(W.hcap), 256, 0, c.stream>>>(W.htab[sd].as<uint64_t>(), W.hcap, nt.as<uint64_t>(),
                                                               uint64_t(cap - 1));
        NBG_HIP(hipGetLastError());
        W.htab[sd] = std::move(nt);
      }
      W.hcap = cap;
    }
    st.htab[0] = W.htab[0].as<uint64_t>();
    st.htab[1] = W.htab[1].as<uint64_t>();
    st.hmask = uint64_t(W.hcap - 1);
  };
  SpCsr gout{cout->row_ptr.as<int64_t>(), cout->col.as<int32_t>(), cout->row_ok.as<uint8_t>()};
  SpCsr gin{cin->row_ptr.as<int64_t>(), cin->col.as<int32_t>(), cin->row_ok.as<uint8_t>()};
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
  if (hash && c.sp_dirty && W.hcap > 0)  // a failed call's claims
    for (auto& t : W.htab) NBG_HIP(hipMemsetAsync(t.p, 0xFF, size_t(W.hcap) * 8, c.stream));
  c.sp_dirty = true;  // until the batch's bytes are reset
  for (size_t b0 = 0; b0 < npairs; b0 += size_t(B)) {
    const int64_t nb = std::min<int64_t>(B, int64_t(npairs - b0));
    SpState st{};
    st.B = int32_t(nb);
    hash_fit(st, 2 * nb);
    st.deg = W.state.as<unsigned long long>();
    st.state = reinterpret_cast<int32_t*>(st.deg + 2 * nb);
    st.res = st.state + nb;
    st.lvl = st.res + nb;
    st.side = st.lvl + 2 * nb;
    st.pside = st.side + nb;
    st.met = st.pside + nb;
    st.vmajor = int32_t(c.opt("sp_vmajor", 0));
    if (c.opt("sp_lvbits", 1) != 0) {  // level filter: 2 * kLv maps, cleared per batch
      // bits per level: the power of two >= n, capped (option sp_lvbits_log2, default 23)
      const int cap = int(std::min<int64_t>(std::max<int64_t>(c.opt("sp_lvbits_log2", 23), 5), 31));
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
      const int grid = int(std::max<int64_t>(1, std::min<int64_t>(tiles, c.opt("sp_grid", 256 * 8))));
      hipEventRecord(c.ev[2], c.stream);
      a.tile_row = nullptr;
      if (c.opt("expand_tile_rows", 1) && nX < (int64_t(1) << 31)) {
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
    unsigned long long diag[2] = {0, 0};  // option sp_sweep_stats: distinct X vertices, their degree sum
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
      if (hash) {
        DevBuf flag;
        flag.alloc(size_t(nb) + 64);
        NBG_HIP(hipMemsetAsync(flag.p, 0, size_t(nb) + 64, c.stream));
        k_set_flags<<<grid_n(np), 256, 0, c.stream>>>(W.plist.as<int32_t>(), np, flag.as<uint8_t>());
        k_sp_regen_hash<<<grid_n(W.hcap), 256, 0, c.stream>>>(mode, side, j, flag.as<uint8_t>(), st, n, outl, cap, cnt,
                                                              which);
        NBG_HIP(hipGetLastError());
        return;
      }
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
        hash_fit(st, int64_t(hc[C_ARENA]) + max_chunks);
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
            int(std::max<int64_t>(1, std::min<int64_t>((max_chunks + 3) / 4, c.opt("sp_probe_grid", 4096))));
        chx.alloc(size_t(max_chunks) * 4);
        k_chunk_x<<<grid_n(nX), 256, 0, c.stream>>>(choff.as<int64_t>(), nX, chx.as<int32_t>(), slot.as<uint64_t>());
        if (c.opt("sp_probe_occ", 7) >= 8)
          k_sp_probe<8><<<pgrid, 256, 0, c.stream>>>(W.X.as<uint64_t>(), nX, choff.as<int64_t>(), chx.as<int32_t>(),
                                                     gout, gin, d0, d1, n, lo, st, slot.as<uint64_t>(), cnt);
        else
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
        hash_fit(st, int64_t(hc[C_ARENA]) + max_chunks + E);
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
            pullc, pushc, int32_t(nb), push_pair, (unsigned long long)std::max<int64_t>(0, c.opt("sp_push_bias", 16)));
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
      if (c.opt("sp_sweep_stats", 0) && nX <= (int64_t(1) << 26)) {
        // diagnostics: how many distinct vertices the step's adjacency scans come from (pairs
        // sharing a meet vertex scan its row once each)
        std::vector<uint64_t> hx(static_cast<size_t>(nX));
        std::vector<int64_t> hd(static_cast<size_t>(nX));
        NBG_HIP(hipMemcpyAsync(hx.data(), W.X.p, size_t(nX) * 8, hipMemcpyDeviceToHost, c.stream));
        NBG_HIP(hipMemcpyAsync(hd.data(), W.Xdeg.p, size_t(nX) * 8, hipMemcpyDeviceToHost, c.stream));
        NBG_HIP(hipStreamSynchronize(c.stream));
        std::unordered_map<uint64_t, int64_t> seen;
        for (int64_t i = 0; i < nX; i++) seen[(hx[size_t(i)] >> 63) << 32 | uint32_t(hx[size_t(i)])] = hd[size_t(i)];
        diag[0] = seen.size();
        for (auto& kv : seen) diag[1] += uint64_t(kv.second);
      }
      c.timing.edges_scanned += uint64_t(E);
      hash_fit(st, 2 * int64_t(hc[C_ARENA]));
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
        const int sgrid = int(std::max<int64_t>(1, std::min<int64_t>((max_ch + 3) / 4, c.opt("sp_sweep_grid", 8192))));
        const int64_t socc = c.opt("sp_sweep_occ", 5);
        if (socc >= 8)
          k_sp_sweep<8><<<sgrid, 256, 0, c.stream>>>(W.X.as<uint64_t>(), choff.as<int64_t>(), chx.as<int32_t>(), nX,
                                                      gout, gin, d0, d1, n, lo, st, bf, cnt);
        else if (socc >= 6)
          k_sp_sweep<6><<<sgrid, 256, 0, c.stream>>>(W.X.as<uint64_t>(), choff.as<int64_t>(), chx.as<int32_t>(), nX,
                                                      gout, gin, d0, d1, n, lo, st, bf, cnt);
        else
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
        char* q = static_cast<char*>(wk.p);
        auto take = [&](size_t b) { char* r = q; q += (b + 63) & ~size_t(63); return r; };
        int32_t* dcur = reinterpret_cast<int32_t*>(take(size_t(nb) * 4));
        long long* dbest = reinterpret_cast<long long*>(take(size_t(nb) * 8));
        int64_t* wdeg = reinterpret_cast<int64_t*>(take(size_t(nb + 1) * 8));
        int64_t* woff = reinterpret_cast<int64_t*>(take(size_t(nb + 1) * 8));
        int32_t* wtr = reinterpret_cast<int32_t*>(take(size_t(max_tiles) * 4));
        NBG_HIP(hipMemcpyAsync(dcur, dgs, size_t(nb) * 4, hipMemcpyDeviceToDevice, c.stream));
        size_t tb = 0;
        NBG_HIP(rocprim::exclusive_scan(nullptr, tb, wdeg, woff, int64_t(0), size_t(nb + 1), rocprim::plus<int64_t>(),
                                        c.stream));
        c.ws_tmp.ensure(tb);
        const int wgrid = int(std::max<int64_t>(1, std::min<int64_t>(c.opt("sp_grid", 256 * 8), max_tiles)));
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
    sync_counters();  // every copy above has landed (stream order) and C_WALKERR is current
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
    if (hash) {
      for (auto& t : W.htab) NBG_HIP(hipMemsetAsync(t.p, 0xFF, size_t(W.hcap) * 8, c.stream));
    } else if (arena_lost) {
      const size_t used = ((size_t(nb) * size_t(n) + 3) & ~size_t(3)) + 64;
      for (auto& d : c.sp_dist) NBG_HIP(hipMemsetAsync(d.p, 0xFF, std::min(used, c.sp_dist_bytes), c.stream));
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
