// device_common.h -- small device helpers shared by the .hip translation units.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace nbg {

constexpr int kWave = 64;  // CDNA wavefront

__host__ __device__ inline uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

__host__ __device__ inline uint64_t bswap64(uint64_t x) {
  x = ((x & 0x00FF00FF00FF00FFull) << 8) | ((x >> 8) & 0x00FF00FF00FF00FFull);
  x = ((x & 0x0000FFFF0000FFFFull) << 16) | ((x >> 16) & 0x0000FFFF0000FFFFull);
  return (x << 32) | (x >> 32);
}

// partition of a vid: (uint64)vid % parts + 1 (StorageClient.cpp:10-11); rank = part % world
__host__ __device__ inline int32_t dev_part_of(int64_t vid, int32_t parts) {
  return int32_t(uint64_t(vid) % uint64_t(parts) + 1);
}
__host__ __device__ inline int32_t dev_owner(int64_t vid, int32_t parts, int32_t world) {
  return dev_part_of(vid, parts) % world;
}

// Open-addressing vid -> gidx table (linear probing, INT64_MIN = empty).
__host__ __device__ inline uint64_t ht_hash(int64_t vid) { return splitmix64(uint64_t(vid)); }

__device__ inline int32_t ht_lookup(const int64_t* __restrict__ keys, const int32_t* __restrict__ vals,
                                    uint64_t mask, int64_t vid, bool has_min, int32_t min_gidx) {
  if (vid == INT64_MIN) return has_min ? min_gidx : -1;
  uint64_t h = ht_hash(vid) & mask;
  while (true) {
    int64_t k = keys[h];
    if (k == vid) return vals[h];
    if (k == INT64_MIN) return -1;
    h = (h + 1) & mask;
  }
}

// The LDS hub copy of a bottom-up kernel: words [0, cw) of the frontier bitmap into s_fb, plus
// a zero word at [cw] when `zero_word`.  Every thread issues all its 16-byte loads before its
// LDS stores, so a block waits one global latency, not one per blockDim words (the element loop
// compiled to load / vmcnt(0) / ds_write per iteration: 16 dependent L2 round trips for a 64 KiB
// hub at 1024 threads).  Ends with the block barrier.
__device__ inline void hub_fill(uint32_t* s_fb, const uint32_t* __restrict__ fbits, int cw, bool zero_word) {
  constexpr int kB = 4;  // 16-byte loads in flight per thread per round
  const int nt = int(blockDim.x), tid = int(threadIdx.x);
  int done = 0;
  if (((reinterpret_cast<uintptr_t>(fbits) | reinterpret_cast<uintptr_t>(s_fb)) & 15u) == 0u) {
    const int nv = cw >> 2;
    const uint4* src = reinterpret_cast<const uint4*>(fbits);
    uint4* dst = reinterpret_cast<uint4*>(s_fb);
    for (int base = 0; base < nv; base += kB * nt) {
      uint4 v[kB];
#pragma unroll
      for (int k = 0; k < kB; k++) {
        const int i = base + k * nt + tid;
        v[k] = i < nv ? src[i] : make_uint4(0u, 0u, 0u, 0u);
      }
#pragma unroll
      for (int k = 0; k < kB; k++) {
        const int i = base + k * nt + tid;
        if (i < nv) dst[i] = v[k];
      }
    }
    done = nv << 2;
  }
  for (int base = done; base < cw; base += kB * nt) {
    uint32_t v[kB];
#pragma unroll
    for (int k = 0; k < kB; k++) {
      const int i = base + k * nt + tid;
      v[k] = i < cw ? fbits[i] : 0u;
    }
#pragma unroll
    for (int k = 0; k < kB; k++) {
      const int i = base + k * nt + tid;
      if (i < cw) s_fb[i] = v[k];
    }
  }
  if (zero_word && tid == 0) s_fb[cw] = 0u;
  __syncthreads();
}

// wave-aggregated append: returns this lane's slot in `*counter` space (lanes with !pred get -1)
__device__ inline int64_t wave_append(unsigned long long* counter, bool pred) {
  uint64_t mask = __ballot(pred);
  if (mask == 0) return -1;
  int lane = threadIdx.x & (kWave - 1);
  int leader = __ffsll((long long)mask) - 1;
  uint64_t base = 0;
  if (lane == leader) base = atomicAdd(counter, (unsigned long long)__popcll(mask));
  base = __shfl(base, leader);
  if (!pred) return -1;
  uint64_t below = mask & ((lane == 0) ? 0ull : (~0ull >> (64 - lane)));
  return int64_t(base + __popcll(below));
}

// ---- edge-balanced tiles over a frontier's flattened adjacency (k_expand, k_sp_expand) -------
// tile_row[t] = the frontier entry holding slot t * TILE of the flattened range: every non-empty
// entry k writes the tiles whose first slot falls in [off[k], off[k + 1]) (each tile start lies
// in exactly one non-empty entry).  One coalesced pass over off[] instead of two dependent binary
// searches of off[] by one thread at the head of every tile.
// Every wave takes 64 consecutive entries (one per lane); a lane fills a range of up to 4 items
// itself, longer ranges [i0, i1) are filled by the whole wave, entry by entry, 64 items a step: a hub entry's thousands of tiles / chunks are no
// longer one thread's serial loop (~20 us for the C4 probe's largest rows).  Wave-uniform;
// blockDim a multiple of 64.  range(k, i0, i1) gives entry k's items; fill(item, k) writes one.
template <typename Range, typename Fill>
__device__ inline void wave_fill_ranges(int64_t nk, Range range, Fill fill) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = (int64_t(blockIdx.x) * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = (int64_t(gridDim.x) * blockDim.x) >> 6;
  for (int64_t k0 = wave * 64; k0 < nk; k0 += nwaves * 64) {
    int64_t i0 = 0, i1 = 0;
    if (k0 + lane < nk) range(k0 + lane, i0, i1);
    // short ranges (most entries: one or two items) by their own lane, the rest together
    if (i1 - i0 <= 4) {
      for (int64_t i = i0; i < i1; i++) fill(i, k0 + lane);
      i1 = i0;
    }
    uint64_t m = __ballot(i1 > i0);
    while (m) {
      const int j = __ffsll((long long)m) - 1;
      m &= m - 1;
      const int64_t a = __shfl(i0, j), z = __shfl(i1, j);
      for (int64_t i = a + lane; i < z; i += 64) fill(i, k0 + j);
    }
  }
}
template <int TILE>
__global__ void k_tile_rows(const int64_t* __restrict__ off, int64_t nF, int32_t* __restrict__ tile_row) {
  wave_fill_ranges(
      nF,
      [&](int64_t k, int64_t& t0, int64_t& t1) {
        const int64_t b = off[k], e = off[k + 1];
        if (b < e) t0 = (b + TILE - 1) / TILE, t1 = (e + TILE - 1) / TILE;  // tiles with t * TILE in [b, e)
      },
      [&](int64_t t, int64_t k) { tile_row[t] = int32_t(k); });
}
// The entries [i0, i0 + cnt) staged for tile t (slots [e0, e1) of E): i0 holds e0; the last one
// holds e1 - 1, i.e. the entry before the one holding e1 when that one starts at e1 (entries of
// zero degree in between are staged too, harmlessly: their slots are empty).
__device__ inline void tile_entries(const int32_t* tile_row, const int64_t* off, int64_t nF, int64_t t, int64_t e1,
                                    int64_t E, int64_t& i0, int64_t& cnt) {
  i0 = tile_row[t];
  int64_t i1 = nF - 1;
  if (e1 < E) {
    const int64_t r = tile_row[t + 1];
    i1 = off[r] == e1 ? r - 1 : r;
  }
  cnt = i1 - i0 + 1;
}
// Owner map of a tile in LDS: s_off[k] (k < cnt <= TILE) holds entry k's first slot relative to
// the tile (<= 0 for the entry holding slot 0); on return s_off[j] (j < TILE) is the entry owning
// slot j: the largest k starting at or before j (entries of zero degree share their successor's
// start; the max picks the non-empty one) - one atomicMax per entry and a block max-scan instead
// of a binary search per slot.  Block-wide (THREADS threads, all of them must call it).
template <int TILE, int THREADS>
__device__ inline void tile_owner_map(int32_t* s_off, int cnt, int32_t* s_scan /* [THREADS / 64] */) {
  constexpr int kRows = TILE / THREADS;
  int st[kRows];
#pragma unroll
  for (int i = 0; i < kRows; i++) {
    const int k = threadIdx.x + i * THREADS;
    st[i] = k < cnt ? s_off[k] : TILE;
  }
  __syncthreads();
  for (int j = threadIdx.x; j < TILE; j += THREADS) s_off[j] = 0;
  __syncthreads();
#pragma unroll
  for (int i = 0; i < kRows; i++)
    if (st[i] < TILE) atomicMax(&s_off[st[i] < 0 ? 0 : st[i]], int(threadIdx.x + i * THREADS));
  __syncthreads();
  // inclusive max-scan: kRows consecutive slots per thread, then across the wave and the block
  int m = 0;
  int loc[kRows];
#pragma unroll
  for (int i = 0; i < kRows; i++) {
    m = max(m, s_off[threadIdx.x * kRows + i]);
    loc[i] = m;
  }
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  int x = m;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(x, o);
    if (lane >= o) x = max(x, y);
  }
  if (lane == 63) s_scan[wv] = x;
  int prev = __shfl_up(x, 1);
  if (lane == 0) prev = 0;
  __syncthreads();
  for (int w = 0; w < wv; w++) prev = max(prev, s_scan[w]);
#pragma unroll
  for (int i = 0; i < kRows; i++) s_off[threadIdx.x * kRows + i] = max(prev, loc[i]);
  __syncthreads();
}

}  // namespace nbg
