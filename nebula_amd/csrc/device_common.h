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

}  // namespace nbg
