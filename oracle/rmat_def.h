// oracle/rmat_def.h -- TEST INFRASTRUCTURE ONLY (see refcpu.h).
// The synthetic RMAT definition shared by the oracle's two restatements (refcpu.cpp: the KV
// store + processors; rmat_graph.cpp: the index-space CSR used at the configured sizes).  The
// product generator (nebula_amd/csrc/snapshot.hip) restates the same arithmetic on the device.
#pragma once
#include <cstdint>

namespace refcpu {
// ---------------------------------------------------------------------------------------------
// Synthetic RMAT definition (the product generator restates the same arithmetic on device).
//   sample i of E = ef << scale:  for level pairs draw h = splitmix64(seed ^ H1*(i+1) ^ H2*(l+1))
//   each 32-bit half picks a quadrant against (A, A+B, A+B+C) * 2^32 (Graph500 0.57/0.19/0.19).
//   vid(idx) = bijective 63-bit mix; weight(src, dst) = splitmix64(src ^ rotl(dst,32) ^ seed) % 1000
// ---------------------------------------------------------------------------------------------
inline uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}
constexpr uint32_t kTA = 2448131358u;    // floor(0.57 * 2^32)
constexpr uint32_t kTAB = 3264175144u;   // floor(0.76 * 2^32)
constexpr uint32_t kTABC = 4080218931u;  // floor(0.95 * 2^32)
inline void rmatPick(uint32_t r, uint64_t& u, uint64_t& v) {
  uint64_t bu = (r >= kTAB) ? 1 : 0;
  uint64_t bv = (r >= kTA && r < kTAB) || r >= kTABC ? 1 : 0;
  u = (u << 1) | bu;
  v = (v << 1) | bv;
}
inline void rmatEdge(uint64_t seed, int32_t scale, uint64_t i, uint64_t& u, uint64_t& v) {
  u = 0;
  v = 0;
  for (int32_t l = 0; l < scale; l += 2) {
    uint64_t h = splitmix64(seed ^ (0xD6E8FEB86659FD93ull * (i + 1)) ^
                            (0xA0761D6478BD642Full * uint64_t(l + 1)));
    rmatPick(uint32_t(h >> 32), u, v);
    if (l + 1 < scale) rmatPick(uint32_t(h), u, v);
  }
}
inline int64_t rmatVid(uint64_t idx, uint64_t seed) {
  const uint64_t M = (1ull << 63) - 1;
  uint64_t x = (idx + (splitmix64(seed) & M)) & M;
  x ^= x >> 29;
  x = (x * 0xBF58476D1CE4E5B9ull) & M;
  x ^= x >> 32;
  x = (x * 0x94D049BB133111EBull) & M;
  x ^= x >> 29;
  return int64_t(x);
}
inline int64_t rmatWeight(int64_t src, int64_t dst, uint64_t seed) {
  uint64_t d = uint64_t(dst);
  return int64_t(splitmix64(uint64_t(src) ^ ((d << 32) | (d >> 32)) ^ seed) % 1000);
}

}  // namespace refcpu
