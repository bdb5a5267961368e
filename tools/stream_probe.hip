// Streaming-read calibration for the bottom-up slab kernels (standalone, no torch):
//   hipcc -O3 --offload-arch=gfx950 tools/stream_probe.hip -o tools/stream_probe && tools/stream_probe
// Reads two arrays of n rows x 8 B (the quad slab's halves) with the access shapes the kernels
// use and prints the achieved read bandwidth of each; one JSON line per case.  Also the byte
// count for calibrating rocprofv3 FETCH_SIZE at 4-, 8- and 16-byte lanes (run under --pmc).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                 \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                \
    }                                                                         \
  } while (0)

// flat grid-stride read of one array, V bytes per lane
template <typename V>
__global__ void k_flat(const V* __restrict__ a, int64_t m, unsigned* out) {
  unsigned x = 0;
  for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < m; i += int64_t(gridDim.x) * blockDim.x) {
    const V v = a[i];
    if constexpr (sizeof(V) == 16) x ^= v.x ^ v.y ^ v.z ^ v.w;
    else if constexpr (sizeof(V) == 8) x ^= v.x ^ v.y;
    else x ^= v;
  }
  if (x == 0x12345678u) out[0] = x;
}

// the slab kernels' shape: a wave owns a tile (64 * RPL rows), tiles strided by the wave count;
// RPL = 1: 8-byte lanes (one row), RPL = 2: 16-byte lanes (two adjacent rows); both halves read;
// BITS: a 64-bit ballot word stored per 64 rows (the next-frontier / pending words)
template <int RPL, int BITS>
__global__ __launch_bounds__(1024) void k_tiles(const uint2* __restrict__ lo, const uint2* __restrict__ hi, int64_t n,
                                                unsigned long long* bits, unsigned* out) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = (int64_t(blockIdx.x) * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = (int64_t(gridDim.x) * blockDim.x) >> 6;
  const int64_t ntiles = n / (64 * RPL);
  unsigned x = 0;
  for (int64_t t = wave; t < ntiles; t += nwaves) {
    bool f0, f1 = false;
    if constexpr (RPL == 2) {
      const uint4 a = reinterpret_cast<const uint4*>(lo)[t * 64 + lane];
      const uint4 b = reinterpret_cast<const uint4*>(hi)[t * 64 + lane];
      f0 = int(a.x ^ b.x) < 0;
      f1 = int(a.z ^ b.z) < 0;
      x ^= a.y ^ b.w;
    } else {
      const uint2 a = lo[t * 64 + lane];
      const uint2 b = hi[t * 64 + lane];
      f0 = int(a.x ^ b.x) < 0;
      x ^= a.y ^ b.y;
    }
    if (BITS) {
      const unsigned long long e = __ballot(f0), o = __ballot(f1);
      if (lane == 0) bits[t * RPL] = e;
      if (RPL == 2 && lane == 1) bits[t * RPL + 1] = o;
    }
  }
  if (x == 0x12345678u) out[0] = x;
}

// random 4-byte probes into a table of tw words (the frontier-bitmap probes of the bottom-up
// kernels): m probes, word index = a multiplicative hash of the probe number
__global__ void k_probe(const unsigned* __restrict__ table, int64_t tw, int64_t m, unsigned* out) {
  unsigned x = 0;
  for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < m; i += int64_t(gridDim.x) * blockDim.x) {
    const uint64_t h = uint64_t(i) * 0x9E3779B97F4A7C15ull;
    x ^= table[(h >> 20) % uint64_t(tw)];
  }
  if (x == 0x12345678u) out[0] = x;
}

template <typename F>
static float time_ms(F f, int reps) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  f();
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(a));
  for (int i = 0; i < reps; i++) f();
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms / reps;
}

int main(int argc, char** argv) {
  const int64_t n = argc > 1 ? atoll(argv[1]) : (int64_t(1) << 25);  // rows (2^25 = the RMAT-26 slab)
  const int reps = 10;
  uint2 *lo, *hi;
  unsigned long long* bits;
  unsigned* out;
  CK(hipMalloc(&lo, n * 8));
  CK(hipMalloc(&hi, n * 8));
  CK(hipMalloc(&bits, n / 8 + 64));
  CK(hipMalloc(&out, 64));
  CK(hipMemset(lo, 1, n * 8));
  CK(hipMemset(hi, 2, n * 8));
  const double bytes2 = double(n) * 16;
  auto line = [&](const char* name, int grid, int block, double bytes, float ms) {
    printf("{\"case\": \"%s\", \"grid\": %d, \"block\": %d, \"bytes\": %.0f, \"us\": %.1f, \"GBps\": %.1f}\n", name, grid,
           block, bytes, ms * 1e3, bytes / (ms * 1e-3) / 1e9);
    fflush(stdout);
  };
  for (int grid : {1024, 4096, 16384}) {
    float ms = time_ms([&] { k_flat<uint4><<<grid, 256>>>(reinterpret_cast<const uint4*>(lo), n / 2, out); }, reps);
    line("flat16_one_array", grid, 256, double(n) * 8, ms);
    ms = time_ms([&] { k_flat<uint2><<<grid, 256>>>(lo, n, out); }, reps);
    line("flat8_one_array", grid, 256, double(n) * 8, ms);
    ms = time_ms([&] { k_flat<unsigned><<<grid, 256>>>(reinterpret_cast<const unsigned*>(lo), n * 2, out); }, reps);
    line("flat4_one_array", grid, 256, double(n) * 8, ms);
  }
  for (int grid : {256, 512, 1024, 2048}) {
    float ms = time_ms([&] { k_tiles<1, 0><<<grid, 1024>>>(lo, hi, n, bits, out); }, reps);
    line("tiles_8B_lanes", grid, 1024, bytes2, ms);
    ms = time_ms([&] { k_tiles<2, 0><<<grid, 1024>>>(lo, hi, n, bits, out); }, reps);
    line("tiles_16B_lanes", grid, 1024, bytes2, ms);
    ms = time_ms([&] { k_tiles<1, 1><<<grid, 1024>>>(lo, hi, n, bits, out); }, reps);
    line("tiles_8B_lanes_bits", grid, 1024, bytes2, ms);
    ms = time_ms([&] { k_tiles<2, 1><<<grid, 1024>>>(lo, hi, n, bits, out); }, reps);
    line("tiles_16B_lanes_bits", grid, 1024, bytes2, ms);
  }
  // random probes: 4 MiB table (the RMAT-26 frontier bitmap) and 1 GiB (no cache reuse)
  for (int64_t tw : {int64_t(1) << 20, int64_t(1) << 28}) {
    unsigned* table;
    CK(hipMalloc(&table, tw * 4));
    CK(hipMemset(table, 3, tw * 4));
    const int64_t m = int64_t(1) << 25;
    float ms = time_ms([&] { k_probe<<<4096, 256>>>(table, tw, m, out); }, reps);
    line(tw == (int64_t(1) << 20) ? "probe4_table4MiB" : "probe4_table1GiB", 4096, 256, double(m) * 4, ms);
    CK(hipFree(table));
  }
  CK(hipFree(lo));
  CK(hipFree(hi));
  CK(hipFree(bits));
  CK(hipFree(out));
  return 0;
}
