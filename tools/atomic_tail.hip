// atomic_tail.hip -- what the block-sum tail of a resident grid costs: every block of a grid adds
// K per-block sums into device counters at its end (block_add_sums in traverse.hip).  Variants:
//   dense : the K counters of one hop on one 128-byte line (the engine's layout)
//   spread: each counter on a line of its own
//   shard : spread, and blocks add into one of S shards (blockIdx % S), S lines apart
// Each variant runs an empty grid (the tail alone) and a grid that first streams `mb` MB (the
// tail behind real work).  hipcc --offload-arch=gfx950 -O3 tools/atomic_tail.hip -o tools/atomic_tail
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                             \
  do {                                                                    \
    hipError_t e_ = (x);                                                  \
    if (e_ != hipSuccess) {                                               \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));             \
      exit(1);                                                            \
    }                                                                     \
  } while (0)

__global__ __launch_bounds__(1024) void k_tail(const uint4* __restrict__ src, size_t n16, unsigned long long* out,
                                               int K, int stride, int shards, unsigned long long* sink) {
  __shared__ unsigned long long s[16];
  unsigned long long acc = 0;
  for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n16; i += size_t(gridDim.x) * blockDim.x) {
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(src) + i);
    acc += v.x ^ v.w;
  }
  if (acc == 0x123456789ull) sink[0] = acc;  // keeps the loads
  if (threadIdx.x < 16) s[threadIdx.x] = threadIdx.x + 1;
  __syncthreads();
  if (threadIdx.x < unsigned(K)) {
    unsigned long long* o = out + size_t(blockIdx.x % unsigned(shards)) * size_t(K) * size_t(stride);
    __hip_atomic_fetch_add(o + size_t(threadIdx.x) * size_t(stride), s[threadIdx.x], __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
  }
}

int main(int argc, char** argv) {
  const int grid = argc > 1 ? atoi(argv[1]) : 512;
  const size_t mb = argc > 2 ? size_t(atol(argv[2])) : 200;
  const size_t bytes = mb << 20;
  uint4* src;
  unsigned long long *out, *sink;
  CK(hipMalloc(&src, bytes + 16));
  CK(hipMemset(src, 1, bytes + 16));
  CK(hipMalloc(&out, size_t(64) << 20));
  CK(hipMalloc(&sink, 64));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  struct V {
    const char* name;
    int K, stride, shards;
  } vs[] = {{"dense K=8", 8, 1, 1},      {"dense K=3", 3, 1, 1},        {"spread K=8", 8, 16, 1},
            {"shard8 K=8", 8, 16, 8},    {"shard32 K=8", 8, 16, 32},    {"none K=0", 0, 1, 1}};
  for (size_t work : {size_t(0), bytes}) {
    for (const V& v : vs) {
      float best = 1e30f;
      for (int rep = 0; rep < 20; rep++) {
        CK(hipMemset(out, 0, size_t(64) << 20));
        CK(hipEventRecord(a));
        k_tail<<<grid, 1024>>>(src, work / 16, out, v.K, v.stride, v.shards, sink);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        if (rep >= 3 && ms < best) best = ms;
      }
      printf("{\"grid\": %d, \"stream_mb\": %zu, \"variant\": \"%s\", \"us\": %.2f}\n", grid, work >> 20, v.name,
             best * 1e3);
    }
  }
  return 0;
}
