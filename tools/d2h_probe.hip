// Device -> pinned-host copy rates for result hand-out (standalone, no torch):
//   hipcc -O3 --offload-arch=gfx950 tools/d2h_probe.hip -o tools/d2h_probe && tools/d2h_probe
// Copies B bytes (default 173 MB, C3's DISTINCT _dst result) from HBM into hipHostMalloc'd
// memory: hipMemcpyAsync (DMA engines), the same in 2 / 4 chunks on as many streams, and a
// kernel storing straight into the mapped host block.  One JSON line per case (best of 5).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
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

__global__ void k_copy16(const uint4* __restrict__ src, uint4* dst, size_t n) {
  for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x)
    dst[i] = src[i];
}

int main(int argc, char** argv) {
  const size_t bytes = argc > 1 ? size_t(atoll(argv[1])) : size_t(173076000);
  const size_t n16 = bytes / 16;
  void *d = nullptr, *h = nullptr;
  CK(hipMalloc(&d, bytes));
  CK(hipMemset(d, 1, bytes));
  CK(hipHostMalloc(&h, bytes, hipHostMallocDefault));
  memset(h, 0, bytes);
  hipStream_t s[4];
  for (auto& x : s) CK(hipStreamCreateWithFlags(&x, hipStreamNonBlocking));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  auto run = [&](const char* name, auto body) {
    float best = 1e30f;
    for (int r = 0; r < 5; r++) {
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(a, s[0]));
      body();
      for (int k = 1; k < 4; k++) {  // join the side streams into s[0]
        hipEvent_t e;
        CK(hipEventCreate(&e));
        CK(hipEventRecord(e, s[k]));
        CK(hipStreamWaitEvent(s[0], e, 0));
        CK(hipEventDestroy(e));
      }
      CK(hipEventRecord(b, s[0]));
      CK(hipEventSynchronize(b));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, a, b));
      best = std::min(best, ms);
    }
    printf("{\"case\": \"%s\", \"bytes\": %zu, \"ms\": %.3f, \"GBps\": %.1f}\n", name, bytes, best, bytes / (best * 1e6));
    fflush(stdout);
  };
  run("memcpy_async_1", [&] { CK(hipMemcpyAsync(h, d, bytes, hipMemcpyDeviceToHost, s[0])); });
  for (int k : {2, 4}) {
    char nm[64];
    snprintf(nm, sizeof nm, "memcpy_async_%d_streams", k);
    run(nm, [&] {
      const size_t part = (bytes / k + 4095) & ~size_t(4095);
      for (int i = 0; i < k; i++) {
        const size_t o = part * i, len = std::min(part, bytes - std::min(bytes, o));
        if (len) CK(hipMemcpyAsync(static_cast<char*>(h) + o, static_cast<char*>(d) + o, len, hipMemcpyDeviceToHost, s[i]));
      }
    });
  }
  for (int grid : {256, 1024, 4096}) {
    char nm[64];
    snprintf(nm, sizeof nm, "kernel_store_grid%d", grid);
    run(nm, [&] { k_copy16<<<grid, 256, 0, s[0]>>>(static_cast<const uint4*>(d), static_cast<uint4*>(h), n16); });
  }
  CK(hipHostFree(h));
  CK(hipFree(d));
  return 0;
}
