// Launch-gap calibration (GPU box): N dependent small kernels on one stream, launched eagerly
// vs captured once into a hipGraph and replayed.  Prints us per kernel for both.
//   hipcc --offload-arch=gfx950 -O2 tools/launch_gap.hip -o tools/launch_gap && tools/launch_gap
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>

__global__ void k_step(unsigned* x, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) x[i] = x[i] * 3u + 1u;
}

int main() {
  const int N = 200, n = 1 << 20;
  unsigned* x;
  hipMalloc(&x, n * 4);
  hipMemset(x, 0, n * 4);
  hipStream_t s;
  hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int grid : {64, 1024, 4096}) {
    for (int rep = 0; rep < 3; rep++) {
      hipEventRecord(a, s);
      for (int k = 0; k < N; k++) k_step<<<grid, 256, 0, s>>>(x, n);
      hipEventRecord(b, s);
      hipEventSynchronize(b);
      float ms = 0;
      hipEventElapsedTime(&ms, a, b);
      if (rep == 2) printf("eager  grid %5d: %.2f us per kernel\n", grid, ms * 1e3 / N);
    }
    hipGraph_t g;
    hipGraphExec_t ge;
    hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal);
    for (int k = 0; k < N; k++) k_step<<<grid, 256, 0, s>>>(x, n);
    hipStreamEndCapture(s, &g);
    hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
    for (int rep = 0; rep < 3; rep++) {
      hipEventRecord(a, s);
      hipGraphLaunch(ge, s);
      hipEventRecord(b, s);
      hipEventSynchronize(b);
      float ms = 0;
      hipEventElapsedTime(&ms, a, b);
      if (rep == 2) printf("graph  grid %5d: %.2f us per kernel\n", grid, ms * 1e3 / N);
    }
    hipGraphExecDestroy(ge);
    hipGraphDestroy(g);
  }
  // host round trip: kernel, copy 8 B to pinned host, sync, repeat
  unsigned long long* h;
  hipHostMalloc(&h, 64, hipHostMallocDefault);
  auto t0 = std::chrono::steady_clock::now();
  for (int k = 0; k < N; k++) {
    k_step<<<64, 256, 0, s>>>(x, n);
    hipMemcpyAsync(h, x, 8, hipMemcpyDeviceToHost, s);
    hipStreamSynchronize(s);
  }
  auto t1 = std::chrono::steady_clock::now();
  printf("round trip (kernel + 8 B d2h + sync): %.2f us each\n",
         std::chrono::duration<double, std::micro>(t1 - t0).count() / N);
  return 0;
}
