// Random-lookup ceiling of the MI355X for k_probe's access pattern: independent random
// 16-B loads from a large table (power-of-two size, masked index: no 64-bit modulo in the
// loop, unlike calib_traffic's k_rand_read16), Q loads in flight per lane, over table sizes
// 2, 8 and 16 GiB (the 50k x 10 kb index table is 16 GiB).  Prints G loads/s per (size, Q);
// k_probe's rate (~40 G windows/s, HIP events in bench.py) is read against these.
//
// build: hipcc --offload-arch=gfx950 -O3 -o tools/bin/rand_ceiling tools/rand_ceiling.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                      \
      return 1;                                                                    \
    }                                                                              \
  } while (0)

__device__ __forceinline__ uint64_t mix(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

template <int Q>
__global__ void __launch_bounds__(256) k_rand(const uint4 *t, uint64_t mask, uint64_t iters,
                                              uint32_t *sink) {
  uint32_t acc = 0;
  const uint64_t tid = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  uint64_t x = mix(tid + 1);
  for (uint64_t i = 0; i < iters; i++) {
    uint4 v[Q];
#pragma unroll
    for (int q = 0; q < Q; q++) {
      x = x * 6364136223846793005ull + 1442695040888963407ull;   // LCG: cheap, independent
      v[q] = t[(x >> 17) & mask];
    }
#pragma unroll
    for (int q = 0; q < Q; q++) acc ^= v[q].x ^ v[q].w;
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

template <int Q>
static int run(const uint4 *t, uint64_t mask, uint32_t *sink, int blocks, double gib) {
  const uint64_t iters = 64;
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  hipLaunchKernelGGL(k_rand<Q>, dim3(blocks), dim3(256), 0, 0, t, mask, iters, sink);  // warm
  CK(hipEventRecord(a));
  for (int r = 0; r < 3; r++)
    hipLaunchKernelGGL(k_rand<Q>, dim3(blocks), dim3(256), 0, 0, t, mask, iters, sink);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  const double loads = 3.0 * blocks * 256.0 * iters * Q;
  printf("table %5.1f GiB  Q %2d  blocks %6d  %7.2f ms  %6.1f G loads/s  (%5.0f GB/s of 64-B sectors)\n",
         gib, Q, blocks, ms / 3, loads / (ms * 1e-3) / 1e9, loads * 64 / (ms * 1e-3) / 1e9);
  CK(hipEventDestroy(a));
  CK(hipEventDestroy(b));
  return 0;
}

int main() {
  const uint64_t max_bytes = 16ull << 30;
  uint4 *t = nullptr;
  uint32_t *sink = nullptr;
  CK(hipMalloc(&t, max_bytes));
  CK(hipMalloc(&sink, 4));
  CK(hipMemset(t, 1, max_bytes));
  for (uint64_t gib : {2ull, 8ull, 16ull}) {
    const uint64_t n = (gib << 30) / 16;
    const uint64_t mask = n - 1;
    for (int blocks : {2048, 8192}) {
      if (run<4>(t, mask, sink, blocks, (double)gib)) return 1;
      if (run<8>(t, mask, sink, blocks, (double)gib)) return 1;
      if (run<16>(t, mask, sink, blocks, (double)gib)) return 1;
    }
  }
  CK(hipFree(t));
  CK(hipFree(sink));
  return 0;
}
