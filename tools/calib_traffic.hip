// calib_traffic.hip -- what rocprofv3's FETCH_SIZE / WRITE_SIZE report for the access
// patterns of this repository's kernels, on a known byte count (MI355X_MICROARCH.md: the
// counters are calibrated only for 16-B/lane streaming; "calibrate on a known byte count in
// your own access pattern before trusting an absolute").
//
// Each kernel is launched once (after one untimed warm-up launch of a different size so the
// dispatch ids separate); stdout names every kernel with the bytes it moves by construction:
//   k_stream_read16   coalesced 16 B / lane loads of a 4 GiB array          (reference)
//   k_rand_read16     random 16-B loads from an 8 GiB table, 4 per lane      (k_probe's table)
//   k_stream_write8   coalesced 8 B / lane stores                            (k_probe's records)
//   k_stream_write16  coalesced 16 B / lane stores                           (reference)
//   k_log_write2      per wave 128-B rows of 2-B cells, 2 per step, own 1 MiB region
//                     per wave (k_extend's row log)
//   k_scatter_write16 random 16-B stores into a 4 GiB array                  (k_coarse_scatter)
//   k_log_read2       per wave, 16-row windows of 64 2-B cells around a drifting column of
//                     the rows k_log_write2 wrote (k_extend's traceback reads)
//   k_lane_read4      per wave, lane-interleaved 4-B words of its own 64 KiB region (the
//                     layout and width of k_extend's spill reloads from scratch)
//
// usage: calib_traffic            (then tools/calib_traffic.py turns the two PMC passes into
//                                  profiles/calib_traffic.json)
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

__global__ void k_stream_read16(const uint4 *a, uint64_t n, uint32_t *sink) {
  uint32_t acc = 0;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * blockDim.x) {
    const uint4 v = a[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678u) sink[0] = acc;        // keeps the loads, writes (almost) nothing
}

__global__ void k_rand_read16(const uint4 *t, uint64_t tn, uint64_t loads, uint32_t *sink) {
  uint32_t acc = 0;
  const uint64_t tid = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  const uint64_t nt = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = tid; i * 4 < loads; i += nt) {
    uint4 v[4];
#pragma unroll
    for (int q = 0; q < 4; q++) v[q] = t[mix(4 * i + q) % tn];
#pragma unroll
    for (int q = 0; q < 4; q++) acc ^= v[q].x ^ v[q].w;
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

__global__ void k_stream_write8(uint2 *a, uint64_t n) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * blockDim.x)
    a[i] = make_uint2((uint32_t)i, (uint32_t)(i >> 32));
}

__global__ void k_stream_write16(uint4 *a, uint64_t n) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * blockDim.x)
    a[i] = make_uint4((uint32_t)i, 1u, 2u, 3u);
}

// one wave per region of `rows` rows x 512 cells; per row 2 chunks of 64 cells written
__global__ void k_log_write2(uint16_t *log, uint32_t rows) {
  const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6, lane = threadIdx.x & 63;
  uint16_t *r = log + (size_t)wave * rows * 512;
  for (uint32_t e = 0; e < rows; e++) {
    const uint32_t b = (e * 37u) & 511u;           // the band drifts through the stripe
    r[(size_t)e * 512 + ((b + lane) & 511)] = (uint16_t)e;
    r[(size_t)e * 512 + ((b + 64 + lane) & 511)] = (uint16_t)(e + 1);
  }
}

// the traceback: rows e-1 .. e-16 read at 64 cells around the walk's column, window by
// window down to row 0
__global__ void k_log_read2(const uint16_t *log, uint32_t rows, uint32_t *sink) {
  const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6, lane = threadIdx.x & 63;
  const uint16_t *r = log + (size_t)wave * rows * 512;
  uint32_t acc = 0;
  for (uint32_t e0 = rows; e0 >= 16; e0 -= 16) {
    const uint32_t col = (e0 * 37u) & 511u;
#pragma unroll
    for (uint32_t i = 0; i < 16; i++)
      acc += r[(size_t)(e0 - 1 - i) * 512 + ((col + lane) & 511)];
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

// spill reloads: a wave's 64 KiB region as 256 words per lane, word j of lane l at
// 64 * j + l (the private-segment swizzle), each read once
__global__ void k_lane_read4(const uint32_t *a, uint32_t words, uint32_t *sink) {
  const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6, lane = threadIdx.x & 63;
  const uint32_t *r = a + (size_t)wave * words * 64;
  uint32_t acc = 0;
  for (uint32_t j = 0; j < words; j++) acc ^= r[64 * j + lane];
  if (acc == 0x12345678u) sink[0] = acc;
}

__global__ void k_scatter_write16(uint4 *a, uint64_t an, uint64_t n) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * blockDim.x)
    a[mix(i) % an] = make_uint4((uint32_t)i, 1u, 2u, 3u);
}

int main() {
  const uint64_t GiB = 1ull << 30;
  uint4 *big = nullptr, *table = nullptr;
  uint32_t *sink = nullptr;
  CK(hipMalloc(&big, 4 * GiB));
  CK(hipMalloc(&table, 8 * GiB));
  CK(hipMalloc(&sink, 64));
  CK(hipMemset(big, 1, 4 * GiB));
  CK(hipMemset(table, 2, 8 * GiB));
  const dim3 grid(256 * 64), block(256);
  const uint64_t n16 = 4 * GiB / 16, tn = 8 * GiB / 16;

  // warm-ups (small), then the measured launches
  hipLaunchKernelGGL(k_stream_read16, grid, block, 0, 0, big, n16 / 64, sink);
  hipLaunchKernelGGL(k_stream_read16, grid, block, 0, 0, big, n16, sink);
  printf("CALIB k_stream_read16 read_bytes %llu write_bytes 0\n", (unsigned long long)(n16 * 16));

  const uint64_t loads = 256ull << 20;            // 256 M random 16-B loads
  hipLaunchKernelGGL(k_rand_read16, grid, block, 0, 0, table, tn, loads / 64, sink);
  hipLaunchKernelGGL(k_rand_read16, grid, block, 0, 0, table, tn, loads, sink);
  printf("CALIB k_rand_read16 read_bytes %llu write_bytes 0 loads %llu\n",
         (unsigned long long)(loads * 16), (unsigned long long)loads);

  const uint64_t n8 = 4 * GiB / 8;
  hipLaunchKernelGGL(k_stream_write8, grid, block, 0, 0, (uint2 *)big, n8 / 64);
  hipLaunchKernelGGL(k_stream_write8, grid, block, 0, 0, (uint2 *)big, n8);
  printf("CALIB k_stream_write8 read_bytes 0 write_bytes %llu\n", (unsigned long long)(n8 * 8));

  hipLaunchKernelGGL(k_stream_write16, grid, block, 0, 0, big, n16 / 64);
  hipLaunchKernelGGL(k_stream_write16, grid, block, 0, 0, big, n16);
  printf("CALIB k_stream_write16 read_bytes 0 write_bytes %llu\n", (unsigned long long)(n16 * 16));

  const uint32_t rows = 1024;                      // 1 MiB per wave
  const uint32_t waves = (uint32_t)(4 * GiB / ((uint64_t)rows * 1024));   // 4096 waves
  hipLaunchKernelGGL(k_log_write2, dim3(waves / 64), dim3(256), 0, 0, (uint16_t *)big, rows / 16);
  hipLaunchKernelGGL(k_log_write2, dim3(waves / 4), dim3(256), 0, 0, (uint16_t *)big, rows);
  printf("CALIB k_log_write2 read_bytes 0 write_bytes %llu\n",
         (unsigned long long)waves * rows * 256ull);
  // reads of those rows (4 GiB written just before: past the 256 MiB Infinity Cache)
  hipLaunchKernelGGL(k_log_read2, dim3(waves / 64), dim3(256), 0, 0, (const uint16_t *)big,
                     rows / 16, sink);
  hipLaunchKernelGGL(k_log_read2, dim3(waves / 4), dim3(256), 0, 0, (const uint16_t *)big, rows,
                     sink);
  printf("CALIB k_log_read2 read_bytes %llu write_bytes 0\n",
         (unsigned long long)waves * rows * 128ull);

  // spill-reload layout over the 8 GiB table region (cold), 64 KiB per wave
  const uint32_t lw = 256, lwaves = (uint32_t)(8 * GiB / (64ull * 1024));   // 131072 waves
  hipLaunchKernelGGL(k_lane_read4, dim3(lwaves / 256), dim3(256), 0, 0, (const uint32_t *)table,
                     lw, sink);
  hipLaunchKernelGGL(k_lane_read4, dim3(lwaves / 4), dim3(256), 0, 0, (const uint32_t *)table, lw,
                     sink);
  printf("CALIB k_lane_read4 read_bytes %llu write_bytes 0\n",
         (unsigned long long)lwaves * lw * 256ull);

  const uint64_t ns = 256ull << 20;                // 256 M random 16-B stores
  hipLaunchKernelGGL(k_scatter_write16, grid, block, 0, 0, big, n16, ns / 64);
  hipLaunchKernelGGL(k_scatter_write16, grid, block, 0, 0, big, n16, ns);
  printf("CALIB k_scatter_write16 read_bytes 0 write_bytes %llu\n", (unsigned long long)(ns * 16));
  CK(hipDeviceSynchronize());
  CK(hipFree(big));
  CK(hipFree(table));
  CK(hipFree(sink));
  return 0;
}
