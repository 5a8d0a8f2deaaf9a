// hipcub::DeviceRadixSort::SortPairs over partial bit ranges of 64-bit keys: checks that the
// output is a permutation of the input pairs, ordered on the range's bits (DESIGN.md round
// 4: the range [40, 64) returned duplicated values on an 882,524-item run).
// build: hipcc --offload-arch=gfx950 -O2 -o tools/sortcheck tools/sortcheck.hip
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <cstdio>
#include <cstdint>
#include <vector>

static uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

static int check(size_t n, int b0, int b1) {
  std::vector<uint64_t> hk(n);
  std::vector<uint32_t> hv(n);
  for (size_t i = 0; i < n; i++) { hk[i] = mix64(i * 0x9E3779B97F4A7C15ull + 7); hv[i] = (uint32_t)i; }
  uint64_t *ki, *ko; uint32_t *vi, *vo; void *tmp = nullptr; size_t tb = 0;
  if (hipMalloc(&ki, 8 * n) || hipMalloc(&ko, 8 * n) || hipMalloc(&vi, 4 * n) || hipMalloc(&vo, 4 * n)) return 2;
  hipMemcpy(ki, hk.data(), 8 * n, hipMemcpyHostToDevice);
  hipMemcpy(vi, hv.data(), 4 * n, hipMemcpyHostToDevice);
  hipcub::DeviceRadixSort::SortPairs(nullptr, tb, ki, ko, vi, vo, (int)n, b0, b1, 0);
  if (hipMalloc(&tmp, tb)) return 2;
  hipcub::DeviceRadixSort::SortPairs(tmp, tb, ki, ko, vi, vo, (int)n, b0, b1, 0);
  if (hipDeviceSynchronize() != hipSuccess) return 3;
  std::vector<uint64_t> ok(n);
  std::vector<uint32_t> ov(n);
  hipMemcpy(ok.data(), ko, 8 * n, hipMemcpyDeviceToHost);
  hipMemcpy(ov.data(), vo, 4 * n, hipMemcpyDeviceToHost);
  std::vector<uint8_t> seen(n, 0);
  size_t dup = 0, brk = 0, pair = 0;
  const uint64_t mask = (b1 - b0 == 64) ? ~0ull : (((1ull << (b1 - b0)) - 1) << b0);
  for (size_t i = 0; i < n; i++) {
    if (ov[i] >= n || seen[ov[i]]++) dup++;
    else if (hk[ov[i]] != ok[i]) pair++;
    if (i && (ok[i] & mask) < (ok[i - 1] & mask)) brk++;
  }
  printf("n %zu bits [%d, %d): temp %zu B, %zu duplicate values, %zu broken pairs, %zu order breaks -> %s\n",
         n, b0, b1, tb, dup, pair, brk, (dup || pair || brk) ? "WRONG" : "ok");
  hipFree(ki); hipFree(ko); hipFree(vi); hipFree(vo); hipFree(tmp);
  return 0;
}

int main() {
  const size_t sizes[] = {100000, 882524, 1441007, 8000000, 1ull << 27};
  const int ranges[][2] = {{40, 64}, {32, 64}, {48, 64}, {0, 64}, {0, 32}};
  for (size_t n : sizes)
    for (auto &r : ranges)
      if (int rc = check(n, r[0], r[1])) return rc;
  return 0;
}
