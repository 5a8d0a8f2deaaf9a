// hipcub::DeviceRadixSort::SortPairs over partial bit ranges of 64-bit keys: checks that the
// output is a permutation of the input pairs, ordered on the range's bits (DESIGN.md round
// 4: the range [40, 64) returned duplicated values on an 882,524-item run).  Round 5 adds the
// [0, end_bit) sorts mhap.hip runs, with keys below 2^end_bit as there: SortPairs of
// (hash function << 32 | value, read) at end_bit 32 + bits(H) (the MinHash index), SortKeys
// of 64-bit (read, code) keys with a 64-bit item count (k > 16), and the per-read
// DeviceSegmentedRadixSort::SortKeys of 32-bit codes at end_bit 2k -- each output checked to
// be a permutation of its input (a multiset compare), ordered.
// build: hipcc --offload-arch=gfx950 -O2 -o tools/sortcheck tools/sortcheck.hip
// run:   tools/sortcheck (the OverlapDriver ranges), tools/sortcheck mhap (mhap.hip's)
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <algorithm>
#include <string>

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

// keys below 2^end_bit (MHAP's), SortPairs [0, end_bit) or SortKeys (vals == false, 64-bit count)
static int check_low(size_t n, int end_bit, bool vals) {
  const uint64_t km = end_bit >= 64 ? ~0ull : ((1ull << end_bit) - 1);
  std::vector<uint64_t> hk(n);
  for (size_t i = 0; i < n; i++) hk[i] = mix64(i * 0x9E3779B97F4A7C15ull + 11) & km;
  uint64_t *ki, *ko; uint32_t *vi = nullptr, *vo = nullptr; void *tmp = nullptr; size_t tb = 0;
  if (hipMalloc(&ki, 8 * n) || hipMalloc(&ko, 8 * n)) return 2;
  hipMemcpy(ki, hk.data(), 8 * n, hipMemcpyHostToDevice);
  std::vector<uint32_t> hv;
  if (vals) {
    hv.resize(n);
    for (size_t i = 0; i < n; i++) hv[i] = (uint32_t)i;
    if (hipMalloc(&vi, 4 * n) || hipMalloc(&vo, 4 * n)) return 2;
    hipMemcpy(vi, hv.data(), 4 * n, hipMemcpyHostToDevice);
    hipcub::DeviceRadixSort::SortPairs(nullptr, tb, ki, ko, vi, vo, (int)n, 0, end_bit, 0);
    if (hipMalloc(&tmp, tb)) return 2;
    hipcub::DeviceRadixSort::SortPairs(tmp, tb, ki, ko, vi, vo, (int)n, 0, end_bit, 0);
  } else {
    hipcub::DeviceRadixSort::SortKeys(nullptr, tb, ki, ko, n, 0, end_bit, 0);
    if (hipMalloc(&tmp, tb)) return 2;
    hipcub::DeviceRadixSort::SortKeys(tmp, tb, ki, ko, n, 0, end_bit, 0);
  }
  if (hipDeviceSynchronize() != hipSuccess) return 3;
  std::vector<uint64_t> ok(n);
  hipMemcpy(ok.data(), ko, 8 * n, hipMemcpyDeviceToHost);
  size_t dup = 0, pair = 0, brk = 0, multiset = 0;
  if (vals) {
    std::vector<uint32_t> ov(n);
    hipMemcpy(ov.data(), vo, 4 * n, hipMemcpyDeviceToHost);
    std::vector<uint8_t> seen(n, 0);
    for (size_t i = 0; i < n; i++) {
      if (ov[i] >= n || seen[ov[i]]++) dup++;
      else if (hk[ov[i]] != ok[i]) pair++;
    }
  } else {
    std::vector<uint64_t> want(hk);
    std::sort(want.begin(), want.end());
    for (size_t i = 0; i < n; i++) multiset += want[i] != ok[i];
  }
  for (size_t i = 1; i < n; i++) brk += ok[i] < ok[i - 1];
  printf("n %zu bits [0, %d) %s: temp %zu B, %zu duplicate values, %zu broken pairs, %zu keys "
         "unlike the input's, %zu order breaks -> %s\n", n, end_bit, vals ? "SortPairs" : "SortKeys",
         tb, dup, pair, multiset, brk, (dup || pair || multiset || brk) ? "WRONG" : "ok");
  hipFree(ki); hipFree(ko); if (vals) { hipFree(vi); hipFree(vo); } hipFree(tmp);
  return 0;
}

// per-segment 32-bit codes below 2^end_bit, DeviceSegmentedRadixSort::SortKeys [0, end_bit)
static int check_seg(uint32_t nseg, uint32_t seglen, int end_bit) {
  const size_t n = (size_t)nseg * seglen;
  const uint32_t km = end_bit >= 32 ? ~0u : ((1u << end_bit) - 1);
  std::vector<uint32_t> hk(n);
  std::vector<int> off(nseg + 1);
  size_t at = 0;
  for (uint32_t s = 0; s < nseg; s++) {       // ragged segments: 1/2 .. 3/2 of seglen
    off[s] = (int)at;
    const size_t len = s + 1 == nseg ? n - at : std::min<size_t>(n - at, seglen / 2 + (mix64(s) % (seglen + 1)));
    at += len;
  }
  off[nseg] = (int)n;
  for (size_t i = 0; i < n; i++) hk[i] = (uint32_t)mix64(i + 99) & km;
  uint32_t *ki, *ko; int *doff; void *tmp = nullptr; size_t tb = 0;
  if (hipMalloc(&ki, 4 * n) || hipMalloc(&ko, 4 * n) || hipMalloc(&doff, 4 * (nseg + 1))) return 2;
  hipMemcpy(ki, hk.data(), 4 * n, hipMemcpyHostToDevice);
  hipMemcpy(doff, off.data(), 4 * (nseg + 1), hipMemcpyHostToDevice);
  hipcub::DeviceSegmentedRadixSort::SortKeys(nullptr, tb, ki, ko, (int)n, (int)nseg, doff, doff + 1, 0, end_bit, 0);
  if (hipMalloc(&tmp, std::max<size_t>(tb, 1))) return 2;
  hipcub::DeviceSegmentedRadixSort::SortKeys(tmp, tb, ki, ko, (int)n, (int)nseg, doff, doff + 1, 0, end_bit, 0);
  if (hipDeviceSynchronize() != hipSuccess) return 3;
  std::vector<uint32_t> ok(n);
  hipMemcpy(ok.data(), ko, 4 * n, hipMemcpyDeviceToHost);
  size_t bad = 0;
  for (uint32_t s = 0; s < nseg; s++) {
    std::vector<uint32_t> want(hk.begin() + off[s], hk.begin() + off[s + 1]);
    std::sort(want.begin(), want.end());
    for (int i = off[s]; i < off[s + 1]; i++) bad += want[i - off[s]] != ok[i];
  }
  printf("%u segments x ~%u, %zu keys, bits [0, %d) SegmentedSortKeys: %zu keys out of place -> %s\n",
         nseg, seglen, n, end_bit, bad, bad ? "WRONG" : "ok");
  hipFree(ki); hipFree(ko); hipFree(doff); hipFree(tmp);
  return 0;
}

int main(int argc, char **argv) {
  if (argc > 1 && std::string(argv[1]) == "mhap") {
    // the MinHash index: n = reads x H at the tests' sizes (120-400 reads, H 128-512) and
    // configs[3]'s (200k x 512), end_bit = 32 + bits(H)
    const size_t npairs[] = {120 * 128, 400 * 256, 400 * 512, 1441007, 200000ull * 512};
    const int ebits[] = {40, 41, 42};
    for (size_t n : npairs)
      for (int e : ebits)
        if (int rc = check_low(n, e, true)) return rc;
    // (read, code) keys for k = 20 (end_bit 40 + bits(reads + 1)), 64-bit counts
    const size_t nkeys[] = {100000, 2000000, 50000000};
    for (size_t n : nkeys)
      for (int e : {49, 50, 58})
        if (int rc = check_low(n, e, false)) return rc;
    // per-read segmented sorts of 32-bit codes, k = 12..16 (end_bit 24..32)
    for (int e : {24, 28, 32})
      for (uint32_t ns : {200u, 4000u})
        if (int rc = check_seg(ns, 15000, e)) return rc;
    return 0;
  }
  const size_t sizes[] = {100000, 882524, 1441007, 8000000, 1ull << 27};
  const int ranges[][2] = {{40, 64}, {32, 64}, {48, 64}, {0, 64}, {0, 32}};
  for (size_t n : sizes)
    for (auto &r : ranges)
      if (int rc = check(n, r[0], r[1])) return rc;
  return 0;
}
