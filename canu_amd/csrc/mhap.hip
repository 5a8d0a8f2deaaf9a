// mhap.hip -- MHAP's MinHash sketch / filter stage on gfx950, behind include/canu_mhap.h.
//
// Replaces the MHAP jar canu runs for overlapper=mhap (src/pipelines/canu/OverlapMhap.pm:
// precompute :374-399, compare :476-498); output keeps MHAP's text line, which
// src/mhap/mhapConvert.C:114-150 converts to ovOverlap records.  The algorithm is
// specified in oracle/mhap_oracle.py (the CPU restatement; parity against the jar itself is
// unpinned -- see DESIGN.md), and implemented here with the same integer arithmetic:
//
//   k_mh_sketch    one block per read: MinHash sketch.  Each thread rolls 16 consecutive
//                  k-mers into registers (canonical 2-bit codes -> splitmix64), then walks the
//                  H xorshift64 hash functions; per function the block's minimum is a DPP
//                  wave reduction + one LDS update per wave.  Integer-VALU bound.
//   k_mh_ordered   one block per read: the ordered (second-stage) sketch -- a 4096-bin
//                  histogram of the k'-mer hashes picks the bins that hold the S smallest,
//                  those entries are collected and bitonic-sorted in LDS, deduplicated,
//                  the first S kept.
//   index          (j, value) -> read pairs sorted by hipcub radix sort, per-table offsets.
//   k_mh_candidates one wave per query: binary-search its H values in their tables, count
//                  matches per target in an LDS open-addressing table, emit targets with
//                  count >= min_matches.
//   k_mh_compare   one wave per candidate: merge the two ordered sketches (binary search in
//                  LDS), vote the orientation, radix-select the median offset, count the
//                  sketch entries inside the implied overlap, Jaccard -> Mash distance.
#include <hip/hip_runtime.h>
#include <type_traits>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cerrno>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/canu_mhap.h"

namespace mh {

constexpr int32_t I32MAX = 0x7FFFFFFF;
constexpr int RK = 32;            // k-mers per thread per round in k_mh_sketch
constexpr int OCAP = 4096;        // collected ordered-sketch entries per read (LDS)
constexpr int NBIN = 4096;        // histogram bins (hash >> 20)
constexpr int TSLOTS = 1024;      // candidate table slots per wave
constexpr int TSHIFT = 22;        // 32 - log2(TSLOTS)

struct Cand {
  uint32_t q, t, cnt, pad;
};

struct RecDev {
  uint32_t a, b;
  double erate;
  uint32_t count;
  int32_t a_bgn, a_end, a_len;
  uint32_t o;
  int32_t b_bgn, b_end, b_len;
};

__device__ __host__ __forceinline__ uint64_t splitmix64(uint64_t c) {
  uint64_t z = c + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__device__ __forceinline__ uint32_t base_code(uint8_t b) {
  b |= 0x20;
  return b == 'a' ? 0u : b == 'c' ? 1u : b == 'g' ? 2u : b == 't' ? 3u : 255u;
}

__device__ __forceinline__ int32_t wave_min(int32_t v) {
  int32_t t;
  t = __builtin_amdgcn_update_dpp(I32MAX, v, 0x111, 0xf, 0xf, false); v = v < t ? v : t;
  t = __builtin_amdgcn_update_dpp(I32MAX, v, 0x112, 0xf, 0xf, false); v = v < t ? v : t;
  t = __builtin_amdgcn_update_dpp(I32MAX, v, 0x114, 0xf, 0xf, false); v = v < t ? v : t;
  t = __builtin_amdgcn_update_dpp(I32MAX, v, 0x118, 0xf, 0xf, false); v = v < t ? v : t;
  t = __builtin_amdgcn_update_dpp(I32MAX, v, 0x142, 0xa, 0xf, false); v = v < t ? v : t;
  t = __builtin_amdgcn_update_dpp(I32MAX, v, 0x143, 0xc, 0xf, false); v = v < t ? v : t;
  return __builtin_amdgcn_readlane(v, 63);
}

// Rolling canonical k-mer over a read: push one base, report whether the k-mer ending at
// the pushed base is valid (no non-ACGT byte among its k bases).
struct Roller {
  uint64_t fwd = 0, rc = 0, mask;
  int32_t k, since_bad;         // bases pushed since the last bad one
  __device__ Roller(int32_t k_) : k(k_), since_bad(0) {
    mask = (k_ >= 32) ? ~0ull : ((1ull << (2 * k_)) - 1);
  }
  __device__ __forceinline__ bool push(uint32_t c) {
    if (c > 3) {
      since_bad = 0;
      c = 0;
    } else {
      since_bad++;
    }
    fwd = ((fwd << 2) | c) & mask;
    rc = (rc >> 2) | ((uint64_t)(3 - c) << (2 * (k - 1)));
    return since_bad >= k;
  }
  __device__ __forceinline__ uint64_t canon() const { return fwd < rc ? fwd : rc; }
  __device__ __forceinline__ uint32_t strand() const { return rc < fwd ? 1u : 0u; }
};

struct SketchArgs {
  const uint8_t *bases;
  const uint64_t *off;
  const uint32_t *len;
  uint32_t r0;                  // first read (0-based) of this launch
  uint32_t nreads;
  int32_t k, H;
  const uint64_t *filter;       // sorted canonical codes, or null
  uint32_t nfilter;
  int32_t *minhash;             // [read][H]
  unsigned long long *kmers;    // hashed k-mers (stats)
};

__device__ __forceinline__ bool filtered(const uint64_t *f, uint32_t n, uint64_t c) {
  uint32_t lo = 0, hi = n;
  while (lo < hi) {
    uint32_t mid = (lo + hi) >> 1;
    if (f[mid] < c) lo = mid + 1;
    else hi = mid;
  }
  return lo < n && f[lo] == c;
}

// One xorshift64 step (<<21, >>35, <<4) on the state's two 32-bit halves.  64-bit shifts
// (v_lshlrev_b64) measured faster than a v_alignbit split of the same step (108 vs 129 ms
// for the 50k-read sketch).
__device__ __forceinline__ void xs64(uint32_t &lo, uint32_t &hi) {
  uint64_t x = ((uint64_t)hi << 32) | lo;
  x ^= x << 21;
  x ^= x >> 35;
  x ^= x << 4;
  lo = (uint32_t)x;
  hi = (uint32_t)(x >> 32);
}

// One xorshift64 step of N independent chains, each sub-step over all chains before the
// next (shift results in their own registers): written chain by chain, the compiler emitted
// every chain's 9 instructions back to back, each on the previous one's result.  On the
// configs[3] sketch 845 -> 831 ms (profiles/r05h_mhap_xorshift_ab.txt, sketches equal); the
// kernel is VALU-bound on the draws themselves (~9.5 VALU per draw, the PMC's count:
// profiles/r05f_mhap_pmc.txt), so interleaving gains little
template <int N>
__device__ __forceinline__ void xs64_n(uint32_t (&lo)[N], uint32_t (&hi)[N]) {
  uint64_t x[N];
#pragma unroll
  for (int i = 0; i < N; i++) x[i] = ((uint64_t)hi[i] << 32) | lo[i];
  uint64_t t[N];
#pragma unroll
  for (int i = 0; i < N; i++) t[i] = x[i] << 21;
#pragma unroll
  for (int i = 0; i < N; i++) x[i] ^= t[i];
#pragma unroll
  for (int i = 0; i < N; i++) t[i] = x[i] >> 35;
#pragma unroll
  for (int i = 0; i < N; i++) x[i] ^= t[i];
#pragma unroll
  for (int i = 0; i < N; i++) t[i] = x[i] << 4;
#pragma unroll
  for (int i = 0; i < N; i++) x[i] ^= t[i];
#pragma unroll
  for (int i = 0; i < N; i++) { lo[i] = (uint32_t)x[i]; hi[i] = (uint32_t)(x[i] >> 32); }
}

// Stage 1 (oracle: mhap_oracle.sketch)
__global__ void __launch_bounds__(256) k_mh_sketch(SketchArgs A) {
  extern __shared__ int32_t s_min[];               // [4 waves][H]
  const uint32_t r = A.r0 + blockIdx.x;
  const uint32_t tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int32_t H = A.H, k = A.k;
  for (int32_t j = tid; j < 4 * H; j += 256) s_min[j] = I32MAX;
  __syncthreads();
  const uint8_t *s = A.bases + A.off[r];
  const int32_t L = (int32_t)A.len[r];
  const int32_t npos = L - k + 1;                  // k-mer start positions
  unsigned long long nk = 0;
  for (int32_t base = 0; base < npos; base += 256 * RK) {
    const int32_t p0 = base + (int32_t)tid * RK;   // this thread: starts p0 .. p0+RK-1
    uint64_t X[RK];
    uint32_t vm = 0;
    if (p0 < npos) {
      Roller R(k);
      for (int32_t i = 0; i < k - 1; i++) R.push(base_code(s[p0 + i]));
#pragma unroll
      for (int i = 0; i < RK; i++) {
        X[i] = 0;
        const int32_t p = p0 + i;
        if (p < npos) {
          bool ok = R.push(base_code(s[p + k - 1]));
          uint64_t c = R.canon();
          if (ok && A.filter && filtered(A.filter, A.nfilter, c)) ok = false;
          if (ok) {
            X[i] = splitmix64(c);
            vm |= 1u << i;
          }
        }
      }
    } else {
#pragma unroll
      for (int i = 0; i < RK; i++) X[i] = 0;
    }
    nk += __builtin_popcount(vm);
    if (__builtin_amdgcn_ballot_w64(vm != 0) == 0) continue;   // wave has nothing here
    // invalid slots take a copy of a valid k-mer's state (min is idempotent), so the
    // per-function loop needs no per-slot masking; a thread with no valid k-mer at all
    // contributes INT32_MAX
    {
      uint64_t x0 = 0;
#pragma unroll
      for (int i = RK - 1; i >= 0; i--) x0 = (vm >> i) & 1u ? X[i] : x0;
#pragma unroll
      for (int i = 0; i < RK; i++) X[i] = (vm >> i) & 1u ? X[i] : x0;
    }
    const bool live = vm != 0;
    int32_t *wm = s_min + wave * H;
    uint32_t XL[RK], XH[RK];
#pragma unroll
    for (int i = 0; i < RK; i++) { XL[i] = (uint32_t)X[i]; XH[i] = (uint32_t)(X[i] >> 32); }
    for (int32_t j = 0; j < H; j++) {
      int32_t v[RK];
#pragma unroll
      for (int i = 0; i < RK; i++) {
        xs64(XL[i], XH[i]);
        v[i] = (int32_t)XL[i];
      }
      // min over the slots as a min3 tree
      int32_t m = v[0];
#pragma unroll
      for (int i = 1; i + 1 < RK; i += 2) {
        const int32_t a = v[i] < v[i + 1] ? v[i] : v[i + 1];
        m = m < a ? m : a;
      }
      if ((RK & 1) == 0) m = m < v[RK - 1] ? m : v[RK - 1];
      m = live ? m : I32MAX;
      m = wave_min(m);
      if (lane == 0 && m < wm[j]) wm[j] = m;
    }
  }
  __syncthreads();
  for (int32_t j = tid; j < H; j += 256) {
    int32_t m = s_min[j];
    for (int w = 1; w < 4; w++) m = s_min[w * H + j] < m ? s_min[w * H + j] : m;
    A.minhash[(size_t)r * H + j] = m;
  }
  if (A.kmers) {
    for (int s2 = 32; s2 > 0; s2 >>= 1) nk += __shfl_xor(nk, s2);
    if (lane == 0 && nk) atomicAdd(A.kmers, nk);
  }
}

// ---- weighted MinHash (MHAP 2.x tf-idf repeat weighting, restated; canu_mhap.h) --------
// Each distinct k-mer of a read counts once with weight w >= 1 (w draws of its xorshift64
// chain per hash function), so the reads' k-mers are first made distinct and counted:
//   k_mh_kmer_keys  one block per read: (read index << 2k | canonical code) per valid k-mer
//                   (a sentinel for the rest), RKK consecutive positions per thread
//   radix sort      of the batch's keys (hipcub): each read's k-mers contiguous, equal
//                   k-mers adjacent -- tf is a run length
//   k_mh_sketch_w   one block per read over its sorted run: run starts only, weight from
//                   the run length and the -f table, then the sketch loop of k_mh_sketch
//                   with w draws per slot and function
constexpr int RKK = 16;           // positions per thread in k_mh_kmer_keys
#ifndef MH_RKW
#define MH_RKW 8
#endif
constexpr int RKW = MH_RKW;       // distinct k-mers per thread per round in k_mh_sketch_w

struct KeyArgs {
  const uint8_t *bases;
  const uint64_t *off;
  const uint32_t *len;
  uint32_t r0, nreads;
  int32_t k;
  const uint64_t *koff;         // per read of the batch: its first key
  uint64_t sentinel;            // key of an invalid position (sorts after every real key)
  void *keys;                   // K[]
  uint32_t *vcnt;               // 32-bit keys: valid k-mers per read
  unsigned long long *kmers;
};

// K = uint32_t (2k <= 32): each read's keys are its codes, sorted per read (segmented
// sort); K = uint64_t: read index << 2k | code, one sort over the batch.  4^k - 1 (all T)
// is never a canonical code, so it can mark an invalid position in the 32-bit form.
template <typename K>
__global__ void __launch_bounds__(256) k_mh_kmer_keys(KeyArgs A) {
  const uint32_t ri = blockIdx.x, r = A.r0 + ri;
  const int32_t k = A.k;
  const uint8_t *s = A.bases + A.off[r];
  const int32_t L = (int32_t)A.len[r];
  const int32_t npos = L - k + 1;
  K *out = (K *)A.keys + A.koff[ri];
  const uint64_t hi = sizeof(K) == 8 ? ((uint64_t)ri << (2 * k)) : 0;
  unsigned long long nk = 0;
  for (int32_t base = 0; base < npos; base += 256 * RKK) {
    const int32_t p0 = base + (int32_t)threadIdx.x * RKK;
    if (p0 >= npos) continue;
    Roller R(k);
    for (int32_t i = 0; i < k - 1; i++) R.push(base_code(s[p0 + i]));
#pragma unroll
    for (int i = 0; i < RKK; i++) {
      const int32_t p = p0 + i;
      if (p < npos) {
        const bool ok = R.push(base_code(s[p + k - 1]));
        out[p] = ok ? (K)(hi | R.canon()) : (K)A.sentinel;
        nk += ok;
      }
    }
  }
  for (int s2 = 32; s2 > 0; s2 >>= 1) nk += __shfl_xor(nk, s2);
  if ((threadIdx.x & 63) == 0 && nk) {
    if (A.kmers) atomicAdd(A.kmers, nk);
    if (sizeof(K) == 4) atomicAdd(&A.vcnt[ri], (uint32_t)nk);
  }
}

// The -f multipliers as an open-addressing table (a binary search over the sorted codes
// cost ~17 dependent loads per distinct k-mer): slot = splitmix64(code) & mask, linear
// probing, empty slots hold FEMPTY (no 2k-bit code reaches it).
constexpr uint64_t FEMPTY = ~0ull;
struct FreqSlot {
  uint64_t code;
  double mult;
};

struct WSketchArgs {
  const void *keys;             // K[], sorted (per read, or over the batch)
  uint64_t nkeys;
  const uint64_t *koff;         // 32-bit keys: per read its first key ...
  const uint32_t *vcnt;         // ... and its valid ones
  uint32_t r0, nreads;
  int32_t k, H;
  const FreqSlot *ftab;         // -f k-mers and their multipliers m(c), or null
  uint64_t fmask;               // table slots - 1
  double dmult;                 // m(c) of every other k-mer (< 0: it never enters a sketch)
  int32_t no_tf;
  int32_t *minhash;             // [read][H]
};

__device__ __forceinline__ uint64_t lower_bound_u64(const uint64_t *a, uint64_t n, uint64_t v) {
  uint64_t lo = 0, hi = n;
  while (lo < hi) {
    const uint64_t mid = (lo + hi) >> 1;
    if (a[mid] < v) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

// Stage 1, weighted (oracle: mhap_oracle.sketch_weighted)
template <typename K>
__global__ void __launch_bounds__(256) k_mh_sketch_w(WSketchArgs A) {
  const K *keys = (const K *)A.keys;
  extern __shared__ int32_t s_min[];               // [4 waves][H]
  __shared__ uint64_t s_rng[2];
  const uint32_t ri = blockIdx.x, r = A.r0 + ri;
  const uint32_t tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int32_t H = A.H, k = A.k;
  const uint64_t cmask = (k >= 32) ? ~0ull : ((1ull << (2 * k)) - 1);
  for (int32_t j = tid; j < 4 * H; j += 256) s_min[j] = I32MAX;
  if (tid == 0) {
    if (sizeof(K) == 4) {
      s_rng[0] = A.koff[ri];
      s_rng[1] = A.koff[ri] + A.vcnt[ri];
    } else {
      s_rng[0] = lower_bound_u64((const uint64_t *)keys, A.nkeys, (uint64_t)ri << (2 * k));
      s_rng[1] = lower_bound_u64((const uint64_t *)keys, A.nkeys, (uint64_t)(ri + 1) << (2 * k));
    }
  }
  __syncthreads();
  const uint64_t s0 = s_rng[0], s1 = s_rng[1];
  int32_t *wm = s_min + wave * H;
  for (uint64_t base = s0; base < s1; base += 256 * RKW) {
    const uint64_t p0 = base + (uint64_t)tid * RKW;
    uint32_t XL[RKW], XH[RKW];
    int32_t W[RKW];
    uint32_t vm = 0;
#pragma unroll
    for (int i = 0; i < RKW; i++) {
      XL[i] = XH[i] = 0;
      W[i] = 0;
      const uint64_t p = p0 + i;
      if (p < s1) {
        const K key = keys[p];
        if (p == s0 || keys[p - 1] != key) {             // a run start: a distinct k-mer
          uint64_t e = p + 1;
          while (e < s1 && keys[e] == key) e++;
          const uint64_t c = (uint64_t)key & cmask;
          double m = A.dmult;
          if (A.ftab) {
            for (uint64_t h = splitmix64(c) & A.fmask;; h = (h + 1) & A.fmask) {
              const FreqSlot fs = A.ftab[h];
              if (fs.code == c) { m = fs.mult; break; }
              if (fs.code == FEMPTY) break;
            }
          }
          if (m >= 0.0) {                       // m < 0: removed (--supress-noise 1)
            const double tf = A.no_tf ? 1.0 : (double)(e - p);
            const double wf = floor(tf * m + 0.5);
            W[i] = wf < 1.0 ? 1 : (int32_t)wf;
            const uint64_t x = splitmix64(c);
            XL[i] = (uint32_t)x;
            XH[i] = (uint32_t)(x >> 32);
            vm |= 1u << i;
          }
        }
      }
    }
    if (__builtin_amdgcn_ballot_w64(vm != 0) == 0) continue;
    // empty slots take a copy of a live slot's chain and weight (min is idempotent)
    {
      uint32_t l0 = 0, h0 = 0;
      int32_t w0 = 0;
#pragma unroll
      for (int i = RKW - 1; i >= 0; i--)
        if ((vm >> i) & 1u) { l0 = XL[i]; h0 = XH[i]; w0 = W[i]; }
#pragma unroll
      for (int i = 0; i < RKW; i++)
        if (!((vm >> i) & 1u)) { XL[i] = l0; XH[i] = h0; W[i] = w0; }
    }
    const bool live = vm != 0;
    // The draws per slot are a per-lane loop; when every live slot of the wave has the same
    // small weight (w = 2: a distinct k-mer at the default multiplier r + (1 - r) X = 1.9,
    // canu's case; or w = 1) the draws are straight-line code instead (no exec-mask loop
    // per slot and function)
    bool all1 = true, all2 = true;
#pragma unroll
    for (int i = 0; i < RKW; i++) { all1 &= W[i] == 1; all2 &= W[i] == 2; }
    const int32_t wu = __builtin_amdgcn_ballot_w64(live && !all2) == 0 ? 2
                     : __builtin_amdgcn_ballot_w64(live && !all1) == 0 ? 1 : 0;
    auto run = [&](auto wc) {
      constexpr int WC = decltype(wc)::value;
      for (int32_t j = 0; j < H; j++) {
        int32_t m = I32MAX;
        if constexpr (WC > 0) {
#pragma unroll
          for (int t = 0; t < WC; t++) {
            xs64_n<RKW>(XL, XH);
#pragma unroll
            for (int i = 0; i < RKW; i++) m = (int32_t)XL[i] < m ? (int32_t)XL[i] : m;
          }
        } else {
#pragma unroll
          for (int i = 0; i < RKW; i++) {
            for (int32_t t = 0; t < W[i]; t++) {
              xs64(XL[i], XH[i]);
              const int32_t v = (int32_t)XL[i];
              m = v < m ? v : m;
            }
          }
        }
        m = live ? m : I32MAX;
        m = wave_min(m);
        if (lane == 0 && m < wm[j]) wm[j] = m;
      }
    };
    if (wu == 2)      run(std::integral_constant<int, 2>());
    else if (wu == 1) run(std::integral_constant<int, 1>());
    else              run(std::integral_constant<int, 0>());
  }
  __syncthreads();
  for (int32_t j = tid; j < H; j += 256) {
    int32_t m = s_min[j];
    for (int w = 1; w < 4; w++) m = s_min[w * H + j] < m ? s_min[w * H + j] : m;
    A.minhash[(size_t)r * H + j] = m;
  }
}

struct OrderedArgs {
  const uint8_t *bases;
  const uint64_t *off;
  const uint32_t *len;
  uint32_t r0, nreads;
  int32_t k, S;
  uint64_t *ordered;            // [read][S]: hash << 32 | pos << 1 | strand
  uint32_t *ocount;
};

// Stage 3 input (oracle: mhap_oracle.ordered_sketch)
__global__ void __launch_bounds__(256) k_mh_ordered(OrderedArgs A) {
  __shared__ uint32_t hist[NBIN];
  __shared__ uint64_t list[OCAP];
  __shared__ uint32_t part[256];
  __shared__ int32_t sB;
  __shared__ uint32_t sN, sCnt;
  const uint32_t r = A.r0 + blockIdx.x;
  const uint32_t tid = threadIdx.x;
  const int32_t k = A.k, S = A.S;
  for (int32_t i = tid; i < NBIN; i += 256) hist[i] = 0;
  if (tid == 0) sCnt = 0;
  __syncthreads();
  const uint8_t *s = A.bases + A.off[r];
  const int32_t L = (int32_t)A.len[r];
  const int32_t npos = L - k + 1;
  const int32_t seg = npos > 0 ? (npos + 255) / 256 : 0;
  const int32_t p0 = (int32_t)tid * seg, p1 = min(p0 + seg, npos > 0 ? npos : 0);
  // pass 1: histogram of hash >> 20
  if (p0 < p1) {
    Roller R(k);
    for (int32_t i = 0; i < k - 1; i++) R.push(base_code(s[p0 + i]));
    for (int32_t p = p0; p < p1; p++) {
      if (R.push(base_code(s[p + k - 1]))) {
        uint32_t h = (uint32_t)(splitmix64(R.canon()) >> 32);
        atomicAdd(&hist[h >> 20], 1u);
      }
    }
  }
  __syncthreads();
  if (tid == 0) {
    // smallest bin B whose cumulative count reaches S (the last bin if none does), then
    // drop whole bins from the top while the collected entries exceed the LDS capacity
    uint32_t cs = 0;
    int32_t B = NBIN - 1;
    for (int32_t b = 0; b < NBIN; b++) {
      cs += hist[b];
      if (cs >= (uint32_t)S) { B = b; break; }
    }
    while (B >= 0 && cs > (uint32_t)OCAP) { cs -= hist[B]; B--; }
    sB = B;
    sN = cs;
  }
  __syncthreads();
  const int32_t B = sB;
  const uint32_t n = sN;
  // pass 2: collect the entries of bins <= B
  if (B >= 0 && p0 < p1) {
    Roller R(k);
    for (int32_t i = 0; i < k - 1; i++) R.push(base_code(s[p0 + i]));
    for (int32_t p = p0; p < p1; p++) {
      if (R.push(base_code(s[p + k - 1]))) {
        uint32_t h = (uint32_t)(splitmix64(R.canon()) >> 32);
        if ((int32_t)(h >> 20) <= B) {
          uint32_t idx = atomicAdd(&sCnt, 1u);
          if (idx < (uint32_t)OCAP)
            list[idx] = ((uint64_t)h << 32) | ((uint64_t)(uint32_t)p << 1) | R.strand();
        }
      }
    }
  }
  __syncthreads();
  uint32_t P = 1;
  while (P < n) P <<= 1;
  for (uint32_t i = n + tid; i < P; i += 256) list[i] = ~0ull;
  __syncthreads();
  // bitonic sort list[0 .. P) ascending
  for (uint32_t kk = 2; kk <= P; kk <<= 1) {
    for (uint32_t jj = kk >> 1; jj > 0; jj >>= 1) {
      for (uint32_t i = tid; i < P; i += 256) {
        uint32_t ix = i ^ jj;
        if (ix > i) {
          uint64_t a = list[i], b = list[ix];
          bool up = (i & kk) == 0;
          if ((a > b) == up) { list[i] = b; list[ix] = a; }
        }
      }
      __syncthreads();
    }
  }
  // dedup by hash (first = smallest position), keep the first S
  const uint32_t per = (n + 255) / 256;
  const uint32_t i0 = tid * per, i1 = min(i0 + per, n);
  uint32_t c = 0;
  for (uint32_t i = i0; i < i1; i++)
    if (i == 0 || (list[i] >> 32) != (list[i - 1] >> 32)) c++;
  part[tid] = c;
  __syncthreads();
  if (tid == 0) {
    uint32_t acc = 0;
    for (int t = 0; t < 256; t++) { uint32_t v = part[t]; part[t] = acc; acc += v; }
    A.ocount[r] = acc < (uint32_t)S ? acc : (uint32_t)S;
  }
  __syncthreads();
  uint32_t rank = part[tid];
  uint64_t *dst = A.ordered + (size_t)r * S;
  for (uint32_t i = i0; i < i1; i++) {
    if (i == 0 || (list[i] >> 32) != (list[i - 1] >> 32)) {
      if (rank < (uint32_t)S) dst[rank] = list[i];
      rank++;
    }
  }
}

// MinHash index keys: (j << 32 | value ^ 0x80000000), value = read; invalid -> table H.
// rows r0 .. r0 + nreads - 1 of the sketch (the indexed reads)
__global__ void k_mh_index_keys(const int32_t *mh, uint32_t r0, uint32_t nreads, int32_t H,
                                uint64_t *keys, uint32_t *vals) {
  size_t n = (size_t)nreads * H;
  for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < n;
       e += (size_t)gridDim.x * blockDim.x) {
    uint32_t r = r0 + (uint32_t)(e / H), j = (uint32_t)(e % H);
    int32_t v = mh[(size_t)r0 * H + e];
    keys[e] = (v == I32MAX) ? ((uint64_t)H << 32)
                            : (((uint64_t)j << 32) | ((uint32_t)v ^ 0x80000000u));
    vals[e] = r;
  }
}

__global__ void k_mh_table_offsets(const uint64_t *keys, size_t n, int32_t H, uint64_t *off) {
  int32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j > H) return;
  uint64_t key = (uint64_t)j << 32;
  size_t lo = 0, hi = n;
  while (lo < hi) {
    size_t mid = (lo + hi) >> 1;
    if (keys[mid] < key) lo = mid + 1;
    else hi = mid;
  }
  off[j] = lo;
}

struct CandArgs {
  const int32_t *mh;
  const uint64_t *keys;
  const uint32_t *vals;
  const uint64_t *toff;
  int32_t H;
  uint32_t q0, q1;              // queries [q0, q1), 0-based
  uint32_t all_targets;         // 0: targets t > q (all-vs-all, each pair once); 1: t != q
  uint32_t min_matches;
  Cand *out;
  uint32_t *nout;
  uint32_t cap;
  uint32_t *overflow;
};

// Stage 2 (oracle: mhap_oracle.candidates)
__global__ void __launch_bounds__(256) k_mh_candidates(CandArgs A) {
  extern __shared__ uint32_t s_tab[];              // [4][TSLOTS] keys, then [4][TSLOTS] counts
  const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const uint32_t q = A.q0 + blockIdx.x * 4 + wave;
  if (q >= A.q1) return;                           // whole wave leaves together
  uint32_t *tk = s_tab + wave * TSLOTS;
  uint32_t *tc = s_tab + 4 * TSLOTS + wave * TSLOTS;
  for (uint32_t i = lane; i < TSLOTS; i += 64) { tk[i] = 0; tc[i] = 0; }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  bool ovf = false;
  for (int32_t j = lane; j < A.H; j += 64) {
    const int32_t v = A.mh[(size_t)q * A.H + j];
    if (v == I32MAX) continue;
    const uint64_t key = ((uint64_t)j << 32) | ((uint32_t)v ^ 0x80000000u);
    uint64_t lo = A.toff[j], hi = A.toff[j + 1];
    while (lo < hi) {
      uint64_t mid = (lo + hi) >> 1;
      if (A.keys[mid] < key) lo = mid + 1;
      else hi = mid;
    }
    const uint64_t end = A.toff[j + 1];
    for (uint64_t i = lo; i < end && A.keys[i] == key; i++) {
      const uint32_t t = A.vals[i];
      if (A.all_targets ? t == q : t <= q) continue;
      uint32_t sl = (t * 2654435761u) >> TSHIFT;
      uint32_t probes = 0;
      for (;;) {
        uint32_t old = atomicCAS(&tk[sl], 0u, t + 1);
        if (old == 0u || old == t + 1) { atomicAdd(&tc[sl], 1u); break; }
        sl = (sl + 1) & (TSLOTS - 1);
        if (++probes >= TSLOTS) { ovf = true; break; }
      }
      if (ovf) break;
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  if (ovf) atomicOr(A.overflow, 1u);
  for (uint32_t i = lane; i < TSLOTS; i += 64) {
    const uint32_t key = tk[i], c = tc[i];
    if (key && c >= A.min_matches) {
      uint32_t idx = atomicAdd(A.nout, 1u);
      if (idx < A.cap) A.out[idx] = Cand{q, key - 1, c, 0};
      else atomicOr(A.overflow, 2u);
    }
  }
}

struct CmpArgs {
  const Cand *cand;
  uint32_t ncand;
  const uint64_t *ordered;
  const uint32_t *ocount;
  const uint32_t *len;
  uint32_t first_iid;
  int32_t S, kk, min_olap;
  double threshold;
  RecDev *out;
  uint32_t *nout;
  uint32_t cap;
  uint32_t *overflow;
};

__device__ __forceinline__ uint32_t lds_lower_bound_hash(const uint64_t *b, uint32_t n,
                                                         uint32_t h) {
  uint32_t lo = 0, hi = n;
  while (lo < hi) {
    uint32_t mid = (lo + hi) >> 1;
    if ((uint32_t)(b[mid] >> 32) < h) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ uint32_t popc64(uint64_t m) { return (uint32_t)__builtin_popcountll(m); }

// Stage 3 (oracle: mhap_oracle.compare).  Two waves per block; per wave LDS:
// B's sketch (S u64), the shared list (S x {pA, pB | same << 31}), a 256-bin histogram.
__global__ void __launch_bounds__(128) k_mh_compare(CmpArgs A) {
  extern __shared__ uint64_t s_cmp[];
  const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int32_t S = A.S, kk = A.kk;
  const size_t wave_words = (size_t)S + S + 128;   // u64 words: B, shared (2 x u32), hist
  uint64_t *bk = s_cmp + wave * wave_words;
  uint32_t *shA = (uint32_t *)(bk + S);
  uint32_t *shB = shA + S;
  uint32_t *hist = (uint32_t *)(bk + 2 * S);
  const uint64_t lane_lt = (1ull << lane) - 1;
  for (uint32_t c = blockIdx.x * 2 + wave; c < A.ncand; c += gridDim.x * 2) {
    wave_sync();                                   // the previous pair's LDS reads are done
    const Cand cd = A.cand[c];
    const uint32_t q = cd.q, t = cd.t;
    const uint32_t na = A.ocount[q], nb = A.ocount[t];
    const int32_t la = (int32_t)A.len[q], lb = (int32_t)A.len[t];
    const uint64_t *ak = A.ordered + (size_t)q * S;
    const uint64_t *bg = A.ordered + (size_t)t * S;
    for (uint32_t i = lane; i < nb; i += 64) bk[i] = bg[i];
    wave_sync();
    // shared entries (each A entry with the first B entry of its hash; the median and the
    // counts below only need them as a set): lane l merges its own run of A,
    // A[l c .. l c + c), against B from one binary search for the run's first hash -- about
    // c + nb / 64 LDS reads per lane instead of a binary search (log2 nb reads) per entry
    uint32_t nsh = 0, nsame = 0;
    const uint32_t crun = (na + 63) / 64;
    const uint32_t a_lo = lane * crun, a_hi = a_lo + crun < na ? a_lo + crun : na;
    uint32_t bp = a_lo < a_hi ? lds_lower_bound_hash(bk, nb, (uint32_t)(ak[a_lo] >> 32)) : nb;
    for (uint32_t st = 0; st < crun; st++) {
      const uint32_t i = a_lo + st;
      bool found = false, same = false;
      uint32_t pa = 0, pb = 0;
      if (i < a_hi) {
        const uint64_t ka = ak[i];
        const uint32_t h = (uint32_t)(ka >> 32);
        while (bp < nb && (uint32_t)(bk[bp] >> 32) < h) bp++;
        if (bp < nb && (uint32_t)(bk[bp] >> 32) == h) {
          const uint64_t kb = bk[bp];
          found = true;
          pa = (uint32_t)(ka >> 1) & 0x7FFFFFFFu;
          pb = (uint32_t)(kb >> 1) & 0x7FFFFFFFu;
          same = (ka & 1) == (kb & 1);
        }
      }
      const uint64_t fm = __builtin_amdgcn_ballot_w64(found);
      const uint64_t smm = __builtin_amdgcn_ballot_w64(found && same);
      if (found) {
        const uint32_t slot = nsh + popc64(fm & lane_lt);
        shA[slot] = pa;
        shB[slot] = pb | (same ? 0x80000000u : 0u);
      }
      nsh += popc64(fm);
      nsame += popc64(smm);
    }
    wave_sync();
    if (nsh == 0) continue;
    const uint32_t o = (nsame >= nsh - nsame) ? 0u : 1u;
    const uint32_t ncons = o == 0 ? nsame : nsh - nsame;
    if (ncons == 0) continue;
    // lower median of d = pA - pB' over the consistent entries: 4-pass radix select
    uint32_t kth = (ncons - 1) / 2, prefix = 0, pmask = 0;
    for (int pass = 3; pass >= 0; pass--) {
      for (uint32_t i = lane; i < 256; i += 64) hist[i] = 0;
      wave_sync();
      for (uint32_t i = lane; i < nsh; i += 64) {
        const uint32_t pb_raw = shB[i];
        const bool sm = (pb_raw >> 31) != 0;
        if (sm != (o == 0)) continue;
        const int32_t pb = (int32_t)(pb_raw & 0x7FFFFFFFu);
        const int32_t pbp = o == 0 ? pb : lb - kk - pb;
        const uint32_t u = (uint32_t)((int32_t)shA[i] - pbp) ^ 0x80000000u;
        if ((u & pmask) == prefix) atomicAdd(&hist[(u >> (8 * pass)) & 255u], 1u);
      }
      wave_sync();
      // bin holding the kth element: lane l owns bins 4l .. 4l+3
      uint32_t h0 = hist[4 * lane], h1 = hist[4 * lane + 1], h2 = hist[4 * lane + 2],
               h3 = hist[4 * lane + 3];
      uint32_t tot = h0 + h1 + h2 + h3;
      uint32_t incl = tot;                          // inclusive scan over lanes
      for (int sft = 1; sft < 64; sft <<= 1) {
        uint32_t v = __shfl_up(incl, sft);
        if ((int)lane >= sft) incl += v;
      }
      const uint32_t excl = incl - tot;
      const bool mine = excl <= kth && kth < incl;
      const uint64_t who = __builtin_amdgcn_ballot_w64(mine);
      const uint32_t owner = (uint32_t)__builtin_ctzll(who);
      uint32_t bin = 0, before = excl;
      if (mine) {
        uint32_t rem = kth - excl;
        if (rem < h0) bin = 0;
        else if (rem < h0 + h1) { bin = 1; before += h0; }
        else if (rem < h0 + h1 + h2) { bin = 2; before += h0 + h1; }
        else { bin = 3; before += h0 + h1 + h2; }
        bin += 4 * lane;
      }
      bin = __shfl(bin, owner);
      before = __shfl(before, owner);
      kth -= before;
      prefix |= bin << (8 * pass);
      pmask |= 255u << (8 * pass);
      wave_sync();
    }
    const int32_t dm = (int32_t)(prefix ^ 0x80000000u);
    const int32_t a_bgn = dm > 0 ? dm : 0;
    const int32_t a_end = la < lb + dm ? la : lb + dm;
    if (a_end - a_bgn < A.min_olap) continue;
    const int32_t b_bgn = a_bgn - dm, b_end = a_end - dm;
    uint32_t cA = 0, cB = 0, m = 0;
    for (uint32_t i0 = 0; i0 < na; i0 += 64) {
      const uint32_t i = i0 + lane;
      bool in = false;
      if (i < na) {
        const int32_t p = (int32_t)((uint32_t)(ak[i] >> 1) & 0x7FFFFFFFu);
        in = p >= a_bgn && p <= a_end - kk;
      }
      cA += popc64(__builtin_amdgcn_ballot_w64(in));
    }
    for (uint32_t i0 = 0; i0 < nb; i0 += 64) {
      const uint32_t i = i0 + lane;
      bool in = false;
      if (i < nb) {
        const int32_t pb = (int32_t)((uint32_t)(bk[i] >> 1) & 0x7FFFFFFFu);
        const int32_t p = o == 0 ? pb : lb - kk - pb;
        in = p >= b_bgn && p <= b_end - kk;
      }
      cB += popc64(__builtin_amdgcn_ballot_w64(in));
    }
    for (uint32_t i0 = 0; i0 < nsh; i0 += 64) {
      const uint32_t i = i0 + lane;
      bool in = false;
      if (i < nsh) {
        const uint32_t pb_raw = shB[i];
        const bool sm = (pb_raw >> 31) != 0;
        if (sm == (o == 0)) {
          const int32_t pa = (int32_t)shA[i];
          const int32_t pb = (int32_t)(pb_raw & 0x7FFFFFFFu);
          const int32_t pbp = o == 0 ? pb : lb - kk - pb;
          in = pa >= a_bgn && pa <= a_end - kk && pbp >= b_bgn && pbp <= b_end - kk;
        }
      }
      m += popc64(__builtin_amdgcn_ballot_w64(in));
    }
    if (m == 0) continue;
    const double J = (double)m / (double)(cA + cB - m);
    const double D = -log(2.0 * J / (1.0 + J)) / (double)kk;
    if (1.0 - D < A.threshold) continue;
    if (lane == 0) {
      uint32_t idx = atomicAdd(A.nout, 1u);
      if (idx < A.cap) {
        RecDev rr;
        rr.a = A.first_iid + q;
        rr.b = A.first_iid + t;
        rr.erate = D < 1.0 ? D : 1.0;
        rr.count = cd.cnt;
        rr.a_bgn = a_bgn; rr.a_end = a_end; rr.a_len = la;
        rr.o = o;
        rr.b_bgn = b_bgn; rr.b_end = b_end; rr.b_len = lb;
        A.out[idx] = rr;
      } else {
        atomicOr(A.overflow, 1u);
      }
    }
  }
}

}  // namespace mh

using namespace mh;

// ---------------------------------------------------------------------------------------
static thread_local std::string g_merr;

static int mfail(int code, const char *fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_merr = buf;
  return code;
}

enum { M_OK = 0, M_NO_DEVICE = -1, M_BAD_PARAM = -2, M_BAD_INPUT = -4, M_HIP = -5,
       M_OOM = -6, M_STATE = -7 };

#define MHC(x)                                                                          \
  do {                                                                                  \
    hipError_t _e = (x);                                                                \
    if (_e != hipSuccess)                                                               \
      return mfail(M_HIP, "%s:%d %s: %s", __FILE__, __LINE__, #x, hipGetErrorString(_e)); \
  } while (0)

template <typename T>
struct MBuf {
  T *p = nullptr;
  size_t n = 0;
  ~MBuf() { release(); }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    n = 0;
  }
  hipError_t alloc(size_t count) {
    if (count <= n && p) return hipSuccess;
    release();
    hipError_t e = hipMalloc((void **)&p, sizeof(T) * std::max<size_t>(count, 1));
    if (e == hipSuccess) n = count;
    return e;
  }
};

struct mhap_ctx {
  mhap_params P;
  int device = 0;
  hipStream_t stream = nullptr;
  hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};   // [2..3]: the MinHash kernel
  uint32_t first_iid = 1, nreads = 0;
  std::vector<uint32_t> h_len;
  MBuf<uint8_t> bases_own;
  const uint8_t *d_bases = nullptr;
  MBuf<uint64_t> off_own;
  const uint64_t *d_off = nullptr;
  MBuf<uint32_t> d_len;
  MBuf<uint64_t> filter;
  uint32_t nfilter = 0;
  // repeat weighting (mhap_set_kmer_frequencies): weighted sketch when repeat_weight >= 0
  mhap_weighting W{-1.0, 10.0, 1e-5, 0};
  bool weighted = false;
  MBuf<uint64_t> wkeys, wkeys2;
  MBuf<FreqSlot> ftab;
  uint64_t fmask = 0;
  uint32_t nf = 0;
  double dmult = 1.0;
  MBuf<uint8_t> wsort_tmp;
  MBuf<int32_t> minhash;
  MBuf<uint64_t> ordered;
  MBuf<uint32_t> ocount;
  MBuf<uint64_t> keys, keys2, toff;
  MBuf<uint32_t> vals, vals2;
  MBuf<uint8_t> sort_tmp;
  size_t nkeys = 0;
  bool indexed = false;
  MBuf<Cand> cand;
  MBuf<RecDev> rec;
  MBuf<uint32_t> ctr;
  MBuf<unsigned long long> kctr;
  uint64_t nrec = 0;
  mhap_stats stats{};
};

static float elapsed(mhap_ctx *c) {
  float t = 0;
  (void)hipEventElapsedTime(&t, c->ev[0], c->ev[1]);
  return t;
}

extern "C" {

int mhap_abi_version(void) { return MHAP_ABI_VERSION; }
const char *mhap_last_error(void) { return g_merr.c_str(); }

void mhap_params_init(mhap_params *p) {
  p->k = 16;
  p->num_hashes = 512;
  p->min_matches = 3;
  p->ordered_sketch = 1536;
  p->ordered_k = 12;
  p->min_olap = 500;
  p->threshold = 0.78;
}

int mhap_ctx_create(const mhap_params *p, int device, mhap_ctx **out) {
  *out = nullptr;
  if (!p) return mfail(M_BAD_PARAM, "null params");
  if (p->k < 1 || p->k > 32 || p->ordered_k < 1 || p->ordered_k > 32)
    return mfail(M_BAD_PARAM, "k-mer sizes must be 1..32");
  if (p->num_hashes < 1 || p->num_hashes > 1024)
    return mfail(M_BAD_PARAM, "num_hashes must be 1..1024");
  if (p->ordered_sketch < 1 || p->ordered_sketch > 1984)   // k_mh_compare LDS: 2 waves x 8(2S+128) B
    return mfail(M_BAD_PARAM, "ordered_sketch must be 1..1984");
  if (p->min_matches < 1) return mfail(M_BAD_PARAM, "min_matches must be >= 1");
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= device || device < 0)
    return mfail(M_NO_DEVICE, "no HIP device %d", device);
  hipDeviceProp_t prop;
  MHC(hipGetDeviceProperties(&prop, device));
  if (strncmp(prop.gcnArchName, "gfx950", 6) != 0)
    return mfail(M_NO_DEVICE, "device %d is %s, not gfx950", device, prop.gcnArchName);
  MHC(hipSetDevice(device));
  mhap_ctx *c = new mhap_ctx();
  c->P = *p;
  c->device = device;
  if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreate(&c->ev[0]) != hipSuccess || hipEventCreate(&c->ev[1]) != hipSuccess ||
      hipEventCreate(&c->ev[2]) != hipSuccess || hipEventCreate(&c->ev[3]) != hipSuccess) {
    delete c;
    return mfail(M_HIP, "stream/event creation failed");
  }
  if (c->ctr.alloc(16) != hipSuccess || c->kctr.alloc(1) != hipSuccess) {
    delete c;
    return mfail(M_OOM, "counters");
  }
  *out = c;
  return M_OK;
}

void mhap_ctx_destroy(mhap_ctx *c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  for (auto &e : c->ev)
    if (e) (void)hipEventDestroy(e);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
}

// the MinHash kernel's launch just completed (events ev[2] .. ev[3]): its time, summed
static void sketch_kernel_time(mhap_ctx *c) {
  float t = 0;
  (void)hipEventElapsedTime(&t, c->ev[2], c->ev[3]);
  c->stats.ms_sketch_kernel += t;
  c->stats.sketch_launches++;
}

static int alloc_sketches(mhap_ctx *c) {
  const size_t n = c->nreads;
  if (c->minhash.alloc(n * c->P.num_hashes) || c->ordered.alloc(n * c->P.ordered_sketch) ||
      c->ocount.alloc(n))
    return mfail(M_OOM, "sketch arrays for %zu reads", n);
  MHC(hipMemsetAsync(c->ocount.p, 0, 4 * n, c->stream));
  c->indexed = false;
  return M_OK;
}

static int set_lengths(mhap_ctx *c, uint32_t first_iid, uint32_t nreads, const uint32_t *lens) {
  if (first_iid == 0) return mfail(M_BAD_PARAM, "gkStore IDs start at 1");
  for (uint32_t i = 0; i < nreads; i++)
    if (lens[i] >= 0x7FFFFFFFu) return mfail(M_BAD_INPUT, "read %u too long", first_iid + i);
  c->first_iid = first_iid;
  c->nreads = nreads;
  c->h_len.assign(lens, lens + nreads);
  if (c->d_len.alloc(nreads)) return mfail(M_OOM, "lengths");
  MHC(hipMemcpyAsync(c->d_len.p, lens, 4ull * nreads, hipMemcpyHostToDevice, c->stream));
  return alloc_sketches(c);
}

int mhap_load_reads(mhap_ctx *c, uint32_t first_iid, uint32_t nreads, const uint8_t *bases,
                    const uint64_t *offsets, const uint32_t *lengths) {
  if (!c) return mfail(M_STATE, "null context");
  MHC(hipSetDevice(c->device));
  uint64_t total = 0;
  for (uint32_t i = 0; i < nreads; i++)
    total = std::max<uint64_t>(total, offsets[i] + lengths[i]);
  if (c->bases_own.alloc(total + 64) || c->off_own.alloc(nreads))
    return mfail(M_OOM, "reads (%llu bytes)", (unsigned long long)total);
  MHC(hipMemcpyAsync(c->bases_own.p, bases, total, hipMemcpyHostToDevice, c->stream));
  MHC(hipMemcpyAsync(c->off_own.p, offsets, 8ull * nreads, hipMemcpyHostToDevice, c->stream));
  c->d_bases = c->bases_own.p;
  c->d_off = c->off_own.p;
  int rc = set_lengths(c, first_iid, nreads, lengths);
  if (rc) return rc;
  MHC(hipStreamSynchronize(c->stream));
  return M_OK;
}

int mhap_load_reads_device(mhap_ctx *c, uint32_t first_iid, uint32_t nreads,
                           const uint8_t *d_bases, const uint64_t *d_offsets,
                           const uint32_t *h_lengths) {
  if (!c) return mfail(M_STATE, "null context");
  MHC(hipSetDevice(c->device));
  c->d_bases = d_bases;
  c->d_off = d_offsets;
  int rc = set_lengths(c, first_iid, nreads, h_lengths);
  if (rc) return rc;
  MHC(hipStreamSynchronize(c->stream));
  return M_OK;
}

int mhap_set_filter_kmers(mhap_ctx *c, const char *kmers, uint64_t n) {
  if (!c) return mfail(M_STATE, "null context");
  const uint32_t k = c->P.k;
  std::vector<uint64_t> codes;
  for (uint64_t i = 0; i < n; i++) {
    uint64_t f = 0, r = 0;
    bool ok = true;
    for (uint32_t t = 0; t < k; t++) {
      char ch = kmers[i * k + t] | 0x20;
      uint64_t b = ch == 'a' ? 0 : ch == 'c' ? 1 : ch == 'g' ? 2 : ch == 't' ? 3 : 9;
      if (b > 3) { ok = false; break; }
      f = (f << 2) | b;
      r |= (3 - b) << (2 * t);
    }
    if (ok) codes.push_back(f < r ? f : r);
  }
  std::sort(codes.begin(), codes.end());
  codes.erase(std::unique(codes.begin(), codes.end()), codes.end());
  MHC(hipSetDevice(c->device));
  if (c->filter.alloc(codes.size())) return mfail(M_OOM, "filter");
  if (!codes.empty())
    MHC(hipMemcpy(c->filter.p, codes.data(), 8 * codes.size(), hipMemcpyHostToDevice));
  c->nfilter = (uint32_t)codes.size();
  return M_OK;
}

void mhap_weighting_init(mhap_weighting *w) {
  w->repeat_weight = -1.0;
  w->repeat_idf_scale = 10.0;
  w->filter_threshold = 1e-5;
  w->no_tf = 0;
  w->supress_noise = 0;
}

static bool kmer_code(const char *km, uint32_t k, uint64_t *canon) {
  uint64_t f = 0, r = 0;
  for (uint32_t t = 0; t < k; t++) {
    const char ch = km[t] | 0x20;
    const uint64_t b = ch == 'a' ? 0 : ch == 'c' ? 1 : ch == 'g' ? 2 : ch == 't' ? 3 : 9;
    if (b > 3) return false;
    f = (f << 2) | b;
    r |= (3 - b) << (2 * t);
  }
  *canon = f < r ? f : r;
  return true;
}

int mhap_set_kmer_frequencies(mhap_ctx *c, const char *kmers, const double *fractions,
                              uint64_t n, const mhap_weighting *w) {
  if (!c || !w) return mfail(M_STATE, "null argument");
  if (n && (!kmers || !fractions)) return mfail(M_BAD_PARAM, "null k-mers / fractions");
  if (!(w->filter_threshold > 0.0) || !(w->repeat_idf_scale >= 1.0))
    return mfail(M_BAD_PARAM, "filter_threshold must be > 0 and repeat_idf_scale >= 1");
  const uint32_t k = c->P.k;
  if (w->repeat_weight >= 0.0 && 2 * k > 56)
    return mfail(M_BAD_PARAM, "weighted sketches need k <= 28 (read index beside the code)");
  if (w->supress_noise < 0 || w->supress_noise > 2)
    return mfail(M_BAD_PARAM, "--supress-noise %d (0, 1 or 2)", w->supress_noise);
  if (w->supress_noise && w->repeat_weight < 0.0)
    return mfail(M_BAD_PARAM, "--supress-noise needs the weighted sketch (--repeat-weight >= 0)");
  // --supress-noise: every -f k-mer is in the table (those below the threshold at the top
  // multiplier), so that a k-mer NOT in the file can be told apart
  const bool noise = w->supress_noise != 0 && n != 0;
  c->W = *w;
  c->weighted = w->repeat_weight >= 0.0;
  // the -f k-mers at or above the threshold, canonical (both strands are listed), the
  // largest fraction per k-mer
  std::vector<std::pair<uint64_t, double>> F;
  for (uint64_t i = 0; i < n; i++) {
    uint64_t cc;
    if (!kmer_code(kmers + i * k, k, &cc)) continue;
    if (!(fractions[i] >= w->filter_threshold) && !noise) continue;
    F.emplace_back(cc, fractions[i]);
  }
  std::sort(F.begin(), F.end());
  std::vector<uint64_t> codes;
  std::vector<double> fr;
  for (size_t i = 0; i < F.size(); i++) {
    if (!codes.empty() && codes.back() == F[i].first) {
      fr.back() = std::max(fr.back(), F[i].second);
      continue;
    }
    codes.push_back(F[i].first);
    fr.push_back(F[i].second);
  }
  MHC(hipSetDevice(c->device));
  if (!c->weighted) {                 // MHAP 1.x: the repeats are dropped
    if (c->filter.alloc(codes.size())) return mfail(M_OOM, "filter");
    if (!codes.empty())
      MHC(hipMemcpy(c->filter.p, codes.data(), 8 * codes.size(), hipMemcpyHostToDevice));
    c->nfilter = (uint32_t)codes.size();
    c->nf = 0;
    return M_OK;
  }
  c->nfilter = 0;
  // multipliers m(c) = r + (1 - r) * (1 + (X - 1) * (idf - idf_min) / (idf_max - idf_min))
  const double r = w->repeat_weight, X = w->repeat_idf_scale;
  const double idf_max = log(1.0 / w->filter_threshold);
  double idf_min = idf_max;
  std::vector<double> idf(codes.size());
  for (size_t i = 0; i < codes.size(); i++) {
    // below the threshold (only listed with --supress-noise): the top idf
    idf[i] = fr[i] >= w->filter_threshold ? log(1.0 / fr[i]) : idf_max;
    idf_min = std::min(idf_min, idf[i]);
  }
  auto mult = [&](double v) {
    if (r >= 1.0 || codes.empty()) return 1.0;
    const double sc = idf_max > idf_min ? 1.0 + (X - 1.0) * (v - idf_min) / (idf_max - idf_min) : X;
    return r + (1.0 - r) * sc;
  };
  std::vector<double> m(codes.size());
  for (size_t i = 0; i < codes.size(); i++) m[i] = mult(idf[i]);
  // a k-mer not in the table: the top multiplier; with --supress-noise 2 the most frequent
  // k-mer's (suppressed like a repeat), with 1 none (-1: it never enters a sketch)
  c->dmult = !noise ? mult(idf_max) : w->supress_noise == 2 ? mult(idf_min) : -1.0;
  // open addressing at load <= 1/2
  uint64_t slots = 16;
  while (slots < 2 * codes.size() + 1) slots <<= 1;
  std::vector<FreqSlot> tab(slots, FreqSlot{FEMPTY, 0.0});
  for (size_t i = 0; i < codes.size(); i++) {
    uint64_t h = splitmix64(codes[i]) & (slots - 1);
    while (tab[h].code != FEMPTY) h = (h + 1) & (slots - 1);
    tab[h] = FreqSlot{codes[i], m[i]};
  }
  if (c->ftab.alloc(slots)) return mfail(M_OOM, "k-mer frequency table");
  MHC(hipMemcpy(c->ftab.p, tab.data(), sizeof(FreqSlot) * slots, hipMemcpyHostToDevice));
  c->fmask = slots - 1;
  c->nf = (uint32_t)codes.size();
  return M_OK;
}

// The weighted MinHash of reads r0 .. r0+nr-1 in batches of <= WKEY_BUDGET positions: keys,
// radix sort, sketch (the ordered sketch is the caller's, unweighted as in the jar).
static int sketch_weighted(mhap_ctx *c, uint32_t r0, uint32_t nr) {
  hipStream_t s = c->stream;
  const uint32_t k = c->P.k;
  // k <= 16: 32-bit codes sorted per read (a segmented sort, 4 B per key); longer k-mers:
  // 64-bit (read index, code) keys in one sort over the batch
  const bool k32 = 2 * k <= 32;
  const uint64_t WKEY_BUDGET = 1ull << 30;                  // keys per batch
  const uint32_t idx_bits = 64 - 2 * k;
  const uint64_t max_reads = k32 ? (1u << 20)
                                 : (idx_bits >= 32 ? 0xFFFFFFF0ull : (1ull << idx_bits) - 2);
  for (uint32_t a = 0; a < nr;) {
    std::vector<uint64_t> koff;
    uint64_t tot = 0;
    uint32_t b = a;
    while (b < nr && b - a < max_reads && b - a < (1u << 20)) {
      const int64_t np = (int64_t)c->h_len[r0 + b] - (int64_t)k + 1;
      const uint64_t add = np > 0 ? (uint64_t)np : 0;
      if (tot + add > WKEY_BUDGET && b > a) break;
      koff.push_back(tot);
      tot += add;
      b++;
    }
    koff.push_back(tot);                                    // the segments' end offsets
    const uint32_t nb = b - a;
    uint32_t end_bit;
    uint64_t sentinel;
    if (k32) {
      end_bit = 2 * k;
      sentinel = (1ull << (2 * k)) - 1;                     // never a canonical code
    } else {
      end_bit = 2 * k + (uint32_t)std::max<int>(1, 64 - __builtin_clzll((uint64_t)nb + 1));
      sentinel = end_bit >= 64 ? ~0ull : ((1ull << end_bit) - 1);
    }
    const size_t ksz = k32 ? 4 : 8;
    MBuf<uint64_t> d_koff;
    MBuf<uint32_t> d_vcnt;
    const uint64_t kwords = (std::max<uint64_t>(tot, 1) * ksz + 7) / 8;
    if (d_koff.alloc(nb + 1) || d_vcnt.alloc(nb) || c->wkeys.alloc(kwords) ||
        c->wkeys2.alloc(kwords))
      return mfail(M_OOM, "weighted-sketch keys (%llu)", (unsigned long long)tot);
    MHC(hipMemcpyAsync(d_koff.p, koff.data(), 8ull * (nb + 1), hipMemcpyHostToDevice, s));
    MHC(hipMemsetAsync(d_vcnt.p, 0, 4ull * nb, s));
    KeyArgs KA{c->d_bases, c->d_off, c->d_len.p, r0 + a, nb, (int32_t)k, d_koff.p, sentinel,
               c->wkeys.p, d_vcnt.p, c->kctr.p};
    if (k32) hipLaunchKernelGGL(k_mh_kmer_keys<uint32_t>, dim3(nb), dim3(256), 0, s, KA);
    else     hipLaunchKernelGGL(k_mh_kmer_keys<uint64_t>, dim3(nb), dim3(256), 0, s, KA);
    MHC(hipGetLastError());
    size_t tb = 0;
    if (k32) {
      uint32_t *ki = (uint32_t *)c->wkeys.p, *ko = (uint32_t *)c->wkeys2.p;
      MHC(hipcub::DeviceSegmentedRadixSort::SortKeys(nullptr, tb, ki, ko, (int)tot, (int)nb,
                                                     d_koff.p, d_koff.p + 1, 0, (int)end_bit, s));
      if (c->wsort_tmp.alloc(std::max<size_t>(tb, 1))) return mfail(M_OOM, "sort scratch");
      MHC(hipcub::DeviceSegmentedRadixSort::SortKeys(c->wsort_tmp.p, tb, ki, ko, (int)tot, (int)nb,
                                                     d_koff.p, d_koff.p + 1, 0, (int)end_bit, s));
    } else {
      // key counts can pass 2^31: the 64-bit-count form of the sort
      MHC(hipcub::DeviceRadixSort::SortKeys(nullptr, tb, c->wkeys.p, c->wkeys2.p, tot, 0,
                                            (int)end_bit, s));
      if (c->wsort_tmp.alloc(std::max<size_t>(tb, 1))) return mfail(M_OOM, "sort scratch");
      MHC(hipcub::DeviceRadixSort::SortKeys(c->wsort_tmp.p, tb, c->wkeys.p, c->wkeys2.p, tot, 0,
                                            (int)end_bit, s));
    }
    WSketchArgs WA{c->wkeys2.p, tot, d_koff.p, d_vcnt.p, r0 + a, nb, (int32_t)k,
                   (int32_t)c->P.num_hashes, c->nf ? c->ftab.p : nullptr, c->fmask, c->dmult,
                   c->W.no_tf, c->minhash.p};
    MHC(hipEventRecord(c->ev[2], s));
    if (k32)
      hipLaunchKernelGGL(k_mh_sketch_w<uint32_t>, dim3(nb), dim3(256), 4 * 4 * c->P.num_hashes, s, WA);
    else
      hipLaunchKernelGGL(k_mh_sketch_w<uint64_t>, dim3(nb), dim3(256), 4 * 4 * c->P.num_hashes, s, WA);
    MHC(hipGetLastError());
    MHC(hipEventRecord(c->ev[3], s));
    MHC(hipStreamSynchronize(s));                           // d_koff / d_vcnt are freed here
    sketch_kernel_time(c);
    a = b;
  }
  return M_OK;
}

int mhap_sketch(mhap_ctx *c, uint32_t bgn, uint32_t end) {
  if (!c || !c->nreads) return mfail(M_STATE, "no reads loaded");
  if (!c->d_bases || !c->d_off)
    return mfail(M_STATE, "no bases loaded (lengths only: import sketches instead)");
  if (bgn < c->first_iid || end >= c->first_iid + c->nreads || bgn > end)
    return mfail(M_BAD_PARAM, "sketch range %u-%u outside the loaded reads", bgn, end);
  MHC(hipSetDevice(c->device));
  hipStream_t s = c->stream;
  const uint32_t r0 = bgn - c->first_iid, nr = end - bgn + 1;
  MHC(hipMemsetAsync(c->kctr.p, 0, 8, s));
  c->stats.ms_sketch_kernel = 0;
  c->stats.sketch_launches = 0;
  MHC(hipEventRecord(c->ev[0], s));
  // one block per read; launches of <= 65535 * 16 reads keep grids modest
  if (c->weighted) {
    const int rc = sketch_weighted(c, r0, nr);
    if (rc) return rc;
  }
  for (uint32_t a = 0; a < nr; a += 1u << 20) {
    const uint32_t nb = std::min<uint32_t>(nr - a, 1u << 20);
    if (!c->weighted) {
      SketchArgs SA{c->d_bases, c->d_off, c->d_len.p, r0 + a, nb, (int32_t)c->P.k,
                    (int32_t)c->P.num_hashes, c->nfilter ? c->filter.p : nullptr, c->nfilter,
                    c->minhash.p, c->kctr.p};
      MHC(hipEventRecord(c->ev[2], s));
      hipLaunchKernelGGL(k_mh_sketch, dim3(nb), dim3(256), 4 * 4 * c->P.num_hashes, s, SA);
      MHC(hipGetLastError());
      MHC(hipEventRecord(c->ev[3], s));
      MHC(hipEventSynchronize(c->ev[3]));
      sketch_kernel_time(c);
    }
    OrderedArgs OA{c->d_bases, c->d_off, c->d_len.p, r0 + a, nb, (int32_t)c->P.ordered_k,
                   (int32_t)c->P.ordered_sketch, c->ordered.p, c->ocount.p};
    hipLaunchKernelGGL(k_mh_ordered, dim3(nb), dim3(256), 0, s, OA);
    MHC(hipGetLastError());
  }
  MHC(hipEventRecord(c->ev[1], s));
  unsigned long long nk = 0;
  MHC(hipMemcpyAsync(&nk, c->kctr.p, 8, hipMemcpyDeviceToHost, s));
  MHC(hipStreamSynchronize(s));
  c->stats.ms_sketch = elapsed(c);
  c->stats.sketched_reads = nr;
  c->stats.sketch_kmers = nk;
  c->indexed = false;
  return M_OK;
}

int mhap_sketch_buffers(mhap_ctx *c, void **d_minhash, void **d_ordered, void **d_ocount) {
  if (!c || !c->nreads) return mfail(M_STATE, "no reads loaded");
  *d_minhash = c->minhash.p;
  *d_ordered = c->ordered.p;
  *d_ocount = c->ocount.p;
  return M_OK;
}

int mhap_copy_sketches(mhap_ctx *c, uint32_t first, uint32_t n, void *d_minhash,
                       void *d_ordered, void *d_ocount, int to_ctx) {
  if (!c || !c->nreads) return mfail(M_STATE, "no reads loaded");
  if (n == 0) return M_OK;
  if (first < c->first_iid || (uint64_t)first + n > (uint64_t)c->first_iid + c->nreads)
    return mfail(M_BAD_PARAM, "rows %u..%u outside the loaded reads", first, first + n - 1);
  MHC(hipSetDevice(c->device));
  const size_t r0 = first - c->first_iid;
  const size_t H = c->P.num_hashes, S = c->P.ordered_sketch;
  struct { void *ctx; void *user; size_t bytes; } parts[3] = {
      {c->minhash.p + r0 * H, d_minhash, 4 * H * n},
      {c->ordered.p + r0 * S, d_ordered, 8 * S * n},
      {c->ocount.p + r0, d_ocount, 4ull * n}};
  for (auto &pt : parts) {
    if (!pt.user) return mfail(M_BAD_PARAM, "null buffer");
    if (to_ctx) MHC(hipMemcpyAsync(pt.ctx, pt.user, pt.bytes, hipMemcpyDeviceToDevice, c->stream));
    else        MHC(hipMemcpyAsync(pt.user, pt.ctx, pt.bytes, hipMemcpyDeviceToDevice, c->stream));
  }
  MHC(hipStreamSynchronize(c->stream));
  if (to_ctx) c->indexed = false;
  return M_OK;
}

int mhap_copy_sketches_host(mhap_ctx *c, uint32_t first, uint32_t n, void *h_minhash,
                            void *h_ordered, void *h_ocount, int to_ctx) {
  if (!c || !c->nreads) return mfail(M_STATE, "no reads loaded");
  if (n == 0) return M_OK;
  if (first < c->first_iid || (uint64_t)first + n > (uint64_t)c->first_iid + c->nreads)
    return mfail(M_BAD_PARAM, "rows %u..%u outside the loaded reads", first, first + n - 1);
  if (!h_minhash || !h_ordered || !h_ocount) return mfail(M_BAD_PARAM, "null buffer");
  MHC(hipSetDevice(c->device));
  const size_t r0 = first - c->first_iid;
  const size_t H = c->P.num_hashes, S = c->P.ordered_sketch;
  struct { void *ctx; void *user; size_t bytes; } parts[3] = {
      {c->minhash.p + r0 * H, h_minhash, 4 * H * n},
      {c->ordered.p + r0 * S, h_ordered, 8 * S * n},
      {c->ocount.p + r0, h_ocount, 4ull * n}};
  for (auto &pt : parts) {
    if (to_ctx) MHC(hipMemcpyAsync(pt.ctx, pt.user, pt.bytes, hipMemcpyHostToDevice, c->stream));
    else        MHC(hipMemcpyAsync(pt.user, pt.ctx, pt.bytes, hipMemcpyDeviceToHost, c->stream));
  }
  MHC(hipStreamSynchronize(c->stream));
  if (to_ctx) c->indexed = false;
  return M_OK;
}

int mhap_build_index(mhap_ctx *c) {
  if (!c || !c->nreads) return mfail(M_STATE, "no reads loaded");
  return mhap_build_index_range(c, c->first_iid, c->first_iid + c->nreads - 1);
}

int mhap_build_index_range(mhap_ctx *c, uint32_t bgn, uint32_t end) {
  if (!c || !c->nreads) return mfail(M_STATE, "no reads loaded");
  if (bgn < c->first_iid || end >= c->first_iid + c->nreads || bgn > end)
    return mfail(M_BAD_PARAM, "index range %u-%u outside the loaded reads", bgn, end);
  MHC(hipSetDevice(c->device));
  hipStream_t s = c->stream;
  const int32_t H = (int32_t)c->P.num_hashes;
  const uint32_t r0 = bgn - c->first_iid, nr = end - bgn + 1;
  const size_t n = (size_t)nr * H;
  if (c->keys.alloc(n) || c->vals.alloc(n) || c->keys2.alloc(n) || c->vals2.alloc(n) ||
      c->toff.alloc(H + 1))
    return mfail(M_OOM, "index (%zu entries)", n);
  MHC(hipEventRecord(c->ev[0], s));
  hipLaunchKernelGGL(k_mh_index_keys, dim3(4096), dim3(256), 0, s, c->minhash.p, r0, nr, H,
                     c->keys.p, c->vals.p);
  MHC(hipGetLastError());
  int end_bit = 32;
  while ((1ll << (end_bit - 32)) <= H) end_bit++;
  size_t tmp = 0;
  MHC(hipcub::DeviceRadixSort::SortPairs(nullptr, tmp, c->keys.p, c->keys2.p, c->vals.p,
                                         c->vals2.p, (int)n, 0, end_bit, s));
  if (c->sort_tmp.alloc(tmp)) return mfail(M_OOM, "sort scratch");
  MHC(hipcub::DeviceRadixSort::SortPairs(c->sort_tmp.p, tmp, c->keys.p, c->keys2.p, c->vals.p,
                                         c->vals2.p, (int)n, 0, end_bit, s));
  hipLaunchKernelGGL(k_mh_table_offsets, dim3((H + 1 + 255) / 256), dim3(256), 0, s,
                     c->keys2.p, n, H, c->toff.p);
  MHC(hipGetLastError());
  MHC(hipEventRecord(c->ev[1], s));
  MHC(hipStreamSynchronize(s));
  c->stats.ms_index = elapsed(c);
  c->nkeys = n;
  c->indexed = true;
  return M_OK;
}

static int compare_impl(mhap_ctx *c, uint32_t bgn, uint32_t end, uint32_t all_targets,
                        uint64_t *n_out);

int mhap_compare(mhap_ctx *c, uint32_t bgn, uint32_t end, uint64_t *n_out) {
  return compare_impl(c, bgn, end, 0, n_out);
}

int mhap_compare_all(mhap_ctx *c, uint32_t bgn, uint32_t end, uint64_t *n_out) {
  return compare_impl(c, bgn, end, 1, n_out);
}

static int compare_impl(mhap_ctx *c, uint32_t bgn, uint32_t end, uint32_t all_targets,
                        uint64_t *n_out) {
  if (!c || !c->indexed) return mfail(M_STATE, "mhap_build_index() first");
  if (bgn < c->first_iid || end >= c->first_iid + c->nreads || bgn > end)
    return mfail(M_BAD_PARAM, "query range %u-%u outside the loaded reads", bgn, end);
  MHC(hipSetDevice(c->device));
  hipStream_t s = c->stream;
  const uint32_t q0 = bgn - c->first_iid, q1 = end - c->first_iid + 1;
  const uint32_t nq = q1 - q0;
  // stage 2 (grow the candidate buffer and redo on overflow)
  size_t cap = std::max<size_t>((size_t)nq * 64, 1u << 16);
  uint32_t h[4];
  float ms_cand = 0;
  for (;;) {
    if (cap > 0xFFFFFFF0ull) return mfail(M_OOM, "candidate list too large");
    if (c->cand.alloc(cap)) return mfail(M_OOM, "candidates");
    MHC(hipMemsetAsync(c->ctr.p, 0, 64, s));
    CandArgs CA{c->minhash.p, c->keys2.p, c->vals2.p, c->toff.p, (int32_t)c->P.num_hashes,
                q0, q1, all_targets, c->P.min_matches, c->cand.p, c->ctr.p, (uint32_t)cap,
                c->ctr.p + 1};
    MHC(hipEventRecord(c->ev[0], s));
    hipLaunchKernelGGL(k_mh_candidates, dim3((nq + 3) / 4), dim3(256),
                       2 * 4 * TSLOTS * sizeof(uint32_t), s, CA);
    MHC(hipGetLastError());
    MHC(hipEventRecord(c->ev[1], s));
    MHC(hipMemcpyAsync(h, c->ctr.p, 16, hipMemcpyDeviceToHost, s));
    MHC(hipStreamSynchronize(s));
    ms_cand += elapsed(c);
    if (h[1] & 1u) return mfail(M_BAD_INPUT, "a query has more than %d candidate targets", TSLOTS);
    if (h[1] & 2u) { cap = (size_t)h[0] + (h[0] >> 2) + 1024; continue; }
    break;
  }
  const uint32_t ncand = h[0];
  // stage 3
  size_t rcap = std::max<size_t>(ncand, 1024);
  if (c->rec.alloc(rcap)) return mfail(M_OOM, "records");
  MHC(hipMemsetAsync(c->ctr.p + 4, 0, 16, s));
  const int32_t S = (int32_t)c->P.ordered_sketch;
  CmpArgs MA{c->cand.p, ncand, c->ordered.p, c->ocount.p, c->d_len.p, c->first_iid, S,
             (int32_t)c->P.ordered_k, c->P.min_olap, c->P.threshold, c->rec.p, c->ctr.p + 4,
             (uint32_t)rcap, c->ctr.p + 5};
  const size_t lds = 2 * 8 * ((size_t)S + S + 128);
  MHC(hipEventRecord(c->ev[0], s));
  if (ncand) {
    uint32_t blocks = std::min<uint32_t>((ncand + 1) / 2, 256u * 64u);
    hipLaunchKernelGGL(k_mh_compare, dim3(blocks), dim3(128), lds, s, MA);
    MHC(hipGetLastError());
  }
  MHC(hipEventRecord(c->ev[1], s));
  MHC(hipMemcpyAsync(h, c->ctr.p + 4, 8, hipMemcpyDeviceToHost, s));
  MHC(hipStreamSynchronize(s));
  if (h[1]) return mfail(M_OOM, "record capacity exceeded");
  c->stats.ms_candidates = ms_cand;
  c->stats.ms_compare = elapsed(c);
  c->stats.candidates = ncand;
  c->stats.overlaps = h[0];
  c->nrec = h[0];
  *n_out = c->nrec;
  return M_OK;
}

int mhap_fetch(mhap_ctx *c, mhap_record *out, uint64_t max_records, uint64_t *n_copied) {
  if (!c) return mfail(M_STATE, "null context");
  MHC(hipSetDevice(c->device));
  std::vector<RecDev> h(c->nrec);
  if (c->nrec) MHC(hipMemcpy(h.data(), c->rec.p, sizeof(RecDev) * c->nrec, hipMemcpyDeviceToHost));
  std::sort(h.begin(), h.end(), [](const RecDev &x, const RecDev &y) {
    return x.a != y.a ? x.a < y.a : x.b < y.b;
  });
  uint64_t n = std::min<uint64_t>(max_records, h.size());
  for (uint64_t i = 0; i < n; i++) {
    const RecDev &r = h[i];
    out[i] = mhap_record{r.a, r.b, r.erate, r.count, r.a_bgn, r.a_end, r.a_len, r.o,
                         r.b_bgn, r.b_end, r.b_len};
  }
  *n_copied = n;
  return M_OK;
}

int mhap_write_text(mhap_ctx *c, const char *path, uint32_t hash_base, uint32_t num_hash,
                    uint32_t query_base) {
  if (!c || !path) return mfail(M_STATE, "null argument");
  if (hash_base == 0 || query_base == 0) return mfail(M_BAD_PARAM, "bases are 1-based IDs");
  std::vector<mhap_record> r(c->nrec);
  uint64_t n = 0;
  int rc = mhap_fetch(c, r.data(), r.size(), &n);
  if (rc) return rc;
  FILE *F = fopen(path, "w");
  if (!F) return mfail(M_BAD_INPUT, "open '%s': %s", path, strerror(errno));
  for (uint64_t i = 0; i < n; i++) {
    const mhap_record &x = r[i];
    // mhapConvert.C:122-123: a_iid = W0 + (query_base - 1) - num_hash, b_iid = W1 + hash_base - 1
    const uint64_t w0 = (uint64_t)x.a_iid - (query_base - 1) + num_hash;
    const uint64_t w1 = (uint64_t)x.b_iid - (hash_base - 1);
    fprintf(F, "%llu %llu %.6f %u 0 %d %d %d %u %d %d %d\n", (unsigned long long)w0,
            (unsigned long long)w1, x.erate, x.count, x.a_bgn, x.a_end, x.a_len, x.b_rc,
            x.b_bgn, x.b_end, x.b_len);
  }
  if (fclose(F) != 0) return mfail(M_BAD_INPUT, "write '%s': %s", path, strerror(errno));
  return M_OK;
}

int mhap_get_stats(mhap_ctx *c, mhap_stats *out) {
  if (!c) return mfail(M_STATE, "null context");
  *out = c->stats;
  return M_OK;
}

}  // extern "C"
