// mhap.hip -- MHAP 2.1.2's sketch / two-stage filter on gfx950, behind include/canu_mhap.h.
//
// Replaces the MHAP jar canu runs for overlapper=mhap (src/pipelines/canu/OverlapMhap.pm:
// precompute :374-399, compare :476-498); the text line it writes is MatchResult.toString's,
// which src/mhap/mhapConvert.C:114-150 converts to ovOverlap records.  What the jar computes
// was read from its bytecode and is restated, method by method, in oracle/mhap_jar.py (the
// parity checker); the kernels below compute the same integers:
//
//   k_mh_ordered   one block per strand: BottomOverlapSketch -- Murmur3_x86_32 of every
//                  k'-mer's UTF-16 chars; the S smallest (hash, position) keys by a 4096-bin
//                  radix select (one histogram pass in practice, deeper digits when a bin
//                  overflows LDS), then a bitonic sort of the selected keys in LDS.
//   k_mh_keys      Murmur3_x64_128 h1 of every k-mer of every strand (the MinHash keys);
//                  a segmented radix sort (hipcub) makes each strand's keys runs: a run is a
//                  distinct k-mer, its length the count, its first value the first position.
//   k_mh_minhash   one block per strand over its sorted keys: per distinct k-mer the weight
//                  w (tf-idf), then for every hash function j, w xorshift64 draws of the
//                  k-mer's chain; the signed-smallest draw (earliest first occurrence on ties)
//                  stores the key's low / high 32 bits.  Integer-VALU bound (the draws).
//   index          (j, value) -> stored strand, hipcub radix sort, per-function offsets.
//   k_mh_candidates one wave per query: its forward row's H values looked up, matches counted
//                  per stored strand in an LDS table, the self / length rules of
//                  MinHashSearch.findMatches applied, >= min_matches emitted.
//   k_mh_compare   one wave per candidate: BottomOverlapSketch.getOverlapInfo.  The jar's
//                  sequential merge (recordMatchingKmers) decomposes into independent groups
//                  of equal hashes, so lanes take groups; the three medians are radix
//                  selects over regenerated records; the final bottom-sketch Jaccard merge is
//                  evaluated in closed form from per-group counts and prefix sums.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <charconv>
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

constexpr int64_t LMAX = 0x7FFFFFFFFFFFFFFFll;
constexpr int OCAP = 4096;        // ordered-sketch keys collected per strand (LDS)
constexpr int NBIN = 4096;        // radix-select bins (12-bit digits)
constexpr int TSLOTS = 2048;      // candidate table slots per wave
constexpr int TSHIFT = 21;        // 32 - log2(TSLOTS)
constexpr int RKW = 8;            // distinct k-mers per thread per round in k_mh_minhash
constexpr int RKK = 16;           // positions per thread in k_mh_keys

struct Cand {
  uint32_t q, t, cnt, pad;        // query read, stored strand (2 r + rc), shared entries
};

struct RecDev {
  uint32_t a, b;                  // reads (0-based in the context)
  uint32_t o, cnt;                // b strand, first-stage count
  uint32_t inter, n, raw, pad;    // Jaccard numerator / denominator, edges count
  int32_t a1, a2, a_len, b1, b2, b_len;
};

// Utils$Translate (Utils.rc): the complement of an upper-case IUPAC byte, 0 for the rest
__constant__ uint8_t c_comp[256];

__device__ __host__ __forceinline__ uint32_t upper_byte(uint32_t b) {
  return (b >= 'a' && b <= 'z') ? b - 32u : b;
}

// One strand of a read as the jar sees it: the forward string, or Utils.rc of it
struct Strand {
  const uint8_t *s;
  int32_t L;
  int32_t rc;
  __device__ __forceinline__ uint64_t ch(int32_t p) const {
    return rc ? (uint64_t)c_comp[upper_byte(s[L - 1 - p])] : (uint64_t)upper_byte(s[p]);
  }
};

__device__ __host__ __forceinline__ uint64_t rotl64(uint64_t x, int r) {
  return (x << r) | (x >> (64 - r));
}

__device__ __host__ __forceinline__ uint64_t fmix64(uint64_t k) {
  k ^= k >> 33;
  k *= 0xFF51AFD7ED558CCDull;
  k ^= k >> 33;
  k *= 0xC4CEB9FE1A85EC53ull;
  k ^= k >> 33;
  return k;
}

// Guava Hashing.murmur3_128(0).hashUnencodedChars(kmer).asLong(): MurmurHash3_x64_128 of
// the chars as little-endian UTF-16, first 8 bytes (h1)  (HashUtils.computeSequenceHashesLong
// @0-108; oracle mhap_jar.murmur3_128_h1)
template <class CH>
__device__ __host__ __forceinline__ uint64_t murmur128_h1(CH ch, int32_t k) {
  const uint64_t c1 = 0x87C37B91114253D5ull, c2 = 0x4CF5AD432745937Full;
  uint64_t h1 = 0, h2 = 0;
  const int32_t nb = k >> 3;
  int32_t q = 0;
  for (int32_t b = 0; b < nb; b++, q += 8) {
    uint64_t k1 = ch(q) | (ch(q + 1) << 16) | (ch(q + 2) << 32) | (ch(q + 3) << 48);
    uint64_t k2 = ch(q + 4) | (ch(q + 5) << 16) | (ch(q + 6) << 32) | (ch(q + 7) << 48);
    k1 *= c1; k1 = rotl64(k1, 31); k1 *= c2; h1 ^= k1;
    h1 = rotl64(h1, 27); h1 += h2; h1 = h1 * 5 + 0x52DCE729;
    k2 *= c2; k2 = rotl64(k2, 33); k2 *= c1; h2 ^= k2;
    h2 = rotl64(h2, 31); h2 += h1; h2 = h2 * 5 + 0x38495AB5;
  }
  const int32_t t = k - 8 * nb;
  if (t > 4) {
    uint64_t k2 = 0;
    for (int32_t j = 0; j < t - 4; j++) k2 |= ch(q + 4 + j) << (16 * j);
    k2 *= c2; k2 = rotl64(k2, 33); k2 *= c1; h2 ^= k2;
  }
  if (t > 0) {
    uint64_t k1 = 0;
    for (int32_t j = 0; j < (t < 4 ? t : 4); j++) k1 |= ch(q + j) << (16 * j);
    k1 *= c1; k1 = rotl64(k1, 31); k1 *= c2; h1 ^= k1;
  }
  h1 ^= (uint64_t)(2 * k);
  h2 ^= (uint64_t)(2 * k);
  h1 += h2;
  h2 += h1;
  h1 = fmix64(h1);
  h2 = fmix64(h2);
  return h1 + h2;
}

// --supress-noise 1: the jar's bundled Guava 19.0 BloomFilter (MURMUR128_MITZ_64) over the
// -f file's keys (FrequencyCounts.<init> @189-207, lambda$1 @162-185; keepKmer @0-21).  The
// Long funnel hashes the key's 8 little-endian bytes with murmur3_128(0); bit i of a key is
// (h1 + i * h2 & Long.MAX_VALUE) % bitSize (BloomFilterStrategies$2.put / mightContain;
// oracle mhap_jar.GuavaBloom)
__device__ __host__ __forceinline__ void murmur128_u64(uint64_t key, uint64_t &h1, uint64_t &h2) {
  const uint64_t c1 = 0x87C37B91114253D5ull, c2 = 0x4CF5AD432745937Full;
  uint64_t k1 = key * c1;
  k1 = rotl64(k1, 31);
  k1 *= c2;
  h1 = k1 ^ 8u;                                   // one 8-byte tail, length 8
  h2 = 8u;
  h1 += h2;
  h2 += h1;
  h1 = fmix64(h1);
  h2 = fmix64(h2);
  h1 += h2;
  h2 += h1;
}

struct BloomDev {
  const uint64_t *words;        // null: keep every k-mer
  uint64_t bit_size;            // 64 x words
  int32_t k;                    // hash functions
};

__device__ __host__ __forceinline__ bool bloom_has(const uint64_t *words, uint64_t bit_size,
                                                   int32_t k, uint64_t key) {
  uint64_t h1, h2;
  murmur128_u64(key, h1, h2);
  uint64_t c = h1;
  for (int32_t i = 0; i < k; i++, c += h2) {
    const uint64_t b = (c & 0x7FFFFFFFFFFFFFFFull) % bit_size;
    if (!((words[b >> 6] >> (b & 63)) & 1ull)) return false;
  }
  return true;
}

__device__ __forceinline__ uint32_t rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }

// Guava Hashing.murmur3_32(0) of the chars as UTF-16 (HashUtils.computeSequenceHashes
// @0-106; oracle mhap_jar.murmur3_32)
__device__ __forceinline__ uint32_t murmur32(const Strand &S, int32_t p, int32_t k) {
  const uint32_t c1 = 0xCC9E2D51u, c2 = 0x1B873593u;
  uint32_t h = 0;
  const int32_t nb = k >> 1;
  for (int32_t b = 0; b < nb; b++) {
    uint32_t kk = (uint32_t)S.ch(p + 2 * b) | ((uint32_t)S.ch(p + 2 * b + 1) << 16);
    kk *= c1; kk = rotl32(kk, 15); kk *= c2;
    h ^= kk;
    h = rotl32(h, 13); h = h * 5 + 0xE6546B64u;
  }
  if (k & 1) {
    uint32_t kk = (uint32_t)S.ch(p + k - 1);
    kk *= c1; kk = rotl32(kk, 15); kk *= c2;
    h ^= kk;
  }
  h ^= (uint32_t)(2 * k);
  h ^= h >> 16; h *= 0x85EBCA6Bu;
  h ^= h >> 13; h *= 0xC2B2AE35u;
  h ^= h >> 16;
  return h;
}

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ uint32_t popc64(uint64_t m) { return (uint32_t)__builtin_popcountll(m); }

__device__ __forceinline__ int32_t wave_sum_i32(int32_t v) {
  for (int s = 32; s > 0; s >>= 1) v += __shfl_xor(v, s);
  return v;
}
__device__ __forceinline__ int32_t wave_min_i32(int32_t v) {
  for (int s = 32; s > 0; s >>= 1) { const int32_t t = __shfl_xor(v, s); v = t < v ? t : v; }
  return v;
}
__device__ __forceinline__ int32_t wave_max_i32(int32_t v) {
  for (int s = 32; s > 0; s >>= 1) { const int32_t t = __shfl_xor(v, s); v = t > v ? t : v; }
  return v;
}
__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v) {
  for (int s = 32; s > 0; s >>= 1) { const uint32_t t = __shfl_xor(v, s); v = t < v ? t : v; }
  return v;
}

// signed 64-bit minimum over the wave, result uniform: DPP row shifts within 16-lane rows,
// then the row broadcasts (lanes whose source is outside the row read LMAX)
template <int CTRL, int RM>
__device__ __forceinline__ int64_t dpp_i64(int64_t v) {
  const int lo = __builtin_amdgcn_update_dpp((int)0xFFFFFFFF, (int)(uint32_t)v, CTRL, RM, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp((int)0x7FFFFFFF, (int)(uint32_t)((uint64_t)v >> 32),
                                             CTRL, RM, 0xf, false);
  return (int64_t)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
}
__device__ __forceinline__ int64_t wave_min_i64(int64_t v) {
  int64_t t;
  t = dpp_i64<0x111, 0xf>(v); v = t < v ? t : v;
  t = dpp_i64<0x112, 0xf>(v); v = t < v ? t : v;
  t = dpp_i64<0x114, 0xf>(v); v = t < v ? t : v;
  t = dpp_i64<0x118, 0xf>(v); v = t < v ? t : v;
  t = dpp_i64<0x142, 0xa>(v); v = t < v ? t : v;
  t = dpp_i64<0x143, 0xc>(v); v = t < v ? t : v;
  const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)v, 63);
  const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)((uint64_t)v >> 32), 63);
  return (int64_t)(((uint64_t)hi << 32) | lo);
}

// ---- ordered sketch -----------------------------------------------------------------------
struct OrderedArgs {
  const uint8_t *bases;
  const uint64_t *off;
  const uint32_t *len;
  uint32_t r0, nstrands;          // strands 2 r0 .. 2 r0 + nstrands - 1
  int32_t kk, S, min_use;         // k', ordered sketch size, shortest used read
  int32_t no_rc;
  uint64_t *ordered;              // [strand][S]: (hash ^ 0x80000000) << 32 | position
  uint32_t *ocount;
};

// key of the k'-mer at p: signed hash order, then position (stable radix sort of the jar)
__device__ __forceinline__ uint64_t okey(const Strand &S, int32_t p, int32_t kk) {
  return ((uint64_t)(murmur32(S, p, kk) ^ 0x80000000u) << 32) | (uint32_t)p;
}

// BottomOverlapSketch.<init>(s, k', S, false) @0-177 (oracle mhap_jar.ordered_sketch)
__global__ void __launch_bounds__(256) k_mh_ordered(OrderedArgs A) {
  __shared__ uint32_t hist[NBIN];
  __shared__ uint64_t list[OCAP];
  __shared__ uint32_t sD, sCnt, sBelow, sDone;
  const uint32_t sid = 2 * A.r0 + blockIdx.x;
  const uint32_t r = sid >> 1, tid = threadIdx.x;
  const int32_t L = (int32_t)A.len[r];
  const int32_t kk = A.kk;
  const int32_t npos = L - kk + 1;
  // a read shorter than --min-olap-length, or without a k'-mer, is not used; --no-rc: the
  // reverse strand is not stored
  if (L < A.min_use || npos <= 0 || ((sid & 1) && A.no_rc)) {
    if (tid == 0) A.ocount[sid] = 0;
    return;
  }
  const Strand St{A.bases + A.off[r], L, (int32_t)(sid & 1)};
  const uint32_t want = (uint32_t)min(A.S, npos);
  // radix select of the `want` smallest keys: digits of 12 bits from the top; prefix =
  // the digits fixed so far, below = keys known to be smaller than the prefix's range
  uint64_t prefix = 0;
  int32_t fixed = 0;
  uint32_t below = 0;
  uint64_t bound = 0;             // collect keys whose top (fixed + 12) bits <= bound
  int32_t bshift = 0;
  for (;;) {
    for (int32_t i = tid; i < NBIN; i += 256) hist[i] = 0;
    __syncthreads();
    const int32_t width = fixed + 12 <= 64 ? 12 : 64 - fixed;
    const int32_t sh = 64 - fixed - width;
    for (int32_t p = tid; p < npos; p += 256) {
      const uint64_t key = okey(St, p, kk);
      if (fixed == 0 || (key >> (64 - fixed)) == prefix)
        atomicAdd(&hist[(uint32_t)((key >> sh) & ((1ull << width) - 1))], 1u);
    }
    __syncthreads();
    if (tid == 0) {
      const uint32_t need = want - below;
      uint32_t cs = 0, D = (1u << width) - 1;
      for (uint32_t b = 0; b < (1u << width); b++) {
        if (cs + hist[b] >= need) { D = b; break; }
        cs += hist[b];
      }
      sD = D;
      sBelow = below + cs;                        // keys below digit D (all selected)
      sDone = (below + cs + hist[D] <= (uint32_t)OCAP) ? 1u : 0u;
    }
    __syncthreads();
    const uint32_t D = sD;
    if (sDone) {
      bound = (fixed == 0 ? 0 : prefix << width) | D;
      bshift = sh;
      break;
    }
    below = sBelow;
    prefix = (fixed == 0 ? 0 : prefix << width) | D;
    fixed += width;
    __syncthreads();
  }
  // collect every key whose top bits are <= (prefix, D): exactly the selected ones below
  // plus all of bin D (>= want in total, <= OCAP)
  if (tid == 0) sCnt = 0;
  __syncthreads();
  for (int32_t p = tid; p < npos; p += 256) {
    const uint64_t key = okey(St, p, kk);
    if ((key >> bshift) <= bound) {
      const uint32_t idx = atomicAdd(&sCnt, 1u);
      if (idx < (uint32_t)OCAP) list[idx] = key;
    }
  }
  __syncthreads();
  const uint32_t n = min(sCnt, (uint32_t)OCAP);
  uint32_t P = 1;
  while (P < n) P <<= 1;
  for (uint32_t i = n + tid; i < P; i += 256) list[i] = ~0ull;
  __syncthreads();
  for (uint32_t kb = 2; kb <= P; kb <<= 1) {
    for (uint32_t jb = kb >> 1; jb > 0; jb >>= 1) {
      for (uint32_t i = tid; i < P; i += 256) {
        const uint32_t ix = i ^ jb;
        if (ix > i) {
          const uint64_t a = list[i], b = list[ix];
          const bool up = (i & kb) == 0;
          if ((a > b) == up) { list[i] = b; list[ix] = a; }
        }
      }
      __syncthreads();
    }
  }
  uint64_t *dst = A.ordered + (size_t)sid * A.S;
  for (uint32_t i = tid; i < want; i += 256) dst[i] = list[i];
  if (tid == 0) A.ocount[sid] = want;
}

// ---- MinHash keys ---------------------------------------------------------------------------
struct KeyArgs {
  const uint8_t *bases;
  const uint64_t *off;
  const uint32_t *len;
  const uint32_t *sids;           // the batch's strands
  const uint64_t *koff;           // per batch strand: its first key
  int32_t k;
  uint64_t *keys;
  uint32_t *pos;
};

// HashUtils.computeSequenceHashesLong(s, k, 0, false) of one strand per block
__global__ void __launch_bounds__(256) k_mh_keys(KeyArgs A) {
  const uint32_t bi = blockIdx.x, sid = A.sids[bi], r = sid >> 1;
  const int32_t L = (int32_t)A.len[r], k = A.k;
  const int32_t npos = L - k + 1;
  const Strand St{A.bases + A.off[r], L, (int32_t)(sid & 1)};
  uint64_t *out = A.keys + A.koff[bi];
  uint32_t *po = A.pos + A.koff[bi];
  for (int32_t p = threadIdx.x; p < npos; p += 256) {
    out[p] = murmur128_h1([&](int32_t q) { return St.ch(p + q); }, k);
    po[p] = (uint32_t)p;
  }
}

// ---- MinHash sketch -------------------------------------------------------------------------
// The -f table (FrequencyCounts.fractionCounts): open addressing on the 64-bit key.
struct FreqSlot {
  uint64_t key;
  double sidf;                    // scaledIdf of the k-mer (weighting mode 1)
  uint32_t used, pad;
};

enum { W_ONE = 0, W_TFIDF = 1, W_COUNT = 2 };

struct SketchArgs {
  const uint64_t *keys;           // sorted per strand
  const uint32_t *pos;            // first positions ride along (stable sort)
  const uint64_t *koff;           // per batch strand: segment start, [nb + 1]
  const uint32_t *sids;
  int32_t H;
  int32_t mode;                   // W_ONE (repeat_weight < 0), W_TFIDF, W_COUNT
  const FreqSlot *ftab;           // null: no -f table
  uint64_t fmask;
  double range;                   // scaledIdf of a k-mer not in the table
  int32_t no_tf;
  int32_t *minhash;               // [strand][H]
  uint32_t *ocount;               // zeroed for a strand with no k-mer of weight > 0
  unsigned long long *stat;       // [0] distinct k-mers, [1] draws
  // bit-sliced draws (k_mh_bitslice; bs_w = 0: every k-mer here).  The k-mers of weight bs_w
  // past the strand's first round go to its list (bs_key / bs_fp at koff[b], bs_cnt[b] of
  // them) and this kernel leaves its exact minima in best_out instead of the sketch
  int32_t bs_w;
  uint32_t bs_sample;             // a strand's first bs_sample sorted k-mers are drawn here
  uint64_t *bs_key;
  uint32_t *bs_fp;
  uint32_t *bs_cnt;
  struct BestOut *best_out;       // [batch strand][H]
  BloomDev keep;                  // --supress-noise 1: k-mers the filter rejects never count
};

// one hash function's minimum so far: the exact draw, the k-mer's first position
// (FP_NONE: none yet) and the value stored (a key half)
struct BestOut {
  int64_t val;
  uint32_t fp;
  uint32_t v;
};

__device__ __forceinline__ uint64_t slot_hash(uint64_t key) {
  return fmix64(key ^ 0x9E3779B97F4A7C15ull);
}

__device__ __forceinline__ const FreqSlot *table_find(const FreqSlot *t, uint64_t mask,
                                                      uint64_t key) {
  for (uint64_t h = slot_hash(key) & mask;; h = (h + 1) & mask) {
    const FreqSlot *s = t + h;
    if (!s->used) return nullptr;
    if (s->key == key) return s;
  }
}

// Math.round(double): the closest long, ties toward positive infinity
__device__ __forceinline__ int64_t java_round(double x) {
  const double f = floor(x);
  return (int64_t)f + (__dsub_rn(x, f) >= 0.5 ? 1 : 0);
}

// one xorshift64 step (<<21, >>>35, <<4)
__device__ __forceinline__ uint64_t xs64(uint64_t x) {
  x ^= x << 21;
  x ^= x >> 35;
  x ^= x << 4;
  return x;
}

// exact minimum (signed) of w xorshift64 draws from chain state x (w = 0: x is the value)
__device__ __forceinline__ int64_t exact_min(uint64_t x, int32_t w) {
  if (w == 0) return (int64_t)x;
  int64_t m = LMAX;
  for (int32_t t = 0; t < w; t++) {
    x = xs64(x);
    m = (int64_t)x < m ? (int64_t)x : m;
  }
  return m;
}

// A best draw of one hash function: its high word decides almost every comparison; the
// exact value is recomputed from (state, w) -- the k-mer's chain before the function's w
// draws -- only when two candidates tie on the high word (w = 0: state is the value).
struct BestRec {
  int32_t hi;
  uint32_t fp;                    // first position of the k-mer (0xFFFFFFFF: none yet)
  uint32_t v;                     // the value stored: the key's low / high 32 bits
  int32_t w;
  uint64_t state;
};

constexpr uint32_t FP_NONE = 0xFFFFFFFFu;

// the jar's order of candidates: the smaller draw, then the earlier first occurrence
__device__ __forceinline__ bool rec_less(const BestRec &a, const BestRec &b) {
  if (b.fp == FP_NONE) return a.fp != FP_NONE;
  if (a.fp == FP_NONE) return false;
  if (a.hi != b.hi) return a.hi < b.hi;
  const int64_t xa = exact_min(a.state, a.w), xb = exact_min(b.state, b.w);
  return xa < xb || (xa == xb && a.fp < b.fp);
}

// MinHashSketch.computeNgramMinHashesWeighted @0-476 (oracle mhap_jar.minhash); one block
// per strand, RKW distinct k-mers per thread per round.  LDS: per wave and hash function the
// best candidate so far (BestRec).
__global__ void __launch_bounds__(256) k_mh_minhash(SketchArgs A) {
  extern __shared__ uint8_t s_raw[];
  const int32_t H = A.H;
  const uint32_t tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  BestRec *best_all = (BestRec *)s_raw;                      // [4][H]
  __shared__ uint32_t s_live, s_bsn;
  for (int32_t j = tid; j < 4 * H; j += 256) best_all[j] = BestRec{0x7FFFFFFF, FP_NONE, 0, 0, 0};
  if (tid == 0) { s_live = 0; s_bsn = 0; }
  __syncthreads();
  const uint32_t bi = blockIdx.x, sid = A.sids[bi];
  const uint64_t s0 = A.koff[bi], s1 = A.koff[bi + 1];
  BestRec *best = best_all + wave * H;
  unsigned long long nkm = 0, ndraw = 0;
  for (uint64_t base = s0; base < s1; base += 256 * RKW) {
    const uint64_t p0 = base + (uint64_t)tid * RKW;
    uint64_t X[RKW];
    uint32_t KL[RKW], KH[RKW], FP[RKW];
    int32_t W[RKW];
    uint32_t listed = 0;                 // bit i: slot i's k-mer goes to the bit-sliced list
#pragma unroll
    for (int i = 0; i < RKW; i++) {
      X[i] = 0; KL[i] = KH[i] = 0; FP[i] = FP_NONE; W[i] = 0;
      const uint64_t p = p0 + i;
      if (p < s1) {
        const uint64_t key = A.keys[p];
        if (p == s0 || A.keys[p - 1] != key) {             // a run start: a distinct k-mer
          uint64_t e = p + 1;
          while (e < s1 && A.keys[e] == key) e++;
          const uint32_t cnt = (uint32_t)(e - p);
          int64_t w = cnt;
          if (A.keep.words && !bloom_has(A.keep.words, A.keep.bit_size, A.keep.k, key)) {
            w = 0;                         // keepKmer @70-83: never in the map, never drawn
          } else if (A.mode == W_ONE) {
            w = (A.ftab && table_find(A.ftab, A.fmask, key)) ? 0 : 1;
          } else if (A.mode == W_TFIDF) {
            const FreqSlot *f = A.ftab ? table_find(A.ftab, A.fmask, key) : nullptr;
            const double sidf = f ? f->sidf : A.range;
            const double tf = A.no_tf ? 1.0 : (double)cnt;
            w = java_round(__dmul_rn(tf, sidf));
            if (w < 1) w = 1;
          }
          if (w > 0 && w == A.bs_w && p >= s0 + A.bs_sample) {
            // past the strand's first bs_sample sorted positions (a sample whose minima make
            // the bit-sliced threshold tight), the dominant weight's k-mers are drawn
            // bit-sliced (k_mh_bitslice, from the minima this kernel leaves): listed below
            listed |= 1u << i;
            nkm++;
            ndraw += (unsigned long long)w * (unsigned long long)H;
            w = 0;
          }
          if (w > 0) {
            W[i] = (int32_t)(w > 0x7FFFFFFF ? 0x7FFFFFFF : w);
            X[i] = key;
            KL[i] = (uint32_t)key;
            KH[i] = (uint32_t)(key >> 32);
            FP[i] = A.pos[p];
            nkm++;
            ndraw += (unsigned long long)W[i] * (unsigned long long)H;
          }
        }
      }
    }
    if (A.bs_w) {
      // the listed k-mers appended to the strand's list, one LDS atomic per wave and slot
      const uint64_t lt = (1ull << lane) - 1ull;
#pragma unroll
      for (int i = 0; i < RKW; i++) {
        const uint64_t m = __builtin_amdgcn_ballot_w64((listed >> i) & 1u);
        if (!m) continue;
        uint32_t at = 0;
        if (lane == 0) at = atomicAdd(&s_bsn, (uint32_t)popc64(m));
        at = (uint32_t)__shfl((int)at, 0) + popc64(m & lt);
        if ((listed >> i) & 1u) {
          const uint64_t p = p0 + i;
          A.bs_key[s0 + at] = A.keys[p];
          A.bs_fp[s0 + at] = A.pos[p];
        }
      }
    }
    // dead slots (W = 0) take a live slot's chain, weight and payload: a duplicate candidate
    // changes no minimum and no tie; a lane with no live slot is masked at the wave minimum
    bool live = false;
    {
      uint64_t x0 = 0;
      uint32_t l0 = 0, h0 = 0, f0 = FP_NONE;
      int32_t w0 = 0;
#pragma unroll
      for (int i = RKW - 1; i >= 0; i--)
        if (W[i] > 0) { x0 = X[i]; l0 = KL[i]; h0 = KH[i]; f0 = FP[i]; w0 = W[i]; live = true; }
#pragma unroll
      for (int i = 0; i < RKW; i++)
        if (W[i] == 0) { X[i] = x0; KL[i] = l0; KH[i] = h0; FP[i] = f0; W[i] = w0; }
    }
    if (__builtin_amdgcn_ballot_w64(live) == 0) continue;   // nothing in this wave
    // one weight for every live slot of the wave (canu's weighting: a k-mer seen once and not
    // in the -f table weighs round(1 x 10) = 10, nearly all of them): the draws are a
    // wave-uniform loop instead of a per-lane one under an exec mask per slot and draw
    int32_t wmn = 0x7FFFFFFF, wmx = 0;
#pragma unroll
    for (int i = 0; i < RKW; i++) { wmn = min(wmn, W[i]); wmx = max(wmx, W[i]); }
    if (!live) { wmn = 0x7FFFFFFF; wmx = 0; }
    wmn = wave_min_i32(wmn);
    wmx = wave_max_i32(wmx);
    const int32_t wu = wmn == wmx ? __builtin_amdgcn_readfirstlane(wmx) : 0;
    for (int32_t j = 0; j < H; j++) {
      const BestRec cur = best[j];                     // uniform (LDS broadcast)
      if (wu >= 2) {
        // high-word minima: one v_min per draw instead of a 64-bit compare and two selects
        uint64_t X0[RKW];
        int32_t mh[RKW];
#pragma unroll
        for (int i = 0; i < RKW; i++) { X0[i] = X[i]; mh[i] = 0x7FFFFFFF; }
        for (int32_t t = 0; t < wu; t++) {
#pragma unroll
          for (int i = 0; i < RKW; i++) {
            X[i] = xs64(X[i]);
            const int32_t h = (int32_t)(X[i] >> 32);
            mh[i] = h < mh[i] ? h : mh[i];
          }
        }
        int32_t lh = mh[0];
#pragma unroll
        for (int i = 1; i < RKW; i++) lh = mh[i] < lh ? mh[i] : lh;
        if (!live) lh = 0x7FFFFFFF;
        const int32_t wh = wave_min_i32(lh);
        if (cur.fp != FP_NONE && wh > cur.hi) continue;       // cannot beat the best so far
        // slots holding the wave's smallest high word
        uint32_t nmine = 0, li = 0;
#pragma unroll
        for (int i = RKW - 1; i >= 0; i--)
          if (live && mh[i] == wh) { nmine++; li = i; }
        const uint64_t who = __builtin_amdgcn_ballot_w64(nmine > 0);
        const uint32_t ln = (uint32_t)__builtin_ctzll(who);
        const bool unique = popc64(who) == 1 && __builtin_amdgcn_readlane(nmine, ln) == 1 &&
                            wh != 0x7FFFFFFF && (cur.fp == FP_NONE || wh < cur.hi);
        BestRec nb;
        if (unique) {
          // the candidate's own (state, w) stand for its exact value, fetched from lane ln
          uint64_t st = 0;
          uint32_t fp = 0, v = 0;
#pragma unroll
          for (int i = 0; i < RKW; i++)
            if ((uint32_t)i == li) { st = X0[i]; fp = FP[i]; v = (j & 1) ? KH[i] : KL[i]; }
          nb.hi = wh;
          nb.fp = __builtin_amdgcn_readlane(fp, ln);
          nb.v = __builtin_amdgcn_readlane(v, ln);
          nb.w = wu;
          // (readlane returns an int: the low word is widened unsigned, or a set bit 31 would
          // smear over the high word -- the state is a number k_mh_bitslice compares with)
          nb.state = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((uint32_t)(st >> 32), ln) << 32) |
                     (uint64_t)(uint32_t)__builtin_amdgcn_readlane((uint32_t)st, ln);
        } else {
          // a tie on the high word (rare): exact values by replaying the tied slots' draws
          int64_t ex = LMAX;
          uint32_t ep = FP_NONE, ev = 0;
          uint64_t es = 0;
#pragma unroll
          for (int i = 0; i < RKW; i++) {
            if (live && mh[i] == wh) {
              const int64_t e = exact_min(X0[i], wu);
              if (e < ex || (e == ex && FP[i] < ep)) {
                ex = e; ep = FP[i]; es = X0[i]; ev = (j & 1) ? KH[i] : KL[i];
              }
            }
          }
          const int64_t wx = wave_min_i64(ex);
          const uint32_t wp = wave_min_u32(ex == wx ? ep : FP_NONE);
          const uint64_t w2 = __builtin_amdgcn_ballot_w64(ex == wx && ep == wp);
          const uint32_t l2 = (uint32_t)__builtin_ctzll(w2);
          if (wx == LMAX) continue;                   // never below the jar's initial value
          nb.hi = (int32_t)((uint64_t)wx >> 32);
          nb.fp = wp;
          nb.v = __builtin_amdgcn_readlane(ev, l2);
          nb.w = 0;
          nb.state = (uint64_t)wx;
          (void)es;
        }
        if (rec_less(nb, cur) && lane == 0) best[j] = nb;
      } else {
        // exact 64-bit minima (one draw per function, or weights that differ in the wave)
        int64_t mi[RKW];
#pragma unroll
        for (int i = 0; i < RKW; i++) mi[i] = LMAX;
        if (wu == 1) {
#pragma unroll
          for (int i = 0; i < RKW; i++) {
            X[i] = xs64(X[i]);
            mi[i] = (int64_t)X[i];
          }
        } else {
#pragma unroll
          for (int i = 0; i < RKW; i++) {
            for (int32_t t = 0; t < W[i]; t++) {
              X[i] = xs64(X[i]);
              mi[i] = (int64_t)X[i] < mi[i] ? (int64_t)X[i] : mi[i];
            }
          }
        }
        // the jar's strict '<' in key order: equal draws keep the earlier first occurrence
        int64_t mx = LMAX;
        uint32_t mp = FP_NONE, mv = 0;
#pragma unroll
        for (int i = 0; i < RKW; i++) {
          if (mi[i] < mx || (mi[i] == mx && FP[i] < mp)) {
            mx = mi[i];
            mp = FP[i];
            mv = (j & 1) ? KH[i] : KL[i];
          }
        }
        if (!live) mx = LMAX;
        const int64_t wx = wave_min_i64(mx);
        if (wx == LMAX) continue;                     // no draw below the initial value
        if (cur.fp != FP_NONE && (int32_t)((uint64_t)wx >> 32) > cur.hi) continue;
        const uint64_t hold = __builtin_amdgcn_ballot_w64(mx == wx);
        uint32_t wp, wv;
        if (popc64(hold) == 1) {
          const uint32_t ln = (uint32_t)__builtin_ctzll(hold);
          wp = __builtin_amdgcn_readlane(mp, ln);
          wv = __builtin_amdgcn_readlane(mv, ln);
        } else {
          wp = wave_min_u32(mx == wx ? mp : FP_NONE);
          const uint64_t who = __builtin_amdgcn_ballot_w64(mx == wx && mp == wp);
          wv = __builtin_amdgcn_readlane(mv, (uint32_t)__builtin_ctzll(who));
        }
        const BestRec nb{(int32_t)((uint64_t)wx >> 32), wp, wv, 0, (uint64_t)wx};
        if (rec_less(nb, cur) && lane == 0) best[j] = nb;
      }
    }
  }
  for (int s = 32; s > 0; s >>= 1) {
    nkm += __shfl_xor(nkm, s);
    ndraw += __shfl_xor(ndraw, s);
  }
  if (lane == 0 && nkm) {
    atomicAdd(&s_live, 1u);
    if (A.stat) {
      atomicAdd(&A.stat[0], nkm);
      atomicAdd(&A.stat[1], ndraw);
    }
  }
  __syncthreads();
  if (A.bs_w && tid == 0) A.bs_cnt[bi] = s_bsn;
  for (int32_t j = tid; j < H; j += 256) {
    BestRec b = best_all[j];
    for (int w = 1; w < 4; w++) {
      const BestRec c = best_all[w * H + j];
      if (rec_less(c, b)) b = c;
    }
    if (A.bs_w) {
      BestOut o;
      o.val = b.fp == FP_NONE ? LMAX : exact_min(b.state, b.w);
      o.fp = b.fp;
      o.v = b.v;
      A.best_out[(size_t)bi * H + j] = o;
    } else {
      A.minhash[(size_t)sid * H + j] = b.fp == FP_NONE ? 0 : (int32_t)b.v;
    }
  }
  // no k-mer of positive weight: the jar's sketch constructor fails and the read (or this
  // strand) is skipped
  if (tid == 0 && s_live == 0) A.ocount[sid] = 0;
}

// ---- bit-sliced draws ------------------------------------------------------------------
// Nearly every k-mer of a canu sketch has the same weight (seen once, not in the -f table:
// round(1 x 10) = 10), so after a strand's first round (k_mh_minhash, exact, which leaves the
// minima so far in best_out) its k-mers of that weight are drawn 32 to a lane in BIT PLANES:
// plane b (one VGPR) holds bit b of 32 chains' states (bit p: the lane's chain p, list entry
// base + 64 p + lane).  A xorshift64 step is then 132 plane XORs for 32 chains -- the shifts
// are renamings of planes -- instead of 2 64-bit shifts, 5 XORs and a right shift per chain.
// The minimum is not tracked per chain: a draw matters only if it is <= the function's best
// so far T, and since T is small after the exact round (the minimum of ~20 k draws), a draw
// can be below it only if the top Z bits of x ^ 2^63 are zero, Z = clz(T ^ 2^63): one OR over
// Z planes tests 32 chains.  The few chains that pass are read out of the planes (the exact
// 64-bit draw) and compared with the best in the jar's order -- smaller draw, then earlier
// first occurrence -- so the result is the exact minimum whatever the draw order.
constexpr uint32_t BS_CHAINS = 2048;     // k-mers per wave per batch (64 lanes x 32 planes)

__device__ __forceinline__ void bs_step(uint32_t (&S)[64]) {
#pragma unroll
  for (int b = 63; b >= 21; b--) S[b] ^= S[b - 21];       // x ^= x << 21
#pragma unroll
  for (int b = 0; b <= 28; b++) S[b] ^= S[b + 35];        // x ^= x >>> 35
#pragma unroll
  for (int b = 63; b >= 4; b--) S[b] ^= S[b - 4];         // x ^= x << 4
}

// draws t.. of the current function until one leaves a chain that may be <= T (its top Z
// bits of x ^ 2^63 all zero) or the function's w draws are done; returns the next draw
template <int Z>
__device__ __forceinline__ int32_t bs_draws(uint32_t (&S)[64], uint32_t valid, int32_t t,
                                            int32_t w, uint32_t &cand) {
  for (; t < w;) {
    bs_step(S);
    t++;
    uint32_t c = valid;
    if constexpr (Z > 0) {
      uint32_t z = ~S[63];                                  // the sign bit, flipped
#pragma unroll
      for (int i = 1; i < Z; i++) z |= S[63 - i];
      c &= ~z;
    }
    if (__builtin_amdgcn_ballot_w64(c != 0)) { cand = c; return t; }
  }
  cand = 0;
  return t;
}

struct BsArgs {
  const uint64_t *bs_key;         // per batch strand at koff[b]: keys of its listed k-mers
  const uint32_t *bs_fp;          //   and their first positions
  const uint32_t *bs_cnt;
  const uint64_t *koff;
  const uint32_t *sids;
  const BestOut *best_in;         // [batch strand][H]: k_mh_minhash's minima
  int32_t H;
  int32_t w;                      // the listed k-mers' weight
  int32_t *minhash;               // [strand][H]
  int32_t zmax;                   // planes tested at most (MHAP_BS_ZMAX, A/B and checks: 64)
};

__device__ __forceinline__ uint32_t uni_u32(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_readfirstlane((int32_t)v);
}

// one wave per strand
__global__ void __launch_bounds__(64, 5) k_mh_bitslice(BsArgs A) {
  extern __shared__ uint8_t s_raw[];
  BestOut *best = (BestOut *)s_raw;                          // [H]
  const uint32_t lane = threadIdx.x, bi = blockIdx.x, sid = A.sids[bi];
  const int32_t H = A.H, w = A.w;
  for (int32_t j = lane; j < H; j += 64) best[j] = A.best_in[(size_t)bi * H + j];
  wave_sync();
  const uint64_t s0 = A.koff[bi];
  const uint32_t n = A.bs_cnt[bi];
  const uint64_t *keys = A.bs_key + s0;
  const uint32_t *fps = A.bs_fp + s0;
  for (uint32_t base = 0; base < n; base += BS_CHAINS) {
    uint32_t S[64];
#pragma unroll
    for (int b = 0; b < 64; b++) S[b] = 0;
    uint32_t valid = 0;
    for (uint32_t p = 0; p < 32; p++) {
      const uint32_t idx = base + p * 64 + lane;
      if (idx < n) {
        const uint64_t key = keys[idx];
        const uint32_t lo = (uint32_t)key, hi = (uint32_t)(key >> 32);
        valid |= 1u << p;
#pragma unroll
        for (int b = 0; b < 32; b++) {
          S[b] |= ((lo >> b) & 1u) << p;
          S[b + 32] |= ((hi >> b) & 1u) << p;
        }
      }
    }
    for (int32_t j = 0; j < H; j++) {
      BestOut cur = best[j];
      cur.fp = uni_u32(cur.fp);
      cur.v = uni_u32(cur.v);
      cur.val = (int64_t)(((uint64_t)uni_u32((uint32_t)((uint64_t)cur.val >> 32)) << 32) |
                          uni_u32((uint32_t)cur.val));
      bool changed = false;
      for (int32_t t = 0; t < w;) {
        // draws may be <= T only with their top Z bits (of x ^ 2^63) clear; fewer planes
        // tested is a looser filter, never a wrong one
        const uint64_t U = cur.fp == FP_NONE ? ~0ull : ((uint64_t)cur.val ^ (1ull << 63));
        const int32_t Z = min(U == 0 ? 64 : (int32_t)__builtin_clzll(U), A.zmax);
        uint32_t cand = 0;
        // a filter of fewer planes than Z lets up to 2^(Z - planes) x the true candidates
        // through: a step per plane where the sample leaves Z (13-16), coarser outside
        if (Z >= 20)      t = bs_draws<20>(S, valid, t, w, cand);
        else if (Z >= 18) t = bs_draws<18>(S, valid, t, w, cand);
        else if (Z >= 16) t = bs_draws<16>(S, valid, t, w, cand);
        else if (Z == 15) t = bs_draws<15>(S, valid, t, w, cand);
        else if (Z == 14) t = bs_draws<14>(S, valid, t, w, cand);
        else if (Z == 13) t = bs_draws<13>(S, valid, t, w, cand);
        else if (Z >= 10) t = bs_draws<10>(S, valid, t, w, cand);
        else if (Z >= 6)  t = bs_draws<6>(S, valid, t, w, cand);
        else              t = bs_draws<0>(S, valid, t, w, cand);
        if (!__builtin_amdgcn_ballot_w64(cand != 0)) continue;
        const uint32_t T_hi = (uint32_t)((uint64_t)cur.val >> 32);
        // the lane's smallest (draw, first position) among its passing chains that beats the
        // best so far (a strict '<' on the draw, then the earlier first occurrence)
        int64_t bv = LMAX;
        uint32_t bfp = FP_NONE, bidx = 0;
        for (uint32_t m = cand; m;) {
          const uint32_t c = (uint32_t)__builtin_ctz(m);
          m &= m - 1;
          // the high word first: most passing chains are above T there
          uint32_t hi = 0;
#pragma unroll
          for (int b = 0; b < 32; b++) hi |= ((S[b + 32] >> c) & 1u) << b;
          if (cur.fp != FP_NONE && (int32_t)hi > (int32_t)T_hi) continue;
          uint32_t lo = 0;
#pragma unroll
          for (int b = 0; b < 32; b++) lo |= ((S[b] >> c) & 1u) << b;
          const int64_t v = (int64_t)(((uint64_t)hi << 32) | lo);
          const uint32_t idx = base + c * 64 + lane;
          const uint32_t fp = fps[idx];
          const bool beats = cur.fp == FP_NONE ? v < LMAX
                                               : (v < cur.val || (v == cur.val && fp < cur.fp));
          if (beats && (v < bv || (v == bv && fp < bfp))) { bv = v; bfp = fp; bidx = idx; }
        }
        if (!__builtin_amdgcn_ballot_w64(bv != LMAX)) continue;   // no draw beat it
        const int64_t wv = wave_min_i64(bv);
        const uint32_t wp = wave_min_u32(bv == wv ? bfp : FP_NONE);
        const uint64_t who = __builtin_amdgcn_ballot_w64(bv == wv && bfp == wp);
        const uint32_t widx = uni_u32(__builtin_amdgcn_readlane(bidx, (uint32_t)__builtin_ctzll(who)));
        const uint64_t key = keys[widx];
        cur.val = wv;
        cur.fp = wp;
        cur.v = (j & 1) ? (uint32_t)(key >> 32) : (uint32_t)key;
        changed = true;
      }
      if (changed) {
        if (lane == 0) best[j] = cur;
        wave_sync();
      }
    }
  }
  wave_sync();
  for (int32_t j = lane; j < H; j += 64) {
    const BestOut b = best[j];
    A.minhash[(size_t)sid * H + j] = b.fp == FP_NONE ? 0 : (int32_t)b.v;
  }
}

// a read whose forward strand was skipped is skipped whole (SequenceSketchStreamer
// .enqueue @67-95: the reverse strand is made only after the forward one)
__global__ void k_mh_strand_fixup(uint32_t *ocount, uint32_t r0, uint32_t nr) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < nr && ocount[2 * (r0 + i)] == 0) ocount[2 * (r0 + i) + 1] = 0;
}

// ---- index ----------------------------------------------------------------------------------
// (j << 32 | value ^ 0x80000000) -> stored strand; strands not stored -> table H
__global__ void k_mh_index_keys(const int32_t *mh, const uint32_t *ocount, uint32_t s0,
                                uint32_t ns, int32_t H, uint64_t *keys, uint32_t *vals) {
  const size_t n = (size_t)ns * H;
  for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < n;
       e += (size_t)gridDim.x * blockDim.x) {
    const uint32_t sid = s0 + (uint32_t)(e / H), j = (uint32_t)(e % H);
    const int32_t v = mh[(size_t)s0 * H + e];
    keys[e] = ocount[sid] == 0 ? ((uint64_t)H << 32)
                               : (((uint64_t)j << 32) | ((uint32_t)v ^ 0x80000000u));
    vals[e] = sid;
  }
}

__global__ void k_mh_table_offsets(const uint64_t *keys, size_t n, int32_t H, uint64_t *off) {
  const int32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j > H) return;
  const uint64_t key = (uint64_t)j << 32;
  size_t lo = 0, hi = n;
  while (lo < hi) {
    const size_t mid = (lo + hi) >> 1;
    if (keys[mid] < key) lo = mid + 1;
    else hi = mid;
  }
  off[j] = lo;
}

// ---- first stage ----------------------------------------------------------------------------
struct CandArgs {
  const int32_t *mh;
  const uint32_t *ocount;
  const uint32_t *len;
  const uint64_t *keys;
  const uint32_t *vals;
  const uint64_t *toff;
  int32_t H;
  uint32_t q0, q1;                // query reads [q0, q1)
  uint32_t self;                  // 1: toSelf (stored reads of smaller ID), 0: all but q
  int32_t min_store;
  uint32_t min_matches;
  Cand *out;
  uint32_t *nout;
  uint32_t cap;
  uint32_t *overflow;
};

// MinHashSearch.findMatches(query, toSelf) @0-492 (oracle mhap_jar.find_matches)
__global__ void __launch_bounds__(256) k_mh_candidates(CandArgs A) {
  extern __shared__ uint32_t s_tab[];              // [4][TSLOTS] keys, then [4][TSLOTS] counts
  const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const uint32_t q = A.q0 + blockIdx.x * 4 + wave;
  if (q >= A.q1) return;                           // whole wave leaves together
  if (A.ocount[2 * q] == 0) return;                // query not used
  uint32_t *tk = s_tab + wave * TSLOTS;
  uint32_t *tc = s_tab + 4 * TSLOTS + wave * TSLOTS;
  for (uint32_t i = lane; i < TSLOTS; i += 64) { tk[i] = 0; tc[i] = 0; }
  wave_sync();
  const int32_t qlen = (int32_t)A.len[q], ms = A.min_store;
  bool ovf = false;
  for (int32_t j = lane; j < A.H; j += 64) {
    const int32_t v = A.mh[(size_t)(2 * q) * A.H + j];
    const uint64_t key = ((uint64_t)j << 32) | ((uint32_t)v ^ 0x80000000u);
    uint64_t lo = A.toff[j], hi = A.toff[j + 1];
    while (lo < hi) {
      const uint64_t mid = (lo + hi) >> 1;
      if (A.keys[mid] < key) lo = mid + 1;
      else hi = mid;
    }
    const uint64_t end = A.toff[j + 1];
    for (uint64_t i = lo; i < end && A.keys[i] == key; i++) {
      const uint32_t t = A.vals[i], tr = t >> 1;
      if (tr == q) continue;
      const int32_t tlen = (int32_t)A.len[tr];
      if (tlen < ms && qlen < ms) continue;                                 // @393-416
      if (A.self && tr > q && tlen >= ms && qlen >= ms) continue;           // @419-462
      if (A.self && tlen < ms && qlen >= ms) continue;                      // @465-492
      uint32_t sl = ((t + 1) * 2654435761u) >> TSHIFT;
      uint32_t probes = 0;
      for (;;) {
        const uint32_t old = atomicCAS(&tk[sl], 0u, t + 1);
        if (old == 0u || old == t + 1) { atomicAdd(&tc[sl], 1u); break; }
        sl = (sl + 1) & (TSLOTS - 1);
        if (++probes >= TSLOTS) { ovf = true; break; }
      }
      if (ovf) break;
    }
  }
  wave_sync();
  if (ovf) atomicOr(A.overflow, 1u);
  for (uint32_t i = lane; i < TSLOTS; i += 64) {
    const uint32_t key = tk[i], c = tc[i];
    if (key && c >= A.min_matches) {
      const uint32_t idx = atomicAdd(A.nout, 1u);
      if (idx < A.cap) A.out[idx] = Cand{q, key - 1, c, 0};
      else atomicOr(A.overflow, 2u);
    }
  }
}

// ---- second stage ---------------------------------------------------------------------------
struct CmpArgs {
  const Cand *cand;
  uint32_t ncand;
  const uint64_t *ordered;
  const uint32_t *ocount;
  const uint32_t *len;
  int32_t S, kk;
  double max_shift;
  const uint32_t *pass;           // bit n (S + 1) + inter: identity(inter / n) >= threshold
  uint32_t pass_empty;            // identity 0 (n = 0) >= threshold
  RecDev *out;
  uint32_t *nout;
  uint32_t cap;
  uint32_t *overflow;
};

__device__ __forceinline__ uint32_t hash_of(uint64_t e) { return (uint32_t)(e >> 32); }
__device__ __forceinline__ int32_t pos_of(uint64_t e) { return (int32_t)(uint32_t)e; }

// A group: the entries of one hash present in both sketches, A[a0, a1) and B[b0, b1)
struct Group {
  uint32_t a0, a1, b0, b1;
};
__device__ __forceinline__ uint64_t pack_group(uint32_t a0, uint32_t a1, uint32_t b0, uint32_t b1) {
  return (uint64_t)a0 | ((uint64_t)a1 << 16) | ((uint64_t)b0 << 32) | ((uint64_t)b1 << 48);
}
__device__ __forceinline__ Group unpack_group(uint64_t g) {
  return Group{(uint32_t)(g & 0xFFFF), (uint32_t)((g >> 16) & 0xFFFF),
               (uint32_t)((g >> 32) & 0xFFFF), (uint32_t)(g >> 48)};
}

// MatchData's state for one recordMatchingKmers pass: median shift, its absMax and the
// valid position windows (performUpdate @0-134, valid1/2Lower/Upper)
struct Window {
  int32_t m, amax, v1lo, v1hi, v2lo, v2hi;
};

__device__ __forceinline__ Window make_window(int32_t m, int32_t amax, int32_t sl1, int32_t sl2) {
  Window w;
  w.m = m;
  w.amax = amax;
  w.v1lo = max(0, -m - amax);
  w.v2lo = max(0, m - amax);
  w.v1hi = min(sl1, sl2 - m + amax);
  w.v2hi = min(sl2, sl1 + m + amax);
  return w;
}

// performUpdate with records whose median shift is m
__device__ __forceinline__ int32_t abs_max(int32_t m, int32_t sl1, int32_t sl2, double msp) {
  const int32_t lo = max(0, -m);
  const int32_t hi = min(sl1, sl2 - m);
  const int32_t olap = max(10, hi - lo);
  return min(max(sl1, sl2), (int32_t)__dmul_rn((double)olap, msp));
}

// recordMatchingKmers @0-450 restricted to one group (the jar's merge only ever compares
// entries of equal hash when it records, and enters each group at its first entries on both
// sides, so groups are independent): emit(p1, p2) per recorded match, in the jar's order
template <class Emit>
__device__ __forceinline__ void group_records(const uint64_t *A, const uint64_t *B, Group g,
                                              const Window &w, Emit emit) {
  uint32_t i1 = g.a0, i2 = g.b0;
  while (i1 < g.a1 && i2 < g.b1) {
    const int32_t p1 = pos_of(A[i1]);
    if (p1 < w.v1lo || p1 >= w.v1hi) { i1++; continue; }
    const int32_t p2 = pos_of(B[i2]);
    if (p2 < w.v2lo || p2 >= w.v2hi) { i2++; continue; }
    const int32_t d = (p2 - p1) - w.m;
    if (d > w.amax) { i1++; continue; }
    if (d < -w.amax) { i2++; continue; }
    emit(p1, p2);
    uint32_t l1 = i1, l2 = i2;
    for (uint32_t j = i1 + 1; j < g.a1; j++) {
      const int32_t p = pos_of(A[j]);
      if (p < w.v1lo || p >= w.v1hi) break;
      l1 = j;
    }
    for (uint32_t j = i2 + 1; j < g.b1; j++) {
      const int32_t p = pos_of(B[j]);
      if (p < w.v2lo || p >= w.v2hi) break;
      l2 = j;
    }
    if (l1 == i1 && l2 == i2) {
      i1++;
      i2++;
    } else {
      emit(pos_of(A[l1]), pos_of(B[l2]));
      i1 = l1 + 1;
      i2 = l2 + 1;
    }
  }
}

// the same records after optimizeShifts @0-165 (consecutive records of one p1 keep the one
// whose shift is nearest the median m; equal p1 only ever occur inside a group)
template <class Emit>
__device__ __forceinline__ void group_records_opt(const uint64_t *A, const uint64_t *B, Group g,
                                                  const Window &w, int32_t m, Emit emit) {
  bool has = false;
  int32_t q1 = 0, q2 = 0;
  group_records(A, B, g, w, [&](int32_t p1, int32_t p2) {
    if (has && q1 == p1) {
      if (abs(q2 - q1 - m) > abs(p2 - p1 - m)) q2 = p2;
    } else {
      if (has) emit(q1, q2);
      has = true;
      q1 = p1;
      q2 = p2;
    }
  });
  if (has) emit(q1, q2);
}

// The (count / 2)-th smallest shift p2 - p1 over the records gen() emits (Utils.quickSelect
// of performUpdate): a radix select over u = shift + off (off = sl1, so u > 0) in 8-bit
// digits; count = the number of records (0: none)
template <class Gen>
__device__ int32_t wave_median(Gen gen, int32_t off, uint32_t bits, uint32_t *hist,
                               uint32_t lane, uint32_t &count) {
  const int npass = (int)((bits + 7) / 8);
  uint32_t prefix = 0, pmask = 0, kth = 0;
  count = 0;
  for (int pass = npass - 1; pass >= 0; pass--) {
    for (uint32_t i = lane; i < 256; i += 64) hist[i] = 0;
    wave_sync();
    gen([&](int32_t p1, int32_t p2) {
      const uint32_t u = (uint32_t)(p2 - p1 + off);
      if ((u & pmask) == prefix) atomicAdd(&hist[(u >> (8 * pass)) & 255u], 1u);
    });
    wave_sync();
    const uint32_t h0 = hist[4 * lane], h1 = hist[4 * lane + 1], h2 = hist[4 * lane + 2],
                   h3 = hist[4 * lane + 3];
    const uint32_t tot = h0 + h1 + h2 + h3;
    uint32_t incl = tot;
    for (int sft = 1; sft < 64; sft <<= 1) {
      const uint32_t v = __shfl_up(incl, sft);
      if ((int)lane >= sft) incl += v;
    }
    if (pass == npass - 1) {
      count = __shfl(incl, 63);
      if (count == 0) return 0;
      kth = count / 2;
    }
    const uint32_t excl = incl - tot;
    const bool mine = excl <= kth && kth < incl;
    const uint64_t who = __builtin_amdgcn_ballot_w64(mine);
    const uint32_t owner = (uint32_t)__builtin_ctzll(who);
    uint32_t bin = 0, before = excl;
    if (mine) {
      const uint32_t rem = kth - excl;
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
  return (int32_t)prefix - off;
}

// BottomOverlapSketch.getOverlapInfo(other, maxShift) @0-211 (oracle mhap_jar.overlap_info);
// one wave per candidate; LDS per wave: A [S], B [S], groups [S] (u64) and a 256-bin histogram
__global__ void __launch_bounds__(64) k_mh_compare(CmpArgs A) {
  extern __shared__ uint64_t s_cmp[];
  const uint32_t lane = threadIdx.x;
  const int32_t S = A.S;
  uint64_t *la = s_cmp;
  uint64_t *lb = la + S;
  uint64_t *lg = lb + S;
  uint32_t *hist = (uint32_t *)(lg + S);
  const uint64_t lane_lt = (1ull << lane) - 1;
  for (uint32_t c = blockIdx.x; c < A.ncand; c += gridDim.x) {
    wave_sync();                                   // the previous pair's LDS reads are done
    const Cand cd = A.cand[c];
    const uint32_t sa = 2 * cd.q, sb = cd.t;
    const uint32_t na = A.ocount[sa], nb = A.ocount[sb];
    const int32_t la_len = (int32_t)A.len[cd.q], lb_len = (int32_t)A.len[sb >> 1];
    const int32_t sl1 = la_len - A.kk + 1, sl2 = lb_len - A.kk + 1;   // seqLength
    {
      const uint64_t *ga = A.ordered + (size_t)sa * S;
      const uint64_t *gb = A.ordered + (size_t)sb * S;
      for (uint32_t i = lane; i < na; i += 64) la[i] = ga[i];
      for (uint32_t i = lane; i < nb; i += 64) lb[i] = gb[i];
    }
    wave_sync();
    // groups, in hash order: lane l owns A[l c, l c + c) and the groups starting there
    const uint32_t crun = (na + 63) / 64;
    const uint32_t a_lo = lane * crun, a_hi = min(a_lo + crun, na);
    auto discover = [&](auto found) {
      uint32_t bp = 0;
      if (a_lo < a_hi) {                           // lower bound of A[a_lo]'s hash in B
        const uint32_t h = hash_of(la[a_lo]);
        uint32_t lo = 0, hi = nb;
        while (lo < hi) {
          const uint32_t mid = (lo + hi) >> 1;
          if (hash_of(lb[mid]) < h) lo = mid + 1;
          else hi = mid;
        }
        bp = lo;
      }
      for (uint32_t i = a_lo; i < a_hi; i++) {
        const uint32_t h = hash_of(la[i]);
        if (i > 0 && hash_of(la[i - 1]) == h) continue;   // not a group start
        while (bp < nb && hash_of(lb[bp]) < h) bp++;
        if (bp < nb && hash_of(lb[bp]) == h) {
          uint32_t ae = i + 1, be = bp + 1;
          while (ae < na && hash_of(la[ae]) == h) ae++;
          while (be < nb && hash_of(lb[be]) == h) be++;
          found(i, ae, bp, be);
        }
      }
    };
    uint32_t mine = 0;
    discover([&](uint32_t, uint32_t, uint32_t, uint32_t) { mine++; });
    uint32_t goff = mine;                          // exclusive scan over lanes
    for (int sft = 1; sft < 64; sft <<= 1) {
      const uint32_t v = __shfl_up(goff, sft);
      if ((int)lane >= sft) goff += v;
    }
    const uint32_t ngroups = __shfl(goff, 63);
    goff -= mine;
    if (ngroups == 0) continue;                    // no shared k'-mer: EMPTY
    discover([&](uint32_t a0, uint32_t a1, uint32_t b0, uint32_t b1) {
      lg[goff++] = pack_group(a0, a1, b0, b1);
    });
    wave_sync();
    const uint32_t bits = 32u - (uint32_t)__builtin_clz((uint32_t)(sl1 + sl2));
    // pass 0: no records yet -> median 0, absMax = max(seqLength) + 1, everything valid
    const Window w0 = make_window(0, max(sl1, sl2) + 1, sl1, sl2);
    uint32_t n0 = 0;
    const int32_t m0 = wave_median([&](auto emit) {
      for (uint32_t g = lane; g < ngroups; g += 64) group_records(la, lb, unpack_group(lg[g]), w0, emit);
    }, sl1, bits, hist, lane, n0);
    if (n0 == 0) continue;
    // pass 1 in the windows of pass 0's median
    const Window w1 = make_window(m0, abs_max(m0, sl1, sl2, A.max_shift), sl1, sl2);
    uint32_t n1 = 0;
    const int32_t m1 = wave_median([&](auto emit) {
      for (uint32_t g = lane; g < ngroups; g += 64) group_records(la, lb, unpack_group(lg[g]), w1, emit);
    }, sl1, bits, hist, lane, n1);
    if (n1 == 0) continue;
    // optimizeShifts with pass 1's median, then computeEdges with the new median
    uint32_t n2 = 0;
    const int32_t m2 = wave_median([&](auto emit) {
      for (uint32_t g = lane; g < ngroups; g += 64)
        group_records_opt(la, lb, unpack_group(lg[g]), w1, m1, emit);
    }, sl1, bits, hist, lane, n2);
    const int32_t a2m = abs_max(m2, sl1, sl2, A.max_shift);
    int32_t cnt = 0, l1 = 0x7FFFFFFF, l2 = 0x7FFFFFFF, r1 = (int32_t)0x80000000,
            r2 = (int32_t)0x80000000;
    for (uint32_t g = lane; g < ngroups; g += 64) {
      group_records_opt(la, lb, unpack_group(lg[g]), w1, m1, [&](int32_t p1, int32_t p2) {
        if (abs(p2 - p1 - m2) > a2m) return;
        l1 = min(l1, p1); l2 = min(l2, p2);
        r1 = max(r1, p1); r2 = max(r2, p2);
        cnt++;
      });
    }
    cnt = wave_sum_i32(cnt);
    if (cnt < 3) continue;
    l1 = wave_min_i32(l1); l2 = wave_min_i32(l2);
    r1 = wave_max_i32(r1); r2 = wave_max_i32(r2);
    // computeEdges @118-236: int imul / isub (wrapping), i2d, ddiv, Math.round, l2i
    auto edge = [&](int32_t x, int32_t y) {
      const int32_t num = (int32_t)((uint32_t)((uint32_t)cnt * (uint32_t)x) - (uint32_t)y);
      return (int32_t)java_round((double)num / (double)(cnt - 1));
    };
    const int32_t e_a1 = max(0, edge(l1, r1));
    const int32_t e_a2 = min(sl1, edge(r1, l1));
    const int32_t e_b1 = max(0, edge(l2, r2));
    const int32_t e_b2 = min(sl2, edge(r2, l2));
    // computeKBottomSketchJaccard @0-227: the entries of each sketch whose position lies in
    // its edge range (in hash order), n = min of the two counts, a merge of n steps counting
    // equal hashes.  Closed form: a value v present in both with rx / ry entries in range
    // takes max(rx, ry) steps, min(rx, ry) of them equal, after xr + yr - E(< v) steps (xr,
    // yr: entries in range below v; E: equal steps of smaller values); a value in one
    // sketch only adds steps, no equality.  The hash halves of la / lb are replaced by the
    // exclusive prefix counts of in-range entries (group discovery is done).
    uint32_t nx = 0, ny = 0;
    for (uint32_t i0 = 0; i0 < na; i0 += 64) {
      const uint32_t i = i0 + lane;
      bool in = false;
      int32_t p = 0;
      if (i < na) { p = pos_of(la[i]); in = p >= e_a1 && p <= e_a2; }
      const uint64_t m = __builtin_amdgcn_ballot_w64(in);
      if (i < na) la[i] = ((uint64_t)(nx + popc64(m & lane_lt)) << 32) | (uint32_t)p;
      nx += popc64(m);
    }
    for (uint32_t i0 = 0; i0 < nb; i0 += 64) {
      const uint32_t i = i0 + lane;
      bool in = false;
      int32_t p = 0;
      if (i < nb) { p = pos_of(lb[i]); in = p >= e_b1 && p <= e_b2; }
      const uint64_t m = __builtin_amdgcn_ballot_w64(in);
      if (i < nb) lb[i] = ((uint64_t)(ny + popc64(m & lane_lt)) << 32) | (uint32_t)p;
      ny += popc64(m);
    }
    wave_sync();
    const uint32_t n = min(nx, ny);
    uint32_t inter = 0;
    if (n > 0) {
      uint32_t carry = 0;                         // E over the groups before this chunk
      for (uint32_t g0 = 0; g0 < ngroups; g0 += 64) {
        const uint32_t g = g0 + lane;
        uint32_t eq = 0, xr = 0, yr = 0;
        if (g < ngroups) {
          const Group G = unpack_group(lg[g]);
          xr = hash_of(la[G.a0]);
          yr = hash_of(lb[G.b0]);
          const uint32_t xe = G.a1 < na ? hash_of(la[G.a1]) : nx;
          const uint32_t ye = G.b1 < nb ? hash_of(lb[G.b1]) : ny;
          eq = min(xe - xr, ye - yr);
        }
        uint32_t incl = eq;
        for (int sft = 1; sft < 64; sft <<= 1) {
          const uint32_t v = __shfl_up(incl, sft);
          if ((int)lane >= sft) incl += v;
        }
        const int64_t steps = (int64_t)xr + yr - (int64_t)(carry + incl - eq);
        const int64_t left = (int64_t)n - steps;
        uint32_t got = 0;
        if (eq && left > 0) got = (uint32_t)min<int64_t>(eq, left);
        inter += got;
        carry += __shfl(incl, 63);
      }
      inter = (uint32_t)wave_sum_i32((int32_t)inter);
    }
    const bool ok = n == 0 ? A.pass_empty != 0
                           : ((A.pass[((size_t)n * (S + 1) + inter) >> 5] >> (((size_t)n * (S + 1) + inter) & 31)) & 1u) != 0;
    if (!ok) continue;
    if (lane == 0) {
      const uint32_t idx = atomicAdd(A.nout, 1u);
      if (idx < A.cap) {
        RecDev rr;
        rr.a = cd.q;
        rr.b = sb >> 1;
        rr.o = sb & 1;
        rr.cnt = cd.cnt;
        rr.inter = inter;
        rr.n = n;
        rr.raw = (uint32_t)cnt;
        rr.pad = 0;
        rr.a1 = e_a1; rr.a2 = e_a2; rr.a_len = la_len;
        // MatchResult.<init> @86-143: reverse-strand coordinates mirrored on the read
        rr.b1 = rr.o ? lb_len - e_b2 - 1 : e_b1;
        rr.b2 = rr.o ? lb_len - e_b1 - 1 : e_b2;
        rr.b_len = lb_len;
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
  // weighting (MhapMain options + FrequencyCounts)
  mhap_weighting W{0.9, 3.0, 1e-5, 0, 0};
  bool has_table = false;
  MBuf<FreqSlot> ftab;
  uint64_t fmask = 0;
  bool has_bloom = false;               // --supress-noise 1 with a -f table
  MBuf<uint64_t> bloom;
  uint64_t bloom_bits = 0;
  int32_t bloom_k = 0;
  // second-stage acceptance: identity(inter / n) >= threshold, per (n, inter)
  MBuf<uint32_t> pass;
  uint32_t pass_empty = 0;
  // sketches
  MBuf<int32_t> minhash;
  MBuf<uint64_t> ordered;
  MBuf<uint32_t> ocount;
  MBuf<uint64_t> mkeys, mkeys2;
  MBuf<uint32_t> mpos, mpos2, msids;
  MBuf<uint64_t> mkoff;
  MBuf<uint8_t> msort_tmp;
  MBuf<uint32_t> mbscnt;          // bit-sliced draws: per batch strand, its listed k-mers
  MBuf<BestOut> mbest;            //   and the exact pass's minima [batch strand][H]
  // index
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

// the jar's score of a Jaccard value (BottomOverlapSketch.jaccardToIdentity @0-25)
static double jaccard_identity(double J, int kk) {
  if (!(J > 0.0)) return 0.0;
  const double d = (-1.0 / (double)kk) * log(2.0 * J / (1.0 + J));
  return exp(-d);
}

// computeKBottomSketchJaccard's J = inter / n (0 when n = 0)
static double jaccard_of(uint32_t inter, uint32_t n) {
  return n == 0 ? 0.0 : (double)inter / (double)n;
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
  p->max_shift = 0.2;
  p->min_store = 0;
  p->no_rc = 0;
}

void mhap_weighting_init(mhap_weighting *w) {
  w->repeat_weight = 0.9;
  w->repeat_idf_scale = 3.0;
  w->filter_threshold = 1e-5;
  w->no_tf = 0;
  w->supress_noise = 0;
}

int mhap_ctx_create(const mhap_params *p, int device, mhap_ctx **out) {
  *out = nullptr;
  if (!p) return mfail(M_BAD_PARAM, "null params");
  if (p->k < 1 || p->k > 32 || p->ordered_k < 1 || p->ordered_k > 32)
    return mfail(M_BAD_PARAM, "k-mer sizes must be 1..32");
  if (p->num_hashes < 1 || p->num_hashes > 1024)
    return mfail(M_BAD_PARAM, "num_hashes must be 1..1024");
  if (p->ordered_sketch < 1 || p->ordered_sketch > 2048)   // k_mh_compare LDS: 3 x 8 S + 1 KB
    return mfail(M_BAD_PARAM, "ordered_sketch must be 1..2048");
  if (p->min_matches < 1) return mfail(M_BAD_PARAM, "min_matches must be >= 1");
  if (!(p->max_shift >= -1.0)) return mfail(M_BAD_PARAM, "--max-shift must be >= -1");
  if (p->min_store < 0) return mfail(M_BAD_PARAM, "--min-store-length must be >= 0");
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
  if (c->ctr.alloc(16) != hipSuccess || c->kctr.alloc(2) != hipSuccess) {
    delete c;
    return mfail(M_OOM, "counters");
  }
  // the complement table (Utils$Translate)
  uint8_t comp[256] = {0};
  const char *from = "ABCDGHKMNRSTVWY", *to = "TVGHCDMKNYSABWR";
  for (int i = 0; from[i]; i++) comp[(uint8_t)from[i]] = (uint8_t)to[i];
  if (hipMemcpyToSymbol(HIP_SYMBOL(c_comp), comp, 256) != hipSuccess) {
    delete c;
    return mfail(M_HIP, "complement table");
  }
  // acceptance bits: the identity is computed here, on the host, exactly as the oracle does
  const uint32_t S = p->ordered_sketch;
  const size_t nbits = (size_t)(S + 1) * (S + 1);
  std::vector<uint32_t> bits((nbits + 31) / 32, 0);
  for (uint32_t n = 1; n <= S; n++)
    for (uint32_t i = 0; i <= n; i++)
      if (jaccard_identity(jaccard_of(i, n), (int)p->ordered_k) >= p->threshold) {
        const size_t b = (size_t)n * (S + 1) + i;
        bits[b >> 5] |= 1u << (b & 31);
      }
  c->pass_empty = jaccard_identity(0.0, (int)p->ordered_k) >= p->threshold ? 1u : 0u;
  if (c->pass.alloc(bits.size()) != hipSuccess ||
      hipMemcpy(c->pass.p, bits.data(), 4 * bits.size(), hipMemcpyHostToDevice) != hipSuccess) {
    delete c;
    return mfail(M_OOM, "acceptance table");
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

static int alloc_sketches(mhap_ctx *c) {
  const size_t n = 2ull * c->nreads;
  if (c->minhash.alloc(n * c->P.num_hashes) || c->ordered.alloc(n * c->P.ordered_sketch) ||
      c->ocount.alloc(n))
    return mfail(M_OOM, "sketch arrays for %u reads", c->nreads);
  MHC(hipMemsetAsync(c->ocount.p, 0, 4 * n, c->stream));
  c->indexed = false;
  return M_OK;
}

static int set_lengths(mhap_ctx *c, uint32_t first_iid, uint32_t nreads, const uint32_t *lens) {
  if (first_iid == 0) return mfail(M_BAD_PARAM, "gkStore IDs start at 1");
  if (nreads >= 0x7FFFFFF0u) return mfail(M_BAD_PARAM, "too many reads");
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

static int check_weighting(const mhap_weighting *w) {
  if (!w) return mfail(M_BAD_PARAM, "null weighting");
  if (!(w->repeat_idf_scale >= 1.0))
    return mfail(M_BAD_PARAM, "The minimum repeat idf scale must be >=1.0.");
  if (w->supress_noise < 0 || w->supress_noise > 2)            // FrequencyCounts.<init> @10-50
    return mfail(M_BAD_PARAM, "Unknown removeUnique option %d.", w->supress_noise);
  return M_OK;
}

int mhap_set_weighting(mhap_ctx *c, const mhap_weighting *w) {
  if (!c) return mfail(M_STATE, "null context");
  const int rc = check_weighting(w);
  if (rc) return rc;
  c->W = *w;
  c->has_table = false;                 // no -f: no FrequencyCounts, so no keepKmer either
  c->has_bloom = false;
  return M_OK;
}

int mhap_set_kmer_frequencies(mhap_ctx *c, const char *kmers, const double *fractions,
                              uint64_t n, const mhap_weighting *w) {
  return mhap_set_kmer_frequencies_ex(c, kmers, fractions, n, n, w);
}

// FrequencyCounts.<init> @0-429 and its lambda$1 (oracle mhap_jar.FrequencyCounts); with
// --supress-noise 1 also its Bloom filter of every line's key (oracle mhap_jar.GuavaBloom)
int mhap_set_kmer_frequencies_ex(mhap_ctx *c, const char *kmers, const double *fractions,
                                 uint64_t n, uint64_t expected, const mhap_weighting *w) {
  if (!c) return mfail(M_STATE, "null context");
  int rc = check_weighting(w);
  if (rc) return rc;
  if (n && (!kmers || !fractions)) return mfail(M_BAD_PARAM, "null k-mers / fractions");
  // Guava BloomFilter.create(funnel, expected (0 -> 1), 1e-5): optimalNumOfBits,
  // optimalNumOfHashFunctions, BitArray of ceil(bits / 64) longs.  removeUnique 2 builds it
  // and never reads it (keepKmer @0-21), so only 1 does here.
  const bool bloom = w->supress_noise == 1;
  std::vector<uint64_t> bw;
  uint64_t bloom_bits = 0;
  int32_t bloom_k = 0;
  if (bloom) {
    const int64_t ne = expected ? (int64_t)expected : 1;
    const int64_t bits = (int64_t)((double)(-ne) * log(1e-5) / (log(2.0) * log(2.0)));
    const double hk = (double)bits / (double)ne * log(2.0);
    const double fk = floor(hk);
    bloom_k = std::max<int32_t>(1, (int32_t)((int64_t)fk + (hk - fk >= 0.5 ? 1 : 0)));
    bw.assign((size_t)((bits + 63) / 64), 0ull);
    if (bw.empty()) return mfail(M_BAD_PARAM, "Bloom filter of 0 bits");
    bloom_bits = 64ull * bw.size();
  }
  const uint32_t k = c->P.k;
  const bool do_rc = !c->P.no_rc;
  const double offset = (w->repeat_weight >= 0.0 && w->repeat_weight < 1.0) ? w->repeat_weight : 0.0;
  const double cutoff = w->filter_threshold, range = w->repeat_idf_scale;
  // key -> fraction, file order, a later line of the same key replacing an earlier one
  std::vector<std::pair<uint64_t, double>> kv;
  double max_value = -INFINITY;
  std::vector<uint8_t> km(k), rk(k);
  for (uint64_t i = 0; i < n; i++) {
    const double f = fractions[i];
    if (!(f >= cutoff) && !bloom) continue;
    for (uint32_t t = 0; t < k; t++) km[t] = (uint8_t)kmers[i * k + t];
    const uint8_t *use = km.data();
    if (do_rc) {                                  // Utils.rc: reverse, upper case, complement
      static const char *from = "ABCDGHKMNRSTVWY", *to = "TVGHCDMKNYSABWR";
      for (uint32_t t = 0; t < k; t++) {
        const uint8_t b = (uint8_t)upper_byte(km[k - 1 - t]);
        uint8_t o = 0;
        for (int q = 0; from[q]; q++)
          if ((uint8_t)from[q] == b) o = (uint8_t)to[q];
        rk[t] = o;
      }
      if (memcmp(rk.data(), km.data(), k) < 0) use = rk.data();   // String.compareTo
    }
    const uint64_t key = murmur128_h1([&](int32_t q) { return (uint64_t)use[q]; }, (int32_t)k);
    if (bloom) {                              // lambda$1 @162-185: every line, any fraction
      uint64_t h1, h2;
      murmur128_u64(key, h1, h2);
      uint64_t x = h1;
      for (int32_t j = 0; j < bloom_k; j++, x += h2) {
        const uint64_t b = (x & 0x7FFFFFFFFFFFFFFFull) % bloom_bits;
        bw[b >> 6] |= 1ull << (b & 63);
      }
    }
    if (!(f >= cutoff)) continue;
    max_value = std::max(max_value, f);
    kv.emplace_back(key, f);
  }
  const auto idf = [&](double x) { return log(max_value / x - offset); };
  const double min_idf = idf(max_value), max_idf = idf(cutoff);
  const double scale = (max_idf - min_idf) / (range - 1.0);
  // open addressing at load <= 1/2; later lines overwrite
  uint64_t slots = 16;
  while (slots < 2 * kv.size() + 1) slots <<= 1;
  std::vector<FreqSlot> tab(slots, FreqSlot{0, 0.0, 0, 0});
  for (const auto &e : kv) {
    uint64_t h = fmix64(e.first ^ 0x9E3779B97F4A7C15ull) & (slots - 1);
    while (tab[h].used && tab[h].key != e.first) h = (h + 1) & (slots - 1);
    tab[h].key = e.first;
    tab[h].used = 1;
    tab[h].sidf = 1.0 + (idf(e.second) - min_idf) / scale;     // scaledIdf @31-94
  }
  MHC(hipSetDevice(c->device));
  if (c->ftab.alloc(slots)) return mfail(M_OOM, "k-mer frequency table");
  MHC(hipMemcpy(c->ftab.p, tab.data(), sizeof(FreqSlot) * slots, hipMemcpyHostToDevice));
  c->fmask = slots - 1;
  if (bloom) {
    if (c->bloom.alloc(bw.size())) return mfail(M_OOM, "k-mer Bloom filter");
    MHC(hipMemcpy(c->bloom.p, bw.data(), 8ull * bw.size(), hipMemcpyHostToDevice));
    c->bloom_bits = bloom_bits;
    c->bloom_k = bloom_k;
  }
  c->has_bloom = bloom;
  c->W = *w;
  c->has_table = true;
  return M_OK;
}

// The weight of a k-mer seen once in its strand and not in the -f table -- nearly all of a
// sketch's k-mers -- whose draws k_mh_bitslice takes (0: off; MHAP_BITSLICE=0 for A/Bs)
static int32_t bitslice_weight(const mhap_ctx *c, int mode) {
  if (const char *e = getenv("MHAP_BITSLICE"))
    if (atoi(e) == 0) return 0;
  if (mode != W_TFIDF) return 1;                    // W_ONE: 1 (not popular); W_COUNT: count
  const double x = c->W.repeat_idf_scale;           // tf(1) x scaledIdf of an absent k-mer
  const double f = floor(x);
  const int64_t w = (int64_t)f + (x - f >= 0.5 ? 1 : 0);   // Math.round
  return (int32_t)std::min<int64_t>(std::max<int64_t>(w, 1), 0x7FFFFFFF);
}

// The MinHash sketches of strands (sids) in batches of <= KEY_BUDGET k-mers: keys, segmented
// radix sort of (key, position), draws (exact for the first round of every strand and for
// k-mers of other weights, bit-sliced for the rest).
static int sketch_minhash(mhap_ctx *c, const std::vector<uint32_t> &sids) {
  hipStream_t s = c->stream;
  const int32_t k = (int32_t)c->P.k;
  const uint64_t KEY_BUDGET = 1ull << 29;
  const int mode = c->W.repeat_weight < 0.0 ? W_ONE
                 : (c->has_table && c->W.repeat_weight < 1.0) ? W_TFIDF : W_COUNT;
  const int32_t bs_w = bitslice_weight(c, mode);
  const int32_t H = (int32_t)c->P.num_hashes;
  // the exact sample: a strand's first 2,048 sorted k-mers (x w draws) put a function's
  // minimum near 2^64 / 20,480 above -2^63, so the bit-sliced filter starts at ~14 planes;
  // measured on configs[3]: sketch 5.62 s with 2,048, 6.37 s with 512, 6.61 s with 128
  // (profiles/r06s_mhap_sample_ab.txt; MHAP_BS_SAMPLE for A/Bs)
  uint32_t bs_sample = 2048;
  if (const char *e = getenv("MHAP_BS_SAMPLE")) bs_sample = (uint32_t)std::max(0, atoi(e));
  for (size_t a = 0; a < sids.size();) {
    std::vector<uint64_t> koff;
    uint64_t tot = 0;
    size_t b = a;
    while (b < sids.size() && b - a < (1u << 20)) {
      const int64_t np = (int64_t)c->h_len[sids[b] >> 1] - k + 1;
      const uint64_t add = np > 0 ? (uint64_t)np : 0;
      if (tot + add > KEY_BUDGET && b > a) break;
      koff.push_back(tot);
      tot += add;
      b++;
    }
    koff.push_back(tot);
    const uint32_t nb = (uint32_t)(b - a);
    if (c->mkoff.alloc(nb + 1) || c->msids.alloc(nb) || c->mkeys.alloc(tot) ||
        c->mkeys2.alloc(tot) || c->mpos.alloc(tot) || c->mpos2.alloc(tot))
      return mfail(M_OOM, "MinHash keys (%llu)", (unsigned long long)tot);
    MHC(hipMemcpyAsync(c->mkoff.p, koff.data(), 8ull * (nb + 1), hipMemcpyHostToDevice, s));
    MHC(hipMemcpyAsync(c->msids.p, sids.data() + a, 4ull * nb, hipMemcpyHostToDevice, s));
    KeyArgs KA{c->d_bases, c->d_off, c->d_len.p, c->msids.p, c->mkoff.p, k, c->mkeys.p, c->mpos.p};
    hipLaunchKernelGGL(k_mh_keys, dim3(nb), dim3(256), 0, s, KA);
    MHC(hipGetLastError());
    size_t tb = 0;
    MHC(hipcub::DeviceSegmentedRadixSort::SortPairs(nullptr, tb, c->mkeys.p, c->mkeys2.p,
                                                    c->mpos.p, c->mpos2.p, (int)tot, (int)nb,
                                                    c->mkoff.p, c->mkoff.p + 1, 0, 64, s));
    if (c->msort_tmp.alloc(std::max<size_t>(tb, 1))) return mfail(M_OOM, "sort scratch");
    MHC(hipcub::DeviceSegmentedRadixSort::SortPairs(c->msort_tmp.p, tb, c->mkeys.p, c->mkeys2.p,
                                                    c->mpos.p, c->mpos2.p, (int)tot, (int)nb,
                                                    c->mkoff.p, c->mkoff.p + 1, 0, 64, s));
    if (bs_w && (c->mbscnt.alloc(nb) || c->mbest.alloc((size_t)nb * H)))
      return mfail(M_OOM, "bit-sliced draws (%u strands)", nb);
    // the sorted keys are in mkeys2 / mpos2: mkeys / mpos hold the bit-sliced lists
    SketchArgs SA{c->mkeys2.p, c->mpos2.p, c->mkoff.p, c->msids.p, H,
                  mode, c->has_table ? c->ftab.p : nullptr, c->fmask, c->W.repeat_idf_scale,
                  c->W.no_tf, c->minhash.p, c->ocount.p, c->kctr.p,
                  bs_w, bs_sample, c->mkeys.p, c->mpos.p, c->mbscnt.p, c->mbest.p,
                  BloomDev{c->has_bloom ? c->bloom.p : nullptr, c->bloom_bits, c->bloom_k}};
    const size_t lds = sizeof(BestRec) * 4 * c->P.num_hashes;
    MHC(hipEventRecord(c->ev[2], s));
    hipLaunchKernelGGL(k_mh_minhash, dim3(nb), dim3(256), lds, s, SA);
    MHC(hipGetLastError());
    if (bs_w && getenv("MHAP_BS_DUMP")) {      // checks: the exact pass's minima and lists
      MHC(hipStreamSynchronize(s));
      std::vector<BestOut> hb((size_t)nb * H);
      std::vector<uint32_t> hc(nb);
      MHC(hipMemcpy(hb.data(), c->mbest.p, sizeof(BestOut) * hb.size(), hipMemcpyDeviceToHost));
      MHC(hipMemcpy(hc.data(), c->mbscnt.p, 4ull * nb, hipMemcpyDeviceToHost));
      if (FILE *f = fopen(getenv("MHAP_BS_DUMP"), "wb")) {
        fwrite(&nb, 4, 1, f);
        fwrite(sids.data() + a, 4, nb, f);
        fwrite(hc.data(), 4, nb, f);
        fwrite(hb.data(), sizeof(BestOut), hb.size(), f);
        fclose(f);
      }
    }
    if (bs_w) {
      const char *zm = getenv("MHAP_BS_ZMAX");
      BsArgs BA{c->mkeys.p, c->mpos.p, c->mbscnt.p, c->mkoff.p, c->msids.p, c->mbest.p, H, bs_w,
                c->minhash.p, zm ? atoi(zm) : 64};
      hipLaunchKernelGGL(k_mh_bitslice, dim3(nb), dim3(64), sizeof(BestOut) * H, s, BA);
      MHC(hipGetLastError());
    }
    MHC(hipEventRecord(c->ev[3], s));
    MHC(hipStreamSynchronize(s));                 // koff / sids are rewritten next batch
    float t = 0;
    (void)hipEventElapsedTime(&t, c->ev[2], c->ev[3]);
    c->stats.ms_sketch_kernel += t;
    c->stats.sketch_launches++;
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
  MHC(hipMemsetAsync(c->kctr.p, 0, 16, s));
  c->stats.ms_sketch_kernel = 0;
  c->stats.sketch_launches = 0;
  MHC(hipEventRecord(c->ev[0], s));
  // ordered sketches first: they decide which strands are used (ocount > 0)
  const int32_t min_use = std::max<int32_t>(c->P.min_olap, (int32_t)c->P.k);
  for (uint32_t a = 0; a < nr; a += 1u << 19) {
    const uint32_t n = std::min<uint32_t>(nr - a, 1u << 19);
    OrderedArgs OA{c->d_bases, c->d_off, c->d_len.p, r0 + a, 2 * n, (int32_t)c->P.ordered_k,
                   (int32_t)c->P.ordered_sketch, min_use, c->P.no_rc, c->ordered.p, c->ocount.p};
    hipLaunchKernelGGL(k_mh_ordered, dim3(2 * n), dim3(256), 0, s, OA);
    MHC(hipGetLastError());
  }
  // the MinHash sketches of the strands in use (host lengths decide the same way)
  std::vector<uint32_t> sids;
  uint64_t used = 0;
  for (uint32_t i = 0; i < nr; i++) {
    const uint32_t r = r0 + i;
    const int64_t L = c->h_len[r];
    if (L < min_use || L < (int64_t)c->P.ordered_k) continue;
    used++;
    sids.push_back(2 * r);
    if (!c->P.no_rc) sids.push_back(2 * r + 1);
  }
  int rc = sketch_minhash(c, sids);
  if (rc) return rc;
  hipLaunchKernelGGL(k_mh_strand_fixup, dim3((nr + 255) / 256), dim3(256), 0, s, c->ocount.p,
                     r0, nr);
  MHC(hipGetLastError());
  MHC(hipEventRecord(c->ev[1], s));
  unsigned long long st[2] = {0, 0};
  MHC(hipMemcpyAsync(st, c->kctr.p, 16, hipMemcpyDeviceToHost, s));
  MHC(hipStreamSynchronize(s));
  c->stats.ms_sketch = elapsed(c);
  c->stats.sketched_reads = used;
  c->stats.sketch_kmers = st[0];
  c->stats.sketch_draws = st[1];
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

static int copy_rows(mhap_ctx *c, uint32_t first, uint32_t n, void *mh, void *od, void *oc,
                     int to_ctx, bool host) {
  if (!c || !c->nreads) return mfail(M_STATE, "no reads loaded");
  if (n == 0) return M_OK;
  if (first < c->first_iid || (uint64_t)first + n > (uint64_t)c->first_iid + c->nreads)
    return mfail(M_BAD_PARAM, "rows %u..%u outside the loaded reads", first, first + n - 1);
  if (!mh || !od || !oc) return mfail(M_BAD_PARAM, "null buffer");
  MHC(hipSetDevice(c->device));
  const size_t s0 = 2ull * (first - c->first_iid), ns = 2ull * n;
  const size_t H = c->P.num_hashes, S = c->P.ordered_sketch;
  struct { void *ctx; void *user; size_t bytes; } parts[3] = {
      {c->minhash.p + s0 * H, mh, 4 * H * ns},
      {c->ordered.p + s0 * S, od, 8 * S * ns},
      {c->ocount.p + s0, oc, 4 * ns}};
  const hipMemcpyKind in = host ? hipMemcpyHostToDevice : hipMemcpyDeviceToDevice;
  const hipMemcpyKind outk = host ? hipMemcpyDeviceToHost : hipMemcpyDeviceToDevice;
  for (auto &pt : parts) {
    if (to_ctx) MHC(hipMemcpyAsync(pt.ctx, pt.user, pt.bytes, in, c->stream));
    else        MHC(hipMemcpyAsync(pt.user, pt.ctx, pt.bytes, outk, c->stream));
  }
  MHC(hipStreamSynchronize(c->stream));
  if (to_ctx) c->indexed = false;
  return M_OK;
}

int mhap_copy_sketches(mhap_ctx *c, uint32_t first, uint32_t n, void *d_minhash,
                       void *d_ordered, void *d_ocount, int to_ctx) {
  return copy_rows(c, first, n, d_minhash, d_ordered, d_ocount, to_ctx, false);
}

int mhap_copy_sketches_host(mhap_ctx *c, uint32_t first, uint32_t n, void *h_minhash,
                            void *h_ordered, void *h_ocount, int to_ctx) {
  return copy_rows(c, first, n, h_minhash, h_ordered, h_ocount, to_ctx, true);
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
  const uint32_t s0 = 2 * (bgn - c->first_iid), ns = 2 * (end - bgn + 1);
  const size_t n = (size_t)ns * H;
  if (n >= 0x7FFFFFFFull) return mfail(M_BAD_PARAM, "index of %zu entries too large", n);
  if (c->keys.alloc(n) || c->vals.alloc(n) || c->keys2.alloc(n) || c->vals2.alloc(n) ||
      c->toff.alloc(H + 1))
    return mfail(M_OOM, "index (%zu entries)", n);
  MHC(hipEventRecord(c->ev[0], s));
  hipLaunchKernelGGL(k_mh_index_keys, dim3(4096), dim3(256), 0, s, c->minhash.p, c->ocount.p,
                     s0, ns, H, c->keys.p, c->vals.p);
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

static int compare_impl(mhap_ctx *c, uint32_t bgn, uint32_t end, uint32_t self,
                        uint64_t *n_out) {
  if (!c || !c->indexed) return mfail(M_STATE, "mhap_build_index() first");
  if (bgn < c->first_iid || end >= c->first_iid + c->nreads || bgn > end)
    return mfail(M_BAD_PARAM, "query range %u-%u outside the loaded reads", bgn, end);
  MHC(hipSetDevice(c->device));
  hipStream_t s = c->stream;
  const uint32_t q0 = bgn - c->first_iid, q1 = end - c->first_iid + 1;
  const uint32_t nq = q1 - q0;
  // first stage (grow the candidate buffer and redo on overflow)
  size_t cap = std::max<size_t>((size_t)nq * 64, 1u << 16);
  uint32_t h[4];
  float ms_cand = 0;
  for (;;) {
    if (cap > 0xFFFFFFF0ull) return mfail(M_OOM, "candidate list too large");
    if (c->cand.alloc(cap)) return mfail(M_OOM, "candidates");
    MHC(hipMemsetAsync(c->ctr.p, 0, 64, s));
    CandArgs CA{c->minhash.p, c->ocount.p, c->d_len.p, c->keys2.p, c->vals2.p, c->toff.p,
                (int32_t)c->P.num_hashes, q0, q1, self, c->P.min_store, c->P.min_matches,
                c->cand.p, c->ctr.p, (uint32_t)cap, c->ctr.p + 1};
    MHC(hipEventRecord(c->ev[0], s));
    hipLaunchKernelGGL(k_mh_candidates, dim3((nq + 3) / 4), dim3(256),
                       2 * 4 * TSLOTS * sizeof(uint32_t), s, CA);
    MHC(hipGetLastError());
    MHC(hipEventRecord(c->ev[1], s));
    MHC(hipMemcpyAsync(h, c->ctr.p, 16, hipMemcpyDeviceToHost, s));
    MHC(hipStreamSynchronize(s));
    ms_cand += elapsed(c);
    if (h[1] & 1u) return mfail(M_BAD_INPUT, "a query has more than %d candidate strands", TSLOTS);
    if (h[1] & 2u) { cap = (size_t)h[0] + (h[0] >> 2) + 1024; continue; }
    break;
  }
  const uint32_t ncand = h[0];
  // second stage
  const size_t rcap = std::max<size_t>(ncand, 1024);
  if (c->rec.alloc(rcap)) return mfail(M_OOM, "records");
  MHC(hipMemsetAsync(c->ctr.p + 4, 0, 16, s));
  const int32_t S = (int32_t)c->P.ordered_sketch;
  CmpArgs MA{c->cand.p, ncand, c->ordered.p, c->ocount.p, c->d_len.p, S,
             (int32_t)c->P.ordered_k, c->P.max_shift, c->pass.p, c->pass_empty, c->rec.p,
             c->ctr.p + 4, (uint32_t)rcap, c->ctr.p + 5};
  const size_t lds = 3 * 8 * (size_t)S + 1024;
  MHC(hipEventRecord(c->ev[0], s));
  if (ncand) {
    const uint32_t blocks = std::min<uint32_t>(ncand, 256u * 64u);
    hipLaunchKernelGGL(k_mh_compare, dim3(blocks), dim3(64), lds, s, MA);
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

int mhap_compare(mhap_ctx *c, uint32_t bgn, uint32_t end, uint64_t *n_out) {
  return compare_impl(c, bgn, end, 1, n_out);
}

int mhap_compare_all(mhap_ctx *c, uint32_t bgn, uint32_t end, uint64_t *n_out) {
  return compare_impl(c, bgn, end, 0, n_out);
}

int mhap_fetch(mhap_ctx *c, mhap_record *out, uint64_t max_records, uint64_t *n_copied) {
  if (!c) return mfail(M_STATE, "null context");
  MHC(hipSetDevice(c->device));
  std::vector<RecDev> h(c->nrec);
  if (c->nrec) MHC(hipMemcpy(h.data(), c->rec.p, sizeof(RecDev) * c->nrec, hipMemcpyDeviceToHost));
  std::sort(h.begin(), h.end(), [](const RecDev &x, const RecDev &y) {
    return x.a != y.a ? x.a < y.a : x.b != y.b ? x.b < y.b : x.o < y.o;
  });
  const uint64_t n = std::min<uint64_t>(max_records, h.size());
  for (uint64_t i = 0; i < n; i++) {
    const RecDev &r = h[i];
    const double score = jaccard_identity(jaccard_of(r.inter, r.n), (int)c->P.ordered_k);
    out[i] = mhap_record{c->first_iid + r.a, c->first_iid + r.b, 1.0 - std::min(score, 1.0),
                         (double)r.raw, r.a1, r.a2, r.a_len, r.o, r.b1, r.b2, r.b_len, r.cnt};
  }
  *n_copied = n;
  return M_OK;
}

// Java's String.format("%.6f", x): the shortest decimal that reads back as x
// (FloatingDecimal), rounded half-up to 6 places (FormattedFloatingDecimal.applyPrecision)
static std::string java_fixed6(double x) {
  char buf[64];
  auto res = std::to_chars(buf, buf + sizeof buf, x, std::chars_format::scientific);
  *res.ptr = 0;
  // d.ddddde[+-]xx -> digits, exponent
  std::string mant(buf, strchr(buf, 'e'));
  const int ex = atoi(strchr(buf, 'e') + 1);
  bool neg = false;
  if (!mant.empty() && mant[0] == '-') { neg = true; mant.erase(0, 1); }
  std::string dig;
  for (char ch : mant)
    if (ch != '.') dig += ch;
  // value = 0.dig * 10^(ex + 1); keep integer part + 6 decimals
  const int ip = ex + 1;                         // digits before the point
  std::string intpart, frac;
  if (ip <= 0) {
    intpart = "0";
    frac = std::string(-ip, '0') + dig;
  } else {
    if ((int)dig.size() < ip) dig += std::string(ip - dig.size(), '0');
    intpart = dig.substr(0, ip);
    frac = dig.substr(ip);
  }
  if (frac.size() < 7) frac += std::string(7 - frac.size(), '0');
  const bool up = frac[6] >= '5';
  std::string num = intpart + frac.substr(0, 6);
  if (up) {
    int i = (int)num.size() - 1;
    while (i >= 0 && num[i] == '9') num[i--] = '0';
    if (i >= 0) num[i]++;
    else num.insert(num.begin(), '1');
  }
  std::string s = num.substr(0, num.size() - 6) + "." + num.substr(num.size() - 6);
  return neg ? "-" + s : s;
}

int mhap_format_line(const mhap_record *x, uint32_t hash_base, uint32_t num_hash,
                     uint32_t query_base, char *buf, size_t cap) {
  if (!x || !buf) return mfail(M_BAD_PARAM, "null argument");
  if (hash_base == 0 || query_base == 0) return mfail(M_BAD_PARAM, "bases are 1-based IDs");
  // mhapConvert.C:122-123: a_iid = W0 + (query_base - 1) - num_hash, b_iid = W1 + hash_base - 1
  const uint64_t w0 = (uint64_t)x->a_iid - (query_base - 1) + num_hash;
  const uint64_t w1 = (uint64_t)x->b_iid - (hash_base - 1);
  const int n = snprintf(buf, cap, "%llu %llu %s %s 0 %d %d %d %u %d %d %d",
                         (unsigned long long)w0, (unsigned long long)w1,
                         java_fixed6(x->erate).c_str(), java_fixed6(x->raw).c_str(), x->a_bgn,
                         x->a_end, x->a_len, x->b_rc, x->b_bgn, x->b_end, x->b_len);
  if (n < 0 || (size_t)n >= cap) return mfail(M_BAD_PARAM, "line buffer too small");
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
  char line[256];
  for (uint64_t i = 0; i < n; i++) {
    rc = mhap_format_line(&r[i], hash_base, num_hash, query_base, line, sizeof line);
    if (rc) { fclose(F); return rc; }
    fputs(line, F);
    fputc('\n', F);
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
