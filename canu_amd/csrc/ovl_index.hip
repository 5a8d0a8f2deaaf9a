// ovl_index.hip -- read packing and the k-mer index (Build_Hash_Index replacement).
//
// Reference: src/overlapInCore/overlapInCore-Build_Hash_Index.C
//   Put_String_In_Hash (:360)  every window of k ACGT bases is an occurrence
//   Hash_Insert        (:296)  occurrences of one k-mer are chained newest-first
//   Mark_Skip_Kmers    (:235)  -k file k-mers become Empty entries; their occurrences
//                              mark the reads' screened ends (Mark_Screened_Ends_Single)
//
// MI355X design: instead of a CPU bucket table filled one insert at a time, the index is a
// two-level bucket sort of (mix(kmer), position) records:
//   coarse pass  : 4096 buckets by the top 12 bits of mix(kmer); per-block LDS histograms,
//                  one global atomic per (block, bucket) to claim space
//   fine pass    : one workgroup per coarse bucket splits it into 2^FB fine buckets in LDS,
//                  then each wave sorts one fine bucket in LDS (bitonic, by mix asc /
//                  position desc = the reference's chain order)
//   table pass   : each wave turns one sorted fine bucket into one slice of an open-
//                  addressing table (16-B entries, the slice is the fine bucket's own range
//                  of the table, so no two workgroups ever touch the same slots)
// The occurrence array is the sorted position array itself.
#include "ovl_common.h"

namespace ovl {

// ---------------------------------------------------------------------------------------
// Packing: ASCII reads -> 2-bit strands + exception masks.  One block per read.
// Accepts acgtn / ACGTN; anything else sets *err (the GPU path cannot represent it).
__device__ __forceinline__ int base_code(uint8_t c, int *is_n, int *bad) {
  switch (c | 0x20) {
    case 'a': return 0;
    case 'c': return 1;
    case 'g': return 2;
    case 't': return 3;
    case 'n': *is_n = 1; return 0;
    default:  *bad = 1; return 0;
  }
}

__global__ void k_pack(const uint8_t *__restrict__ bases, const uint64_t *__restrict__ offs,
                       const uint32_t *__restrict__ lens, const uint64_t *__restrict__ wofs,
                       uint64_t *fwd, uint64_t *rc, uint32_t *fwdN, uint32_t *rcNul,
                       uint32_t *flags, uint32_t *rcFirstNul, uint32_t *err, uint32_t k) {
  uint32_t r = blockIdx.x;
  uint32_t L = lens[r];
  uint64_t o = offs[r], w0 = wofs[r];
  uint32_t nw = (L + 31) / 32 + 1;        // + guard word
  __shared__ int s_hasn;
  __shared__ int s_lastn;
  if (threadIdx.x == 0) { s_hasn = 0; s_lastn = -1; }
  __syncthreads();
  int bad = 0, anyn = 0, lastn = -1;
  for (uint32_t w = threadIdx.x; w < nw; w += blockDim.x) {
    uint64_t f = 0, c = 0;
    uint32_t fn = 0, cn = 0;
    for (uint32_t i = 0; i < 32; i++) {
      uint32_t p = w * 32 + i;
      if (p < L) {
        int isn = 0;
        int code = base_code(bases[o + p], &isn, &bad);
        f |= (uint64_t)code << (2 * i);
        if (isn) {
          fn |= 1u << i;
          anyn = 1;
          // only NULs at rc positions >= k can end the window scan (see below)
          if (p + k <= L - 1 && (int)p > lastn) lastn = (int)p;
        }
      }
      // rc base at position p comes from fwd base L-1-p
      if (p < L) {
        int isn2 = 0;
        int code2 = base_code(bases[o + (L - 1 - p)], &isn2, &bad);
        if (isn2) cn |= 1u << i;          // complement of 'n' is NUL
        else      c |= (uint64_t)(3 - code2) << (2 * i);
      }
    }
    fwd[w0 + w] = f;
    rc[w0 + w] = c;
    fwdN[w0 + w] = fn;
    rcNul[w0 + w] = cn;
  }
  if (bad) atomicOr(err, 1u);
  if (anyn) atomicOr(&s_hasn, 1);
  if (lastn >= 0) atomicMax(&s_lastn, lastn);
  __syncthreads();
  if (threadIdx.x == 0) {
    flags[r] = s_hasn ? 1u : 0u;
    // Find_Overlaps.C:341 tests `*P` only for the last base of windows 1, 2, ..., so a
    // NUL ends the scan only from rc position k on: the first such NUL is the rc image of
    // the last forward 'n' at or before L-1-k.
    rcFirstNul[r] = (s_lastn >= 0) ? (L - 1 - (uint32_t)s_lastn) : L;
  }
}

// ---------------------------------------------------------------------------------------
// Index build

struct BuildArgs {
  ReadsDev R;
  uint32_t h0, h1;           // local read range [h0, h1) of hash reads
  uint32_t reads_per_block;
  uint32_t k;
  int32_t  min_len;          // G.Min_Olap_Len: shorter reads are not hashed
  uint64_t kmask;
  const uint64_t *skip;      // skip k-mers (both strands), may be null
  uint32_t n_skip;
  uint32_t cb_bits;          // coarse bucket bits
  uint32_t fb_bits;          // fine bucket bits
};

#define OVL_CB_MAX 4096
#ifndef OVL_COARSE_SWEEPS
#define OVL_COARSE_SWEEPS 4      // bucket windows the coarse scatter stores in turn (1: 29.1, 4: 28.8, 8: 32.5 ms index, r06z)
#endif
#define OVL_SKIP_POS 0xFFFFFFFFFFFFFFFFull

template <typename F>
__device__ __forceinline__ void for_block_windows(const BuildArgs &A, F &&fn) {
  uint32_t rb = A.h0 + blockIdx.x * A.reads_per_block;
  uint32_t re = rb + A.reads_per_block;
  if (re > A.h1) re = A.h1;
  for (uint32_t r = rb; r < re; r++) {
    int32_t L = (int32_t)A.R.len[r];
    // shorter than --minlength, or outside the -H libraries (Build_Hash_Index.C:554-561)
    if (L < A.min_len || L < (int32_t)A.k || (A.R.flags[r] & OVL_RFLAG_NOHASH)) continue;
    uint64_t wo = A.R.wofs[r];
    const uint64_t *w = A.R.fwd + wo;
    const uint32_t *nm = (A.R.flags[r] & 1u) ? A.R.fwdN + wo : nullptr;
    uint64_t iid = A.R.first_iid + r;
    uint32_t kbits = (1u << A.k) - 1u;   // k <= 31
    for (int32_t p = threadIdx.x; p + (int32_t)A.k <= L; p += blockDim.x) {
      if (nm && (mask_at(nm, p) & kbits)) continue;          // key_is_bad
      uint64_t kmer = bases_at(w, p) & A.kmask;
      fn(kmer, (iid << 32) | (uint32_t)p);
    }
  }
  // skip k-mers ride along as marker records, spread over the blocks
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < A.n_skip;
       i += gridDim.x * blockDim.x)
    fn(A.skip[i], OVL_SKIP_POS);
}

__global__ void k_coarse_hist(BuildArgs A, uint32_t *hist) {
  __shared__ uint32_t h[OVL_CB_MAX];
  uint32_t nb = 1u << A.cb_bits;
  for (uint32_t i = threadIdx.x; i < nb; i += blockDim.x) h[i] = 0;
  __syncthreads();
  for_block_windows(A, [&](uint64_t kmer, uint64_t) {
    atomicAdd(&h[mix64(kmer) >> (64 - A.cb_bits)], 1u);
  });
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < nb; i += blockDim.x)
    if (h[i]) atomicAdd(&hist[i], h[i]);
}

// A (mix(kmer), position) record as one 16-B store: the scatter passes write whole
// records, half the transactions of two 8-B arrays.
struct __attribute__((aligned(16))) Rec2 {
  uint64_t m, p;
};

__global__ void k_coarse_scatter(BuildArgs A, uint32_t *cursor, Rec2 *outR) {
  __shared__ uint32_t h[OVL_CB_MAX];
  __shared__ uint32_t base[OVL_CB_MAX];
  uint32_t nb = 1u << A.cb_bits;
  for (uint32_t i = threadIdx.x; i < nb; i += blockDim.x) h[i] = 0;
  __syncthreads();
  for_block_windows(A, [&](uint64_t kmer, uint64_t) {
    atomicAdd(&h[mix64(kmer) >> (64 - A.cb_bits)], 1u);
  });
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < nb; i += blockDim.x) {
    base[i] = h[i] ? atomicAdd(&cursor[i], h[i]) : 0u;
    h[i] = 0;
  }
  __syncthreads();
  // Sweeps: the block's windows are re-read once per window of nb / OVL_COARSE_SWEEPS
  // buckets and only that window's records are stored, so a block has that many write streams
  // open at a time instead of all nb (with every bucket open, the resident blocks' half-written
  // lines overflow the L2 and leave it partially written: 2x the record bytes in PMC writes).
  // The re-reads hit the block's packed reads in the L2; a bucket's order is the fine pass's.
  constexpr uint32_t NS = OVL_COARSE_SWEEPS;
  for (uint32_t sw = 0; sw < NS; sw++) {
    const uint32_t lo = (nb * sw) / NS, span = (nb * (sw + 1)) / NS - lo;
    for_block_windows(A, [&](uint64_t kmer, uint64_t pos) {
      uint64_t M = mix64(kmer);
      uint32_t b = (uint32_t)(M >> (64 - A.cb_bits));
      if (NS > 1 && b - lo >= span) return;
      uint32_t slot = base[b] + atomicAdd(&h[b], 1u);
      Rec2 r;
      r.m = M;
      r.p = pos;
      outR[slot] = r;
    });
    if (NS > 1) __syncthreads();
  }
}

// Sort order: M ascending, then position descending (chain order).
__device__ __forceinline__ bool rec_less(uint64_t m1, uint64_t p1, uint64_t m2, uint64_t p2) {
  return (m1 < m2) || (m1 == m2 && p1 > p2);
}

// Wave-level bitonic sort of n2 (power of 2) records in LDS.
__device__ void wave_bitonic(uint64_t *sM, uint64_t *sP, uint32_t n2, uint32_t lane) {
  for (uint32_t size = 2; size <= n2; size <<= 1) {
    for (uint32_t stride = size >> 1; stride > 0; stride >>= 1) {
      for (uint32_t t = lane; t < n2 / 2; t += OVL_WAVE) {
        uint32_t i = 2 * t - (t & (stride - 1));
        uint32_t j = i + stride;
        bool up = ((i & size) == 0);
        uint64_t mi = sM[i], pi = sP[i], mj = sM[j], pj = sP[j];
        bool sw = up ? rec_less(mj, pj, mi, pi) : rec_less(mi, pi, mj, pj);
        if (sw) { sM[i] = mj; sP[i] = pj; sM[j] = mi; sP[j] = pi; }
      }
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    }
  }
}

// Wave-level grouping of one fine bucket (fn <= H records, H a power of two >= 64):
// every k-mer's records become one contiguous run in position-descending order -- the order
// Hash_Insert chains them (Build_Hash_Index.C:296-341) -- with the runs in the slot order of
// an LDS hash table over the bucket's keys.  The index only needs each k-mer's run
// contiguous and ordered (k_table maps a key to its run, k_first_reads reads a run's last
// record), not the runs ordered by key, so this replaces a comparison sort of the bucket
// (28-36 compare-exchange stages of LDS traffic) with one insert per record, a scan over the
// slots and a rank within the record's own run.  Returns the number of distinct keys.
//   kT: H u64 keys, cT: H u32 counts -> run starts, sP: H u64 staged positions.
template <int EM>
__device__ uint32_t wave_group_runs(const Rec2 *__restrict__ in, uint64_t *__restrict__ outM,
                                    uint64_t *__restrict__ outP, uint32_t fn, uint32_t H,
                                    uint64_t *kT, uint32_t *cT, uint64_t *sP, uint64_t empty,
                                    uint32_t lane) {
  for (uint32_t i = lane; i < H; i += 64) { kT[i] = empty; cT[i] = 0; }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  uint64_t m[EM], p[EM];
  uint32_t sa[EM];                               // slot | arrival << 16
#pragma unroll
  for (int e = 0; e < EM; e++) {
    const uint32_t i = lane + 64u * e;
    m[e] = empty;
    p[e] = 0;
    if (i < fn) { const Rec2 r = in[i]; m[e] = r.m; p[e] = r.p; }
  }
#pragma unroll
  for (int e = 0; e < EM; e++) {
    sa[e] = 0;
    if (lane + 64u * e < fn) {
      uint32_t s = (uint32_t)m[e] & (H - 1);     // low bits of the mix: the bucket fixes the top
      for (;;) {
        const unsigned long long old =
            atomicCAS((unsigned long long *)&kT[s], (unsigned long long)empty,
                      (unsigned long long)m[e]);
        if (old == empty || old == m[e]) break;
        s = (s + 1) & (H - 1);
      }
      sa[e] = s | (atomicAdd(&cT[s], 1u) << 16);
    }
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  // run starts: exclusive scan of the counts in slot order (each lane H/64 slots)
  const uint32_t per = H >> 6, b0 = lane * per;
  uint32_t run = 0, distinct = 0;
  for (uint32_t j = 0; j < per; j++) {
    const uint32_t c = cT[b0 + j];
    run += c;
    distinct += c ? 1u : 0u;
  }
  uint32_t inc = run;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t v = __shfl_up(inc, o);
    if (lane >= (uint32_t)o) inc += v;
  }
  uint32_t acc = inc - run;
  for (uint32_t j = 0; j < per; j++) {
    const uint32_t c = cT[b0 + j];
    cT[b0 + j] = acc;
    acc += c;
  }
  for (int o = 32; o > 0; o >>= 1) distinct += __shfl_xor(distinct, o);
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
#pragma unroll
  for (int e = 0; e < EM; e++)
    if (lane + 64u * e < fn) sP[cT[sa[e] & 0xffffu] + (sa[e] >> 16)] = p[e];
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  // rank within the run: positions descending; equal positions (repeated skip markers) by
  // arrival
#pragma unroll
  for (int e = 0; e < EM; e++) {
    if (lane + 64u * e < fn) {
      const uint32_t s = sa[e] & 0xffffu, a = sa[e] >> 16;
      const uint32_t b = cT[s], end = (s + 1 < H) ? cT[s + 1] : fn;
      uint32_t rank = 0;
      for (uint32_t j = b; j < end; j++) {
        const uint64_t q = sP[j];
        rank += (q > p[e] || (q == p[e] && j - b < a)) ? 1u : 0u;
      }
      outM[b + rank] = m[e];
      outP[b + rank] = p[e];
    }
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  return distinct;
}

#define OVL_FINE_WAVES  8
#ifndef OVL_FINE_PHASE
#define OVL_FINE_PHASE  0        // 1 / 2: stop after the histogram / the split (timing only)
#endif
#define OVL_FB_MAX      4096
#ifndef OVL_FINE_PSCAN
#define OVL_FINE_PSCAN  1
#endif

struct FineArgs {
  const Rec2 *inR;               // coarse-bucketed records
  Rec2 *midR;                    // fine-bucketed (unsorted) records
  uint64_t *outM, *outP;         // fine-bucketed, sorted records (big buckets: unsorted)
  const uint32_t *cstart;        // coarse bucket start (exclusive scan of hist)
  const uint32_t *ccnt;          // coarse bucket counts
  uint32_t *fstart, *fcnt;       // fine bucket start / count (global index)
  uint32_t *big_list, *big_n;    // fine buckets too large for LDS
  uint32_t *max_distinct;
  uint32_t cb_bits, fb_bits;
  uint32_t cap;                  // records a wave sorts in LDS (power of 2); larger fine
                                 // buckets go to k_fine_big
};

// LDS of k_fine: the fine split's bins (h, cur: nf u32 each) and, after it, the waves' sort
// buffers.  Grouped runs (GROUP): per wave [kT: cap u64][sP: cap u64][cT: cap u32], overlaid
// on the bins (the sort phase takes its buckets' bounds from fstart / fcnt); bitonic:
// [sM: 8 x cap u64][sP: 8 x cap u64] then the bins.
#ifndef OVL_SPLIT_TILE
#define OVL_SPLIT_TILE 2048      // records per LDS-staged tile of the fine split (0: direct)
#endif
__host__ __device__ inline size_t fine_lds_bytes(bool group, uint32_t nf, uint32_t cap) {
  if (group) {
    // bins: h, cur (+ the tiled split's tile counts and starts and its staged records)
    const size_t sort = (size_t)OVL_FINE_WAVES * cap * 20,
                 bins = OVL_SPLIT_TILE ? (size_t)nf * 16 + (size_t)OVL_SPLIT_TILE * 16
                                       : (size_t)nf * 8;
    return sort > bins ? sort : bins;
  }
  return 2ull * OVL_FINE_WAVES * cap * 8 + 2ull * nf * 4;
}

// Exclusive scan of nf <= 4096 LDS bins by a block of OVL_FINE_WAVES waves: each thread a
// run of nf/512 bins, a wave scan of the runs, then the wave totals (a one-thread serial
// scan of 4096 bins is a chain of dependent LDS round trips, ~0.1 ms per block).  Ends with
// a barrier.
__device__ __forceinline__ void block_scan_bins(const uint32_t *h, uint32_t *out, uint32_t nf,
                                                uint32_t *s_wsum) {
  const uint32_t per = (nf + blockDim.x - 1) / blockDim.x;
  const uint32_t b0 = threadIdx.x * per;
  uint32_t run = 0;
  for (uint32_t f = b0; f < b0 + per && f < nf; f++) run += h[f];
  uint32_t inc = run;
  const uint32_t ln = threadIdx.x & 63;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t v = __shfl_up(inc, o);
    if (ln >= (uint32_t)o) inc += v;
  }
  if (ln == 63) s_wsum[threadIdx.x >> 6] = inc;
  __syncthreads();
  uint32_t acc = inc - run;
  for (uint32_t w = 0; w < (threadIdx.x >> 6); w++) acc += s_wsum[w];
  for (uint32_t f = b0; f < b0 + per && f < nf; f++) { out[f] = acc; acc += h[f]; }
  __syncthreads();
}

template <int EM, bool GROUP>
__global__ void __launch_bounds__(OVL_FINE_WAVES * 64)
k_fine(FineArgs A) {
  // dynamic LDS sized to the fine buckets (2^fb bins, cap records per wave) so that
  // several blocks share a CU (fine_lds_bytes)
  extern __shared__ __attribute__((aligned(16))) uint64_t s_fine[];
  uint32_t nf = 1u << A.fb_bits;
  const uint32_t cap = A.cap;
  uint32_t *h = GROUP ? (uint32_t *)s_fine : (uint32_t *)(s_fine + 2 * OVL_FINE_WAVES * cap);
  uint32_t *cur = h + nf;
  uint32_t cb = blockIdx.x;
  uint32_t n = A.ccnt[cb], s0 = A.cstart[cb];
  uint32_t shift = 64 - A.cb_bits - A.fb_bits;
  for (uint32_t i = threadIdx.x; i < nf; i += blockDim.x) h[i] = 0;
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < n; i += blockDim.x)
    atomicAdd(&h[(uint32_t)(A.inR[s0 + i].m >> shift) & (nf - 1)], 1u);
  __syncthreads();
  __shared__ uint32_t s_wsum[OVL_FINE_WAVES];
#if OVL_FINE_PSCAN
  block_scan_bins(h, cur, nf, s_wsum);
#else
  if (threadIdx.x == 0) {                        // nf <= 4096: serial scan is cheap
    uint32_t acc = 0;
    for (uint32_t f = 0; f < nf; f++) { cur[f] = acc; acc += h[f]; }
  }
#endif
  __syncthreads();
#if OVL_FINE_PHASE == 1                          // timing experiment: histogram + scan only
  for (uint32_t f = threadIdx.x; f < nf; f += blockDim.x) {   // empty buckets for k_table
    A.fstart[cb * nf + f] = s0;
    A.fcnt[cb * nf + f] = 0;
  }
  return;
#endif
  for (uint32_t f = threadIdx.x; f < nf; f += blockDim.x) {
    A.fstart[cb * nf + f] = s0 + cur[f];
    A.fcnt[cb * nf + f] = h[f];
  }
  __syncthreads();
  if (GROUP && OVL_SPLIT_TILE) {
    // The split through LDS, a tile of records at a time: each tile is ordered by fine
    // bucket in LDS (tile counts, their scan, a rank from the count's atomic), then written
    // out with consecutive threads on consecutive slots of a bucket -- runs instead of one
    // scattered 16-B store per record, whose half-written lines (1,024 open buckets per
    // block, three blocks per CU) cost the direct split 8.3 of k_fine's 14.8 ms at 50k x
    // 10 kb.  A fine bucket's order does not matter: the grouping below orders it.
    constexpr uint32_t T = OVL_SPLIT_TILE > 0 ? OVL_SPLIT_TILE : 512;
    constexpr uint32_t RPT = T / (OVL_FINE_WAVES * 64);
    static_assert(RPT * OVL_FINE_WAVES * 64 == T, "tile = whole rounds of the block");
    uint32_t *tcnt = cur + nf, *tstart = tcnt + nf;
    Rec2 *stage = (Rec2 *)(tstart + nf);
    for (uint32_t t0 = 0; t0 < n; t0 += T) {
      for (uint32_t f = threadIdx.x; f < nf; f += blockDim.x) tcnt[f] = 0;
      __syncthreads();
      Rec2 r[RPT];
      uint32_t fb[RPT], rk[RPT];
#pragma unroll
      for (uint32_t q = 0; q < RPT; q++) {
        const uint32_t i = t0 + q * blockDim.x + threadIdx.x;
        fb[q] = 0xFFFFFFFFu;
        if (i < n) {
          r[q] = A.inR[s0 + i];
          fb[q] = (uint32_t)(r[q].m >> shift) & (nf - 1);
        }
      }
#pragma unroll
      for (uint32_t q = 0; q < RPT; q++)
        if (fb[q] != 0xFFFFFFFFu) rk[q] = atomicAdd(&tcnt[fb[q]], 1u);
      __syncthreads();
      block_scan_bins(tcnt, tstart, nf, s_wsum);
#pragma unroll
      for (uint32_t q = 0; q < RPT; q++)
        if (fb[q] != 0xFFFFFFFFu) stage[tstart[fb[q]] + rk[q]] = r[q];
      __syncthreads();
      const uint32_t tn = n - t0 < T ? n - t0 : T;
      for (uint32_t j = threadIdx.x; j < tn; j += blockDim.x) {
        const Rec2 x = stage[j];
        const uint32_t f = (uint32_t)(x.m >> shift) & (nf - 1);
        A.midR[s0 + cur[f] + (j - tstart[f])] = x;
      }
      __syncthreads();
      for (uint32_t f = threadIdx.x; f < nf; f += blockDim.x) cur[f] += tcnt[f];
      __syncthreads();
    }
  } else {
    for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) {
      const Rec2 r = A.inR[s0 + i];
      uint32_t f = (uint32_t)(r.m >> shift) & (nf - 1);
      uint32_t slot = atomicAdd(&cur[f], 1u);
      A.midR[s0 + slot] = r;
    }
  }
  __threadfence_block();
  __syncthreads();
#if OVL_FINE_PHASE == 2                          // timing experiment: + the fine split
  for (uint32_t f = threadIdx.x; f < nf; f += blockDim.x) A.fcnt[cb * nf + f] = 0;
  return;
#endif

  uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  uint64_t *kT = s_fine + (size_t)wave * (2 * cap + cap / 2);
  uint64_t *sPw = kT + cap;
  uint32_t *cT = (uint32_t *)(sPw + cap);
  // no stored key has the bucket's top bits flipped
  const uint64_t empty = ~(((uint64_t)cb) << (64 - A.cb_bits)) & (~0ull << (64 - A.cb_bits));
  uint64_t *wM = s_fine + (size_t)wave * cap, *wP = s_fine + (size_t)(OVL_FINE_WAVES + wave) * cap;
  __shared__ uint32_t s_runmax;                  // distinct k-mers of the block's largest bucket
  if (threadIdx.x == 0) s_runmax = 0;
  __syncthreads();
  uint32_t wave_max_runs = 0;
  for (uint32_t f = wave; f < nf; f += OVL_FINE_WAVES) {
    // grouped: the bins are overwritten by the sort buffers, bounds from the global copies;
    // bitonic: cur[] now holds the fine bucket end
    const uint32_t fn = GROUP ? __builtin_amdgcn_readfirstlane(A.fcnt[cb * nf + f]) : h[f];
    if (fn == 0) continue;
    const uint32_t fs = GROUP ? __builtin_amdgcn_readfirstlane(A.fstart[cb * nf + f])
                              : s0 + cur[f] - fn;
    if (fn > cap) {
      // too large for the LDS sort: copy out unsorted, k_fine_big sorts it in place
      for (uint32_t i = lane; i < fn; i += 64) {
        const Rec2 r = A.midR[fs + i];
        A.outM[fs + i] = r.m;
        A.outP[fs + i] = r.p;
      }
      if (lane == 0) {
        uint32_t j = atomicAdd(A.big_n, 1u);
        A.big_list[2 * j] = fs;
        A.big_list[2 * j + 1] = fn;
      }
      continue;
    }
    if constexpr (GROUP) {
      uint32_t H = 64;
      while (H < 2 * fn && H < cap) H <<= 1;
      const uint32_t runs = wave_group_runs<EM>(A.midR + fs, A.outM + fs, A.outP + fs, fn, H,
                                                kT, cT, sPw, empty, lane);
      wave_max_runs = runs > wave_max_runs ? runs : wave_max_runs;
      continue;
    }
    uint32_t n2 = 1;
    while (n2 < fn) n2 <<= 1;
    for (uint32_t i = lane; i < n2; i += 64) {
      if (i < fn) { const Rec2 r = A.midR[fs + i]; wM[i] = r.m; wP[i] = r.p; }
      else        { wM[i] = ~0ull;          wP[i] = 0; }
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    if (fn > 1) wave_bitonic(wM, wP, n2, lane);
    uint32_t runs = 0;
    for (uint32_t i = lane; i < fn; i += 64) {
      A.outM[fs + i] = wM[i];
      A.outP[fs + i] = wP[i];
      runs += (i == 0 || wM[i] != wM[i - 1]) ? 1u : 0u;
    }
    for (int o = 32; o > 0; o >>= 1) runs += __shfl_xor(runs, o);
    wave_max_runs = runs > wave_max_runs ? runs : wave_max_runs;
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  }
  // one global atomic per block: a per-bucket atomic on the single max_distinct word
  // serialises thousands of blocks in the L2
  if (lane == 0) atomicMax(&s_runmax, wave_max_runs);
  __syncthreads();
  if (threadIdx.x == 0 && s_runmax) atomicMax(A.max_distinct, s_runmax);
}

// Fine buckets larger than the LDS sort: one workgroup each, bitonic in global memory over
// a power-of-two scratch copy.
__global__ void k_fine_big(uint64_t *M, uint64_t *P, const uint32_t *big_list,
                           uint64_t *scrM, uint64_t *scrP, uint32_t n2, uint32_t *max_distinct) {
  uint32_t fs = big_list[2 * blockIdx.x], fn = big_list[2 * blockIdx.x + 1];
  uint64_t *gM = scrM + (uint64_t)blockIdx.x * n2, *gP = scrP + (uint64_t)blockIdx.x * n2;
  uint32_t m2 = 1;
  while (m2 < fn) m2 <<= 1;
  for (uint32_t i = threadIdx.x; i < m2; i += blockDim.x) {
    if (i < fn) { gM[i] = M[fs + i]; gP[i] = P[fs + i]; }
    else        { gM[i] = ~0ull;     gP[i] = 0; }
  }
  __threadfence_block();
  __syncthreads();
  for (uint32_t size = 2; size <= m2; size <<= 1) {
    for (uint32_t stride = size >> 1; stride > 0; stride >>= 1) {
      for (uint32_t t = threadIdx.x; t < m2 / 2; t += blockDim.x) {
        uint32_t i = 2 * t - (t & (stride - 1));
        uint32_t j = i + stride;
        bool up = ((i & size) == 0);
        uint64_t mi = gM[i], pi = gP[i], mj = gM[j], pj = gP[j];
        bool sw = up ? rec_less(mj, pj, mi, pi) : rec_less(mi, pi, mj, pj);
        if (sw) { gM[i] = mj; gP[i] = pj; gM[j] = mi; gP[j] = pi; }
      }
      __threadfence_block();
      __syncthreads();
    }
  }
  __shared__ uint32_t s_runs;
  if (threadIdx.x == 0) s_runs = 0;
  __syncthreads();
  uint32_t runs = 0;
  for (uint32_t i = threadIdx.x; i < fn; i += blockDim.x) {
    M[fs + i] = gM[i];
    P[fs + i] = gP[i];
    runs += (i == 0 || gM[i] != gM[i - 1]) ? 1u : 0u;
  }
  atomicAdd(&s_runs, runs);
  __syncthreads();
  if (threadIdx.x == 0) atomicMax(max_distinct, s_runs);
}

struct TableArgs {
  const uint64_t *M, *P;         // sorted records
  const uint32_t *fstart, *fcnt;
  TabEntry *tab;
  uint32_t nfine;                // total fine buckets (2^(cb+fb))
  uint32_t slice_bits;
  uint32_t tab_bits;
  // screened-end marking for skip k-mers (Mark_Screened_Ends_Single, :147)
  const uint32_t *len;
  uint32_t *rflags;              // bit1 lfrag_end_screened, bit2 rfrag_end_screened
  uint32_t first_iid;
  uint32_t k;
  uint64_t *bloom;               // the batch's Bloom filter (bloom_word), or null
  uint32_t bloom_w;              // log2(filter words per fine bucket)
};

#define OVL_HOPELESS_MATCH 90

// One wave per fine bucket -> one table slice.
__global__ void __launch_bounds__(256) k_table(TableArgs A) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  uint32_t f = blockIdx.x * (blockDim.x >> 6) + wave;
  uint32_t S = 1u << A.slice_bits;
  uint64_t *key = (uint64_t *)smem + (size_t)wave * S * 2;     // S keys then S (off,cnt)
  uint32_t *oc = (uint32_t *)(key + S);
  // the fine bucket's Bloom filter region, after the waves' slices
  const uint32_t BW = A.bloom ? 1u << A.bloom_w : 0u;
  uint64_t *lb = (uint64_t *)smem + (size_t)(blockDim.x >> 6) * S * 2 + (size_t)wave * BW;
  if (f >= A.nfine) return;
  for (uint32_t i = lane; i < S; i += 64) { key[i] = 0; oc[2 * i] = 0; oc[2 * i + 1] = 0; }
  for (uint32_t i = lane; i < BW; i += 64) lb[i] = 0;
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  uint32_t fs = A.fstart[f], fn = A.fcnt[f];
  uint32_t pshift = 64 - A.tab_bits;
  // Run starts come from one ballot per 64 records, with a virtual start at fn; a run ends
  // at the next start: in the same batch, in the next one (looked ahead), or -- for a run
  // longer than a batch -- found by the whole wave scanning on.
  auto starts = [&](uint32_t j0, uint64_t &Mj) -> uint64_t {
    const uint32_t j = j0 + lane;
    bool st = j == fn;
    Mj = 0;
    if (j < fn) {
      Mj = A.M[fs + j];
      st = (j == 0) || (A.M[fs + j - 1] != Mj);
    }
    return __builtin_amdgcn_ballot_w64(st);
  };
  uint64_t Mnext = 0;
  uint64_t cur_m = fn ? starts(0, Mnext) : 0;
  for (uint32_t i0 = 0; i0 < fn; i0 += 64) {
    uint32_t i = i0 + lane;
    const uint64_t M = Mnext;
    const uint64_t nxt_m = (i0 + 64 <= fn) ? starts(i0 + 64, Mnext) : 0;
    const bool start = i < fn && ((cur_m >> lane) & 1ull);
    const uint64_t above = cur_m & ~((2ull << lane) - 1ull);   // starts after this lane
    const bool far = start && !above && !nxt_m;
    uint32_t efar = 0;
    if (__builtin_amdgcn_ballot_w64(far)) {    // a run longer than the next batch
      for (uint32_t j0 = i0 + 128;; j0 += 64) {
        uint64_t dummy;
        const uint64_t m = starts(j0, dummy);
        if (m) { efar = j0 + (uint32_t)__builtin_ctzll(m); break; }
      }
    }
    if (start) {
      const uint32_t e = above ? i0 + (uint32_t)__builtin_ctzll(above)
                       : nxt_m ? i0 + 64 + (uint32_t)__builtin_ctzll(nxt_m) : efar;
      uint32_t off = fs + i, cnt = e - i, flags = 0;
      if (A.P[off] == OVL_SKIP_POS) {          // marker sorts first (position descending)
        flags = OVL_FLAG_SKIP;
        off++; cnt--;
        for (uint32_t j = off; j < off + cnt; j++) {
          uint64_t pos = A.P[j];
          if (pos == OVL_SKIP_POS) continue;
          uint32_t r = (uint32_t)(pos >> 32) - A.first_iid, o = (uint32_t)pos;
          uint32_t bits = 0;
          if (o < OVL_HOPELESS_MATCH) bits |= 2u;
          if ((int64_t)A.len[r] - o - A.k + 1 < OVL_HOPELESS_MATCH) bits |= 4u;
          if (bits) atomicOr(&A.rflags[r], bits);
        }
        while (cnt > 0 && A.P[off] == OVL_SKIP_POS) { off++; cnt--; }   // duplicate markers
      }
      uint32_t slot = (uint32_t)(M >> pshift) & (S - 1);
      for (;;) {
        uint32_t old = atomicCAS(&oc[2 * slot + 1], 0u, (cnt | flags | OVL_PRESENT));
        if (old == 0) break;
        slot = (slot + 1) & (S - 1);
      }
      key[slot] = M;
      oc[2 * slot] = off;
      if (BW) atomicOr((unsigned long long *)&lb[M & (BW - 1)], (unsigned long long)bloom_mask(M));
    }
    cur_m = nxt_m;
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  TabEntry *dst = A.tab + ((size_t)f << A.slice_bits);
  for (uint32_t i = lane; i < S; i += 64) {
    TabEntry e;
    e.key = key[i];
    e.off = oc[2 * i];
    e.cnt = oc[2 * i + 1];
    dst[i] = e;
  }
  for (uint32_t i = lane; i < BW; i += 64) A.bloom[((size_t)f << A.bloom_w) + i] = lb[i];
}

// Hash_Entries of Build_Hash_Index (Hash_Insert :336-341): a distinct k-mer takes a table
// entry when its first occurrence is loaded, i.e. at the lowest read ID that holds it.  A
// sorted run (one k-mer) ends at its lowest position, so the run's last record names that
// read; runs of skip markers alone are not k-mers of the batch.  hist[r - h0] counts the
// k-mers whose first read is r.
__global__ void k_first_reads(const uint64_t *__restrict__ M, const uint64_t *__restrict__ P,
                              uint32_t n, uint32_t h0_iid, uint32_t *hist) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const uint64_t p = P[i];
    if (p == OVL_SKIP_POS) continue;
    if (i + 1 < n && M[i + 1] == M[i]) continue;
    atomicAdd(&hist[(uint32_t)(p >> 32) - h0_iid], 1u);
  }
}

// The same count with the histogram privatised in LDS: every read takes thousands of run
// ends, so the global atomics above queue on a few thousand addresses (7 ms per build of a
// canu-sized batch).  A block counts OVL_FR_CHUNK consecutive records into 16-bit LDS bins
// (two per word: a block's count per read stays below 2^16) and adds its nonzero bins to
// the global histogram.  nr (reads of the build) <= 2 * OVL_FR_WORDS.
#define OVL_FR_WORDS 16384
#define OVL_FR_CHUNK 65535
__global__ void __launch_bounds__(1024) k_first_reads_lds(const uint64_t *__restrict__ M,
                                                          const uint64_t *__restrict__ P,
                                                          uint32_t n, uint32_t h0_iid, uint32_t nr,
                                                          uint32_t *hist) {
  __shared__ uint32_t bins[OVL_FR_WORDS];
  const uint32_t nw = (nr + 1) / 2;
  for (uint32_t w = threadIdx.x; w < nw; w += blockDim.x) bins[w] = 0;
  __syncthreads();
  const uint64_t b0 = (uint64_t)blockIdx.x * OVL_FR_CHUNK;
  const uint32_t i1 = (uint32_t)(b0 + OVL_FR_CHUNK < n ? b0 + OVL_FR_CHUNK : n);
  for (uint32_t i = (uint32_t)b0 + threadIdx.x; i < i1; i += blockDim.x) {
    const uint64_t p = P[i];
    if (p == OVL_SKIP_POS) continue;
    if (i + 1 < n && M[i + 1] == M[i]) continue;
    const uint32_t r = (uint32_t)(p >> 32) - h0_iid;
    atomicAdd(&bins[r >> 1], (r & 1u) ? 0x10000u : 1u);
  }
  __syncthreads();
  for (uint32_t w = threadIdx.x; w < nw; w += blockDim.x) {
    const uint32_t v = bins[w];
    if (v & 0xFFFFu) atomicAdd(&hist[2 * w], v & 0xFFFFu);
    if ((v >> 16) && 2 * w + 1 < nr) atomicAdd(&hist[2 * w + 1], v >> 16);
  }
}

// A load-cut batch (Build_Hash_Index.C:495-541: the table load stops the batch at read
// `last`) from the index of a longer prefix: every k-mer's occurrence run is position-
// descending, so its occurrences in reads past `last` lead the run -- the entry skips them.
// A k-mer left with none keeps its slot (probe sequences stay intact) with an empty run,
// which every lookup reads as the miss it is in the cut batch's own index ({off 0, cnt 0},
// the record a miss writes).  Skip k-mer entries are kept as they are.  The Bloom filter
// keeps the prefix's k-mers: a superset, so still exact.
__global__ void k_cut_index(TabEntry *tab, uint64_t nslots, const uint64_t *__restrict__ occ,
                            uint32_t last) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < nslots;
       i += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t c = tab[i].cnt;
    if (c == 0 || (c & OVL_FLAG_SKIP)) continue;
    const uint32_t off = tab[i].off, n = c & OVL_CNT_MASK;
    uint32_t lo = 0, hi = n;                     // first occurrence in a read <= last
    while (lo < hi) {
      const uint32_t mid = (lo + hi) >> 1;
      if ((uint32_t)(occ[off + mid] >> 32) > last) lo = mid + 1; else hi = mid;
    }
    if (lo == 0) continue;
    tab[i].off = lo < n ? off + lo : 0u;
    tab[i].cnt = (c & ~OVL_CNT_MASK) | (n - lo);
  }
}

// ---------------------------------------------------------------------------------------
// Small utilities

// Single-block exclusive scan, u32 in -> u32 out, any n.  Also writes the total.
__global__ void k_scan_u32(const uint32_t *in, uint32_t *out, uint32_t n, uint32_t *total) {
  __shared__ uint32_t part[1024];
  uint32_t per = (n + blockDim.x - 1) / blockDim.x;
  uint32_t b = threadIdx.x * per, e = b + per;
  if (e > n) e = n;
  uint32_t s = 0;
  for (uint32_t i = b; i < e; i++) s += in[i];
  part[threadIdx.x] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t acc = 0;
    for (uint32_t i = 0; i < blockDim.x; i++) { uint32_t v = part[i]; part[i] = acc; acc += v; }
    if (total) *total = acc;
  }
  __syncthreads();
  uint32_t acc = part[threadIdx.x];
  for (uint32_t i = b; i < e; i++) { uint32_t v = in[i]; out[i] = acc; acc += v; }
}

}  // namespace ovl
