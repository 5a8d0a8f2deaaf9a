// ovl_common.h -- device-side types and helpers shared by the overlapInCore kernels.
//
// Reads live in HBM as 2-bit packed strands (a=0 c=1 g=2 t=3, first base in the low
// bits -- the reference's key layout, Build_Hash_Index.C:376-379), 32 bases per 64-bit
// word, one guard word after every read.  Exceptions are bit masks with one bit per base
// (32-bit words aligned with the base words):
//   fwdN   'n' in the forward strand (a wildcard in the extension: forward.C:176)
//   rcNul  the reverse complement of 'n' is NUL (AS_UTL_reverseComplement.C:39): it
//          matches nothing but an 'n', and it ends Find_Overlaps' window scan
//          (Find_Overlaps.C:341 `while (*P != '\0')`).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <type_traits>

#define OVL_WAVE 64

namespace ovl {

struct ReadsDev {
  const uint64_t *fwd;      // packed forward strands
  const uint64_t *rc;       // packed reverse-complement strands
  const uint32_t *fwdN;     // 'n' masks, forward
  const uint32_t *rcNul;    // NUL masks, reverse complement
  const uint64_t *wofs;     // first word of read r
  const uint32_t *len;      // read lengths
  const uint32_t *flags;    // bit0: read has an 'n'
  const uint32_t *rcFirstNul;  // first rc NUL at position >= k (len if none): ends the scan
  const uint8_t  *qual;     // quality values (-w only): read r base i at wofs[r]*32 + i
  uint32_t        first_iid;
  uint32_t        nreads;
};

// One strand of one read as the extension sees it.  W is the pointer type of the packed
// words: plain (global) or LDS (address space 3) when the strands are staged on chip.
template <typename W>
struct StrandT {
  static constexpr bool kExc = true;
  W               w;
  const uint32_t *ex_wild;  // bases that match anything ('n'), may be null (global)
  const uint32_t *ex_nul;   // bases that match nothing but a wildcard, may be null (global)
  int32_t         len;
};
// A strand without 'n' / NUL exceptions (the common case): no mask pointers at all.
template <typename W>
struct StrandP {
  static constexpr bool kExc = false;
  W       w;
  int32_t len;
};
typedef StrandT<const uint64_t *> Strand;
typedef __attribute__((address_space(3))) uint64_t lds_u64;
typedef __attribute__((address_space(3))) int32_t lds_i32;
typedef StrandT<const lds_u64 *> StrandL;
typedef StrandP<const lds_u64 *> StrandLP;

__device__ __forceinline__ Strand strand_fwd(const ReadsDev &R, uint32_t r) {
  Strand s;
  uint64_t o = R.wofs[r];
  s.w = R.fwd + o;
  bool ex = R.flags[r] & 1u;
  s.ex_wild = ex ? R.fwdN + o : nullptr;
  s.ex_nul = nullptr;
  s.len = (int32_t)R.len[r];
  return s;
}

__device__ __forceinline__ Strand strand_rc(const ReadsDev &R, uint32_t r) {
  Strand s;
  uint64_t o = R.wofs[r];
  s.w = R.rc + o;
  bool ex = R.flags[r] & 1u;
  s.ex_wild = nullptr;
  s.ex_nul = ex ? R.rcNul + o : nullptr;
  s.len = (int32_t)R.len[r];
  return s;
}

// 32 bases starting at p (0 <= p < len); base i of the result in bits 2i..2i+1.
template <typename W>
__device__ __forceinline__ uint64_t bases_at(W w, int32_t p) {
  uint32_t wi = (uint32_t)p >> 5, sh = ((uint32_t)p & 31u) * 2u;
  uint64_t v = w[wi] >> sh;
  if (sh) v |= w[wi + 1] << (64u - sh);
  return v;
}

__device__ __forceinline__ uint32_t mask_at(const uint32_t *m, int32_t p) {
  uint32_t wi = (uint32_t)p >> 5, sh = (uint32_t)p & 31u;
  uint32_t v = m[wi] >> sh;
  if (sh) v |= m[wi + 1] << (32u - sh);
  return v;
}

// Spread 32 bits to the even bit positions of a 64-bit word.
__device__ __forceinline__ uint64_t spread2(uint32_t m) {
  uint64_t x = m;
  x = (x | (x << 16)) & 0x0000FFFF0000FFFFull;
  x = (x | (x << 8)) & 0x00FF00FF00FF00FFull;
  x = (x | (x << 4)) & 0x0F0F0F0F0F0F0F0Full;
  x = (x | (x << 2)) & 0x3333333333333333ull;
  x = (x | (x << 1)) & 0x5555555555555555ull;
  return x;
}

// Mismatch bits (bit 2i) between 32 bases of A at pa and of T at pt, both forward.
// bases_match(a, b) = a == b || a == 'n' || b == 'n'   (forward.C:176)
template <typename SA, typename ST>
__device__ __forceinline__ uint64_t mismatch_fwd(const SA &A, int32_t pa, const ST &T,
                                                 int32_t pt) {
  uint64_t x = bases_at(A.w, pa) ^ bases_at(T.w, pt);
  uint64_t mm = (x | (x >> 1)) & 0x5555555555555555ull;
  if constexpr (SA::kExc && ST::kExc) if (A.ex_nul || T.ex_nul || A.ex_wild || T.ex_wild) {
    if (A.ex_nul) mm |= spread2(mask_at(A.ex_nul, pa));
    if (T.ex_nul) mm |= spread2(mask_at(T.ex_nul, pt));
    uint32_t wild = 0;
    if (A.ex_wild) wild |= mask_at(A.ex_wild, pa);
    if (T.ex_wild) wild |= mask_at(T.ex_wild, pt);
    if (wild) mm &= ~spread2(wild);
  }
  return mm;
}

// 32 bases ending at p, p-31 .. p (group 31 = base p).  p may be < 31.
template <typename W>
__device__ __forceinline__ uint64_t bases_end(W w, int32_t p) {
  if (p >= 31) return bases_at(w, p - 31);
  return bases_at(w, 0) << (2 * (31 - p));
}
__device__ __forceinline__ uint32_t mask_end(const uint32_t *m, int32_t p) {
  if (p >= 31) return mask_at(m, p - 31);
  return mask_at(m, 0) << (31 - p);
}

template <typename SA, typename ST>
__device__ __forceinline__ uint64_t mismatch_bwd(const SA &A, int32_t pa, const ST &T,
                                                 int32_t pt) {
  uint64_t x = bases_end(A.w, pa) ^ bases_end(T.w, pt);
  uint64_t mm = (x | (x >> 1)) & 0x5555555555555555ull;
  if constexpr (SA::kExc && ST::kExc) if (A.ex_nul || T.ex_nul || A.ex_wild || T.ex_wild) {
    if (A.ex_nul) mm |= spread2(mask_end(A.ex_nul, pa));
    if (T.ex_nul) mm |= spread2(mask_end(T.ex_nul, pt));
    uint32_t wild = 0;
    if (A.ex_wild) wild |= mask_end(A.ex_wild, pa);
    if (T.ex_wild) wild |= mask_end(T.ex_wild, pt);
    if (wild) mm &= ~spread2(wild);
  }
  return mm;
}

// How far A[ra..] and T[rt..] agree, going forward, at most lim bases.
template <typename SA, typename ST>
__device__ __forceinline__ int32_t slide_fwd(const SA &A, int32_t ra, const ST &T, int32_t rt,
                                             int32_t lim) {
  int32_t n = 0;
  while (n < lim) {
    uint64_t mm = mismatch_fwd(A, ra + n, T, rt + n);
    int32_t run = mm ? (int32_t)(__builtin_ctzll(mm) >> 1) : 32;
    n += run;
    if (run < 32) break;
  }
  return n < lim ? n : lim;
}

// How far A[ra], A[ra-1], .. and T[rt], T[rt-1], .. agree, at most lim bases.
template <typename SA, typename ST>
__device__ __forceinline__ int32_t slide_bwd(const SA &A, int32_t ra, const ST &T, int32_t rt,
                                             int32_t lim) {
  int32_t n = 0;
  while (n < lim) {
    uint64_t mm = mismatch_bwd(A, ra - n, T, rt - n);
    int32_t run = mm ? (int32_t)(__builtin_clzll(mm) >> 1) : 32;
    n += run;
    if (run < 32) break;
  }
  return n < lim ? n : lim;
}

// Bijective 64-bit mixer (splitmix64 finalizer): k-mer -> table position.
__device__ __host__ __forceinline__ uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

// ---- k-mer index ------------------------------------------------------------------
// Table entry: an open-addressing slot.  key = mix64(k-mer); cnt holds the number of
// occurrences plus flags (OVL_PRESENT on every filled slot, OVL_FLAG_SKIP).  Occurrence lists hold
// (iid << 32 | offset) sorted DESCENDING, i.e. in Hash_Insert's chain order
// (Build_Hash_Index.C:320-323 pushes every new entry in front).
// Per-read flags (ReadsDev::flags): bit 0 the read holds an 'n'; bits 1 / 2 its left /
// right end is screened (String_Info lfrag/rfrag_end_screened); bit 3 the read is not
// hashed (outside the -H libraries).
#define OVL_RFLAG_NOHASH 8u

#define OVL_CNT_MASK    0x3FFFFFFFu
#define OVL_PRESENT     0x40000000u
#define OVL_FLAG_SKIP   0x80000000u      // k-mer from the -k skip list (Empty entry)

struct TabEntry {
  uint64_t key;
  uint32_t off;
  uint32_t cnt;
};

struct IndexDev {
  const TabEntry *tab;
  const uint64_t *occ;       // occurrence lists
  uint32_t        tab_bits;  // log2(table size)
  uint32_t        slice_bits;// log2(slots per slice)
  uint32_t        k;
  uint64_t        kmask;
  const uint64_t *bloom;     // the batch's Bloom filter (partitioned by fine bucket), or null
  uint32_t        bloom_w;   // log2(filter words per fine bucket)
};

// The blocked Bloom filter of a hash batch's distinct k-mers (every table entry, the -k
// skip entries included): one 64-bit word per key, 4 bits in it.  No false negatives, so a
// window it rejects is a window the table lookup would not have found.  The filter is
// partitioned like the table: fine bucket f (the top bits of mix64(kmer), the table slice's
// index) owns words [f << w, (f + 1) << w), so k_table builds each region in LDS beside its
// slice and writes it whole -- no global atomics.  The word within the region comes from
// the low bits of mix64(kmer), the 4 bits from an odd multiple of it.
__host__ __device__ __forceinline__ uint64_t bloom_word(uint64_t slot0, uint32_t slice_bits,
                                                       uint64_t M, uint32_t w) {
  return ((slot0 >> slice_bits) << w) | (M & ((1ull << w) - 1));
}
__host__ __device__ __forceinline__ uint64_t bloom_mask(uint64_t M) {
  const uint64_t h = M * 0x9E3779B97F4A7C15ull;
  return (1ull << (h >> 58)) | (1ull << ((h >> 52) & 63)) | (1ull << ((h >> 46) & 63)) |
         (1ull << ((h >> 40) & 63));
}

// The table is keyed by mix64(kmer); an empty slot has cnt == 0 (every filled slot has
// the 0x40000000 "present" bit).  Linear probing stays inside the k-mer's slice.
__device__ __forceinline__ const TabEntry *index_find(const IndexDev &X, uint64_t kmer) {
  uint64_t M = mix64(kmer);
  uint64_t slot0 = M >> (64 - X.tab_bits);
  uint64_t smask = (1ull << X.slice_bits) - 1;
  uint64_t base = slot0 & ~smask;
  for (uint64_t i = 0; i <= smask; i++) {
    const TabEntry *e = X.tab + (base | ((slot0 + i) & smask));
    if (e->cnt == 0) return nullptr;
    if (e->key == M) return e;
  }
  return nullptr;
}

// ---- seed probe results ----------------------------------------------------------
// Per query position: where its occurrence list starts and how many entries qualify
// (target iid > query iid: Find_Overlaps.C:328); lists are descending so those are a
// prefix.
struct Probe {
  uint32_t off;
  uint32_t cnt;
};

// A (query, orientation) unit.
struct Unit {
  uint32_t r;        // local read index of the query
  uint32_t dir;      // 0 FORWARD, 1 REVERSE
};

// A (query, orientation, target) pair with its ordered match list.
struct PairRec {
  uint32_t unit;
  uint32_t tgt;          // target local read index
  uint32_t node_off;     // first node (list order) in the pair-node array
  uint32_t node_cnt;
  int32_t  diag_ct, diag_bgn, diag_end;
  uint32_t flags;        // bit0 consistent, bit1 unit left_end_screened, bit2 right,
                         // bit3 / bit4 the target's left / right end screened (as the
                         // hash batch that found the pair left them)
};

// Match_Node_t (prefixEditDistance.H:60)
struct Node {
  int32_t Offset, Len, Start, Next;
};

// ovOverlap record (ovOverlap.H:285, 21-bit layout)
struct Rec {
  uint32_t a_iid, b_iid;
  uint64_t w0, w1;
};

}  // namespace ovl
