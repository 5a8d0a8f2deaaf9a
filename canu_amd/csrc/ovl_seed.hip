// ovl_seed.hip -- seed lookup and match chaining (Find_Overlaps replacement).
//
// Reference: src/overlapInCore/overlapInCore-Find_Overlaps.C
//   Find_Overlaps (:284)  every k-window of the query (FORWARD, then its reverse
//                          complement) is looked up; each occurrence in a read with a
//                          larger ID than the query is passed to Add_Ref
//   Add_Ref       (:158)  per-target bookkeeping (diag stats, consistent flag)
//   Add_Match     (:79)   the ordered match list: extend the node whose next expected
//                          window is this one on the same diagonal, else push a new node
//
// Two kernels:
//   k_probe  one wave per (query, orientation) unit; lanes probe 64 windows at a time,
//            write (list offset, qualifying count) per window -- the HBM-bound kernel
//   k_chain  one wave per unit; per 64-window chunk the qualifying occurrences are staged
//            in LDS (wave-level ordered compaction); every target read owns one lane, and
//            that lane replays Add_Match for its target in reference order (window asc,
//            chain order) -- all targets of the unit advance in parallel
#include "ovl_common.h"

namespace ovl {

struct ProbeArgs {
  ReadsDev R;
  IndexDev X;
  const Unit *units;
  const uint64_t *rbase;        // per unit: first Probe slot
  uint32_t nunits;
  Probe *out;
  uint32_t *unit_hits;          // per unit: occurrences (upper bound of qualifying hits)
  uint32_t *unit_flags;         // bit1 left_end_screened, bit2 right_end_screened
  uint32_t k;
};

__device__ __forceinline__ uint32_t unit_windows(const ReadsDev &R, const Unit &u, uint32_t k) {
  int32_t L = (int32_t)R.len[u.r];
  int32_t lim = L;
  if (u.dir) {
    int32_t fn = (int32_t)R.rcFirstNul[u.r];
    if (fn < lim) lim = fn;
  }
  // windows 0 .. lim-k; window 0 is always visited (it cannot match if it holds a NUL)
  int32_t nw = lim - (int32_t)k + 1;
  if (nw < 1) nw = 1;
  return (uint32_t)nw;
}

// Number of leading entries of a descending occurrence list whose read iid > a.
__device__ __forceinline__ uint32_t qualifying(const uint64_t *occ, uint32_t off, uint32_t cnt,
                                               uint32_t a_iid) {
  if (cnt <= 8) {
    uint32_t q = 0;
    while (q < cnt && (uint32_t)(occ[off + q] >> 32) > a_iid) q++;
    return q;
  }
  uint32_t lo = 0, hi = cnt;           // first index with iid <= a
  while (lo < hi) {
    uint32_t mid = (lo + hi) >> 1;
    if ((uint32_t)(occ[off + mid] >> 32) > a_iid) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

// BLOOM: windows whose k-mer the batch's Bloom filter rejects skip the table (OverlapDriver
// batches probed by many more queries than they index: most windows miss, and the filter
// is a fraction of the table's size).
template <bool BLOOM>
__global__ void __launch_bounds__(256) k_probe(ProbeArgs A) {
  uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  uint32_t u = blockIdx.x * (blockDim.x >> 6) + wave;
  if (u >= A.nunits) return;
  Unit un = A.units[u];
  Strand S = un.dir ? strand_rc(A.R, un.r) : strand_fwd(A.R, un.r);
  const uint32_t *bad = un.dir ? S.ex_nul : S.ex_wild;
  uint32_t nw = unit_windows(A.R, un, A.k);
  int32_t L = S.len;
  uint32_t kbits = (1u << A.k) - 1u;
  Probe *out = A.out + A.rbase[u];
  uint32_t hits = 0, flags = 0;
  // PU windows per lane per step: their table slots are computed first and their first
  // 16-B entries loaded together, so each lane keeps PU random loads in flight (the
  // lookups are latency-bound); the rare longer probe sequences continue one by one.
#ifndef OVL_PROBE_PU
#define OVL_PROBE_PU 4
#endif
  constexpr int PU = OVL_PROBE_PU;
  const uint64_t smask = (1ull << A.X.slice_bits) - 1;
  for (uint32_t o0 = 0; o0 < nw; o0 += 64 * PU) {
    uint64_t M[PU], slot0[PU];
    bool ok[PU];
#pragma unroll
    for (int q = 0; q < PU; q++) {
      const uint32_t o = o0 + 64 * q + lane;
      ok[q] = o < nw && (int32_t)(o + A.k) <= L;
      if (ok[q] && bad) ok[q] = (mask_at(bad, (int32_t)o) & kbits) == 0;
      M[q] = 0;
      slot0[q] = 0;
      if (ok[q]) {
        M[q] = mix64(bases_at(S.w, (int32_t)o) & A.X.kmask);
        slot0[q] = M[q] >> (64 - A.X.tab_bits);
      }
    }
    if constexpr (BLOOM) {
      uint64_t bw[PU];
#pragma unroll
      for (int q = 0; q < PU; q++)
        bw[q] = ok[q] ? A.X.bloom[bloom_word(slot0[q], A.X.slice_bits, M[q], A.X.bloom_w)] : 0;
#pragma unroll
      for (int q = 0; q < PU; q++) {
        const uint64_t bm = bloom_mask(M[q]);
        if (ok[q] && (bw[q] & bm) != bm) { ok[q] = false; M[q] = 0; slot0[q] = 0; }
      }
    }
    TabEntry e[PU];
#pragma unroll
    for (int q = 0; q < PU; q++) {
      e[q].key = 0; e[q].off = 0; e[q].cnt = 0;
      if (ok[q]) e[q] = A.X.tab[slot0[q]];
    }
    // finish each window with its values passed in: a loop over q holding the unbounded
    // probe loop is not unrolled, and its dynamically indexed arrays went to scratch (80 B
    // per lane, ~3x the records' bytes of write traffic)
    auto finish = [&](uint32_t o, bool okq, uint64_t Mq, uint64_t s0, TabEntry t) {
      if (o >= nw) return;
      Probe pr;
      pr.off = 0;
      pr.cnt = 0;
      if (okq) {
        // index_find's linear probe within the slice, from the entry already loaded
        bool found = false;
        const uint64_t base = s0 & ~smask;
        for (uint64_t i = 1;; i++) {
          if (t.cnt == 0) break;
          if (t.key == Mq) { found = true; break; }
          if (i > smask) break;
          t = A.X.tab[base | ((s0 + i) & smask)];
        }
        if (found) {
          const uint32_t c = t.cnt;
          if (c & OVL_FLAG_SKIP) {
            // Hash_Find found an Empty entry: hi_hits (Find_Overlaps.C:321-366)
            if (o < 90) flags |= 2u;
            if (o > 0 && L - (int32_t)o - (int32_t)A.k + 1 < 90) flags |= 4u;
          } else {
            // whole occurrence list; the chain kernel keeps its qualifying prefix
            // (targets with iid > query, Find_Overlaps.C:328)
            pr.off = t.off;
            pr.cnt = c & OVL_CNT_MASK;
            hits += pr.cnt;
          }
        }
      }
      out[o] = pr;
    };
    static_assert(PU == 4 || PU == 8, "finish() calls below");
    finish(o0 + lane, ok[0], M[0], slot0[0], e[0]);
    finish(o0 + 64 + lane, ok[1], M[1], slot0[1], e[1]);
    finish(o0 + 128 + lane, ok[2], M[2], slot0[2], e[2]);
    finish(o0 + 192 + lane, ok[3], M[3], slot0[3], e[3]);
    if constexpr (PU == 8) {
      finish(o0 + 256 + lane, ok[4], M[4], slot0[4], e[4]);
      finish(o0 + 320 + lane, ok[5], M[5], slot0[5], e[5]);
      finish(o0 + 384 + lane, ok[6], M[6], slot0[6], e[6]);
      finish(o0 + 448 + lane, ok[7], M[7], slot0[7], e[7]);
    }
  }
  for (int s = 32; s > 0; s >>= 1) {
    hits += __shfl_xor(hits, s);
    flags |= __shfl_xor(flags, s);
  }
  if (lane == 0) {
    A.unit_hits[u] = hits;
    A.unit_flags[u] = flags;
  }
}

// ---------------------------------------------------------------------------------------
// OverlapDriver jobs: the query windows sorted by k-mer once per job.
// Every hash batch of a driver job is searched by the same query reads (every read of the
// -r range below the batch's end; Process_Overlaps.C:101-137), and most of their windows
// miss the batch, so k_probe's one random table lookup per window per batch runs at the
// memory system's random-access rate (~40 G lookups/s, whatever the table's size).  Here the
// job's query windows are keyed by their k-mer's mix64 and radix-sorted ONCE (k_sq_keys, in
// runs of <= 2^29 windows); each batch then streams a run in key order, which is table-slot
// order (a slot is the top tab_bits of the same mix64): consecutive windows read consecutive
// slots, the table and the windows are both read as streams, and only the windows whose
// k-mer the batch holds write a Probe record back to window order (k_probe_sorted).  The
// records, unit hit counts and screened-end flags are exactly k_probe's.

struct SqKeyArgs {
  ReadsDev R;
  const Unit *units;            // the run's units
  const uint64_t *wbase;        // per unit: first window (run-local)
  uint32_t nunits, k;
  uint64_t kmask;
  uint64_t *key;                // run-local window id -> mix64(k-mer)
  uint32_t *wid;                // -> the window id; 0xFFFFFFFF: no k-mer there (an N, a NUL)
  unsigned long long *sig;      // [0..1]: the run's (key, wid) multiset signature
};

// Multiset signature of a run's (key, wid) pairs: two independent 64-bit sums of a mix of
// each pair, computed before the sort (k_sq_keys) and after it (k_sq_sorted_check).  A sort
// that returns its keys in order but with a window id duplicated or lost (what this ROCm's
// partial-range radix sort did) changes both sums.
__device__ __forceinline__ void sq_sig_add(uint64_t key, uint32_t wid, uint64_t &s1,
                                           uint64_t &s2) {
  const uint64_t h = mix64(key ^ ((uint64_t)wid * 0x9E3779B97F4A7C15ull));
  s1 += h;
  s2 += mix64(h ^ 0xD6E8FEB86659FD93ull);
}
__device__ __forceinline__ void sq_sig_flush(uint64_t s1, uint64_t s2, uint32_t lane,
                                             unsigned long long *sig) {
  for (int o = 32; o > 0; o >>= 1) {
    s1 += __shfl_xor(s1, o);
    s2 += __shfl_xor(s2, o);
  }
  if (lane == 0) {
    atomicAdd(&sig[0], (unsigned long long)s1);
    atomicAdd(&sig[1], (unsigned long long)s2);
  }
}

// one wave per unit: its windows' keys, k_probe's window rule (unit_windows, the N / NUL
// masks).  The unit owns wbase[u+1] - wbase[u] slots (L - k + 1, sq_prepare); a reverse unit
// whose strand holds a NUL has fewer windows (unit_windows), and its tail slots are written
// as "no k-mer" too -- left unwritten they would keep an earlier run's (key, wid) pairs,
// which the sort and the probe would then read as windows.
__global__ void __launch_bounds__(256) k_sq_keys(SqKeyArgs A) {
  const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const uint32_t u = blockIdx.x * 4 + wave;
  if (u >= A.nunits) return;
  const Unit un = A.units[u];
  const Strand S = un.dir ? strand_rc(A.R, un.r) : strand_fwd(A.R, un.r);
  const uint32_t *bad = un.dir ? S.ex_nul : S.ex_wild;
  const uint32_t nw = unit_windows(A.R, un, A.k);
  const int32_t L = S.len;
  const uint32_t kbits = (1u << A.k) - 1u;
  const uint64_t b = A.wbase[u];
  const uint32_t ns = (uint32_t)(A.wbase[u + 1] - b);
  uint64_t s1 = 0, s2 = 0;
  for (uint32_t o = lane; o < ns; o += 64) {
    bool ok = o < nw && (int32_t)(o + A.k) <= L;
    if (ok && bad) ok = (mask_at(bad, (int32_t)o) & kbits) == 0;
    const uint64_t key = ok ? mix64(bases_at(S.w, (int32_t)o) & A.kmask) : ~0ull;
    const uint32_t wid = ok ? (uint32_t)(b + o) : 0xFFFFFFFFu;
    A.key[b + o] = key;
    A.wid[b + o] = wid;
    sq_sig_add(key, wid, s1, s2);
  }
  sq_sig_flush(s1, s2, lane, A.sig);
}

struct SqProbeArgs {
  IndexDev X;
  ReadsDev R;
  const uint64_t *key;          // the run's windows, sorted by key
  const uint32_t *wid;
  uint64_t n;
  uint32_t wlim;                // this batch searches the run's windows below wlim
  const Unit *units;            // the run's units
  const uint64_t *wbase;        // per run unit: first window; [nunits] = the run's windows
  const uint32_t *ublk;         // per 512 windows: the unit holding the block's first window
  uint32_t k;
  Probe *out;                   // run-local window id -> its record (zeroed up to wlim)
  uint32_t *unit_flags;         // per run unit (zeroed)
  uint32_t *unit_hits;          // per run unit: occurrences of its windows' k-mers (zeroed)
};

__global__ void __launch_bounds__(256) k_probe_sorted(SqProbeArgs A) {
  const uint64_t smask = (1ull << A.X.slice_bits) - 1;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  const uint32_t shift = 64 - A.X.tab_bits;
  // a window whose k-mer the table holds: its record, or (a skip k-mer) its unit's
  // screened-end flags; the table entry first loaded is passed in
  auto finish = [&](uint32_t w, uint64_t M, TabEntry t) {
    if (w >= A.wlim) return;                     // no k-mer, or a unit this batch skips
    const uint64_t s0 = M >> shift, base = s0 & ~smask;
    bool found = false;
    for (uint64_t j = 1;; j++) {                 // index_find's linear probe (k_probe)
      if (t.cnt == 0) break;
      if (t.key == M) { found = true; break; }
      if (j > smask) break;
      t = A.X.tab[base | ((s0 + j) & smask)];
    }
    if (!found) return;
    const uint32_t c = t.cnt;
    // the window's unit: the 512-window block's first unit, then at most a unit or two on
    // (units hold ~L windows); ublk, wbase and the per-unit counters are L2-resident
    uint32_t u = A.ublk[w >> 9];
    while (A.wbase[u + 1] <= w) u++;
    if (c & OVL_FLAG_SKIP) {
      // Hash_Find found an Empty entry: hi_hits (Find_Overlaps.C:321-366)
      const uint32_t o = w - (uint32_t)A.wbase[u];
      const int32_t L = (int32_t)A.R.len[A.units[u].r];
      uint32_t f = 0;
      if (o < 90) f |= 2u;
      if (o > 0 && L - (int32_t)o - (int32_t)A.k + 1 < 90) f |= 4u;
      if (f) atomicOr(&A.unit_flags[u], f);
    } else {
      Probe pr;
      pr.off = t.off;
      pr.cnt = c & OVL_CNT_MASK;
      A.out[w] = pr;
      // the unit's hit count (k_probe's unit_hits) here rather than by a second pass over
      // every record of the run: only the windows that hit pay, once
      if (pr.cnt) atomicAdd(&A.unit_hits[u], pr.cnt);
    }
  };
  // 4 sorted windows per thread per step: their ids, keys and first table entries are
  // loaded together (the loop is latency-bound: id -> key -> entry -> record)
  for (uint64_t i0 = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i0 < A.n;
       i0 += 4 * stride) {
    uint32_t w[4];
    uint64_t M[4];
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const uint64_t i = i0 + q * stride;
      w[q] = i < A.n ? A.wid[i] : 0xFFFFFFFFu;
      M[q] = i < A.n ? A.key[i] : 0ull;
    }
    // the batch's Bloom filter first (when it has one): most windows miss the batch, and a
    // miss read from the table is a linear probe to the slice's next empty slot -- dependent
    // loads -- where the filter rejects it with one load (sorted keys: few lines per wave)
    if (A.X.bloom) {
      uint64_t bw[4];
#pragma unroll
      for (int q = 0; q < 4; q++)
        bw[q] = w[q] < A.wlim ? A.X.bloom[bloom_word(M[q] >> shift, A.X.slice_bits, M[q],
                                                     A.X.bloom_w)] : 0;
#pragma unroll
      for (int q = 0; q < 4; q++) {
        const uint64_t bm = bloom_mask(M[q]);
        if ((bw[q] & bm) != bm) w[q] = 0xFFFFFFFFu;
      }
    }
    TabEntry t[4];
#pragma unroll
    for (int q = 0; q < 4; q++) {
      t[q].key = 0; t[q].off = 0; t[q].cnt = 0;
      if (w[q] < A.wlim) t[q] = A.X.tab[M[q] >> shift];
    }
    finish(w[0], M[0], t[0]);
    finish(w[1], M[1], t[1]);
    finish(w[2], M[2], t[2]);
    finish(w[3], M[3], t[3]);
  }
}

// A partially sorted run, checked on both properties a sort must keep (see sq_prepare): the
// order of the key bits from `shift` up, and the (key, wid) multiset -- its signature into
// sig[2..3], compared on the host with k_sq_keys' sig[0..1].  bad: any order violation.
__global__ void __launch_bounds__(256) k_sq_sorted_check(const uint64_t *key, const uint32_t *wid,
                                                         uint64_t n, uint32_t shift,
                                                         unsigned long long *sig, uint32_t *bad) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  uint64_t s1 = 0, s2 = 0;
  bool ordered = true;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += stride) {
    const uint64_t k = key[i];
    if (i > 0 && (k >> shift) < (key[i - 1] >> shift)) ordered = false;
    sq_sig_add(k, wid[i], s1, s2);
  }
  sq_sig_flush(s1, s2, threadIdx.x & 63, sig + 2);
  if (!ordered) atomicOr(bad, 1u);
}

// ---------------------------------------------------------------------------------------
// The seed-hit list (ovl_seed_hits): every Add_Ref call of Find_Overlaps (:328-370) as
// {query, target, window | dir << 31, target offset}, in the reference's order -- window
// ascending, then the k-mer's chain order (target iid, offset descending).  One wave per
// unit; count pass (out == null) -> per-unit totals, write pass -> hits at unit_base[u].

struct HitArgs {
  ReadsDev R;
  const uint64_t *occ;
  const Unit *units;
  const uint64_t *rbase;
  const Probe *probes;
  uint32_t nunits;
  uint32_t k;
  uint64_t *unit_hits;          // count pass: qualifying hits per unit
  const uint64_t *unit_base;    // write pass: first output slot per unit
  uint4 *out;
};

__global__ void __launch_bounds__(256) k_hitlist(HitArgs A) {
  const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const uint32_t u = blockIdx.x * 4 + wave;
  if (u >= A.nunits) return;
  const Unit un = A.units[u];
  const uint32_t nw = unit_windows(A.R, un, A.k);
  const Probe *pr = A.probes + A.rbase[u];
  const uint32_t a_iid = A.R.first_iid + un.r;
  uint64_t run = A.out ? A.unit_base[u] : 0;
  for (uint32_t base = 0; base < nw; base += 64) {
    const uint32_t o = base + lane;
    uint32_t q = 0, off = 0;
    if (o < nw) {
      const Probe p = pr[o];
      off = p.off;
      q = p.cnt ? qualifying(A.occ, p.off, p.cnt, a_iid) : 0;
    }
    uint32_t incl = q;
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t v = __shfl_up(incl, d);
      if ((int)lane >= d) incl += v;
    }
    if (A.out) {
      uint4 *dst = A.out + run + (incl - q);
      for (uint32_t i = 0; i < q; i++) {
        const uint64_t e = A.occ[off + i];
        dst[i] = make_uint4(a_iid, (uint32_t)(e >> 32), o | (un.dir << 31), (uint32_t)e);
      }
    }
    run += __shfl(incl, 63);
  }
  if (!A.out && lane == 0) A.unit_hits[u] = run;
}

#define OVL_HCAP   256           // staged occurrences per wave
#define OVL_MAXT   128           // targets per pass (2 per lane)
#define OVL_NODE_BLOCK 4096      // nodes a wave claims at a time
#ifndef OVL_CHAIN_OCC
#define OVL_CHAIN_OCC 5          // k_chain waves per SIMD (96 VGPRs: 13 spilled instead of 47 at 6;
                                 // chain 74 -> 62 ms per step at 50k x 10 kb, r04s A/B)
#endif

struct ChainArgs {
  ReadsDev R;
  const uint64_t *occ;
  const Unit *units;
  const uint64_t *rbase;
  const Probe *probes;
  const uint32_t *unit_flags;
  uint32_t nunits;
  uint32_t k;
  uint32_t *unit_next;          // work counter
  Node *pool;                   // working node pool (index 0 = null)
  uint32_t *pool_next;          // bump (starts at 1)
  uint32_t pool_cap;
  Node *pnodes;                 // per-pair node arrays, list order
  uint32_t *pnodes_next;
  uint32_t pnodes_cap;
  PairRec *pairs;
  uint32_t *npairs;
  uint32_t pairs_cap;
  uint32_t *overflow;           // set when a capacity is exceeded (the host grows the
                                // buffers from the counters and runs the batch again)
  const uint32_t *unit_list;    // units to chain (indices into units), null = 0..nunits-1
  // Units with more than OVL_MAXT targets need several passes.  The first launch
  // (big_units != null) chains every unit whose first pass holds all its targets and only
  // lists the others; a second launch chains the listed units with a done set:
  uint32_t *big_units, *n_big;
  uint32_t *done_slots;         // per wave: set slots of the targets finished so far
  uint32_t *done_set;           // per wave: open-addressing set of those targets (0 = empty)
  uint32_t done_cap;            // targets per wave (>= any listed unit's distinct targets)
  uint32_t set_mask;            // set size - 1 (power of two >= 2 done_cap)
  unsigned long long *seed_hits; // qualifying occurrences (Add_Ref calls)
  unsigned long long *prof;     // OVL_CHAIN_PROF builds: wave-cycles per phase (8 counters)
};

#ifdef OVL_CHAIN_PROF
#define CPROF_T(v) const unsigned long long v = __builtin_amdgcn_s_memtime()
#define CPROF_ADD(i, a, b) cp[i] += (b) - (a)
#else
#define CPROF_T(v)
#define CPROF_ADD(i, a, b)
#endif

__device__ __forceinline__ uint32_t done_hash(uint32_t t, uint32_t mask) {
  return (t * 0x85EBCA6Bu) & mask;
}

__device__ __forceinline__ bool done_has(const uint32_t *set, uint32_t mask, uint32_t t) {
  for (uint32_t h = done_hash(t, mask);; h = (h + 1) & mask) {
    const uint32_t v = set[h];
    if (v == t) return true;
    if (v == 0) return false;
  }
}

__device__ __forceinline__ uint32_t done_insert(uint32_t *set, uint32_t mask, uint32_t t) {
  for (uint32_t h = done_hash(t, mask);; h = (h + 1) & mask) {
    const uint32_t old = atomicCAS(&set[h], 0u, t);
    if (old == 0u || old == t) return h;
  }
}

struct SlotState {
  uint32_t t;          // target iid (0 = none)
  int32_t  head;       // list head index (0 = empty list)
  Node     hd;         // the head node itself; pool[head] is stale until flushed
  uint32_t nn;
  int32_t  diag_ct, diag_bgn, diag_end;
  uint32_t consistent;
};

__device__ __forceinline__ void slot_reset(SlotState &s) {
  s.t = 0; s.head = 0; s.nn = 0; s.diag_ct = 0; s.diag_bgn = 0x7fffffff; s.diag_end = 0;
  s.consistent = 1;
  s.hd.Offset = s.hd.Len = s.hd.Start = s.hd.Next = 0;
}

struct WaveAlloc {
  uint32_t *cur;   // LDS: next free node
  uint32_t *end;   // LDS: end of claimed block
};

// Node slots for the lanes active at the call; one LDS-held block per wave.
__device__ __forceinline__ int32_t lane_alloc(WaveAlloc &W, const ChainArgs &A, uint32_t lane) {
  uint64_t act = __ballot(1);
  uint32_t leader = __builtin_ctzll(act);
  uint32_t n = __builtin_popcountll(act);
  uint32_t rank = __builtin_popcountll(act & ((1ull << lane) - 1));
  uint32_t base = 0;
  if (lane == leader) {
    if (*W.cur + n > *W.end) {
      uint32_t b = atomicAdd(A.pool_next, (uint32_t)OVL_NODE_BLOCK);
      if (b + OVL_NODE_BLOCK > A.pool_cap) {
        atomicOr(A.overflow, 1u);
        b = 0xFFFFFFFFu;
      }
      *W.cur = b;
      *W.end = b + OVL_NODE_BLOCK;
    }
    base = *W.cur;
    if (base != 0xFFFFFFFFu) *W.cur = base + n;
  }
  base = __shfl(base, leader);
  if (base == 0xFFFFFFFFu) return -1;
  return (int32_t)(base + rank);
}

// Add_Match (Find_Overlaps.C:79) on the slot's list.  p = occurrence offset in the
// target, o = window offset in the query.  The head node lives in registers (s.hd): the
// common case -- the next window on the head's diagonal -- touches no memory.
__device__ __forceinline__ void add_match(SlotState &s, int32_t p, int32_t o, int32_t k,
                                          Node *pool, WaveAlloc &W, const ChainArgs &A,
                                          uint32_t lane) {
  int32_t new_diag = p - o;
  int32_t diag = 0, expected_start = 0, num_checked = 0;
  if (s.head != 0) {
    expected_start = s.hd.Start + s.hd.Len - k + 1;
    diag = s.hd.Offset - s.hd.Start;
    if (expected_start == o && new_diag == diag) {   // extend the head
      s.hd.Len++;
      return;
    }
    if (expected_start >= o) {
      // walk past the head (repeats: several nodes end at this window)
      bool move_to_front = (expected_start == o);
      num_checked = 1;
      int32_t prev = s.head, cur = s.hd.Next;
      uint32_t guard = 0;
      while (cur > 0 && guard++ <= s.nn) {
        Node nd = pool[cur];
        expected_start = nd.Start + nd.Len - k + 1;
        diag = nd.Offset - nd.Start;
        if (expected_start < o) break;
        if (expected_start == o) {
          if (new_diag == diag) {
            nd.Len++;
            if (move_to_front) {
              if (prev == s.head) s.hd.Next = nd.Next;
              else pool[prev].Next = nd.Next;
              pool[s.head] = s.hd;                   // flush the old head
              nd.Next = s.head;
              s.hd = nd;
              s.head = cur;
            } else {
              pool[cur].Len = nd.Len;
            }
            return;
          }
          move_to_front = true;
        }
        num_checked++;
        prev = cur;
        cur = nd.Next;
      }
    }
    if (num_checked > 0 || abs(diag - new_diag) > 3 || o < expected_start + k - 2)
      s.consistent = 0;
  }
  int32_t idx = lane_alloc(W, A, lane);
  if (idx > 0) {
    if (s.head != 0) pool[s.head] = s.hd;            // flush the old head
    s.hd.Offset = p; s.hd.Len = k; s.hd.Start = o; s.hd.Next = s.head;
    s.head = idx;
    s.nn++;
  }
}

__device__ __forceinline__ uint32_t thash(uint32_t t) {
  t *= 0x9E3779B1u;
  return t >> 25;                 // 7 bits -> 0..127
}

// Walk the slot's list and store it in list order; write its PairRec.
__device__ __forceinline__ void emit_slot(const SlotState &s, uint32_t u, uint32_t uflags,
                                          const ChainArgs &A, uint32_t lane) {
  bool has = s.t != 0 && s.nn > 0;
  uint64_t m = __ballot(has);
  uint32_t np = __builtin_popcountll(m);
  if (np == 0) return;
  uint32_t rank = __builtin_popcountll(m & ((1ull << lane) - 1));
  uint32_t nn = has ? s.nn : 0;
  uint32_t incl = nn;
  for (int d = 1; d < 64; d <<= 1) {
    uint32_t v = __shfl_up(incl, d);
    if ((int)lane >= d) incl += v;
  }
  uint32_t totn = __shfl(incl, 63);
  uint32_t pbase = 0, nbase = 0;
  if (lane == 0) {
    pbase = atomicAdd(A.npairs, np);
    nbase = atomicAdd(A.pnodes_next, totn);
    if (pbase + np > A.pairs_cap || nbase + totn > A.pnodes_cap) atomicOr(A.overflow, 2u);
  }
  pbase = __shfl(pbase, 0);
  nbase = __shfl(nbase, 0);
  if (has && pbase + rank < A.pairs_cap && nbase + incl <= A.pnodes_cap) {
    uint32_t no = nbase + incl - nn;
    uint32_t c = 0;
    A.pnodes[no] = s.hd;                               // the head, from registers
    c = 1;
    for (int32_t x = s.hd.Next; x > 0 && c < nn; c++) {
      Node nd = A.pool[x];
      A.pnodes[no + c] = nd;
      x = nd.Next;
    }
    PairRec pr2;
    pr2.unit = u;
    pr2.tgt = s.t - A.R.first_iid;
    pr2.node_off = no;
    pr2.node_cnt = c;
    pr2.diag_ct = s.diag_ct;
    pr2.diag_bgn = s.diag_bgn;
    pr2.diag_end = s.diag_end;
    // the target's screened ends (bits 1 / 2 of its read flags, set by this hash batch's
    // k_table) are copied here: the pair may be extended after a later batch's build has
    // cleared them (the extension accumulator holds pairs across hash batches)
    pr2.flags = (s.consistent ? 1u : 0u) | (uflags & 6u) |
                ((A.R.flags[pr2.tgt] & 6u) << 2);
    A.pairs[pbase + rank] = pr2;
  }
}

#define WAVE_SYNC()                                          \
  do {                                                       \
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");   \
    __builtin_amdgcn_wave_barrier();                         \
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");   \
  } while (0)

__global__ void __launch_bounds__(256, OVL_CHAIN_OCC) k_chain(ChainArgs A) {
  // a staged occurrence is its target iid (s_ht) and its payload (s_hp: window << 21 |
  // offset in the target, which is < 2^21, AS_MAX_READLEN); the scatter copies payloads into
  // per-target lists (s_sv), so the replay reads one independent LDS word per occurrence
  __shared__ uint32_t s_ht[4][OVL_HCAP];
  __shared__ uint32_t s_hp[4][OVL_HCAP];
  __shared__ uint8_t  s_hs[4][OVL_HCAP];      // its target slot (0..127), 0xFF: none
  __shared__ uint32_t s_sv[4][OVL_HCAP];      // payloads sorted by (slot, staged order)
  __shared__ uint64_t s_lst[4][OVL_HCAP / 64]; // bit i: sorted entry i starts a target's list
  __shared__ uint32_t s_cnt[4][2 * OVL_MAXT]; // per slot: base, running count
  __shared__ uint32_t s_seg[4][65];
  __shared__ uint32_t s_off[4][64];
  __shared__ uint32_t s_tgt[4][OVL_MAXT];
  __shared__ uint32_t s_alloc[4][2];
  __shared__ uint64_t s_lmask[4][OVL_MAXT];   // stable scatter: lanes of each slot
  __shared__ uint32_t s_over[4];
  uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  uint32_t *ht = s_ht[wave];
  uint32_t *hp = s_hp[wave];
  uint8_t *hs = s_hs[wave];
  uint32_t *sv = s_sv[wave];
  uint64_t *lst = s_lst[wave];
  uint32_t *cnt = s_cnt[wave];
  uint32_t *seg = s_seg[wave];
  uint32_t *soff = s_off[wave];
  uint32_t *tgt = s_tgt[wave];
  uint64_t *lmask = s_lmask[wave];
  for (uint32_t i = lane; i < OVL_MAXT; i += 64) lmask[i] = 0;
  WaveAlloc W;
  W.cur = &s_alloc[wave][0];
  W.end = &s_alloc[wave][1];
  if (lane == 0) { *W.cur = 0; *W.end = 0; }
  const int32_t k = (int32_t)A.k;
  uint32_t gw = blockIdx.x * 4 + wave;
  const bool first_launch = A.big_units != nullptr;
  uint32_t *done_list = first_launch ? nullptr : A.done_slots + (size_t)gw * A.done_cap;
  uint32_t *done_set = first_launch ? nullptr : A.done_set + (size_t)gw * (A.set_mask + 1);
  unsigned long long nhits = 0;
#ifdef OVL_CHAIN_PROF
  // 0 probe records + qualifying + scan, 1 staging, 2 target discovery, 3 slot scan +
  // scatter, 4 replay, 5 emit, 6 chunks, 7 staged occurrences
  unsigned long long cp[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#endif

  for (;;) {
    uint32_t ui = 0;
    if (lane == 0) ui = atomicAdd(A.unit_next, 1u);
    ui = __shfl(ui, 0);
    if (ui >= A.nunits) break;
    const uint32_t u = A.unit_list ? A.unit_list[ui] : ui;
    Unit un = A.units[u];
    uint32_t nw = unit_windows(A.R, un, A.k);
    const Probe *pr = A.probes + A.rbase[u];
    uint32_t uflags = A.unit_flags[u];
    uint32_t ndone = 0;
    uint32_t a_iid = A.R.first_iid + un.r;

    for (uint32_t pass = 0;; pass++) {
      SlotState s0, s1;
      slot_reset(s0);
      slot_reset(s1);
      for (uint32_t i = lane; i < OVL_MAXT; i += 64) tgt[i] = 0;
      if (lane == 0) s_over[wave] = 0;
      WAVE_SYNC();

      for (uint32_t base = 0; base < nw; base += 64) {
        CPROF_T(t_a);
        uint32_t o = base + lane;
        Probe p;
        p.off = 0; p.cnt = 0;
        if (o < nw) {
          p = pr[o];
          // only the qualifying prefix (target iid > query, Find_Overlaps.C:328) is staged:
          // lists are iid-descending, so it is found by a short search of the list itself
          if (p.cnt) p.cnt = qualifying(A.occ, p.off, p.cnt, a_iid);
        }
        uint32_t incl = p.cnt;                       // wave inclusive scan
        for (int d = 1; d < 64; d <<= 1) {
          uint32_t v = __shfl_up(incl, d);
          if ((int)lane >= d) incl += v;
        }
        uint32_t total = __shfl(incl, 63);
        CPROF_T(t_b);
        CPROF_ADD(0, t_a, t_b);
#ifdef OVL_CHAIN_PROF
        cp[6]++;
        cp[7] += total;
#endif
        if (total == 0) continue;
        seg[lane] = incl - p.cnt;
        soff[lane] = p.off;
        if (lane == 63) seg[64] = total;
        WAVE_SYNC();

        for (uint32_t p0 = 0; p0 < total; p0 += OVL_HCAP) {
          CPROF_T(t_c);
          uint32_t p1 = p0 + OVL_HCAP < total ? p0 + OVL_HCAP : total;
          // stage occurrences p0..p1 of this chunk, in order (ordered compaction)
          for (uint32_t idx = p0 + lane; idx < p1; idx += 64) {
            uint32_t lo = 0, hi = 64;            // last j with seg[j] <= idx
            while (hi - lo > 1) {
              uint32_t mid = (lo + hi) >> 1;
              if (seg[mid] <= idx) lo = mid; else hi = mid;
            }
            const uint64_t oc = A.occ[soff[lo] + (idx - seg[lo])];
            ht[idx - p0] = (uint32_t)(oc >> 32);
            hp[idx - p0] = (lo << 21) | (uint32_t)oc;
          }
          for (uint32_t i = lane; i < 2 * OVL_MAXT; i += 64) cnt[i] = 0;
          if (lane < OVL_HCAP / 64) lst[lane] = 0;
          WAVE_SYNC();
          CPROF_T(t_d);
          CPROF_ADD(1, t_c, t_d);
          // discover targets (LDS open-addressing set, 128 slots); remember each staged
          // occurrence's slot and count occurrences per slot
          for (uint32_t idx = p0 + lane; idx < p1; idx += 64) {
            uint32_t t = ht[idx - p0];
            uint8_t slot = 0xFF;
            if (t > a_iid) {                     // Find_Overlaps.C:328
              if (pass == 0 && first_launch) nhits++;
              const bool skip = ndone && done_has(done_set, A.set_mask, t);
              if (!skip) {
                uint32_t h = thash(t);
                bool placed = false;
                for (uint32_t probe = 0; probe < OVL_MAXT; probe++) {
                  uint32_t cur = tgt[h];
                  if (cur == t) { placed = true; break; }
                  if (cur == 0) {
                    uint32_t old = atomicCAS(&tgt[h], 0u, t);
                    if (old == 0 || old == t) { placed = true; break; }
                  }
                  h = (h + 1) & (OVL_MAXT - 1);
                }
                if (placed) { slot = (uint8_t)h; atomicAdd(&cnt[h], 1u); }
                else atomicOr(&s_over[wave], 1u);
              }
            }
            hs[idx - p0] = slot;
          }
          WAVE_SYNC();
          CPROF_T(t_e);
          CPROF_ADD(2, t_d, t_e);
          // slot bases: exclusive scan over the 128 counts (two per lane)
          {
            uint32_t c0 = cnt[2 * lane], c1 = cnt[2 * lane + 1];
            uint32_t incl = c0 + c1;
            for (int d = 1; d < 64; d <<= 1) {
              uint32_t v = __shfl_up(incl, d);
              if ((int)lane >= d) incl += v;
            }
            uint32_t ex = incl - c0 - c1;
            WAVE_SYNC();
            cnt[2 * lane] = ex;                    // base of slot 2*lane
            cnt[2 * lane + 1] = ex + c0;           // base of slot 2*lane+1
            if (c0) atomicOr((unsigned long long *)&lst[ex >> 6], 1ull << (ex & 63));
            if (c1) atomicOr((unsigned long long *)&lst[(ex + c0) >> 6], 1ull << ((ex + c0) & 63));
            cnt[OVL_MAXT + 2 * lane] = 0;          // running counts
            cnt[OVL_MAXT + 2 * lane + 1] = 0;
          }
          WAVE_SYNC();
          // stable scatter: within each 64-entry step a lane's rank among the lanes of its
          // slot is the popcount of the lower lanes in the slot's lane mask (one LDS OR per
          // lane), so every slot's list keeps the staged (window, chain) order
          for (uint32_t b0 = p0; b0 < p1; b0 += 64) {
            uint32_t idx = b0 + lane;
            uint32_t slot = (idx < p1) ? hs[idx - p0] : 0xFFu;
            const bool has = slot != 0xFFu;
            if (has) atomicOr(&lmask[slot], 1ull << lane);
            WAVE_SYNC();
            uint64_t mk = 0;
            if (has) {
              mk = lmask[slot];
              uint32_t rank = __builtin_popcountll(mk & ((1ull << lane) - 1));
              sv[cnt[slot] + cnt[OVL_MAXT + slot] + rank] = hp[idx - p0];
            }
            WAVE_SYNC();
            if (has && lane == (uint32_t)__builtin_ctzll(mk)) {   // the slot's first lane
              cnt[OVL_MAXT + slot] += __builtin_popcountll(mk);
              lmask[slot] = 0;
            }
            WAVE_SYNC();
          }
          WAVE_SYNC();
          // Runs (see replay below): entry i of a target's list only extends the head node
          // when the list's previous entry is the window before on the same diagonal and
          // both are their windows' only occurrence of the target.  The number of such
          // entries following entry i goes into the payload's top 5 bits (saturating: a
          // longer run continues from its 31st entry); found per 64-entry block by a ballot
          // of the run breaks, blocks from the last, carrying the next break.  A block
          // reads its neighbours before any lane writes, and the block after it is done.
          {
            const uint32_t tn = p1 - p0;
            uint32_t next_break = tn;                  // first break at or after the block
            for (int32_t b0 = (int32_t)((tn - 1) & ~63u); b0 >= 0; b0 -= 64) {
              const uint32_t i = (uint32_t)b0 + lane;
              // the list starts around the block: bit 64 + l of (prev, cur) = entry b0 + l
              const uint64_t lc = lst[b0 >> 6];
              const uint64_t lp = b0 ? lst[(b0 >> 6) - 1] : 0ull;
              const uint64_t ln = (uint32_t)b0 + 64 < OVL_HCAP ? lst[(b0 >> 6) + 1] : 0ull;
              const bool st_i = (lc >> lane) & 1ull;
              const bool st_m1 = lane ? (lc >> (lane - 1)) & 1ull : (lp >> 63) & 1ull;
              const bool st_p1 = lane < 63 ? (lc >> (lane + 1)) & 1ull : ln & 1ull;
              // neighbours through lane exchanges (the block's entries) and, at its edges,
              // LDS reads of the entries around it (the block after it already holds its
              // run bits, masked off)
              uint32_t v = i < tn ? (sv[i] & 0x7FFFFFFu) : 0u;
              const uint32_t vm1 = lane ? (uint32_t)__shfl_up((int)v, 1)
                                        : (i > 0 ? (sv[i - 1] & 0x7FFFFFFu) : 0u);
              uint32_t vm2 = (uint32_t)__shfl_up((int)v, 2);
              if (lane < 2) vm2 = i >= 2 ? (sv[i - 2] & 0x7FFFFFFu) : 0u;
              uint32_t vp1 = (uint32_t)__shfl_down((int)v, 1);
              if (lane == 63) vp1 = i + 1 < tn ? (sv[i + 1] & 0x7FFFFFFu) : 0u;
              bool cont = false;
              if (i < tn && i > 0 && !st_i) {
                const uint32_t o = v >> 21, ow = vm1 >> 21;
                const int32_t dg = (int32_t)(v & 0x1FFFFFu) - (int32_t)o;
                const int32_t dw = (int32_t)(vm1 & 0x1FFFFFu) - (int32_t)ow;
                cont = ow + 1 == o && dg == dw &&
                       (i + 1 >= tn || st_p1 || (vp1 >> 21) != o) &&
                       (i < 2 || st_m1 || (vm2 >> 21) != ow);
              }
              const uint64_t brk = __builtin_amdgcn_ballot_w64(!cont);   // lanes past tn break
              const uint64_t above = brk & ~((2ull << lane) - 1ull);
              const uint32_t nb = above ? (uint32_t)b0 + (uint32_t)__builtin_ctzll(above) : next_break;
              if (i < tn) {
                const uint32_t r = nb - i - 1;
                sv[i] = v | ((r < 31 ? r : 31u) << 27);
              }
              if (brk) next_break = (uint32_t)b0 + (uint32_t)__builtin_ctzll(brk);
            }
            WAVE_SYNC();
          }
          WAVE_SYNC();
          CPROF_T(t_f);
          CPROF_ADD(3, t_e, t_f);
          uint32_t t0 = tgt[lane], t1 = tgt[lane + 64];
          if (t0 != s0.t) { slot_reset(s0); s0.t = t0; }
          if (t1 != s1.t) { slot_reset(s1); s1.t = t1; }
          // replay Add_Ref / Add_Match per target over its own occurrences, in order; the
          // next payload is loaded before the current one is applied (no LDS round trip on
          // the loop's dependency chain)
          {
            // An entry followed by rl run entries: once it is applied, if the head node is
            // the one holding it (expected next window o + 1 on its diagonal), each run entry
            // would take Add_Match's first branch -- Len++ -- so the run is applied at once:
            // Len += rl, diag_ct += rl, diag_end = the run's last window (windows ascend).
            // Otherwise the next entry is applied one by one as before.
            auto replay = [&](SlotState &st, uint32_t b, uint32_t n) {
              for (uint32_t i = 0; i < n;) {
                const uint32_t cur = sv[b + i];
                const uint32_t r = cur >> 27;
                const int32_t pp = (int32_t)(cur & 0x1FFFFFu);
                const int32_t o_j = (int32_t)(base + ((cur >> 21) & 63u));
                st.diag_ct++;                                 // Add_Ref (:203-206)
                if (st.diag_bgn > o_j) st.diag_bgn = o_j;
                if (st.diag_end < o_j) st.diag_end = o_j;
                add_match(st, pp, o_j, k, A.pool, W, A, lane);
                i++;
                if (r && st.head != 0 && st.hd.Start + st.hd.Len - k == o_j &&
                    st.hd.Offset - st.hd.Start == pp - o_j) {
                  st.hd.Len += (int32_t)r;
                  st.diag_ct += (int32_t)r;
                  const int32_t o_l = (int32_t)(base + ((sv[b + i + r - 1] >> 21) & 63u));
                  if (st.diag_end < o_l) st.diag_end = o_l;
                  i += r;
                }
              }
            };
            replay(s0, cnt[lane], cnt[OVL_MAXT + lane]);
            replay(s1, cnt[lane + 64], cnt[OVL_MAXT + lane + 64]);
          }
          {
            CPROF_T(t_g);
            CPROF_ADD(4, t_f, t_g);
          }
          WAVE_SYNC();
        }
      }

      bool over = s_over[wave] != 0;
      if (over && first_launch) {
        // more targets than one pass holds: chained by the second launch (its nodes here
        // are abandoned; the pool is sized for that)
        if (lane == 0) A.big_units[atomicAdd(A.n_big, 1u)] = u;
        break;
      }
      CPROF_T(t_h);
      emit_slot(s0, u, uflags, A, lane);
      emit_slot(s1, u, uflags, A, lane);
      {
        CPROF_T(t_i);
        CPROF_ADD(5, t_h, t_i);
      }
      if (!over) break;
      // targets the 128-slot table could not hold: another pass over the unit, skipping
      // the targets emitted so far (done set)
      uint64_t m0 = __ballot(s0.t != 0), m1 = __ballot(s1.t != 0);
      uint32_t c0 = __builtin_popcountll(m0), c1 = __builtin_popcountll(m1);
      if (ndone + c0 + c1 > A.done_cap) {                // the host's bound was wrong
        if (lane == 0) atomicOr(A.overflow, 4u);
        break;
      }
      if (s0.t) done_list[ndone + __builtin_popcountll(m0 & ((1ull << lane) - 1))] =
          done_insert(done_set, A.set_mask, s0.t);
      if (s1.t) done_list[ndone + c0 + __builtin_popcountll(m1 & ((1ull << lane) - 1))] =
          done_insert(done_set, A.set_mask, s1.t);
      ndone += c0 + c1;
      __threadfence_block();
      WAVE_SYNC();
    }
    if (ndone) {                                          // empty the set for the next unit
      for (uint32_t q = lane; q < ndone; q += 64) done_set[done_list[q]] = 0u;
      __threadfence_block();
      WAVE_SYNC();
    }
  }
  for (int d = 32; d > 0; d >>= 1) nhits += __shfl_xor(nhits, d);
  if (lane == 0 && nhits) atomicAdd(A.seed_hits, nhits);
#ifdef OVL_CHAIN_PROF
  if (lane == 0 && A.prof)
    for (int i = 0; i < 8; i++) atomicAdd(&A.prof[i], cp[i]);
#endif
}

}  // namespace ovl
