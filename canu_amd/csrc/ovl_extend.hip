// ovl_extend.hip -- seed extension and overlap output (Process_Matches replacement).
//
// Reference:
//   src/overlapInCore/overlapInCore-Process_String_Overlaps.C
//     Process_String_Olaps (:687)  per target: --minkmers filter, then Process_Matches
//     Process_Matches      (:400)  hopeless check; repeatedly extend the longest match,
//                                   keep up to 3 distinct overlaps, drop matches that lie on
//                                   the alignment; Combine_Into_One_Olap / Merge / Choose
//   src/overlapInCore/liboverlap/prefixEditDistance-extend.C:86   Extend_Alignment
//   src/overlapInCore/liboverlap/prefixEditDistance-forward.C:103 forward (+Set_Right_Delta)
//   src/overlapInCore/liboverlap/prefixEditDistance-reverse.C:119 reverse (+Set_Left_Delta)
//   src/overlapInCore/overlapInCore-Output.C:75/:253               the ovOverlap record
//
// One wave per (query, orientation, target) pair.  The greedy O(ND) edit distance keeps
// its structure: error level e is a row over diagonals [Left, Right]; the 64 lanes compute
// 64 diagonals of a row at once (each lane slides its diagonal 32 bases per step on the
// 2-bit packed strands), the row's end test / Edit_Match_Limit pruning / longest-row
// bookkeeping are wave ballots and reductions.  Rows are stored band-compact per wave so
// the traceback can stage 16-row windows in LDS and walk them there.
#include "ovl_common.h"

namespace ovl {

struct ExtendArgs {
  ReadsDev R;
  const Unit *units;
  const PairRec *pairs;
  uint32_t npairs;
  const uint32_t *npairs_dev;   // non-null: the pair count is there (an earlier launch's defers)
  int32_t restore;              // the list holds deferred pairs: undo their node removals
  Node *pnodes;                 // Len < 0 marks a node removed from its list
  uint32_t *pair_next;
  const uint32_t *list;   // non-null: process pairs[list[0 .. npairs)] instead of pairs[0 .. npairs)
  uint32_t *defer;        // staged kernel: pairs with 'n' bases go here for the generic kernel
  uint32_t *ndefer;
  const int32_t *error_bound;   // ceil(i * maxErate), i <= AS_MAX_READLEN
  const int32_t *match_limit;   // Edit_Match_Limit[e]
  int32_t max_errors;
  double  branch_match_value;
  double  min_branch_tail_slope;
  int32_t min_branch_end_dist;
  int32_t partial, unique, min_olap_len, use_hopeless, k;
  uint64_t filter_by_kmer_count;
  double  minkmer_exp;          // exp(-k * maxErate), host libm
  int32_t *rows;                // per wave: band-compact edit rows
  uint64_t rows_cap;            // ints per wave
  int32_t *rowdir;              // per wave: (offset, lo) per error level
  int32_t *deltas;              // per wave: stack | right | left
  int32_t e_cap;                // error levels the scratch holds
  int32_t sw_words;             // staged kernel: LDS words per strand (even)
  Rec *out;
  uint32_t *nout;
  uint32_t out_cap;
  unsigned long long *stats;    // 0 without 1 with 2 skipped 3 multi 4 total 5 contained 6 dovetail
                                // (7 seed hits: k_chain) 8 bad short window 9 bad long window
  int32_t window;               // -w: Use_Window_Filter
  uint32_t *overflow;
  unsigned long long *dbg;      // optional counters (null: off)
  // -l (Frag_Olap_Limit), the ordered kernel: one wave per unit runs its pairs one after
  // another in the reference's order, counting the unit's A / B overlaps
  // (Process_String_Overlaps.C:721-790)
  uint64_t olim;
  uint32_t nunits;
  const uint32_t *useg;         // unit u's pairs: [useg[u], useg[u+1]) of ord_slot / ord_diag
  const uint32_t *ord_slot;     // String_Olap_Space order (Add_Ref's hash slots)
  const uint32_t *ord_diag;     // By_Diag_Sum order, ties in String_Olap_Space order (stable)
  const uint64_t *dkey;         // per pair: its average diagonal as an order-preserving key
};

// debug counters (dbg != null): 0 ped calls 1 rows 2 chunks 3 slide words 4 tb steps
// 5 process iterations 6 ped cycles 7 tb cycles 8 pairs 9 max rows in one ped

#define TB_ROWS 16
#define TB_W    (2 * TB_ROWS + 3)

struct PedOut {
  int32_t err;
  int32_t a_len, t_len;    // extents in A and T (positive)
  int32_t leftover;
  int32_t mte;
  int32_t nd;              // deltas produced
  int32_t ovf;             // register window overflow: the pair goes to the generic kernel
};

// Orders this wave's global-memory accesses across lanes (lane 0 writes, others read, or
// the reverse): wait for the wave's outstanding vector memory operations.
__device__ __forceinline__ void vm_sync() {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
}

__device__ __forceinline__ void wave_argmax(int32_t &v, int32_t &d) {
  for (int s = 32; s > 0; s >>= 1) {
    int32_t v2 = __shfl_xor(v, s), d2 = __shfl_xor(d, s);
    if (v2 > v || (v2 == v && d2 < d)) { v = v2; d = d2; }
  }
}

// the register kernel's Edit_Match_Limit: a block-shared LDS copy (r4 measured a global
// table read through the constant address space, which frees the LDS for 32 waves per CU:
// no faster)
typedef const __attribute__((address_space(3))) int32_t ml_t;

struct WaveMem {
  int32_t *rows;      // global: band-compact log of every row (read by the traceback)
  int32_t *rowdir;    // global: (offset, lo) per row
  lds_i32 *lrow;      // LDS: two row buffers of wcap ints (previous / current row)
  int32_t  wcap;
  lds_i32 *tbw;       // LDS: traceback window
  lds_i32 *ldc;       // LDS: Left_Delta cache for Lies_On_Alignment
  int32_t  ldcap;
  const lds_i32 *mlim;  // LDS: Edit_Match_Limit[0 .. e_cap+1], shared by the block
  ml_t    *rmlim;       // the register kernel's Edit_Match_Limit (the LDS copy)
};

__device__ __forceinline__ void lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

#define OVL_REG_CHUNKS 2      // row chunks (x64 diagonals) kept in registers

// Greedy prefix edit distance of A against a prefix of T (m <= n).
// DIR=+1: A[i] = A.w[a0+i], T[i] = T.w[t0+i]   (forward.C:103)
// DIR=-1: A[i] = A.w[a0-i], T[i] = T.w[t0-i]   (reverse.C:119)
// Row e (error level) is computed for all its diagonals at once, 64 per wave step; the
// end test, the Edit_Match_Limit pruning (both sides) and the running longest row are
// wave ballots / reductions over values that stay in registers.  The row is kept in LDS
// for the next level and appended to a global log the traceback reads.
template <int DIR, typename SS>
__device__ __forceinline__ int32_t ped_slide(const SS &A, int32_t a0, int32_t m, const SS &T,
                                             int32_t t0, int32_t n, int32_t r, int32_t d) {
  int32_t lim = m - r;
  int32_t l2 = n - r - d;
  if (l2 < lim) lim = l2;
  if (lim <= 0) return 0;
  if (DIR > 0) return slide_fwd(A, a0 + r, T, t0 + r + d, lim);
  return slide_bwd(A, a0 - r, T, t0 - r - d, lim);
}

// Inclusive prefix sum over the 64 lanes (DPP row shifts, then row broadcasts).
__device__ __forceinline__ int32_t wave_incl_scan(int32_t v) {
  v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, true);
  v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, true);
  v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, true);
  v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, true);
  v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xa, 0xf, false);
  v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xc, 0xf, false);
  return v;
}

// Max over the 64 lanes: DPP row shifts within 16-lane rows, then row broadcasts.
__device__ __forceinline__ int32_t wave_max(int32_t v) {
  const int32_t NEG = (int32_t)0x80000000;
  int32_t t;
  t = __builtin_amdgcn_update_dpp(NEG, v, 0x111, 0xf, 0xf, false); v = v > t ? v : t;
  t = __builtin_amdgcn_update_dpp(NEG, v, 0x112, 0xf, 0xf, false); v = v > t ? v : t;
  t = __builtin_amdgcn_update_dpp(NEG, v, 0x114, 0xf, 0xf, false); v = v > t ? v : t;
  t = __builtin_amdgcn_update_dpp(NEG, v, 0x118, 0xf, 0xf, false); v = v > t ? v : t;
  t = __builtin_amdgcn_update_dpp(NEG, v, 0x142, 0xa, 0xf, false); v = v > t ? v : t;
  t = __builtin_amdgcn_update_dpp(NEG, v, 0x143, 0xc, 0xf, false); v = v > t ? v : t;
  return __builtin_amdgcn_readlane(v, 63);
}

// Set_Right_Delta / Set_Left_Delta walk (forward.C:51, reverse.C:49) over the row log:
// rows are staged into LDS 16 at a time, lane 0 walks them.  Row e of the log holds the
// values of diagonals [lo, lo + width) with width = next row's offset - this row's.
__device__ __forceinline__ void ped_traceback(const WaveMem &WM, int32_t tb_e, int32_t tb_d,
                                              int32_t *dst, uint32_t lane, int32_t &last_out,
                                              int32_t &nd_out) {
  int32_t *rows = WM.rows, *rowdir = WM.rowdir;
  lds_i32 *tbw = WM.tbw;
  vm_sync();                                  // the row log is complete
  int32_t d = tb_d;
  int32_t last;
  {
    int32_t o0 = rowdir[2 * tb_e], l0 = rowdir[2 * tb_e + 1];
    last = rows[o0 + d - l0];
  }
  int32_t nd = 0;
  for (int32_t kh = tb_e; kh >= 1; kh -= TB_ROWS) {
    int32_t kl = kh - TB_ROWS + 1;
    if (kl < 1) kl = 1;
    int32_t dc = d;
    int32_t nrows = kh - kl + 1;
    for (int32_t i = lane; i < nrows * TB_W; i += 64) {
      int32_t rr = i / TB_W, w = i - rr * TB_W;
      int32_t row = kl - 1 + rr;
      int32_t ro = rowdir[2 * row], rl = rowdir[2 * row + 1];
      int32_t rwidth = rowdir[2 * (row + 1)] - ro;
      int32_t dd = dc - (TB_ROWS + 1) + w;
      int32_t idx = dd - rl;
      tbw[i] = (idx >= 0 && idx < rwidth) ? rows[ro + idx] : -3;
    }
    lds_sync();
    if (lane == 0) {
      for (int32_t kk = kh; kk >= kl; kk--) {
        const lds_i32 *prow = tbw + (kk - 1 - (kl - 1)) * TB_W - (dc - (TB_ROWS + 1));
        int32_t from = d, mx = 1 + prow[d], j;
        if ((j = prow[d - 1]) > mx) { from = d - 1; mx = j; }
        if ((j = 1 + prow[d + 1]) > mx) { from = d + 1; mx = j; }
        if (from == d - 1) {
          dst[nd++] = mx - last - 1;
          d--;
          last = prow[from];
        } else if (from == d + 1) {
          dst[nd++] = last - (mx - 1);
          d++;
          last = prow[from];
        }
      }
    }
    d = __shfl(d, 0);
    last = __shfl(last, 0);
    nd = __shfl(nd, 0);
    lds_sync();
  }
  last_out = last;
  nd_out = nd;
}

// GR (global rows): the error limit is too large for the two LDS row buffers and the LDS
// Edit_Match_Limit table, so row e-1 is read back from the global row log itself (which
// holds the same values and sentinels) and the table from global memory.
template <int DIR, typename SS, bool GR>
__device__ __attribute__((noinline)) PedOut wave_ped(const ExtendArgs &X, const SS &A, int32_t a0, int32_t m,
                           const SS &T, int32_t t0, int32_t n, int32_t limit,
                           const WaveMem &WM, int32_t *dst, uint32_t lane) {
  int32_t *rows = WM.rows, *rowdir = WM.rowdir;
  typedef typename std::conditional<GR, int32_t, lds_i32>::type row_t;
  const int32_t NONE = 0x7fffffff, NEG = (int32_t)0x80000000;
  PedOut out;
  out.leftover = 0;
  out.nd = 0;
  out.ovf = 0;
  unsigned long long dbg_rows = 0, dbg_chunks = 0;
  unsigned long long t_start = X.dbg ? __builtin_amdgcn_s_memtime() : 0;
  // the scratch is sized for e_cap rows of width <= 2e+5 (ovl_api.hip), so the row loop
  // needs no capacity checks
  if (limit > X.e_cap - 2) {
    if (lane == 0) atomicOr(X.overflow, 8u);
    out.err = 0; out.a_len = 0; out.t_len = 0; out.mte = 0; out.nd = -1;
    return out;
  }

  int32_t row0 = (m > 0) ? ped_slide<DIR>(A, a0, m, T, t0, n, 0, 0) : 0;
  row0 = __builtin_amdgcn_readfirstlane(row0);
  row_t *lbuf0, *lbuf1;
  if constexpr (GR) { lbuf0 = nullptr; lbuf1 = nullptr; }
  else              { lbuf0 = WM.lrow; lbuf1 = WM.lrow + WM.wcap; }
  if (lane == 0) {
    rowdir[0] = 0; rowdir[1] = -2; rows[2] = row0;
    if constexpr (!GR) lbuf0[2] = row0;
  }
  if constexpr (GR) vm_sync(); else lds_sync();
  if (row0 == m) {
    out.err = 0; out.a_len = m; out.t_len = m; out.mte = 1;
    out.leftover = m;          // reverse(): Leftover = m on an exact match
    out.nd = -1;               // no traceback
    return out;
  }

  double  max_score = 0.0;
  int32_t max_score_len = 0, max_score_best_d = 0, max_score_best_e = 0;
  int32_t best_d = 0, best_e = 0, longest = 0;
  int32_t left = 0, right = 0, cursor = 5;
  int32_t prev_off = 0, prev_lo = -2;
  int32_t tb_e = -1, tb_d = 0;
  bool finished = false;
  row_t *lprev = lbuf0;
  const double bmv = X.branch_match_value;
  const bool partial = X.partial != 0;
  const int32_t mbed = X.min_branch_end_dist;
  const double mbts = X.min_branch_tail_slope;

  for (int32_t e = 1; e <= limit; e++) {
    int32_t ML;
    if constexpr (GR) ML = __builtin_amdgcn_readfirstlane(X.match_limit[e]);
    else              ML = WM.mlim[e];         // LDS: no global load in the row loop
    left = (left - 1 > -e) ? left - 1 : -e;
    right = (right + 1 < e) ? right + 1 : e;
    const int32_t lo = left - 2, width = right - left + 5, off = cursor;
    cursor += width;
    if (GR && (uint64_t)cursor > X.rows_cap) {   // past the wave's row log: refuse loudly
      if (lane == 0) atomicOr(X.overflow, 32u);
      out.err = 0; out.a_len = 0; out.t_len = 0; out.mte = 0; out.nd = -1;
      return out;
    }
    // sentinels around the new band in row e-1 (LDS copy and the traceback log)
    if (lane < 4) {
      int32_t d = (lane == 0) ? left : (lane == 1) ? left - 1 : (lane == 2) ? right : right + 1;
      if constexpr (!GR) lprev[d - prev_lo] = -2;
      rows[prev_off + d - prev_lo] = -2;
    }
    if (lane == 0) { rowdir[2 * e] = off; rowdir[2 * e + 1] = lo; }
    int32_t *glog = rows + off - lo;
    row_t *lcur;
    const row_t *prev;                          // index by diagonal
    row_t *cur;
    if constexpr (GR) {
      lcur = nullptr;
      prev = rows + prev_off - prev_lo;
      cur = glog;
      vm_sync();
    } else {
      lcur = (e & 1) ? lbuf1 : lbuf0;
      prev = lprev - prev_lo;
      cur = lcur - lo;
      lds_sync();
    }

    // ---- the row: 64 diagonals per step ------------------------------------------
    int32_t end_d = NONE, end_row = 0, nl = NONE, nr = NEG;
    int32_t rv0 = NEG, rv1 = NEG;
    int32_t nch = 0;
    for (int32_t c = left; c <= right; c += 64) {
      const int32_t d = c + (int32_t)lane;
      const bool act = d <= right;
      const int32_t dd = act ? d : right;
      int32_t r = 1 + prev[dd];
      int32_t j = prev[dd - 1];
      r = j > r ? j : r;
      j = 1 + prev[dd + 1];
      r = j > r ? j : r;
      if (act && r < m && r + d < n) r += ped_slide<DIR>(A, a0, m, T, t0, n, r, d);
      if (act) {
        if constexpr (!GR) cur[d] = r;
        glog[d] = r;
      }
      if (nch == 0) rv0 = act ? r : NEG;
      if (nch == 1) rv1 = act ? r : NEG;
      nch++;
      const uint64_t endm = __ballot(act && (r == m || r + d == n));
      // pruning test (forward.C:236-252): left and right use the same predicate
      const uint64_t km = __ballot(act && ((d < 0) ? !(r < ML) : !(r + d < ML)));
      if (endm) {
        const int32_t l = (int32_t)__builtin_ctzll(endm);
        end_d = c + l;
        end_row = __builtin_amdgcn_readlane(r, l);
        break;
      }
      if (km) {
        if (nl == NONE) nl = c + (int32_t)__builtin_ctzll(km);
        nr = c + 63 - (int32_t)__builtin_clzll(km);
      }
    }
    dbg_rows++;
    dbg_chunks += nch;
    if constexpr (GR) vm_sync(); else lds_sync();

    if (end_d != NONE) {
      double  score = end_row * bmv - e;
      int32_t tail_len = end_row - max_score_len;
      double  slope = (double)(max_score - score) / tail_len;
      bool    abort_here = false;
      if (partial && score < max_score) abort_here = true;
      if (e > mbed / 2 && tail_len >= mbed && slope >= mbts) abort_here = true;
      if (abort_here) {
        out.err = max_score_best_e;
        out.a_len = max_score_len;
        out.t_len = max_score_len + max_score_best_d;
        out.mte = 0;
        tb_e = max_score_best_e; tb_d = max_score_best_d;
      } else {
        int32_t d = end_d;
        // forward.C:212 -- force the last error to be a mismatch rather than an insertion
        if (DIR > 0 && end_row == m && 1 + prev[d + 1] == end_row && d < right) {
          d++;
          if (lane == 0) {
            if constexpr (!GR) cur[d] = end_row;
            glog[d] = end_row;
          }
        }
        out.err = e;
        out.a_len = end_row;
        out.t_len = end_row + d;
        out.mte = 1;
        tb_e = e; tb_d = d;
      }
      finished = true;
      break;
    }

    if (nl == NONE) break;                     // Left > Right
    left = nl;
    right = nr;

    // longest row over the pruned band, first diagonal on ties (forward.C:256-261)
    int32_t bv = NEG, bd = NONE;
    for (int32_t ci = 0; ci < nch; ci++) {
      const int32_t c = lo + 2 + 64 * ci;
      if (c > right) break;
      if (c + 63 < left) continue;
      const int32_t d = c + (int32_t)lane;
      int32_t v = (ci == 0) ? rv0 : (ci == 1) ? rv1 : cur[d <= right ? d : right];
      v = (d >= left && d <= right) ? v : NEG;
      const int32_t cm = wave_max(v);
      if (cm > bv) {
        bv = cm;
        bd = c + (int32_t)__builtin_ctzll(__ballot(v == cm));
      }
    }
    if (bv > longest) { longest = bv; best_d = bd; best_e = e; }
    double score = longest * bmv - e;
    if (score > max_score) {
      max_score = score;
      max_score_len = longest;
      max_score_best_d = best_d;
      max_score_best_e = best_e;
    }
    prev_off = off;
    prev_lo = lo;
    if constexpr (!GR) lprev = lcur;
  }
  if (!finished) {
    out.err = max_score_best_e;
    out.a_len = max_score_len;
    out.t_len = max_score_len + max_score_best_d;
    out.mte = 0;
    tb_e = max_score_best_e; tb_d = max_score_best_d;
  }

  unsigned long long t_mid = X.dbg ? __builtin_amdgcn_s_memtime() : 0;
  int32_t last = 0, nd = 0;
  ped_traceback(WM, tb_e, tb_d, dst, lane, last, nd);
  out.leftover = last;
  out.nd = nd;
  if (X.dbg && lane == 0) {
    unsigned long long t_end = __builtin_amdgcn_s_memtime();
    atomicAdd(&X.dbg[0], 1ull);
    atomicAdd(&X.dbg[1], dbg_rows);
    atomicAdd(&X.dbg[2], dbg_chunks);
    atomicAdd(&X.dbg[4], (unsigned long long)tb_e);
    atomicAdd(&X.dbg[6], t_mid - t_start);
    atomicAdd(&X.dbg[7], t_end - t_mid);
    atomicMax(&X.dbg[9], dbg_rows);
  }
  return out;
}

// ---- register-resident rows (the staged kernel) -------------------------------------
// Row e-1 lives in OVL_RJ registers per lane: lane l of chunk j holds diagonal B+64j+l, the
// window [B, B + 64*OVL_RJ) is re-centred through LDS when the band drifts out of it (rare).
// Every value outside the surviving band [pl, pr] is -2, which is exactly the sentinel
// forward.C:170 writes around the band, so the neighbours d-1 / d+1 come from DPP wave
// shifts with no LDS round trip.  Row e is logged band-compact as [nl-2, nr+2] (masked)
// for the traceback.
#ifndef OVL_RJ
#define OVL_RJ 8
#endif
#define OVL_LOGW 512             // cells per logged row (>= 64 * OVL_RJ, a power of two)
static_assert(64 * OVL_RJ <= OVL_LOGW, "the row log's stripe holds the register window");

#ifdef OVL_PROFILE
#define PROF_T(v) unsigned long long v = __builtin_amdgcn_s_memtime()
#define PROF_ADD(acc, a, b) acc += (b) - (a)
#else
#define PROF_T(v)
#define PROF_ADD(acc, a, b)
#endif

// Staged strands are kept in LDS as BIT PLANES: word w holds bases 32w..32w+31 as
// (plane0 = low code bits) | (plane1 = high code bits) << 32, so 32 bases at any offset are
// two v_alignbit_b32 per strand and a mismatch mask is 32 bits wide.
__device__ __forceinline__ uint32_t compact_even(uint64_t x) {   // bits 0,2,..,62 -> 0..31
  x &= 0x5555555555555555ull;
  x = (x | (x >> 1)) & 0x3333333333333333ull;
  x = (x | (x >> 2)) & 0x0F0F0F0F0F0F0F0Full;
  x = (x | (x >> 4)) & 0x00FF00FF00FF00FFull;
  x = (x | (x >> 8)) & 0x0000FFFF0000FFFFull;
  x = (x | (x >> 16)) & 0x00000000FFFFFFFFull;
  return (uint32_t)x;
}

// Mismatch mask of the 32 bases at a[pa..pa+31] vs t[pt..pt+31] (bit i = base i); pa, pt
// may be negative (the words before a strand are other LDS data: those bases lie beyond
// the comparison limit and are never counted).
__device__ __forceinline__ uint32_t plane_mismatch(const lds_u64 *a, int32_t pa,
                                                   const lds_u64 *t, int32_t pt) {
  const int32_t ia = pa >> 5, it = pt >> 5;
  const uint64_t a0 = a[ia], a1 = a[ia + 1], t0 = t[it], t1 = t[it + 1];
  const uint32_t sa = (uint32_t)pa & 31u, st = (uint32_t)pt & 31u;
  const uint32_t xa0 = __builtin_amdgcn_alignbit((uint32_t)a1, (uint32_t)a0, sa);
  const uint32_t xa1 = __builtin_amdgcn_alignbit((uint32_t)(a1 >> 32), (uint32_t)(a0 >> 32), sa);
  const uint32_t xt0 = __builtin_amdgcn_alignbit((uint32_t)t1, (uint32_t)t0, st);
  const uint32_t xt1 = __builtin_amdgcn_alignbit((uint32_t)(t1 >> 32), (uint32_t)(t0 >> 32), st);
  return (xa0 ^ xt0) | (xa1 ^ xt1);
}

__device__ __forceinline__ int32_t run_fwd(uint32_t mm) {   // matches from bit 0 up
  return mm ? (int32_t)__builtin_ctz(mm) : 32;
}
__device__ __forceinline__ int32_t run_bwd(uint32_t mm) {   // matches from bit 31 down
  return mm ? (int32_t)__builtin_clz(mm) : 32;
}

// slide on exception-free LDS plane strands: DIR=+1 compares A[pa..], T[pt..]; DIR=-1
// compares A[pa], A[pa-1], .. with T[pt], T[pt-1], ..; at most lim (> 0) bases.
template <int DIR>
__device__ __forceinline__ int32_t slide_lds(const lds_u64 *a, int32_t pa, const lds_u64 *t,
                                             int32_t pt, int32_t lim) {
  int32_t k = 0;
  for (;;) {
    int32_t run;
    if (DIR > 0) run = run_fwd(plane_mismatch(a, pa + k, t, pt + k));
    else         run = run_bwd(plane_mismatch(a, pa - k - 31, t, pt - k - 31));
    k += run;
    if (run < 32 || k >= lim) break;
  }
  return k < lim ? k : lim;
}

template <int DIR, typename SS>
__device__ __forceinline__ int32_t slide_any(const SS &A, int32_t a0, const SS &T, int32_t t0,
                                             int32_t r, int32_t d, int32_t lim) {
  if constexpr (SS::kExc) {
    if (DIR > 0) return slide_fwd(A, a0 + r, T, t0 + r + d, lim);
    return slide_bwd(A, a0 - r, T, t0 - r - d, lim);
  } else {
    if (DIR > 0) return slide_lds<1>(A.w, a0 + r, T.w, t0 + r + d, lim);
    return slide_lds<-1>(A.w, a0 - r, T.w, t0 - r - d, lim);
  }
}

__device__ __forceinline__ int32_t dpp_from_lower(int32_t v, int32_t lane0) {   // lane l <- l-1
  return __builtin_amdgcn_update_dpp(lane0, v, 0x138, 0xf, 0xf, false);
}
__device__ __forceinline__ int32_t dpp_from_upper(int32_t v, int32_t lane63) {  // lane l <- l+1
  return __builtin_amdgcn_update_dpp(lane63, v, 0x130, 0xf, 0xf, false);
}
// Chunk-boundary neighbours without a readlane: lane l <- v[l-1], lane 0 <- prev[63]
// (wave_ror:1 of prev supplies lane 0, then wave_shr:1 of v overwrites lanes 1..63), and
// lane l <- v[l+1], lane 63 <- next[0] (wave_rol:1, then wave_shl:1).
// (a rotate writes every lane, so it needs no old value and no initialising move)
__device__ __forceinline__ int32_t dpp_lower_across(int32_t v, int32_t prev) {
  const int32_t u = __builtin_amdgcn_mov_dpp(prev, 0x13C, 0xf, 0xf, false);
  return __builtin_amdgcn_update_dpp(u, v, 0x138, 0xf, 0xf, false);
}
__device__ __forceinline__ int32_t dpp_upper_across(int32_t v, int32_t next) {
  const int32_t u = __builtin_amdgcn_mov_dpp(next, 0x134, 0xf, 0xf, false);
  return __builtin_amdgcn_update_dpp(u, v, 0x130, 0xf, 0xf, false);
}

// Set_Right_Delta / Set_Left_Delta over the code log of wave_ped_reg: cell (k, d) holds
// (r << 2 | code), r = max(1 + L[k-1][d], L[k-1][d-1], 1 + L[k-1][d+1]) and code = which
// one won (0: d, 1: d-1, 2: d+1) with the reference's tie order.  16 rows at a time are
// loaded into registers (lane = diagonal offset -16..16 from the walk's position), and the
// walk is scalar: one readlane per row.
typedef __attribute__((address_space(1))) const int32_t g_ci32;
typedef __attribute__((address_space(1))) const uint16_t g_cu16;
typedef __attribute__((address_space(1))) const uint64_t g_cu64;

// Set_Right_Delta / Set_Left_Delta (forward.C:48, reverse.C:52) over the row log of
// wave_ped_reg: row k's stripe holds L[k][d] (-2 outside the pruned band).  For 16 rows at a
// time the previous rows are loaded into registers (lane = diagonal offset -31..31 from the
// window's first position), every lane's step is decided in parallel, and the walk is
// scalar, one readlane per row.
//
// The walk itself is cheap; what it waits for is the log.  So the rows of OVL_TB_G windows
// are loaded in one burst (one memory round trip instead of one per window), every window of
// the burst centred at the burst's first position dc.  A window can be walked from these
// lanes while its first position d stays within 15 of dc: its 16 steps then read lanes
// 31 + (d - dc) +- 15, inside the lanes 1..61 whose DPP neighbours are real cells.  The
// first window of a burst always can; when a later one cannot (the path drifted), the next
// burst starts there.  Measured (10k x 10 kb, records identical): 2 windows per burst the
// same as 1, 3 windows +3-4 % (the 48 row registers) -- the other waves of the SIMD already
// hide the log's latency, so the default stays one window per load.
#ifndef OVL_TB_G
#define OVL_TB_G 1
#endif
template <bool L16, int LW = OVL_LOGW>
__device__ __forceinline__ void ped_traceback_codes(int32_t *log, int32_t tb_e, int32_t tb_d,
                                                    int32_t last, int32_t *dst, uint32_t lane,
                                                    int32_t &last_out, int32_t &nd_out) {
  constexpr int W = LW;                        // cells per logged row, cell = d mod W
  // rows per window (lanes cover dc-31..dc+31): 16 keeps the unrolled walk and its code
  // registers within wave_ped_reg's 80 VGPRs (24 spills; 16 vs 24: -1 % extension time)
  constexpr int TBR = 16;
  constexpr int G = OVL_TB_G;                  // windows per burst of log loads
  g_ci32 *rows = (g_ci32 *)log;
  typedef __attribute__((address_space(1))) const int16_t g_ci16;
  g_ci16 *rows16 = (g_ci16 *)log;
  typedef __attribute__((address_space(1))) int32_t g_i32;
  g_i32 *gdst = (g_i32 *)dst;                  // global, not flat (see wave_ped_reg's log)
  vm_sync();                                  // the log is complete
  int32_t d = __builtin_amdgcn_readfirstlane(tb_d);
  last = __builtin_amdgcn_readfirstlane(last);
  int32_t kh = __builtin_amdgcn_readfirstlane(tb_e);
  int32_t nd = 0;
  while (kh >= 1) {
    const int32_t dc = d;
    const int32_t cell = (dc - 31 + (int32_t)(lane < 63 ? lane : 62)) & (W - 1);
    int32_t V[G * TBR];
#pragma unroll
    for (int i = 0; i < G * TBR; i++) {
#ifdef OVL_ATTR_TB_FIXED                       // traffic attribution only (wrong results)
      const int32_t kk = 0;
#else
      const int32_t kk = kh - 1 - i < 0 ? 0 : kh - 1 - i;   // row k-1 for k = kh - i
#endif
      if constexpr (L16) V[i] = (int32_t)rows16[(size_t)kk * W + cell];
      else               V[i] = rows[(size_t)kk * W + cell];
    }
#pragma unroll 1
    for (int g = 0; g < G; g++) {
      if (g > 0) {
        const int32_t off = d - dc;
        if (kh < 1 || off > 15 || off < -15) break;
      }
      // Every lane's winner first, lane-parallel (VALU, DPP neighbours): C[i] at lane x is
      // (the value the walk would take as `last`) << 2 | (from + 1), with the reference's
      // order -- d-1 only if strictly better than d, d+1 only if strictly better than both.
      // The walk is then one readlane and a few scalar operations per row; the window's
      // deltas collect in one VGPR (lane j = its j-th delta) stored once per window.
      const int32_t nsteps = kh < TBR ? kh : TBR;
      int32_t C[TBR];
#pragma unroll
      for (int i = 0; i < TBR; i++) {
        const int32_t v = V[i];
        const int32_t vm = dpp_from_lower(v, -2), vp = dpp_from_upper(v, -2);
        const int32_t a = v + 1, c = vp + 1;
        const int32_t m = vm > a ? vm : a;
        const int32_t f = c > m ? 2 : (vm > a ? 0 : 1);
        C[i] = ((f == 0 ? vm : vp) << 2) | f;
      }
      // the next window's rows move down (register moves; with G == 1 there are none)
#pragma unroll
      for (int i = 0; i + TBR < G * TBR; i++) V[i] = V[i + TBR];
      __builtin_amdgcn_sched_barrier(0);
      int32_t buf = 0, nb = 0;
      int32_t x = 31 + d - dc;                 // lane of diagonal d
#pragma unroll
      for (int i = 0; i < TBR; i++) {
        if (i < nsteps) {
          const int32_t w = __builtin_amdgcn_readlane(C[i], x);
          const int32_t f3 = w & 3, nl = w >> 2;   // f3: 0 d-1, 1 d, 2 d+1
          const int32_t val = f3 == 0 ? nl - last - 1 : last - nl;
          buf = (int32_t)lane == nb ? val : buf;
          const int32_t mv = f3 != 1;
          nb += mv;
          last = mv ? nl : last;
          x += f3 - 1;
        }
      }
      d = dc + x - 31;
      if ((int32_t)lane < nb) gdst[nd + (int32_t)lane] = buf;
      nd += nb;
      kh -= TBR;
    }
  }
  last_out = last;
  nd_out = nd;
}

// Scalar copies of wave-uniform values: arguments of a non-inlined function arrive in
// VGPRs, so without these a loop bound or branch on them is compiled as divergent
// (exec-mask bookkeeping on every row).
__device__ __forceinline__ int32_t uni(int32_t v) { return __builtin_amdgcn_readfirstlane(v); }
template <typename P>
__device__ __forceinline__ P *uni_ptr(P *p) {
  const uint64_t b = (uint64_t)(uintptr_t)p;
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int32_t)(uint32_t)b);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int32_t)(uint32_t)(b >> 32));
  return (P *)(uintptr_t)(((uint64_t)hi << 32) | lo);
}
__device__ __forceinline__ double uni(double v) {
  const uint64_t b = __builtin_bit_cast(uint64_t, v);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int32_t)(uint32_t)b);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int32_t)(uint32_t)(b >> 32));
  return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}

// The row loop stays a call: inlined into process_pair (always_inline) the kernel keeps 80
// VGPRs but spills 576 B per lane inside the loop -- extension 218 -> 297 ms (+37 %) on the
// 10k-read job (r02v A/B).
#ifndef OVL_PED_ATTR
#define OVL_PED_ATTR noinline
#endif
//
// Everything the row loop reads arrives as a scalar argument (v0..v31 of the call), not
// through references: a reference to the ExtendArgs / WaveMem / strand copies in the
// kernel's scratch made every call start with flat loads from scratch and a full vmcnt(0)
// wait (which also waited for the caller's spill stores and the row-0 log store).  X is
// only read by the OVL_PROFILE build.
template <int DIR, typename SS, bool L16, int RJ = OVL_RJ>
__device__ __attribute__((OVL_PED_ATTR)) PedOut wave_ped_reg(
    const ExtendArgs &X, int32_t e_cap, int32_t partial_i, int32_t mbed, double bmv_in,
    double mbts, const lds_u64 *aw, int32_t a0, int32_t m, const lds_u64 *tw, int32_t t0,
    int32_t n, int32_t limit, int32_t *rows, ml_t *mlim, int32_t *dst,
    uint32_t lane) {
  SS A, T;
  A.w = aw; A.len = 0;
  T.w = tw; T.len = 0;
  constexpr int J = RJ;
  // cells per logged row (a power of two holding the register window) and the window
  // offset bits of a row key
  constexpr int LW = 64 * RJ > OVL_LOGW ? 64 * RJ : OVL_LOGW;
  constexpr int WB = 64 * RJ > 512 ? 10 : 9;
  static_assert(64 * J <= (1 << WB) && 64 * J <= LW, "key and log layout hold the window");
  static_assert(!SS::kExc, "the register kernel runs on exception-free LDS strands");
  limit = uni(limit);
  auto slide_d = [&](int32_t r, int32_t d, int32_t lim) -> int32_t {
    return slide_any<DIR>(A, a0, T, t0, r, d, lim);
  };
  const int32_t NONE = 0x7fffffff, NEG = (int32_t)0x80000000;
  PedOut out;
  out.leftover = 0;
  out.nd = 0;
  out.ovf = 0;
  if (limit > uni(e_cap) - 2) {                // not this kernel's class: defer the pair
    out.ovf = 1;
    return out;
  }
  int32_t row0 = 0;
  {
    int32_t lim0 = m < n ? m : n;
    if (lim0 > 0) row0 = slide_d(0, 0, lim0);
    row0 = __builtin_amdgcn_readfirstlane(row0);
  }
  if (row0 == m) {
    out.err = 0; out.a_len = m; out.t_len = m; out.mte = 1;
    out.leftover = m;          // reverse(): Leftover = m on an exact match
    out.nd = -1;               // no traceback
    return out;
  }

  int32_t R[J];
#pragma unroll
  for (int j = 0; j < J; j++) R[j] = -2;
  int32_t B = -3;                              // window anchored: B <= pl-3 < B+64
  if (lane == 3) R[0] = row0;

  double  max_score = 0.0;
  int32_t max_score_len = 0, max_score_best_e = 0;
  // Max_Score_Best_d is kept as the row key and window base it decodes from (decoded once,
  // after the loop): B + 64J-1 - (key & 64J-1)
  int32_t ms_key = (1 << WB) - 1, ms_B = 0;
  int32_t longest = 0;
  int32_t pl = 0, pr = 0;
  int32_t tb_e = -1, tb_d = 0, tb_last = 0;
  bool finished = false;
  const double bmv = uni(bmv_in);
  const bool partial = uni(partial_i) != 0;
  mbed = uni(mbed);
  mbts = uni(mbts);
#ifdef OVL_PROFILE
  unsigned long long pc_a = 0, pc_b = 0, pc_cont = 0, pc_c = 0;
  unsigned long long pc_chunks = 0, pc_rest = 0, pc_rows = 0, pc_nch = 0, pc_slide = 0,
                     pc_recenter = 0;
  PROF_T(pt_begin);
#endif

  // Row log for the traceback: row e (after pruning, -2 outside [nl, nr]) is a fixed
  // 64*J-cell stripe at e * 64J, cell = d mod 64J (the window holds 64J consecutive
  // diagonals, so the index is unique and needs no per-row base).  Row 0 is logged here.
  typedef typename std::conditional<L16, int16_t, int32_t>::type cell_t;
  // global (not flat) stores: a flat store also counts against lgkmcnt, so every LDS wait
  // of the next row would wait for the log stores too
  typedef __attribute__((address_space(1))) cell_t g_cell_t;
  g_cell_t *clog = uni_ptr((g_cell_t *)rows);     // scalar base: stores use saddr + offset
  clog[(B + (int32_t)lane) & (LW - 1)] = (cell_t)R[0];
  typedef __attribute__((address_space(1))) uint8_t g_u8;
  g_u8 *clogb = (g_u8 *)clog;
  // chunks 0..JU-1 are processed unconditionally (straight-line code the compiler can
  // interleave); their lanes beyond the band are inactive by the lane predicates
  constexpr int JU = 1;
  const int32_t lkey = (1 << WB) - 1 - (int32_t)lane;

  int32_t e = 1;
  bool ended = false;
  int32_t end_d = 0, end_row = 0, end_pp = 0;
  // One exit: every way a row ends the loop (the end reached, an empty band, the band
  // outgrowing the window, the error limit) makes `go` negative, tested once per row; with
  // four breaks the structurizer carried exit flags through every row's tail (~12 scalar
  // instructions per row).  The window is re-anchored for the next row at the end of this
  // one (row 1 needs none: B = -3, pl = pr = 0).
  int32_t end_e = 0;
  int32_t go = limit - 1;                      // the loop runs while go >= 0
  while (go >= 0) {
    PROF_T(pt_row);
    const int32_t ML = mlim[e];
    const int32_t right = pr + 1;
    const int32_t jr = (right - B) >> 6;

    // ---- A+B per chunk: neighbours from row e-1 (DPP, no LDS), then the first 32-base
    // slide step of every lane, branch-free (one pass: each unrolled chunk costs a scalar
    // compare-and-branch on jr) --------------------------------------------------------
    int32_t NR[J], RM[J];   // row value; lanes: bases left before the end (0 = end)
    uint64_t need[J];
    uint64_t any = 0;
#pragma unroll
    for (int j = 0; j < J; j++) {
      if (j >= JU && j > jr) break;
      const int32_t d = B + 64 * j + (int32_t)lane;
      const int32_t p0 = R[j];
      // row e-1 at d-1 and d+1 (diagonal B-1 and B+64J are outside the band: -2)
      const int32_t pm = (j == 0) ? dpp_from_lower(p0, -2) : dpp_lower_across(p0, R[j > 0 ? j - 1 : 0]);
      const int32_t pp = (j + 1 < J) ? dpp_upper_across(p0, R[j + 1 < J ? j + 1 : j])
                                     : dpp_from_upper(p0, -2);
      // q = Row - 1 = max(pm - 1, p0, pp): the +1 of the max3 folds into the constants
      const int32_t pm1 = pm - 1;
      const int32_t q = (pm1 > p0 ? pm1 : p0) > pp ? (pm1 > p0 ? pm1 : p0) : pp;
      // d outside [left, right] sees only -2 sentinels, so Row == -1 there (inside, >= 1):
      // its limit is hugely negative, so it never slides, ends or survives pruning
      const int32_t l1 = (m - 1) - q, l2 = (n - 1) - q - d;
      const int32_t lmin = l1 < l2 ? l1 : l2;
      const int32_t lim = q >= -1 ? lmin : -(1 << 30);

      const int32_t pa = (DIR > 0) ? (a0 + 1) + q : (a0 - 32) - q;
      const int32_t pt = (DIR > 0) ? (t0 + 1) + q + d : (t0 - 32) - q - d;
      const int32_t ia = pa >> 5, it = pt >> 5;
      const uint64_t wa0 = A.w[ia], wa1 = A.w[ia + 1];
      const uint64_t wt0 = T.w[it], wt1 = T.w[it + 1];
      // v_alignbit_b32 uses the low 5 bits of the shift
      const uint32_t xa0 = __builtin_amdgcn_alignbit((uint32_t)wa1, (uint32_t)wa0, (uint32_t)pa);
      const uint32_t xa1 = __builtin_amdgcn_alignbit((uint32_t)(wa1 >> 32), (uint32_t)(wa0 >> 32),
                                                     (uint32_t)pa);
      const uint32_t xt0 = __builtin_amdgcn_alignbit((uint32_t)wt1, (uint32_t)wt0, (uint32_t)pt);
      const uint32_t xt1 = __builtin_amdgcn_alignbit((uint32_t)(wt1 >> 32), (uint32_t)(wt0 >> 32),
                                                     (uint32_t)pt);
      const uint32_t mm = (xa0 ^ xt0) | (xa1 ^ xt1);
      // the first step examines 31 bases (a sentinel mismatch in the 32nd: no clamp of
      // the bit scan), lanes that matched all 31 with more left continue below
      const int32_t run = (DIR > 0) ? (int32_t)__builtin_ctz(mm | 0x80000000u)
                                    : (int32_t)__builtin_clz(mm | 1u);
      // k = min(run, lim): lim >= 0 (run >= 0), so the row only moves forward
      const int32_t k = run < lim ? run : lim;
      NR[j] = q + 1 + k;                       // lim >= 0 inside the band
      RM[j] = lmin - k;                        // inside: lim - k >= 0; outside: > 0
      // run == 31 && lim > 31  <=>  min(run, lim - 1) == 31 (run <= 31): one ballot, no
      // scalar AND of two
      need[j] = __builtin_amdgcn_ballot_w64((run < lim - 1 ? run : lim - 1) == 31);
      any |= need[j];
    }
#ifdef OVL_PROFILE
    pc_nch += (jr + 1 > JU ? jr + 1 : JU);
#endif
    PROF_T(pt_b);
    PROF_ADD(pc_a, pt_row, pt_b);
    // lanes that matched all 31 bases continue (the on-path diagonals): one loop over all
    // chunks so their LDS loads overlap
    if (any) {
#pragma unroll
      for (int j = 0; j < J; j++) {
        if (j >= JU && j > jr) break;
        if (need[j]) {
          if (need[j] & (1ull << lane)) {
            const int32_t d = B + 64 * j + (int32_t)lane;
            const int32_t sl = slide_d(NR[j], d, RM[j]);
            NR[j] += sl;
            RM[j] -= sl;
          }
#ifdef OVL_PROFILE
          pc_slide++;
#endif
        }
      }
    }

    PROF_T(pt_cont);
    PROF_ADD(pc_cont, pt_b, pt_cont);
    // ---- C: end test and Edit_Match_Limit pruning, one pass ---------------------------
    // Only two masks are reduced on the common row: the kept range's left end lies in chunk
    // 0 (the window is anchored at the band's left edge) and its right end in the last
    // chunk, jr.  So chunk 0's and chunk jr's kept masks are kept and the other chunks cost
    // no scalar work; when either is empty (~2 % of rows: the pruning emptied the band's
    // first or last chunk, or the whole band) every chunk is rescanned below.  The end test
    // is a per-lane min of the bases left, one ballot per row.  (The per-chunk s_ff1 /
    // s_flbit / min reduction was 6 scalar instructions per chunk.)
    int32_t rmin = RM[0];
    uint64_t km0 = 0, kml = 0;
#pragma unroll
    for (int j = 0; j < J; j++) {
      if (j >= JU && j > jr) break;
      const int32_t d = B + 64 * j + (int32_t)lane;
      if (j > 0) rmin = RM[j] < rmin ? RM[j] : rmin;
      kml = __builtin_amdgcn_ballot_w64(NR[j] + (d > 0 ? d : 0) >= ML);
      if (j == 0) km0 = kml;
    }
    const uint64_t endany = __builtin_amdgcn_ballot_w64(rmin == 0);
    uint32_t nlo, nhi;                         // min window offset of a kept lane; min
                                               // reversed offset (64J-1 - o) of one
    // s_ff1 / s_flbit give ~0u on an empty mask: one signed test of their OR sends the row
    // to the rescan (a boolean AND of the two mask tests cost 6 scalar instructions)
    asm("s_ff1_i32_b64 %0, %1" : "=s"(nlo) : "s"(km0));
    asm("s_flbit_i32_b64 %0, %1" : "=s"(nhi) : "s"(kml));
    if ((int32_t)(nlo | nhi) >= 0) {
      nhi += (uint32_t)(64 * (J - 1)) - (uint32_t)(jr << 6);
    } else {
      // the unsigned mins ignore an empty chunk's ~0u
      nlo = 0xffffffffu;
      nhi = 0xffffffffu;
#pragma unroll
      for (int j = 0; j < J; j++) {
        if (j >= JU && j > jr) break;
        const int32_t d = B + 64 * j + (int32_t)lane;
        const uint64_t km = __builtin_amdgcn_ballot_w64(NR[j] + (d > 0 ? d : 0) >= ML);
        uint32_t f1, fb;
        asm("s_ff1_i32_b64 %0, %1" : "=s"(f1) : "s"(km));
        asm("s_flbit_i32_b64 %0, %1" : "=s"(fb) : "s"(km));
        const uint32_t c1 = f1 | (uint32_t)(64 * j);
        nlo = c1 < nlo ? c1 : nlo;
        const uint32_t g = fb | (uint32_t)(64 * (J - 1 - j));
        nhi = g < nhi ? g : nhi;
      }
    }
    const int32_t nro = 64 * J - 1 - (int32_t)nhi;

    PROF_T(pt_chunks);
    PROF_ADD(pc_chunks, pt_row, pt_chunks);
    PROF_ADD(pc_c, pt_cont, pt_chunks);
#ifdef OVL_PROFILE
    pc_rows++;
#endif
    // Every way a row ends the loop sets e past the limit (the end row keeps its own e in
    // end_e; an empty band needs none) and falls through to one signed test of two
    // differences, so the common row reaches the back-edge with no stop flag: e > limit, or
    // the next row would not fit the window (pr + 3 > B + 64J - 1 -- told apart after the
    // loop by e <= limit: the pair is deferred).  The flag of a three-way branch cost ~6
    // scalar instructions per row.
    if (endany) {                              // the first d in order that reached the end
      // lowest chunk last (no break: the rare row stays out of the common row's CFG)
#pragma unroll
      for (int j = J - 1; j >= 0; j--) {
        if (j >= JU && j > jr) continue;
        const uint64_t em = __builtin_amdgcn_ballot_w64(RM[j] == 0);
        if (em) {
          const int32_t l = (int32_t)__builtin_ctzll(em);
          end_d = B + 64 * j + l;
          end_row = __builtin_amdgcn_readlane(NR[j], l);
          // row e-1 at d+1 (R still holds row e-1)
          end_pp = (l < 63) ? __builtin_amdgcn_readlane(R[j], l + 1)
                 : (j + 1 < J) ? __builtin_amdgcn_readlane(R[j + 1 < J ? j + 1 : j], 0) : -2;
        }
      }
      ended = true;
      end_e = e;
      e = limit + 1;
    } else if (nlo == 0xffffffffu) {
      e = limit + 1;                           // Left > Right (e is not read after)
    } else {
      const int32_t nl = B + (int32_t)nlo;
      const int32_t nr = B + nro;

      // prune to [nl, nr] (the rest becomes the -2 sentinel), log the row for the
      // traceback (cells up to nr+2 are read), longest row with the first d on ties: one
      // wave max over keys (value << WB | 64J-1 - window offset), so a larger value wins and
      // among equal values the smaller d (values < 2^21 and -2 keep the order in 32 bits).
      // The row's stripe is a 32-bit byte offset OR-ed with the cell's (the stripe is a power
      // of two): one scalar shift per row instead of a 64-bit row pointer.
      int32_t kmx = NEG;
      const uint32_t kspan = (uint32_t)(nr - nl);
      const int32_t jrs = ((nr + 2 > right ? nr + 2 : right) - B) >> 6;
#ifdef OVL_ATTR_LOG_FIXED                      // traffic attribution only (wrong results)
      const uint32_t erow = 0u;
#else
      const uint32_t erow = (uint32_t)e * (uint32_t)(LW * sizeof(cell_t));
#endif
#pragma unroll
      for (int j = 0; j < J; j++) {
        if (j >= JU && j > jrs) break;
        const int32_t d = B + 64 * j + (int32_t)lane;
        const int32_t v = ((uint32_t)(d - nl) <= kspan) ? NR[j] : -2;
        R[j] = v;
        const int32_t key = (int32_t)(((uint32_t)v << WB) | (uint32_t)(lkey - 64 * j));
        kmx = key > kmx ? key : kmx;
        *(g_cell_t *)(clogb + (erow | ((uint32_t)(d & (LW - 1)) * (uint32_t)sizeof(cell_t)))) =
            (cell_t)v;
      }
      const int32_t K = wave_max(kmx);
      const int32_t M = K >> WB;
      if (M > longest) {                         // Longest, Best_d, Best_e of this row
        longest = M;
        // the score can only beat Max_Score on a row whose Longest grew: otherwise it is the
        // previous row's score minus one (monotone in double too), and that was <= Max_Score
        const double score = longest * bmv - e;
        if (score > max_score) {
          max_score = score;
          max_score_len = longest;
          ms_key = K;
          ms_B = B;
          max_score_best_e = e;
        }
      }
      pl = nl;
      pr = nr;
      PROF_T(pt_rest);
      PROF_ADD(pc_rest, pt_chunks, pt_rest);
      e++;
      // The window is anchored at the band: B <= pl-3 < B+16, so the row's chunks are
      // 0..jr with little waste in chunk 0.  When pl-3 leaves [B, B+16) the window moves to
      // B = pl-9: whole chunks by register moves, the rest by one ds_bpermute per chunk
      // (about one row in ten).  It must also hold pr+3 (the reads of this row and the log
      // of the next).  (Past the limit B is no longer read.)
      if ((uint32_t)(pl - 3 - B) >= 16u) {
        const int32_t nb = pl - 9;
        int32_t sft = nb - B;
        while (sft >= 64) {
#pragma unroll
          for (int j = 0; j < J - 1; j++) R[j] = R[j + 1];
          R[J - 1] = -2;
          sft -= 64;
        }
        while (sft <= -64) {
#pragma unroll
          for (int j = J - 1; j > 0; j--) R[j] = R[j - 1];
          R[0] = -2;
          sft += 64;
        }
        if (sft != 0) {
          const int32_t ls = (int32_t)lane + sft;
          const int32_t src = (ls & 63) << 2;
          int32_t bp[J];
#pragma unroll
          for (int j = 0; j < J; j++) bp[j] = __builtin_amdgcn_ds_bpermute(src, R[j]);
          if (sft > 0) {
            const bool hi = ls >= 64;            // comes from the next chunk up
#pragma unroll
            for (int j = 0; j < J; j++) R[j] = hi ? (j + 1 < J ? bp[j + 1 < J ? j + 1 : j] : -2) : bp[j];
          } else {
            const bool lo = ls < 0;              // comes from the chunk below
#pragma unroll
            for (int j = 0; j < J; j++) R[j] = lo ? (j > 0 ? bp[j > 0 ? j - 1 : 0] : -2) : bp[j];
          }
        }
        B = nb;
#ifdef OVL_PROFILE
        pc_recenter++;
#endif
      }
    }
    go = (limit - e) | (B + 64 * J - 4 - pr);
  }
  // stopped with rows left to compute: the window overflowed (every other stop sets e
  // past the limit)
  if (e <= limit) out.ovf = 1;
  if (out.ovf) return out;
  const int32_t max_score_best_d = ms_B + ((1 << WB) - 1) - (ms_key & ((1 << WB) - 1));
  if (ended) {                               // forward.C:177-232, at row end_e
    const int32_t e = end_e;
    double  score = end_row * bmv - e;
    int32_t tail_len = end_row - max_score_len;
    double  slope = (double)(max_score - score) / tail_len;
    bool    abort_here = false;
    if (partial && score < max_score) abort_here = true;
    if (e > mbed / 2 && tail_len >= mbed && slope >= mbts) abort_here = true;
    if (abort_here) {
      out.err = max_score_best_e;
      out.a_len = max_score_len;
      out.t_len = max_score_len + max_score_best_d;
      out.mte = 0;
      tb_e = max_score_best_e; tb_d = max_score_best_d;
    } else {
      int32_t d = end_d;
      // forward.C:212 -- force the last error to be a mismatch rather than an insertion
      if (DIR > 0 && end_row == m && 1 + end_pp == end_row && d < pr + 1) d++;
      out.err = e;
      out.a_len = end_row;
      out.t_len = end_row + d;
      out.mte = 1;
      tb_e = e; tb_d = d; tb_last = end_row;
    }
    finished = true;
  }
  if (!finished) {
    out.err = max_score_best_e;
    out.a_len = max_score_len;
    out.t_len = max_score_len + max_score_best_d;
    out.mte = 0;
    tb_e = max_score_best_e; tb_d = max_score_best_d;
  }
  if (!finished || out.mte == 0) tb_last = (tb_e == 0) ? row0 : max_score_len;
  int32_t last = 0, nd = 0;
  PROF_T(pt_tb0);
  ped_traceback_codes<L16, LW>(rows, tb_e, tb_d, tb_last, dst, lane, last, nd);
  out.leftover = last;
  out.nd = nd;
#ifdef OVL_PROFILE
  PROF_T(pt_tb1);
  if (X.dbg && lane == 0) {
    atomicAdd(&X.dbg[0], 1ull);
    atomicAdd(&X.dbg[1], pc_rows);
    atomicAdd(&X.dbg[2], pc_nch);
    atomicAdd(&X.dbg[3], pc_slide);
    atomicAdd(&X.dbg[4], (unsigned long long)(tb_e > 0 ? tb_e : 0));
    atomicAdd(&X.dbg[6], pc_chunks);
    atomicAdd(&X.dbg[7], pt_tb1 - pt_tb0);
    atomicAdd(&X.dbg[10], pc_rest);
    atomicAdd(&X.dbg[11], pt_tb1 - pt_begin);
    atomicAdd(&X.dbg[16], pc_a);
    atomicAdd(&X.dbg[17], pc_b);
    atomicAdd(&X.dbg[18], pc_cont);
    atomicAdd(&X.dbg[19], pc_c);
    (void)pc_recenter;
  }
#endif
  return out;
}

struct OlapInfo {
  int32_t s_lo, s_hi, t_lo, t_hi;
  double  quality;
  int32_t delta_ct;
  int32_t slb, srb, tlb, trb;      // s/t left/right boundary
  int32_t min_diag, max_diag;
};

enum { K_NONE = 0, K_LEFT_BRANCH = 1, K_RIGHT_BRANCH = 2, K_DOVETAIL = 3 };

struct ExtOut {
  int32_t kind, S_Lo, S_Hi, T_Lo, T_Hi, Errors, ld_len;
};

// Extend_Alignment (prefixEditDistance-extend.C:86).  Leaves the merged Left_Delta in LD.
#define UNI(v) uni(v)
template <bool FAST, bool L16, int RJ, typename SS>
__device__ ExtOut extend_alignment(const ExtendArgs &X, const Node &Mv, const SS &S,
                                   int32_t S_Len, const SS &T, int32_t T_Len,
                                   const WaveMem &WM, int32_t *stk, int32_t *RD,
                                   int32_t *LD, uint32_t lane) {
  // The match, the lengths and the row-loop results are wave-uniform: held in SGPRs they
  // survive the two row-loop calls without the per-lane spills a VGPR copy needs (141 -> 132
  // spill stores in the staged kernel; extension 217-218 -> 214-217 ms on 10k reads, r02v
  // A/B, records identical).  SGPR copies of the pair's and unit's fields too (125 spill
  // stores) measured the same, and were left out
  Node M;
  M.Start = UNI(Mv.Start); M.Offset = UNI(Mv.Offset); M.Len = UNI(Mv.Len); M.Next = Mv.Next;
  S_Len = UNI(S_Len);
  T_Len = UNI(T_Len);
  ExtOut r;
  int32_t right_errors = 0, left_errors = 0, leftover = 0;
  int32_t rmte = 1, lmte = 1;
  int32_t S_Left_Begin = M.Start - 1, S_Right_Begin = M.Start + M.Len;
  int32_t S_Right_Len = S_Len - S_Right_Begin;
  int32_t T_Left_Begin = M.Offset - 1, T_Right_Begin = M.Offset + M.Len;
  int32_t T_Right_Len = T_Len - T_Right_Begin;
  int32_t total = (M.Start < M.Offset ? M.Start : M.Offset) + M.Len +
                  (S_Right_Len < T_Right_Len ? S_Right_Len : T_Right_Len);
  int32_t error_limit = X.error_bound[total];
  int32_t rd_len = 0, ld_len = 0;
  int32_t S_Hi, T_Hi, S_Lo, T_Lo;

  if (S_Right_Len == 0 || T_Right_Len == 0) {
    S_Hi = 0; T_Hi = 0; rmte = 1;
  } else {
    bool s_first = S_Right_Len <= T_Right_Len;
    SS A = s_first ? S : T, B = s_first ? T : S;
    int32_t a0 = s_first ? S_Right_Begin : T_Right_Begin;
    int32_t b0 = s_first ? T_Right_Begin : S_Right_Begin;
    int32_t am = s_first ? S_Right_Len : T_Right_Len;
    int32_t bn = s_first ? T_Right_Len : S_Right_Len;
    PedOut po;
    PROF_T(pc0);
    if constexpr (FAST) {
      po = wave_ped_reg<1, SS, L16, RJ>(X, X.e_cap, X.partial, X.min_branch_end_dist,
                                        X.branch_match_value, X.min_branch_tail_slope, A.w, a0,
                                        am, B.w, b0, bn, error_limit, WM.rows, WM.rmlim, stk,
                                        lane);
    }
    else
      po = wave_ped<1, SS, L16>(X, A, a0, am, B, b0, bn, error_limit, WM, stk, lane);
#ifdef OVL_PROFILE
    PROF_T(pc1);
    if (X.dbg && lane == 0) atomicAdd(&X.dbg[12], pc1 - pc0);
#endif
    if (po.ovf) { r.kind = -1; return r; }
    po.err = UNI(po.err); po.mte = UNI(po.mte); po.a_len = UNI(po.a_len);
    po.t_len = UNI(po.t_len); po.nd = UNI(po.nd); po.leftover = UNI(po.leftover);
    right_errors = po.err;
    rmte = po.mte;
    if (s_first) { S_Hi = po.a_len; T_Hi = po.t_len; }
    else         { T_Hi = po.a_len; S_Hi = po.t_len; }
    // Set_Right_Delta: stack -> Right_Delta (forward.C:84-90)
    if (po.nd >= 0) {
      int32_t n = po.nd;
      if (lane == 0) stk[n] = po.leftover + 1;     // "last + 1"
      vm_sync();
      n++;
      for (int32_t i = lane; i < n - 1; i += 64) {
        int32_t src = n - 1 - i;
        int32_t a = stk[src], b = stk[src - 1];
        int32_t v = (a < 0 ? -a : a) * ((b > 0) - (b < 0));
        RD[i] = s_first ? -v : v;
      }
      vm_sync();
      rd_len = n - 1;
    }
  }
  S_Hi += S_Right_Begin - 1;
  T_Hi += T_Right_Begin - 1;

  if (S_Left_Begin < 0 || T_Left_Begin < 0) {
    S_Lo = 0; T_Lo = 0; lmte = 1;
  } else {
    bool s_first = S_Right_Begin <= T_Right_Begin;
    int32_t lim = error_limit - right_errors;
    SS A = s_first ? S : T, B = s_first ? T : S;
    int32_t a0 = s_first ? S_Left_Begin : T_Left_Begin;
    int32_t b0 = s_first ? T_Left_Begin : S_Left_Begin;
    PedOut po;
    PROF_T(pc2);
    if constexpr (FAST)
      po = wave_ped_reg<-1, SS, L16, RJ>(X, X.e_cap, X.partial, X.min_branch_end_dist,
                                         X.branch_match_value, X.min_branch_tail_slope, A.w,
                                         a0, a0 + 1, B.w, b0, b0 + 1, lim, WM.rows, WM.rmlim, LD,
                                         lane);
    else
      po = wave_ped<-1, SS, L16>(X, A, a0, a0 + 1, B, b0, b0 + 1, lim, WM, LD, lane);
#ifdef OVL_PROFILE
    PROF_T(pc3);
    if (X.dbg && lane == 0) atomicAdd(&X.dbg[12], pc3 - pc2);
#endif
    if (po.ovf) { r.kind = -1; return r; }
    left_errors = po.err;
    lmte = po.mte;
    int32_t a_end = -po.a_len, t_end = -po.t_len;
    int32_t n_t = b0 + 1;                                  // reverse()'s n
    leftover = po.leftover;
    if (po.nd >= 0) {
      ld_len = po.nd;
      vm_sync();
      // Set_Left_Delta fix-up (reverse.C:89-104): a leading +1 indel becomes a mismatch
      bool fix = ld_len > 1 && LD[0] == 1 && t_end + n_t > 0;
      if (fix) {
        int32_t l1 = LD[1];
        vm_sync();
        // LD[i-1] = LD[i] for i >= 2, lane-parallel: each pass reads above what it writes
        for (int32_t i0 = 2; i0 < ld_len; i0 += 64) {
          const int32_t i = i0 + (int32_t)lane;
          const int32_t v = (i < ld_len) ? LD[i] : 0;
          vm_sync();
          if (i < ld_len) LD[i - 1] = v;
          vm_sync();
        }
        if (lane == 0) LD[0] = (l1 > 0) ? l1 + 1 : l1 - 1;
        ld_len--;
        t_end--;
        if (ld_len == 0) leftover++;
        vm_sync();
      }
    }
    if (s_first) { S_Lo = a_end; T_Lo = t_end; }
    else         { T_Lo = a_end; S_Lo = t_end; }
    if (!s_first && ld_len > 0) {
      for (int32_t i = lane; i < ld_len; i += 64) LD[i] = -LD[i];
      vm_sync();
    }
  }
  S_Lo += S_Left_Begin + 1;
  T_Lo += T_Left_Begin + 1;

  r.Errors = left_errors + right_errors;
  r.kind = (rmte == 0) ? ((lmte == 0) ? K_NONE : K_RIGHT_BRANCH)
                       : ((lmte == 0) ? K_LEFT_BRANCH : K_DOVETAIL);
  if (lane == 0 && rd_len > 0) {
    int32_t v;
    if (RD[0] > 0) v = -(RD[0] + leftover + M.Len);
    else           v = -(RD[0] - leftover - M.Len);
    LD[ld_len] = v;
  }
  if (rd_len > 0) {
    for (int32_t i = 1 + lane; i < rd_len; i += 64) LD[ld_len + i] = -RD[i];
    ld_len += rd_len;
  }
  vm_sync();
  r.S_Lo = S_Lo; r.S_Hi = S_Hi; r.T_Lo = T_Lo; r.T_Hi = T_Hi;
  r.ld_len = ld_len;
  return r;
}


// ovOverlap.H:93 bit layout (AS_MAX_READLEN_BITS == 21)
__device__ __forceinline__ uint32_t encode_evalue(double q) {
  return (q < 4095 / 10000.0) ? (uint32_t)(int)(10000.0 * q + 0.5) : 4095u;
}

// Output.C:75 Output_Overlap (S_Dir: 0 FORWARD, 1 REVERSE; T is always forward)
__device__ Rec output_overlap(uint32_t S_ID, int32_t S_Len, int S_Dir, uint32_t T_ID,
                              int32_t T_Len, const OlapInfo &o, int32_t *bhg_out) {
  Rec r;
  uint32_t span = (uint32_t)(((o.s_hi - o.s_lo) + (o.t_hi - o.t_lo) + o.delta_ct) / 2);
  int32_t S_Right_Hang = S_Len - o.s_hi - 1;
  int32_t T_Right_Hang = T_Len - o.t_hi - 1;
  bool Sleft = (o.s_lo > o.t_lo) || (o.s_lo == o.t_lo && S_Right_Hang > T_Right_Hang);
  char orient;
  int32_t ahg, bhg;
  if (Sleft) { r.a_iid = S_ID; r.b_iid = T_ID; }
  else       { r.a_iid = T_ID; r.b_iid = S_ID; }
  if (Sleft) {
    orient = (S_Dir == 0) ? 'N' : 'O';
    ahg = o.s_lo;
    bhg = T_Right_Hang - S_Right_Hang;
  } else {
    orient = (S_Dir == 0) ? 'N' : 'I';
    ahg = o.t_lo;
    bhg = S_Right_Hang - T_Right_Hang;
  }
  if (orient == 'O' && S_Right_Hang >= T_Right_Hang) {
    orient = 'I';
    ahg = -(T_Right_Hang - S_Right_Hang);
    bhg = -(o.s_lo);
  }
  int32_t a_hang = ahg, b_hang = bhg;
  if (orient == 'O') { a_hang = -bhg; b_hang = -ahg; }
  uint64_t w0 = (1ull << 57) | ((uint64_t)encode_evalue(o.quality) << 42);
  uint64_t w1 = ((uint64_t)(span & 0x1fffff)) << 42;
  w0 |= (uint64_t)((a_hang < 0 ? 0 : a_hang) & 0x1fffff);
  w1 |= (uint64_t)((a_hang < 0 ? -a_hang : 0) & 0x1fffff);
  w1 |= (uint64_t)((b_hang < 0 ? 0 : b_hang) & 0x1fffff) << 21;
  w0 |= (uint64_t)((b_hang < 0 ? -b_hang : 0) & 0x1fffff) << 21;
  if (orient != 'N') w0 |= 1ull << 54;
  r.w0 = w0;
  r.w1 = w1;
  *bhg_out = bhg;
  return r;
}

// Output.C:253 Output_Partial_Overlap
__device__ Rec output_partial(uint32_t s_id, uint32_t t_id, int dir, const OlapInfo &o,
                              int32_t s_len, int32_t t_len) {
  Rec r;
  r.a_iid = s_id;
  r.b_iid = t_id;
  uint32_t span = (uint32_t)(((o.s_hi - o.s_lo) + (o.t_hi - o.t_lo) + o.delta_ct) / 2);
  uint64_t w0 = (1ull << 55) | (1ull << 56) | ((uint64_t)encode_evalue(o.quality) << 42);
  uint64_t w1 = ((uint64_t)(span & 0x1fffff)) << 42;
  uint64_t ahg5, ahg3, bhg5, bhg3;
  if (dir == 0) {
    ahg5 = o.s_lo; ahg3 = s_len - (o.s_hi + 1);
    bhg5 = o.t_lo; bhg3 = t_len - (o.t_hi + 1);
  } else {
    ahg5 = s_len - (o.s_hi + 1); ahg3 = o.s_lo;
    bhg5 = t_len - (o.t_hi + 1); bhg3 = o.t_lo;
    w0 |= 1ull << 54;
  }
  w0 |= (ahg5 & 0x1fffff) | ((ahg3 & 0x1fffff) << 21);
  w1 |= (bhg5 & 0x1fffff) | ((bhg3 & 0x1fffff) << 21);
  r.w0 = w0;
  r.w1 = w1;
  return r;
}

#define MAX_DISTINCT_OLAPS 3
#define MIN_INTERSECTION 10
#define SHIFT_SLACK 1

// Add_Overlap (Process_String_Overlaps.C:222); wave-uniform
// Returns the entry whose alignment was replaced by this one (new entry or better quality),
// i.e. whose Left_Delta the reference memcpy()s, or -1.
__device__ int32_t add_overlap(const ExtendArgs &X, int32_t s_lo, int32_t s_hi, int32_t t_lo,
                               int32_t t_hi, double qual, int32_t delta_ct, OlapInfo *ol,
                               int32_t &ct) {
  if (!X.partial) {
    int32_t new_diag = t_lo - s_lo;
    for (int32_t i = 0; i < ct; i++) {
      int32_t old_diag = ol[i].t_lo - ol[i].s_lo;
      if ((new_diag > 0 && old_diag > 0 &&
           ol[i].trb - new_diag - ol[i].slb >= MIN_INTERSECTION) ||
          (new_diag <= 0 && old_diag <= 0 &&
           ol[i].srb + new_diag - ol[i].tlb >= MIN_INTERSECTION)) {
        if (new_diag < ol[i].min_diag) ol[i].min_diag = new_diag;
        if (new_diag > ol[i].max_diag) ol[i].max_diag = new_diag;
        if (s_lo < ol[i].slb) ol[i].slb = s_lo;
        if (s_hi > ol[i].srb) ol[i].srb = s_hi;
        if (t_lo < ol[i].tlb) ol[i].tlb = t_lo;
        if (t_hi > ol[i].trb) ol[i].trb = t_hi;
        if (qual < ol[i].quality) {
          ol[i].s_lo = s_lo; ol[i].s_hi = s_hi; ol[i].t_lo = t_lo; ol[i].t_hi = t_hi;
          ol[i].quality = qual;
          ol[i].delta_ct = delta_ct;
          return i;
        }
        return -1;
      }
    }
  }
  if (ct >= MAX_DISTINCT_OLAPS) return -1;
  OlapInfo &o = ol[ct];
  o.s_lo = o.slb = s_lo;
  o.s_hi = o.srb = s_hi;
  o.t_lo = o.tlb = t_lo;
  o.t_hi = o.trb = t_hi;
  o.quality = qual;
  o.delta_ct = delta_ct;
  o.min_diag = o.max_diag = t_lo - s_lo;
  ct++;
  return ct - 1;
}

// ---- the window filter (-w, Process_String_Overlaps.C:562-621) ------------------------
#define OVL_QUALITY_CUTOFF 20                  // overlapInCore.H:190
#define OVL_BAD_WINDOW_LEN 50                  // overlapInCore.H:80
#define OVL_BAD_WINDOW_VALUE (8 * OVL_QUALITY_CUTOFF)

struct BaseAt {
  uint32_t code;
  bool wild;     // 'n' (forward strands)
  bool nul;      // NUL (reverse complement of an 'n')
};
__device__ __forceinline__ BaseAt base_at(const Strand &s, int32_t p) {
  BaseAt b;
  b.code = (uint32_t)(s.w[p >> 5] >> (2 * (p & 31))) & 3u;
  b.wild = s.ex_wild && ((s.ex_wild[p >> 5] >> (p & 31)) & 1u);
  b.nul = s.ex_nul && ((s.ex_nul[p >> 5] >> (p & 31)) & 1u);
  return b;
}

// One olap's quality-difference string q (one value per alignment column: 0 on a match or
// an 'n', else min(quality, quality, cutoff); an indel column takes the quality of the
// base it skips) and Has_Bad_Window (:365) over it, lane-parallel: the columns are
// generated from the delta by segment (prefix scans), their prefix sums go to scr, and
// every window is one subtraction.  Returns 0 (kept), 1 (bad short window), 2 (bad long).
__device__ int32_t window_reject(const ExtendArgs &X, const Unit &un, uint32_t tgt,
                                 const OlapInfo &o, const int32_t *od, int32_t *scr,
                                 uint32_t lane) {
  typedef __attribute__((address_space(1))) int32_t g_i32;
  g_i32 *segC = (g_i32 *)scr, *segI = segC + (o.delta_ct + 1), *segJ = segI + (o.delta_ct + 1);
  g_i32 *P = segJ + (o.delta_ct + 1);
  const Strand S = un.dir ? strand_rc(X.R, un.r) : strand_fwd(X.R, un.r);
  const Strand T = strand_fwd(X.R, tgt);
  const uint8_t *sq = X.R.qual + X.R.wofs[un.r] * 32;
  const uint8_t *tq = X.R.qual + X.R.wofs[tgt] * 32;
  const int32_t SL = S.len;
  const int32_t dct = o.delta_ct;
  int32_t cc = 0, ci = o.s_lo, cj = o.t_lo;
  for (int32_t k0 = 0; k0 < dct; k0 += 64) {
    const int32_t k = k0 + (int32_t)lane;
    const bool in = k < dct;
    const int32_t v = in ? od[k] : 0;
    const int32_t a = v < 0 ? -v : v;
    const int32_t ic = in ? a : 0;
    const int32_t ii = in ? a - 1 + (v > 0 ? 1 : 0) : 0;
    const int32_t ij = in ? a - 1 + (v < 0 ? 1 : 0) : 0;
    const int32_t sc = wave_incl_scan(ic), si = wave_incl_scan(ii), sj = wave_incl_scan(ij);
    if (in) { segC[k] = cc + sc - ic; segI[k] = ci + si - ii; segJ[k] = cj + sj - ij; }
    cc += __builtin_amdgcn_readlane(sc, 63);
    ci += __builtin_amdgcn_readlane(si, 63);
    cj += __builtin_amdgcn_readlane(sj, 63);
  }
  if (lane == 0) { segC[dct] = cc; segI[dct] = ci; segJ[dct] = cj; }
  const int32_t tail = o.s_hi - ci + 1;
  const int32_t n = cc + (tail > 0 ? tail : 0);
  if (n < OVL_BAD_WINDOW_LEN) return 0;
  vm_sync();
  int32_t carry = 0;
  if (lane == 0) P[0] = 0;
  for (int32_t c0 = 0; c0 < n; c0 += 64) {
    const int32_t c = c0 + (int32_t)lane;
    int32_t q = 0;
    if (c < n) {
      int32_t lo = 0, hi = dct;               // last segment with segC <= c
      while (lo < hi) {
        const int32_t mid = (lo + hi + 1) >> 1;
        if (segC[mid] <= c) lo = mid; else hi = mid - 1;
      }
      const int32_t u = c - segC[lo];
      const int32_t i = segI[lo] + u, j = segJ[lo] + u;
      int32_t dv = 0;
      if (lo < dct && u == (od[lo] < 0 ? -od[lo] : od[lo]) - 1) {
        dv = od[lo] > 0 ? (int32_t)sq[un.dir ? SL - 1 - i : i] : (int32_t)tq[j];
      } else {
        const BaseAt bs = base_at(S, i), bt = base_at(T, j);
        const bool same = !bs.wild && !bt.wild && !bs.nul && bs.code == bt.code;
        if (!(same || bs.wild || bt.wild)) {
          const int32_t qs = sq[un.dir ? SL - 1 - i : i], qt = tq[j];
          dv = qs < qt ? qs : qt;
        }
      }
      q = dv < OVL_QUALITY_CUTOFF ? dv : OVL_QUALITY_CUTOFF;
    }
    const int32_t sc = wave_incl_scan(q);
    if (c < n) P[c + 1] = carry + sc;
    carry += __builtin_amdgcn_readlane(sc, 63);
  }
  vm_sync();
  bool bad = false;
  for (int32_t p0 = 0; p0 + OVL_BAD_WINDOW_LEN <= n; p0 += 64) {
    const int32_t p = p0 + (int32_t)lane;
    if (p + OVL_BAD_WINDOW_LEN <= n && P[p + OVL_BAD_WINDOW_LEN] - P[p] >= OVL_BAD_WINDOW_VALUE)
      bad = true;
  }
  if (__builtin_amdgcn_ballot_w64(bad)) return 1;
  for (int32_t p0 = 0; p0 + 100 <= n; p0 += 64) {
    const int32_t p = p0 + (int32_t)lane;
    if (p + 100 <= n && P[p + 100] - P[p] >= 240) bad = true;
  }
  return __builtin_amdgcn_ballot_w64(bad) ? 2 : 0;
}

__device__ bool lies_on_alignment(int32_t start, int32_t offset, int32_t s_lo, int32_t t_lo,
                                  const int32_t *LD, int32_t ld_len) {
  int32_t diag = t_lo - s_lo, new_diag = offset - start;
  for (int32_t i = 0; i < ld_len; i++) {
    int32_t v = LD[i];
    s_lo += v < 0 ? -v : v;
    if (start < s_lo) return abs(new_diag - diag) <= SHIFT_SLACK;
    if (v < 0) diag++;
    else { s_lo++; diag--; }
  }
  return abs(new_diag - diag) <= SHIFT_SLACK;
}

#define OVL_SCAP_WORDS 352          // LDS strand cache: up to 11,232 bases per strand
#define OVL_LDCAP 512                 // LDS Left_Delta cache

// Process_Matches (Process_String_Overlaps.C:400) for one pair, strands S (query, in its
// orientation) and T (target, forward) -- global or LDS-staged.
// Returns false when the pair must be redone by the generic kernel (register window
// overflow); nothing has been output for it then, and removed nodes are marked ~Len so the
// generic kernel can restore them.
template <bool FAST, bool L16, bool ORD, int RJ, typename SS>
__device__ bool process_pair(const ExtendArgs &X, const PairRec &P, const Unit &un,
                             const SS &S, const SS &T, const WaveMem &WM, int32_t *stk,
                             int32_t *RD, int32_t *LD, unsigned long long *st, uint32_t lane,
                             int32_t *ab) {
  uint32_t S_ID = X.R.first_iid + un.r, T_ID = X.R.first_iid + P.tgt;
  int32_t S_Len = S.len, t_len = T.len;
  Node *nodes = X.pnodes + P.node_off;
  int32_t nn = (int32_t)P.node_cnt;
  // the target's screened-end bits as its hash batch set them (PairRec bits 3 / 4): the
  // read flags themselves belong to whichever batch was built last
  const uint32_t trf = (P.flags >> 2) & 6u;
  bool consistent = P.flags & 1u;
  bool lscr = P.flags & 2u, rscr = P.flags & 4u;

  // computeMinimumKmers (Process_String_Overlaps.C:81), Process_String_Olaps:725
  if (X.filter_by_kmer_count != 0) {
    double ovl_len = (double)(P.diag_end - P.diag_bgn);
    if (ovl_len < 0) ovl_len = -ovl_len;
    uint64_t expct = 0;
    if (!(ovl_len < (double)X.k))
      expct = (uint64_t)(int)floor(X.minkmer_exp * (ovl_len - X.k + 1));
    uint64_t mk = expct > X.filter_by_kmer_count ? expct : X.filter_by_kmer_count;
    if (mk > (uint64_t)P.diag_ct) { st[2]++; return true; }
  }

  // hopeless check (:433)
  if (X.use_hopeless && nn == 1 && !X.partial) {
    Node h = nodes[0];
    int32_t s_head = h.Start, t_head = h.Offset;
    bool hopeless = false;
    if (s_head <= t_head) {
      if (s_head > 90 && !lscr) hopeless = true;
    } else {
      if (t_head > 90 && !(trf & 2u)) hopeless = true;
    }
    int32_t s_tail = S_Len - s_head - h.Len + 1;
    int32_t t_tail = t_len - t_head - h.Len + 1;
    if (s_tail <= t_tail) {
      if (s_tail > 90 && !rscr) hopeless = true;
    } else {
      if (t_tail > 90 && !(trf & 4u)) hopeless = true;
    }
    if (hopeless) { st[0]++; return true; }
  }
  if (X.dbg && lane == 0) atomicAdd(&X.dbg[8], 1ull);

  OlapInfo ol[MAX_DISTINCT_OLAPS];
  int32_t ct = 0;
  int32_t kind = K_NONE, S_Lo = 0, S_Hi = 0, T_Lo = 0, T_Hi = 0;
  int32_t remaining = nn;
  int32_t ld_len = 0;
#ifdef OVL_PROFILE
  if (X.dbg && lane == 0) atomicAdd(&X.dbg[22], (unsigned long long)nn);
#endif
  // Measured and not kept (r02v A/B, 10k reads, records identical): finding the next longest
  // match inside the removal pass, which loads every node anyway (214.5 vs 215.4 ms); and
  // skipping the removal pass when an extension reproduces the alignment the survivors were
  // last tested against, coordinates and deltas compared (217 / 214 vs 222 ms: the compare,
  // the saved deltas and the state carried across the row-loop calls cost more than the pass)
  while (remaining > 0) {
    // longest remaining match, first in list order on ties (:473-480)
    PROF_T(pa0);
    int32_t bv = -1, bi = 0x7fffffff;
    for (int32_t i = lane; i < nn; i += 64) {
      int32_t L = nodes[i].Len;
      if (L > bv) { bv = L; bi = i; }
    }
    wave_argmax(bv, bi);
    Node M = nodes[bi];
    if (X.dbg && lane == 0) atomicAdd(&X.dbg[5], 1ull);
#ifdef OVL_PROFILE
    { PROF_T(pa1); const int32_t mx = M.Len; if (X.dbg && lane == 0 && mx >= 0) atomicAdd(&X.dbg[20], pa1 - pa0); }
#endif
    // -l: no extension once the unit has its limit of overlaps off that end (:481-487); the
    // match is still dropped with the previous extension's alignment (kind, S_Lo.., deltas)
    bool hit_limit = false;
    if constexpr (ORD) {
      const int32_t a_hang = M.Start - M.Offset, b_hang = a_hang + S_Len - t_len;
      hit_limit = ((uint64_t)ab[0] >= X.olim && a_hang <= 0) ||
                  ((uint64_t)ab[1] >= X.olim && b_hang <= 0);
    }
    if (!hit_limit) {
      PROF_T(px0);
      ExtOut eo = extend_alignment<FAST, L16, RJ>(X, M, S, S_Len, T, t_len, WM, stk, RD, LD, lane);
#ifdef OVL_PROFILE
      PROF_T(px1);
      if (X.dbg && lane == 0) atomicAdd(&X.dbg[15], px1 - px0);
#endif
      if (FAST && eo.kind < 0) return false;
      kind = eo.kind;
      S_Lo = eo.S_Lo; S_Hi = eo.S_Hi; T_Lo = eo.T_Lo; T_Hi = eo.T_Hi;
      ld_len = eo.ld_len;
      if (kind == K_DOVETAIL || X.partial) {
        if (1 + S_Hi - S_Lo >= X.min_olap_len && 1 + T_Hi - T_Lo >= X.min_olap_len) {
          int32_t olap_len = 1 + ((S_Hi - S_Lo) < (T_Hi - T_Lo) ? (S_Hi - S_Lo) : (T_Hi - T_Lo));
          double quality = (double)eo.Errors / olap_len;
          if (eo.Errors <= X.error_bound[olap_len]) {
            const int32_t slot = add_overlap(X, S_Lo, S_Hi, T_Lo, T_Hi, quality, ld_len, ol, ct);
            if (X.window && slot >= 0) {               // memcpy(olap[i].delta, Left_Delta)
              int32_t *od = LD + (2 + slot) * (X.e_cap + 8);
              for (int32_t i = lane; i < ld_len; i += 64) od[i] = LD[i];
              vm_sync();
            }
          }
        }
      }
    }
    if (consistent) break;
    // drop the longest match and every match on this alignment (:517-531)
    PROF_T(pr0);
    int32_t removed = 0;
    const bool on_aln = (kind == K_DOVETAIL || X.partial);
    // thresholds and diagonals as int16 when every read is < 16384 (the staged kernel's
    // L16; for the generic kernel L16 means global rows, GR), else int32
    constexpr bool T16 = FAST && L16;
    typedef typename std::conditional<T16, __attribute__((address_space(3))) int16_t,
                                      lds_i32>::type lds_t;
    constexpr int32_t per = T16 ? 1 : 2;               // ints per (thr, diag) pair
    // Lies_On_Alignment (:307) by binary search: walking the deltas, delta i is reached
    // with (s_i, diag_i); the walk stops at the first i with start < thr_i = s_i + |LD[i]|
    // and compares with diag_i (or with the final diag).  thr is non-decreasing.  The
    // thresholds live in the wave's LDS scratch.
    auto by_search = [&](auto *thr, auto *dgl, auto sync) {
      int32_t cs = S_Lo, cd = T_Lo - S_Lo;
      for (int32_t i0 = 0; i0 < ld_len; i0 += 64) {
        const int32_t i = i0 + (int32_t)lane;
        const bool in = i < ld_len;
        const int32_t v = in ? LD[i] : 0;
        const int32_t a = v < 0 ? -v : v;
        const int32_t inc_s = in ? a + (v >= 0 ? 1 : 0) : 0;
        const int32_t inc_d = in ? (v < 0 ? 1 : -1) : 0;
        const int32_t ss = wave_incl_scan(inc_s), sd = wave_incl_scan(inc_d);
        if (in) {
          thr[i] = cs + (ss - inc_s) + a;
          dgl[i] = cd + (sd - inc_d);
        }
        cs += __builtin_amdgcn_readlane(ss, 63);
        cd += __builtin_amdgcn_readlane(sd, 63);
      }
      if (lane == 0) { thr[ld_len] = T16 ? 32767 : 0x7fffffff; dgl[ld_len] = cd; }
      sync();
      for (int32_t i = lane; i < nn; i += 64) {
        Node nd = nodes[i];
        if (nd.Len < 0) continue;
        bool rm = (i == bi);
        if (!rm && S_Lo - SHIFT_SLACK <= nd.Start &&
            nd.Start + nd.Len <= (S_Hi + 1) + SHIFT_SLACK - 1) {
          int32_t lo = 0, hi = ld_len;               // first index with thr > start
          while (lo < hi) {
            const int32_t mid = (lo + hi) >> 1;
            if ((int32_t)thr[mid] > nd.Start) hi = mid;
            else lo = mid + 1;
          }
          const int32_t dd = (nd.Offset - nd.Start) - (int32_t)dgl[lo];
          rm = (dd < 0 ? -dd : dd) <= SHIFT_SLACK;
        }
        if (rm) { nodes[i].Len = ~nd.Len; removed++; }
      }
      sync();
    };
    if (on_aln && per * (ld_len + 1) <= WM.ldcap) {
      lds_t *thr = (lds_t *)WM.ldc;
      by_search(thr, thr + ld_len + 1, [] { lds_sync(); });
    } else {
      const int32_t *ldp = LD;
      if (ld_len <= WM.ldcap) {
        for (int32_t i = lane; i < ld_len; i += 64) WM.ldc[i] = LD[i];
        lds_sync();
        ldp = (const int32_t *)WM.ldc;
      }
      for (int32_t i = lane; i < nn; i += 64) {
        Node nd = nodes[i];
        if (nd.Len < 0) continue;
        bool rm = (i == bi) ||
                  (on_aln && S_Lo - SHIFT_SLACK <= nd.Start &&
                   nd.Start + nd.Len <= (S_Hi + 1) + SHIFT_SLACK - 1 &&
                   lies_on_alignment(nd.Start, nd.Offset, S_Lo, T_Lo, ldp, ld_len));
        if (rm) { nodes[i].Len = ~nd.Len; removed++; }
      }
    }
    for (int s = 32; s > 0; s >>= 1) removed += __shfl_xor(removed, s);
    remaining -= removed;
    vm_sync();
#ifdef OVL_PROFILE
    PROF_T(pr1);
    if (X.dbg && lane == 0) atomicAdd(&X.dbg[21], pr1 - pr0);
#endif
  }

  int32_t outputs = 0;
  if (ct > 0) {
    bool del[MAX_DISTINCT_OLAPS] = {false, false, false};
    if (X.partial) {
      if (X.unique) {                       // Choose_Best_Partial (:336)
        int32_t best = 0;
        double mb0 = (1.0 - ol[0].quality) *
                     (2 + ol[0].s_hi - ol[0].s_lo + ol[0].t_hi - ol[0].t_lo);
        for (int32_t i = 1; i < ct; i++) {
          double mb = (1.0 - ol[i].quality) *
                      (2 + ol[i].s_hi - ol[i].s_lo + ol[i].t_hi - ol[i].t_lo);
          if (mb0 < mb || (mb0 == mb && ol[i].quality < ol[best].quality)) best = i;
        }
        for (int32_t i = 0; i < ct; i++) del[i] = (i != best);
      }
    } else if (X.unique) {                  // Combine_Into_One_Olap (:95)
      int32_t best = 0;
      for (int32_t i = 1; i < ct; i++)
        if (ol[i].quality < ol[best].quality) best = i;
      for (int32_t i = 0; i < ct; i++) del[i] = (i != best);
    } else {                                // Merge_Intersecting_Olaps (:153)
      for (int32_t i = 0; i < ct - 1; i++)
        for (int32_t j = i + 1; j < ct; j++) {
          if (del[i] || del[j]) continue;
          int32_t lo = ol[i].min_diag, hi = ol[i].max_diag;
          if ((lo <= 0 && ol[j].min_diag > 0) || (lo > 0 && ol[j].min_diag <= 0)) continue;
          if ((lo >= 0 && ol[j].trb - lo - ol[j].slb >= MIN_INTERSECTION) ||
              (lo <= 0 && ol[j].srb + lo - ol[j].tlb >= MIN_INTERSECTION) ||
              (hi >= 0 && ol[j].trb - hi - ol[j].slb >= MIN_INTERSECTION) ||
              (hi <= 0 && ol[j].srb + hi - ol[j].tlb >= MIN_INTERSECTION)) {
            int32_t keep, disc;
            if (ol[i].quality < ol[j].quality) { keep = i; disc = j; del[j] = true; }
            else                               { keep = j; disc = i; del[i] = true; }
            if (ol[disc].min_diag < ol[keep].min_diag) ol[keep].min_diag = ol[disc].min_diag;
            if (ol[disc].max_diag > ol[keep].max_diag) ol[keep].max_diag = ol[disc].max_diag;
            if (ol[disc].slb < ol[keep].slb) ol[keep].slb = ol[disc].slb;
            if (ol[disc].srb > ol[keep].srb) ol[keep].srb = ol[disc].srb;
            if (ol[disc].tlb < ol[keep].tlb) ol[keep].tlb = ol[disc].tlb;
            if (ol[disc].trb > ol[keep].trb) ol[keep].trb = ol[disc].trb;
          }
        }
    }
    for (int32_t i = 0; i < ct; i++) {
      if (del[i]) continue;
      if (X.window) {
        const int32_t rej = window_reject(X, un, P.tgt, ol[i], LD + (2 + i) * (X.e_cap + 8),
                                          WM.rows, lane);
        if (rej) { st[6 + rej]++; continue; }      // Bad_Short / Bad_Long_Window_Ct
      }
      Rec rec;
      int32_t bhg = 0;
      if (X.partial) rec = output_partial(S_ID, T_ID, un.dir, ol[i], S_Len, t_len);
      else           rec = output_overlap(S_ID, S_Len, un.dir, T_ID, t_len, ol[i], &bhg);
      if (lane == 0) {
        uint32_t slot = atomicAdd(X.nout, 1u);
        if (slot < X.out_cap) X.out[slot] = rec;
        else atomicOr(X.overflow, 16u);
      }
      outputs++;
      st[4]++;
      if constexpr (ORD) {                             // A / B_Olaps_For_Frag (:631-635)
        if (ol[i].s_lo == 0) ab[0]++;
        if (ol[i].s_hi >= S_Len - 1) ab[1]++;
      }
      if (!X.partial) {
        if (bhg <= 0) st[5]++;
        else          st[6]++;
      }
    }
  }
  if (outputs == 0) st[0]++;
  else {
    st[1]++;
    if (outputs > 1) st[3]++;
  }
  return true;
}

// Copy a strand's packed words (and the guard) into LDS.  Only exception-free strands are
// staged: the staged kernel defers pairs with 'n' bases to the generic kernel.
__device__ __forceinline__ StrandLP stage_strand(const Strand &G, lds_u64 *dst, uint32_t lane) {
  int32_t nw = (G.len + 31) / 32 + 1;
  for (int32_t i = lane; i < nw; i += 64) {
    const uint64_t w = G.w[i];
    dst[i] = (uint64_t)compact_even(w) | ((uint64_t)compact_even(w >> 1) << 32);
  }
  StrandLP L;
  L.w = dst;
  L.len = G.len;
  return L;
}

// Words w0..w1 of a strand only (a pair's span, below): the returned strand keeps absolute
// positions (its base pointer is dst - w0), and only words in w0..w1 are ever read.
__device__ __forceinline__ StrandLP stage_strand_span(const Strand &G, lds_u64 *dst, int32_t w0,
                                                      int32_t w1, uint32_t lane) {
  for (int32_t i = w0 + (int32_t)lane; i <= w1; i += 64) {
    const uint64_t w = G.w[i];
    dst[i - w0] = (uint64_t)compact_even(w) | ((uint64_t)compact_even(w >> 1) << 32);
  }
  StrandLP L;
  L.w = dst - w0;
  L.len = G.len;
  return L;
}

__device__ __forceinline__ int32_t wave_min_i32(int32_t v) {
  for (int o = 32; o > 0; o >>= 1) {
    const int32_t t = __shfl_xor(v, o);
    v = t < v ? t : v;
  }
  return v;
}

#define OVL_SCR_STAGE 256        // the staged kernel's per-wave LDS scratch ints
                                 // (Lies_On_Alignment thresholds, Left_Delta cache)

// STAGE = true: exception-free pairs, strands staged in LDS, rows in registers; pairs with
// 'n' bases or a band wider than the register window are deferred to the generic kernel.
// STAGE = false: the generic kernel (global strands with exception masks, rows in LDS).
// L16, staged kernel: every read < 16384 bases, so the traceback log holds 16-bit cells.
// L16, generic kernel: GR -- the rows and the Edit_Match_Limit table stay in global memory
// (error limits past what a CU's LDS holds; see wave_ped).
// ORD (with STAGE = false): the -l kernel, one unit per wave (see ExtendArgs.olim).
#ifndef OVL_EXT_OCC
#define OVL_EXT_OCC 6            // waves per SIMD the staged kernel is compiled for
#endif
// RJ: register chunks of the staged kernel's row window (OVL_RJ; the wide class that takes
// the pairs whose band outgrows it runs 2 x OVL_RJ at lower occupancy)
// Block-shared query strands (the pairs of one unit share the query strand, so a block can
// hold a few query strands and each wave stage only its target: 32 waves per CU at 10 kb)
// were built and measured in round 4, and ran slower (waves idle at a slot's end of pairs;
// DESIGN.md round 4): not kept.
template <bool STAGE, bool L16, bool ORD = false, int RJ = OVL_RJ>
__global__ void __launch_bounds__(512, RJ > OVL_RJ ? 3 : OVL_EXT_OCC)
k_extend(ExtendArgs X) {
  extern __shared__ __attribute__((aligned(16))) int32_t s_ext0[];
  uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  uint32_t gw = blockIdx.x * (blockDim.x >> 6) + wave;
  constexpr bool GR = !STAGE && L16;
  constexpr bool NOML = GR;                         // no LDS Edit_Match_Limit table
  int32_t mlsz = NOML ? 0 : ((X.e_cap + 2) + 3) & ~3;
  if constexpr (!NOML) {
    for (int32_t i = threadIdx.x; i < X.e_cap + 2; i += blockDim.x)
      s_ext0[i] = (i <= X.max_errors) ? X.match_limit[i] : 0x7fffffff;
  }
  __syncthreads();
  lds_i32 *l_ext0 = (lds_i32 *)s_ext0;
  lds_i32 *s_ext = l_ext0 + mlsz;
  WaveMem WM;
  WM.rows = X.rows + (size_t)gw * X.rows_cap;
  WM.rowdir = X.rowdir + (size_t)gw * 4 * (X.e_cap + 2);
  WM.mlim = l_ext0;
  WM.rmlim = l_ext0;
  lds_u64 *sw = nullptr, *tw = nullptr;
  if constexpr (STAGE) {
    // per wave: [S words | T words] (u64) then the scratch
    uint32_t wave_ints = 4 * (uint32_t)X.sw_words + OVL_SCR_STAGE;
    lds_i32 *wlds = s_ext + wave * wave_ints;
    sw = (lds_u64 *)wlds;
    tw = sw + X.sw_words;
    WM.lrow = nullptr;
    WM.wcap = 0;
    WM.tbw = wlds + 4 * X.sw_words;
    WM.ldc = WM.tbw;
    WM.ldcap = OVL_SCR_STAGE;
  } else {
    // per wave: row buffers (not with GR), traceback window, delta cache
    int32_t wcap = GR ? 0 : 2 * X.e_cap + 8;
    uint32_t wave_ints = (2 * wcap + TB_ROWS * TB_W + OVL_LDCAP + 3) & ~3u;
    lds_i32 *wlds = s_ext + wave * wave_ints;
    WM.lrow = wlds;
    WM.wcap = wcap;
    WM.tbw = WM.lrow + 2 * wcap;
    WM.ldc = WM.tbw + TB_ROWS * TB_W;
    WM.ldcap = OVL_LDCAP;
  }
  // per wave: stack | Right_Delta | Left_Delta | spare | the three olaps' delta copies (-w)
  int32_t *stk = X.deltas + (size_t)gw * 7 * (X.e_cap + 8);
  int32_t *RD = stk + (X.e_cap + 8);
  int32_t *LD = RD + (X.e_cap + 8);
  unsigned long long st[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
  const uint32_t npairs = X.npairs_dev ? __builtin_amdgcn_readfirstlane(*X.npairs_dev) : X.npairs;

  if constexpr (ORD) {
    static_assert(!STAGE, "the -l kernel is the generic one");
    for (;;) {
      uint32_t ui = 0;
      if (lane == 0) ui = atomicAdd(X.pair_next, 1u);
      ui = __shfl(ui, 0);
      if (ui >= X.nunits) break;
      const uint32_t b = X.useg[ui], e = X.useg[ui + 1];
      int32_t ab[2] = {0, 0};                // A_ / B_Olaps_For_Frag (Find_Overlaps.C:306)
      auto run = [&](uint32_t pi) {
        PairRec P = X.pairs[pi];
        Unit un = X.units[P.unit];
        Strand S = un.dir ? strand_rc(X.R, un.r) : strand_fwd(X.R, un.r);
        Strand T = strand_fwd(X.R, P.tgt);
        process_pair<false, L16, true, OVL_RJ>(X, P, un, S, T, WM, stk, RD, LD, st, lane, ab);
        lds_sync();
      };
      if ((uint64_t)(e - b) <= X.olim) {     // Process_String_Olaps.C:721
        for (uint32_t i = b; i < e; i++) run(X.ord_slot[i]);
      } else {                               // :746-790: by average diagonal, >= 0 first
        uint32_t start = b;
        while (start < e && X.dkey[X.ord_diag[start]] < (1ull << 63)) start++;
        for (uint32_t i = start; i < e && (uint64_t)ab[0] < X.olim; i++) run(X.ord_diag[i]);
        for (uint32_t i = start; i > b && (uint64_t)ab[1] < X.olim; i--) run(X.ord_diag[i - 1]);
      }
    }
  } else
  for (;;) {
    uint32_t pi = 0;
    if (lane == 0) pi = atomicAdd(X.pair_next, 1u);
    pi = __shfl(pi, 0);
    if (pi >= npairs) break;
    if (X.list) pi = X.list[pi];
    PairRec P = X.pairs[pi];
    Unit un = X.units[P.unit];
    Strand S = un.dir ? strand_rc(X.R, un.r) : strand_fwd(X.R, un.r);
    Strand T = strand_fwd(X.R, P.tgt);
    if (X.restore) {
      // a pair deferred by an earlier launch may have had nodes removed (~Len) before it
      // stopped there
      Node *nodes = X.pnodes + P.node_off;
      for (uint32_t i = lane; i < P.node_cnt; i += 64)
        if (nodes[i].Len < 0) nodes[i].Len = ~nodes[i].Len;
      vm_sync();
    }
    if constexpr (STAGE) {
      bool ok = false;
      // The pair's span: every extension of Process_Matches starts on one of its matches'
      // diagonals (a - b), and the greedy rows of e errors stay within e diagonals of it
      // (at most the class's e_cap), sliding at most to the reads' ends along them; the row
      // slides read 64 bases from a 32-base word.  So A is read only inside
      // [max(0, dmin), min(La, Lb + dmax)] and B inside [max(0, -dmax), min(Lb, La - dmin)],
      // each widened by e_cap + 128 bases: those words are staged, not the whole reads, and a
      // pair of long reads whose overlap span fits this class's LDS runs at its occupancy.
      int32_t dmin = 0x7fffffff, dmax = (int32_t)0x80000000;
      {
        const Node *nodes = X.pnodes + P.node_off;
        for (uint32_t i = lane; i < P.node_cnt; i += 64) {
          const Node nd = nodes[i];
          const int32_t d = nd.Start - nd.Offset;
          dmin = d < dmin ? d : dmin;
          dmax = d > dmax ? d : dmax;
        }
        dmin = __builtin_amdgcn_readfirstlane(wave_min_i32(dmin));
        dmax = wave_max(dmax);                 // lanes without a node hold the identities
      }
      const int32_t La = S.len, Lb = T.len, mg = X.e_cap + 128;
      const int32_t a_lo = max(0, max(0, dmin) - mg), a_hi = min(La, min(La, Lb + dmax) + mg);
      const int32_t b_lo = max(0, max(0, -dmax) - mg), b_hi = min(Lb, min(Lb, La - dmin) + mg);
      // words of the span, the guard word (index (L + 31) / 32) included at a read's end
      const int32_t aw0 = a_lo >> 5, aw1 = min((La + 31) >> 5, (a_hi >> 5) + 1);
      const int32_t bw0 = b_lo >> 5, bw1 = min((Lb + 31) >> 5, (b_hi >> 5) + 1);
      if (!(S.ex_wild || S.ex_nul || T.ex_wild) && P.node_cnt > 0 &&
          aw1 - aw0 + 1 <= X.sw_words && bw1 - bw0 + 1 <= X.sw_words) {
        StrandLP SL = stage_strand_span(S, sw, aw0, aw1, lane);
        StrandLP TL = stage_strand_span(T, tw, bw0, bw1, lane);
        lds_sync();
        PROF_T(pp0);
        ok = process_pair<true, L16, false, RJ>(X, P, un, SL, TL, WM, stk, RD, LD, st, lane, nullptr);
#ifdef OVL_PROFILE
        PROF_T(pp1);
        if (X.dbg && lane == 0) atomicAdd(&X.dbg[13], pp1 - pp0);
#endif
      }
      if (!ok && lane == 0) X.defer[atomicAdd(X.ndefer, 1u)] = pi;
    } else {
      process_pair<false, L16, false, OVL_RJ>(X, P, un, S, T, WM, stk, RD, LD, st, lane, nullptr);
    }
    lds_sync();
  }
  if (lane == 0)
    for (int i = 0; i < 9; i++)
      if (st[i]) atomicAdd(&X.stats[i < 7 ? i : i + 1], st[i]);
}

}  // namespace ovl
