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
  Node *pnodes;                 // Len < 0 marks a node removed from its list
  uint32_t *pair_next;
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
  Rec *out;
  uint32_t *nout;
  uint32_t out_cap;
  unsigned long long *stats;    // 0 without 1 with 2 skipped 3 multi 4 total 5 contained 6 dovetail
  uint32_t *overflow;
};

#define TB_ROWS 16
#define TB_W    (2 * TB_ROWS + 3)

struct PedOut {
  int32_t err;
  int32_t a_len, t_len;    // extents in A and T (positive)
  int32_t leftover;
  int32_t mte;
  int32_t nd;              // deltas produced
};

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

// Greedy prefix edit distance of A against a prefix of T (m <= n).
// DIR=+1: A[i] = A.w[a0+i], T[i] = T.w[t0+i]   (forward.C:103)
// DIR=-1: A[i] = A.w[a0-i], T[i] = T.w[t0-i]   (reverse.C:119)
// The traceback (Set_Right_Delta / Set_Left_Delta) writes the raw delta stack to dst.
template <int DIR>
__device__ PedOut wave_ped(const ExtendArgs &X, const Strand &A, int32_t a0, int32_t m,
                           const Strand &T, int32_t t0, int32_t n, int32_t limit,
                           int32_t *rows, int32_t *rowdir, int32_t *dst, int32_t *tbw,
                           uint32_t lane) {
  PedOut out;
  out.leftover = 0;
  out.nd = 0;
  auto slide = [&](int32_t r, int32_t d) -> int32_t {
    int32_t lim = m - r;
    int32_t l2 = n - r - d;
    if (l2 < lim) lim = l2;
    if (lim <= 0) return 0;
    if (DIR > 0) return slide_fwd(A, a0 + r, T, t0 + r + d, lim);
    return slide_bwd(A, a0 - r, T, t0 - r - d, lim);
  };

  int32_t row0 = (m > 0) ? slide(0, 0) : 0;
  if (lane == 0) { rowdir[0] = 0; rowdir[1] = -2; rows[2] = row0; }
  int32_t cursor = 5;
  if (row0 == m) {
    out.err = 0; out.a_len = m; out.t_len = m; out.mte = 1;
    out.leftover = m;          // reverse(): Leftover = m on an exact match
    out.nd = -1;               // no traceback
    return out;
  }

  double  max_score = 0.0;
  int32_t max_score_len = 0, max_score_best_d = 0, max_score_best_e = 0;
  int32_t best_d = 0, best_e = 0, longest = 0;
  int32_t left = 0, right = 0;
  int32_t prev_off = 0, prev_lo = -2;
  int32_t tb_e = -1, tb_d = 0;
  bool finished = false;
  const bool partial = X.partial != 0;

  int32_t e;
  for (e = 1; e <= limit; e++) {
    left = (left - 1 > -e) ? left - 1 : -e;
    right = (right + 1 < e) ? right + 1 : e;
    int32_t *prev = rows + prev_off - prev_lo;
    if (lane == 0) { prev[left] = -2; prev[left - 1] = -2; prev[right] = -2; prev[right + 1] = -2; }
    int32_t lo = left - 2, width = right - left + 5;
    int32_t off = cursor;
    cursor += width;
    if ((uint64_t)cursor > X.rows_cap || e > X.e_cap) {
      if (lane == 0) atomicOr(X.overflow, 8u);
      out.err = 0; out.a_len = 0; out.t_len = 0; out.mte = 0; out.nd = -1;
      return out;
    }
    if (lane == 0) { rowdir[2 * e] = off; rowdir[2 * e + 1] = lo; }
    int32_t *cur = rows + off - lo;
    vm_sync();

    int32_t end_d = 0x7fffffff, end_row = 0;
    for (int32_t c = left; c <= right; c += 64) {
      int32_t d = c + (int32_t)lane;
      bool act = d <= right;
      int32_t r = 0;
      if (act) {
        r = 1 + prev[d];
        int32_t j = prev[d - 1];
        if (j > r) r = j;
        j = 1 + prev[d + 1];
        if (j > r) r = j;
        if (r < m && r + d < n) r += slide(r, d);
        cur[d] = r;
      }
      uint64_t endm = __ballot(act && (r == m || r + d == n));
      if (endm) {
        uint32_t l = __builtin_ctzll(endm);
        end_d = c + (int32_t)l;
        end_row = __shfl(r, l);
        break;
      }
    }
    vm_sync();

    if (end_d != 0x7fffffff) {
      double  score = end_row * X.branch_match_value - e;
      int32_t tail_len = end_row - max_score_len;
      double  slope = (double)(max_score - score) / tail_len;
      bool    abort_here = false;
      if (partial && score < max_score) abort_here = true;
      if (e > X.min_branch_end_dist / 2 && tail_len >= X.min_branch_end_dist &&
          slope >= X.min_branch_tail_slope)
        abort_here = true;
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
          if (lane == 0) cur[d] = end_row;
          vm_sync();
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

    // Edit_Match_Limit pruning (forward.C:236-252)
    int32_t ML = X.match_limit[e];
    int32_t nl = 0x7fffffff;
    for (int32_t c = left; c <= right; c += 64) {
      int32_t d = c + (int32_t)lane;
      bool keep = false;
      if (d <= right) {
        int32_t v = cur[d];
        keep = (d < 0) ? !(v < ML) : !(v + d < ML);
      }
      uint64_t km = __ballot(keep);
      if (km) { nl = c + (int32_t)__builtin_ctzll(km); break; }
    }
    if (nl == 0x7fffffff) break;           // Left > Right
    int32_t nr = nl;
    for (int32_t c = right; c >= nl; c -= 64) {
      int32_t d = c - (int32_t)lane;
      bool keep = false;
      if (d >= nl) {
        int32_t v = cur[d];
        keep = (d > 0) ? !(v + d < ML) : !(v < ML);
      }
      uint64_t km = __ballot(keep);
      if (km) { nr = c - (int32_t)__builtin_ctzll(km); break; }
    }
    left = nl;
    right = nr;

    int32_t bv = -0x7fffffff, bd = 0x7fffffff;
    for (int32_t c = left; c <= right; c += 64) {
      int32_t d = c + (int32_t)lane;
      if (d <= right) {
        int32_t v = cur[d];
        if (v > bv || (v == bv && d < bd)) { bv = v; bd = d; }
      }
    }
    wave_argmax(bv, bd);
    if (bv > longest) { longest = bv; best_d = bd; best_e = e; }
    double score = longest * X.branch_match_value - e;
    if (score > max_score) {
      max_score = score;
      max_score_len = longest;
      max_score_best_d = best_d;
      max_score_best_e = best_e;
    }
    prev_off = off;
    prev_lo = lo;
  }
  if (!finished) {
    out.err = max_score_best_e;
    out.a_len = max_score_len;
    out.t_len = max_score_len + max_score_best_d;
    out.mte = 0;
    tb_e = max_score_best_e; tb_d = max_score_best_d;
  }

  // ---- traceback (Set_Right_Delta / Set_Left_Delta loop), 16-row LDS windows ---------
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
    // stage rows kl-1 .. kh-1, diagonals dc-(TB_ROWS+1) .. dc+(TB_ROWS+1)
    int32_t nrows = kh - kl + 1;
    for (int32_t i = lane; i < nrows * TB_W; i += 64) {
      int32_t rr = i / TB_W, w = i - rr * TB_W;
      int32_t row = kl - 1 + rr;
      int32_t ro = rowdir[2 * row], rl = rowdir[2 * row + 1];
      int32_t width = rowdir[2 * (row + 1)] - ro;
      int32_t dd = dc - (TB_ROWS + 1) + w;
      int32_t idx = dd - rl;
      tbw[i] = (idx >= 0 && idx < width) ? rows[ro + idx] : -3;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (lane == 0) {
      for (int32_t kk = kh; kk >= kl; kk--) {
        const int32_t *prow = tbw + (kk - 1 - (kl - 1)) * TB_W - (dc - (TB_ROWS + 1));
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
    __builtin_amdgcn_wave_barrier();
  }
  out.leftover = last;
  out.nd = nd;
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
__device__ ExtOut extend_alignment(const ExtendArgs &X, const Node &M, const Strand &S,
                                   int32_t S_Len, const Strand &T, int32_t T_Len,
                                   int32_t *rows, int32_t *rowdir, int32_t *stk, int32_t *RD,
                                   int32_t *LD, int32_t *tbw, uint32_t lane) {
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
    PedOut po;
    if (s_first)
      po = wave_ped<1>(X, S, S_Right_Begin, S_Right_Len, T, T_Right_Begin, T_Right_Len,
                       error_limit, rows, rowdir, stk, tbw, lane);
    else
      po = wave_ped<1>(X, T, T_Right_Begin, T_Right_Len, S, S_Right_Begin, S_Right_Len,
                       error_limit, rows, rowdir, stk, tbw, lane);
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
      rd_len = n - 1;
      vm_sync();
    }
  }
  S_Hi += S_Right_Begin - 1;
  T_Hi += T_Right_Begin - 1;

  if (S_Left_Begin < 0 || T_Left_Begin < 0) {
    S_Lo = 0; T_Lo = 0; lmte = 1;
  } else {
    bool s_first = S_Right_Begin <= T_Right_Begin;
    PedOut po;
    int32_t lim = error_limit - right_errors;
    if (s_first)
      po = wave_ped<-1>(X, S, S_Left_Begin, S_Left_Begin + 1, T, T_Left_Begin, T_Left_Begin + 1,
                        lim, rows, rowdir, LD, tbw, lane);
    else
      po = wave_ped<-1>(X, T, T_Left_Begin, T_Left_Begin + 1, S, S_Left_Begin, S_Left_Begin + 1,
                        lim, rows, rowdir, LD, tbw, lane);
    left_errors = po.err;
    lmte = po.mte;
    int32_t a_end = -po.a_len, t_end = -po.t_len;
    int32_t n_t = s_first ? T_Left_Begin + 1 : S_Left_Begin + 1;     // reverse()'s n
    leftover = po.leftover;
    if (po.nd >= 0) {
      ld_len = po.nd;
      vm_sync();
      // Set_Left_Delta fix-up (reverse.C:89-104): a leading +1 indel becomes a mismatch
      bool fix = ld_len > 1 && LD[0] == 1 && t_end + n_t > 0;
      if (fix) {
        int32_t l1 = LD[1];
        vm_sync();
        if (lane == 0) {
          LD[0] = (l1 > 0) ? l1 + 1 : l1 - 1;
          for (int32_t i = 2; i < ld_len; i++) LD[i - 1] = LD[i];
        }
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
__device__ void add_overlap(const ExtendArgs &X, int32_t s_lo, int32_t s_hi, int32_t t_lo,
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
        }
        return;
      }
    }
  }
  if (ct >= MAX_DISTINCT_OLAPS) return;
  OlapInfo &o = ol[ct];
  o.s_lo = o.slb = s_lo;
  o.s_hi = o.srb = s_hi;
  o.t_lo = o.tlb = t_lo;
  o.t_hi = o.trb = t_hi;
  o.quality = qual;
  o.delta_ct = delta_ct;
  o.min_diag = o.max_diag = t_lo - s_lo;
  ct++;
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

__global__ void __launch_bounds__(256) k_extend(ExtendArgs X) {
  __shared__ int32_t s_tb[4][TB_ROWS * TB_W];
  uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  uint32_t gw = blockIdx.x * 4 + wave;
  int32_t *rows = X.rows + (size_t)gw * X.rows_cap;
  int32_t *rowdir = X.rowdir + (size_t)gw * 2 * (X.e_cap + 2);
  int32_t *stk = X.deltas + (size_t)gw * 4 * (X.e_cap + 8);
  int32_t *RD = stk + (X.e_cap + 8);
  int32_t *LD = RD + (X.e_cap + 8);
  int32_t *tbw = s_tb[wave];
  unsigned long long st[7] = {0, 0, 0, 0, 0, 0, 0};

  for (;;) {
    uint32_t pi = 0;
    if (lane == 0) pi = atomicAdd(X.pair_next, 1u);
    pi = __shfl(pi, 0);
    if (pi >= X.npairs) break;
    PairRec P = X.pairs[pi];
    Unit un = X.units[P.unit];
    uint32_t S_ID = X.R.first_iid + un.r, T_ID = X.R.first_iid + P.tgt;
    Strand S = un.dir ? strand_rc(X.R, un.r) : strand_fwd(X.R, un.r);
    Strand T = strand_fwd(X.R, P.tgt);
    int32_t S_Len = S.len, t_len = T.len;
    Node *nodes = X.pnodes + P.node_off;
    int32_t nn = (int32_t)P.node_cnt;
    uint32_t trf = X.R.flags[P.tgt];
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
      if (mk > (uint64_t)P.diag_ct) { st[2]++; continue; }
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
      if (hopeless) { st[0]++; continue; }
    }

    OlapInfo ol[MAX_DISTINCT_OLAPS];
    int32_t ct = 0;
    int32_t kind = K_NONE, S_Lo = 0, S_Hi = 0, T_Lo = 0, T_Hi = 0;
    int32_t remaining = nn;
    int32_t ld_len = 0;
    while (remaining > 0) {
      // longest remaining match, first in list order on ties (:473-480)
      int32_t bv = -1, bi = 0x7fffffff;
      for (int32_t i = lane; i < nn; i += 64) {
        int32_t L = nodes[i].Len;
        if (L > bv) { bv = L; bi = i; }
      }
      wave_argmax(bv, bi);
      Node M = nodes[bi];
      ExtOut eo = extend_alignment(X, M, S, S_Len, T, t_len, rows, rowdir, stk, RD, LD, tbw,
                                   lane);
      kind = eo.kind;
      S_Lo = eo.S_Lo; S_Hi = eo.S_Hi; T_Lo = eo.T_Lo; T_Hi = eo.T_Hi;
      ld_len = eo.ld_len;
      if (kind == K_DOVETAIL || X.partial) {
        if (1 + S_Hi - S_Lo >= X.min_olap_len && 1 + T_Hi - T_Lo >= X.min_olap_len) {
          int32_t olap_len = 1 + ((S_Hi - S_Lo) < (T_Hi - T_Lo) ? (S_Hi - S_Lo) : (T_Hi - T_Lo));
          double quality = (double)eo.Errors / olap_len;
          if (eo.Errors <= X.error_bound[olap_len])
            add_overlap(X, S_Lo, S_Hi, T_Lo, T_Hi, quality, ld_len, ol, ct);
        }
      }
      if (consistent) break;
      // drop the longest match and every match on this alignment (:517-531)
      int32_t removed = 0;
      for (int32_t i = lane; i < nn; i += 64) {
        Node nd = nodes[i];
        if (nd.Len < 0) continue;
        bool rm = (i == bi) ||
                  ((kind == K_DOVETAIL || X.partial) && S_Lo - SHIFT_SLACK <= nd.Start &&
                   nd.Start + nd.Len <= (S_Hi + 1) + SHIFT_SLACK - 1 &&
                   lies_on_alignment(nd.Start, nd.Offset, S_Lo, T_Lo, LD, ld_len));
        if (rm) { nodes[i].Len = -1; removed++; }
      }
      for (int s = 32; s > 0; s >>= 1) removed += __shfl_xor(removed, s);
      remaining -= removed;
      vm_sync();
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
        int32_t mnd = ol[0].min_diag, mxd = ol[0].max_diag;
        int32_t slb = ol[0].slb, srb = ol[0].srb, tlb = ol[0].tlb, trb = ol[0].trb;
        for (int32_t i = 1; i < ct; i++) {
          if (ol[i].quality < ol[best].quality) best = i;
          if (ol[i].min_diag < mnd) mnd = ol[i].min_diag;
          if (ol[i].max_diag > mxd) mxd = ol[i].max_diag;
          if (ol[i].slb < slb) slb = ol[i].slb;
          if (ol[i].srb > srb) srb = ol[i].srb;
          if (ol[i].tlb < tlb) tlb = ol[i].tlb;
          if (ol[i].trb > trb) trb = ol[i].trb;
        }
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
  }
  if (lane == 0)
    for (int i = 0; i < 7; i++)
      if (st[i]) atomicAdd(&X.stats[i], st[i]);
}

}  // namespace ovl
