// ovl_api.hip -- the C-ABI (include/canu_ovl.h) and the host side of the HIP path.
//
// Host responsibilities mirror overlapInCore's driver (overlapInCore.C:190 OverlapDriver,
// :306 main): option fix-ups, the maxErate tables (prefixEditDistance.C:40-116,
// Binomial_Bound.C), read loading, then the per-batch kernel sequence
//   k_probe -> k_chain -> k_extend
// over (query, orientation) units.  There is no CPU fallback for any of it.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <chrono>
#include <cerrno>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <cstdlib>
#include <string>
#include <vector>

#include "../../include/canu_ovl.h"
#include "ovl_common.h"

#include "ovl_index.hip"
#include "ovl_seed.hip"
#include "ovl_extend.hip"
#include "ovl_ovb.h"

using namespace ovl;

// ---------------------------------------------------------------------------------------
static thread_local std::string g_err;

static int fail(int code, const char *fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

#define HIPC(x)                                                                         \
  do {                                                                                  \
    hipError_t _e = (x);                                                                \
    if (_e != hipSuccess)                                                               \
      return fail(OVL_ERR_HIP, "%s:%d %s: %s", __FILE__, __LINE__, #x,                 \
                  hipGetErrorString(_e));                                               \
  } while (0)

// wall time spent in device (re)allocation and frees (OVL_TIMING reports it)
static double g_alloc_ms = 0;
static uint64_t g_alloc_n = 0, g_alloc_bytes = 0;

template <typename T>
struct DBuf {
  T *p = nullptr;
  size_t n = 0;
  ~DBuf() { release(); }
  void release() {
    if (p) {
      const auto t0 = std::chrono::steady_clock::now();
      (void)hipFree(p);
      g_alloc_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    }
    p = nullptr;
    n = 0;
  }
  hipError_t alloc(size_t count) {
    if (count <= n && p) return hipSuccess;
    release();
    size_t bytes = std::max<size_t>(count, 1) * sizeof(T);
    const auto t0 = std::chrono::steady_clock::now();
    hipError_t e = hipMalloc((void **)&p, bytes);
    g_alloc_n++;
    g_alloc_bytes += bytes;
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    g_alloc_ms += ms;
    static const bool trace = getenv("OVL_TIMING") != nullptr;
    if (trace && bytes >= (1ull << 30))
      fprintf(stderr, "OVL_TIMING alloc %.2f GB (%zu x %zu B) %.1f ms%s\n", bytes / 1e9, count,
              sizeof(T), ms, e == hipSuccess ? "" : " FAILED");
    if (e == hipSuccess) n = count;
    else (void)hipGetLastError();                  // an OOM must not surface at a later check
    return e;
  }
  // search working buffers: sizes vary from batch to batch, so a regrow takes 1.5x (each
  // hipMalloc / hipFree of tens of GB costs seconds), or exactly `count` when 1.5x does not fit
  hipError_t grow(size_t count) {
    if (count <= n && p) return hipSuccess;
    if (p && alloc(std::max(count, n + n / 2)) == hipSuccess) return hipSuccess;
    return alloc(count);
  }
};

static const uint32_t AS_MAX_READLEN = (1u << 21) - 1;

// ---------------------------------------------------------------------------------------
// maxErate tables (prefixEditDistance.C:40-116; Binomial_Bound.C:47 and :121)

static int binomial_bound(int e, double p, int start) {
  const double bound = 1e-4, thold = 3.62;
  double q = 1.0 - p;
  if (start < e) start = e;
  for (int n = start; n < (int)AS_MAX_READLEN; n++) {
    if (n <= 35) {
      double sum = 0.0, p_pow = 1.0, q_pow = pow(q, n);
      int bin = 1, ct = 0;
      for (int k = 0; k < e && 1.0 - sum > bound; k++) {
        double x = bin * p_pow * q_pow;
        sum += x;
        bin *= n - ct;
        bin /= ++ct;
        p_pow *= p;
        q_pow /= q;
      }
      if (1.0 - sum > bound) return n;
    } else {
      double z = (e - 0.5 - n * p) / sqrt(n * p * q);
      if (z <= thold) return n;
      double sum = 0.0, mu_pow = 1.0, fact = 1.0, pc = exp(-n * p);
      for (int k = 0; k < e; k++) {
        sum += mu_pow * pc / fact;
        mu_pow *= n * p;
        fact *= k + 1;
      }
      if (1.0 - sum > bound) return n;
    }
  }
  return AS_MAX_READLEN;
}

static void init_match_limit(std::vector<int32_t> &ml, double erate, int32_t max_errors) {
  ml.assign(max_errors + 1, 0);
  int32_t e = 0, s = 1, l = std::min<int32_t>(max_errors, 2000);
  while (e <= 1) ml[e++] = 0;
  while (e < l) {
    s = binomial_bound(e - 1, erate, s);
    ml[e] = s - 1;
    e++;
  }
  double sl = 0.982064188397525 / erate + 0.067835741959926;   // AS_MAX_READLEN_BITS 21
  double vl = ml[e - 1] + sl;
  while (e < max_errors) {
    ml[e] = (int32_t)ceil(vl);
    vl += sl;
    e++;
  }
}

// ---------------------------------------------------------------------------------------

struct ovl_ctx {
  ovl_params P;
  int device = 0;
  int n_cu = 256;
  hipStream_t stream = nullptr;
  hipEvent_t ev[8];
  // find_overlaps runs the extension of hash-batch chunk i on xstream while the probe and
  // chain of chunk i+1 run on stream; xev[slot] / xev[2 + slot] bracket chunk i's extension
  hipStream_t xstream = nullptr;
  hipEvent_t xev[4];

  // tables
  int32_t max_errors = 0;
  double branch_match_value = 0, min_branch_tail_slope = 0;
  DBuf<int32_t> d_error_bound, d_match_limit;
  std::vector<int32_t> h_error_bound;

  // reads
  uint32_t first_iid = 0, nreads = 0;
  std::vector<uint32_t> h_len;
  std::vector<uint64_t> h_wofs;
  DBuf<uint64_t> d_fwd, d_rc, d_wofs;
  DBuf<uint32_t> d_fwdN, d_rcNul, d_len, d_flags, d_rcFirstNul;
  DBuf<uint8_t> d_qual;          // -w only: read r base i at wofs[r] * 32 + i
  bool have_qual = false;
  uint32_t max_len = 0;

  // skip k-mers (both strands, deduplicated codes)
  std::vector<uint64_t> h_skip;
  DBuf<uint64_t> d_skip;

  // index
  bool have_index = false;
  uint32_t hash_bgn_iid = 0, hash_end_iid = 0;
  DBuf<uint64_t> d_occ, d_tmpM2;
  DBuf<Rec2> d_tmpR, d_midR;     // build scratch: coarse- and fine-bucketed records
  // the build's bucket bookkeeping (coarse histogram and starts, fine starts and counts, a
  // few counters, the big-bucket list): kept too -- the driver's load cuts build the index
  // twice per hash batch, and a hipMalloc / hipFree pair per array per build added up
  DBuf<uint32_t> b_hist, b_cstart, b_cursor, b_fstart, b_fcnt, b_misc, b_big;
  DBuf<uint32_t> b_first;        // the driver's first-read histogram (load cuts)
  uint64_t cut_windows_hint = 0; // windows of the job's last load-cut batch (0: none yet)
  DBuf<TabEntry> d_tab;
  uint32_t tab_bits = 0, slice_bits = 0;
  DBuf<uint64_t> d_bloom;        // the batch's Bloom filter (driver batches: k_table)
  bool bloom_ok = false;
  uint32_t bloom_w = 0;

  // find_overlaps working buffers: kept across calls (grow-only), hipMalloc of tens of
  // GB per call would cost seconds
  // [2]: one per pipeline slot (chunk i's extension reads slot i & 1 while the chain of
  // chunk i + 1 writes the other)
  struct {
    DBuf<Unit> units[2];
    DBuf<uint64_t> rbase;
    DBuf<Probe> probe;
    DBuf<uint32_t> uhits, uflags, ctr, done, dset, big, defer, defer2, okey, oidx, okey2, oidx2;
    DBuf<uint32_t> live;          // the chain's units with at least one hit
    DBuf<uint32_t> xctr[2], xnout;
    DBuf<unsigned long long> chits;
    DBuf<uint8_t> otmp;
    DBuf<uint64_t> ok64a, ok64b, dkey;       // -l orders
    DBuf<uint64_t> hcnt, hbase;              // ovl_seed_hits: per-unit hit counts / bases
    DBuf<uint4> hbuf;                        // ovl_seed_hits: one piece of the hit list
    DBuf<uint32_t> oa, ob, ucnt, useg;
    DBuf<Node> pool, pnodes[2];
    DBuf<PairRec> pairs[2];
    DBuf<unsigned long long> stats;
    DBuf<int32_t> rows, rowdir, deltas;
  } fb;

  // library IDs (-H / -R filters); empty = every read in library 0
  std::vector<uint32_t> h_lib;
  bool nohash_set = false;       // some read carries OVL_RFLAG_NOHASH
  uint32_t stats_hash_lib_lo = 0, stats_hash_lib_hi = UINT32_MAX;   // -H of the index
  std::vector<uint32_t> ext_classes;       // read-length cap of each staged launch
  uint32_t stats_ext_waves = 0, stats_gen_waves = 0;
  uint64_t index_records = 0;    // records of the current index (windows + skip markers)
  // an OverlapDriver job's phase 3 (ovl_overlap_driver): the index buffers are allocated for
  // the largest super-batch at once, and the search buffers keep the size the first search
  // gave them -- a hipFree / hipMalloc of tens of GB on a nearly full device costs ~0.5 s
  uint64_t index_reserve = 0, sq_reserve = 0;
  bool sticky_budgets = false;
  // an OverlapDriver job whose sorted query windows need several chunks: tables at half the
  // slots (slices 1x the largest fine bucket's distinct k-mers instead of 2x), so that more
  // of the HBM holds query windows (fewer chunks, fewer super-batch rebuilds and probes)
  bool dense_tables = false;

  // pending extension work (see find_impl): chains of several probe chunks -- and of the
  // driver's hash batches -- are appended here and extended together in one launch
  struct {
    DBuf<Unit> units;
    DBuf<Node> pnodes;
    DBuf<PairRec> pairs;
    uint64_t nu = 0, nn = 0, np = 0;
  } acc;

  // OverlapDriver jobs: the query windows sorted by k-mer once per job (k_sq_keys,
  // k_probe_sorted in ovl_seed.hip; sq_prepare below).  sq_request: the driver asks find_impl
  // to use them from its second hash batch on (OVL_SQ=0 never, =1 from the first).
  bool sq_request = false;
  struct SqRun {
    uint32_t u0, u1;             // the run's units [u0, u1) of sq.units
    uint64_t e0, n;              // its windows: entries [e0, e0 + n) of key / wid
    uint64_t wb0, ub0;           // offsets of its unit bases (n units + 1) and 512-window blocks
  };
  struct {
    bool on = false;
    uint32_t ref_bgn = 0, ref_end = 0, lib_lo = 0, lib_hi = 0, hash_lo = 0;
    std::vector<Unit> units;     // the job's query units, read order
    std::vector<uint32_t> ureadiid;
    std::vector<uint64_t> uwin;  // windows per unit
    std::vector<uint64_t> wb;    // per unit + one per run: run-local first window (as dwbase)
    std::vector<SqRun> runs;
    DBuf<uint64_t> key, key2;
    DBuf<uint32_t> wid, wid2, ublk;
    DBuf<uint64_t> dwbase;
    DBuf<Unit> dunits;
    DBuf<uint8_t> tmp;
    DBuf<uint32_t> uhits, uflags;
    DBuf<unsigned long long> sig;   // a run's (key, wid) signatures before / after its sort + flag
    uint32_t resorted = 0;       // runs whose partial-range sort failed its check
    int probed = -1;             // the run whose records fb.probe holds for this batch
    uint32_t probed_nu = 0;      // ... for this many of its units
    double ms_sort = 0;
  } sq;

  // results
  DBuf<Rec> d_out;
  uint64_t nout = 0;
  ovl_stats stats;
  DBuf<unsigned long long> dbg;  // OVL_DEBUG counters of this context's extension kernels

  ReadsDev reads() const {
    ReadsDev R;
    R.fwd = d_fwd.p;
    R.rc = d_rc.p;
    R.fwdN = d_fwdN.p;
    R.rcNul = d_rcNul.p;
    R.wofs = d_wofs.p;
    R.len = d_len.p;
    R.flags = d_flags.p;
    R.rcFirstNul = d_rcFirstNul.p;
    R.qual = have_qual ? d_qual.p : nullptr;
    R.first_iid = first_iid;
    R.nreads = nreads;
    return R;
  }
};

// ovl_probe_ceiling: Q independent random 16-B loads in flight per lane over the table's
// 2^tab_bits slots (masked index, an LCG per lane: nothing in the loop but the loads)
template <int Q>
__global__ void __launch_bounds__(256) k_rand_lookup(const uint4 *t, uint64_t mask,
                                                     uint32_t iters, uint32_t *sink) {
  uint32_t acc = 0;
  uint64_t x = (blockIdx.x * (uint64_t)blockDim.x + threadIdx.x + 1) * 0x9E3779B97F4A7C15ull;
  for (uint32_t i = 0; i < iters; i++) {
    uint4 v[Q];
#pragma unroll
    for (int q = 0; q < Q; q++) {
      x = x * 6364136223846793005ull + 1442695040888963407ull;
      v[q] = t[(x >> 17) & mask];
    }
#pragma unroll
    for (int q = 0; q < Q; q++) acc ^= v[q].x ^ v[q].y ^ v[q].z ^ v[q].w;   // whole 16-B loads
  }
  if (acc == 0x9E3779B9u) sink[0] = acc;       // keeps the loads live; (almost) never taken
}

// ovl_probe_replay: the table slot of every query window (k_probe's window rule and hash),
// written as a 32-bit slot list (0xFFFFFFFF: no k-mer), one wave per unit
__global__ void __launch_bounds__(256) k_slot_list(ReadsDev R, const Unit *units,
                                                   const uint64_t *wbase, uint32_t nunits,
                                                   uint32_t k, uint64_t kmask, uint32_t tab_bits,
                                                   uint32_t *slot) {
  const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const uint32_t u = blockIdx.x * 4 + wave;
  if (u >= nunits) return;
  const Unit un = units[u];
  const Strand S = un.dir ? strand_rc(R, un.r) : strand_fwd(R, un.r);
  const uint32_t *bad = un.dir ? S.ex_nul : S.ex_wild;
  const uint32_t nw = (uint32_t)(wbase[u + 1] - wbase[u]);
  const uint32_t kbits = (1u << k) - 1u;
  for (uint32_t o = lane; o < nw; o += 64) {
    bool ok = (int32_t)(o + k) <= S.len;
    if (ok && bad) ok = (mask_at(bad, (int32_t)o) & kbits) == 0;
    slot[wbase[u] + o] =
        ok ? (uint32_t)(mix64(bases_at(S.w, (int32_t)o) & kmask) >> (64 - tab_bits)) : 0xFFFFFFFFu;
  }
}

// the same lookups as pure loads: 8 table entries per lane in flight, the next group's 8
// slot indices loaded while they are (so no phase of the loop waits on the slot stream)
__global__ void __launch_bounds__(256) k_slot_replay(const uint4 *t, const uint32_t *slot,
                                                     uint64_t n, uint32_t *sink) {
  uint32_t acc = 0;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  uint64_t i0 = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  uint32_t sl[8];
#pragma unroll
  for (int q = 0; q < 8; q++) {
    const uint64_t i = i0 + q * stride;
    sl[q] = i < n ? slot[i] : 0xFFFFFFFFu;
  }
  for (; i0 < n; i0 += 8 * stride) {
    uint4 v[8];
#pragma unroll
    for (int q = 0; q < 8; q++) v[q] = sl[q] != 0xFFFFFFFFu ? t[sl[q]] : make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int q = 0; q < 8; q++) {
      const uint64_t i = i0 + 8 * stride + q * stride;
      sl[q] = i < n ? slot[i] : 0xFFFFFFFFu;
    }
#pragma unroll
    for (int q = 0; q < 8; q++) acc ^= v[q].x ^ v[q].y ^ v[q].z ^ v[q].w;   // whole 16-B loads
  }
  if (acc == 0x9E3779B9u) sink[0] = acc;
}

extern "C" {

int ovl_abi_version(void) { return OVL_ABI_VERSION; }

const char *ovl_last_error(void) { return g_err.c_str(); }

void ovl_params_init(ovl_params *p) {
  p->kmer_len = 0;
  p->max_erate = 0.06;
  p->min_olap_len = 0;
  p->partial = 0;
  p->unique_olap_per_pair = 1;
  p->use_window_filter = 0;
  p->use_hopeless_check = 1;
  p->frag_olap_limit = UINT64_MAX;
  p->filter_by_kmer_count = 0;
}

void ovl_params_finalize(ovl_params *p) {
  if (p->max_erate > 0.06) {
    p->use_window_filter = 0;
    p->use_hopeless_check = 0;
  }
}

void *ovl_ctx_stream(ovl_ctx *ctx) { return ctx ? (void *)ctx->stream : nullptr; }

int ovl_probe_ceiling(ovl_ctx *c, double *gloads_per_s, uint64_t *table_bytes) {
  if (!c || !gloads_per_s || !table_bytes) return fail(OVL_ERR_STATE, "null argument");
  if (!c->have_index || !c->d_tab.p) return fail(OVL_ERR_STATE, "no index table");
  HIPC(hipSetDevice(c->device));
  hipStream_t s = c->stream;
  const uint64_t slots = 1ull << c->tab_bits;
  DBuf<uint32_t> sink;
  if (sink.alloc(1)) return fail(OVL_ERR_OOM, "sink");
  const uint32_t blocks = 8u * (uint32_t)c->n_cu, iters = 64;
  hipLaunchKernelGGL(k_rand_lookup<8>, dim3(blocks), dim3(256), 0, s,
                     (const uint4 *)c->d_tab.p, slots - 1, iters, sink.p);   // warm
  HIPC(hipEventRecord(c->ev[6], s));
  const int reps = 3;
  for (int r = 0; r < reps; r++)
    hipLaunchKernelGGL(k_rand_lookup<8>, dim3(blocks), dim3(256), 0, s,
                       (const uint4 *)c->d_tab.p, slots - 1, iters, sink.p);
  HIPC(hipGetLastError());
  HIPC(hipEventRecord(c->ev[7], s));
  HIPC(hipEventSynchronize(c->ev[7]));
  float ms = 0;
  HIPC(hipEventElapsedTime(&ms, c->ev[6], c->ev[7]));
  const double loads = (double)reps * blocks * 256.0 * iters * 8.0;
  *gloads_per_s = ms > 0 ? loads / (ms * 1e-3) / 1e9 : 0.0;
  *table_bytes = slots * sizeof(TabEntry);
  return OVL_OK;
}

int ovl_probe_replay(ovl_ctx *c, uint32_t bgn, uint32_t end, double *gloads_per_s,
                     uint64_t *n_windows) {
  if (!c || !gloads_per_s || !n_windows) return fail(OVL_ERR_STATE, "null argument");
  if (!c->have_index || !c->d_tab.p) return fail(OVL_ERR_STATE, "no index table");
  if (c->tab_bits > 32) return fail(OVL_ERR_UNSUPPORTED, "table of 2^%u slots", c->tab_bits);
  HIPC(hipSetDevice(c->device));
  hipStream_t s = c->stream;
  if (bgn < c->first_iid) bgn = c->first_iid;
  const uint32_t last = c->first_iid + c->nreads - 1;
  if (end > last) end = last;
  // the query units of find_impl's rule (both orientations, --minlength, k), up to 2^28
  // windows: a sample of the same lookup stream k_probe runs over these reads
  std::vector<Unit> units;
  std::vector<uint64_t> wb(1, 0);
  const uint32_t k = c->P.kmer_len;
  for (uint32_t a = bgn; a <= end && a >= bgn && wb.back() < (1ull << 28); a++) {
    const uint32_t r = a - c->first_iid;
    const int32_t L = (int32_t)c->h_len[r];
    if (L < c->P.min_olap_len || L < (int32_t)k) continue;
    for (uint32_t dir = 0; dir < 2; dir++) {
      units.push_back(Unit{r, dir});
      wb.push_back(wb.back() + (uint64_t)(L - (int32_t)k + 1));
    }
  }
  const uint64_t n = wb.back();
  *n_windows = n;
  *gloads_per_s = 0.0;
  if (n == 0) return OVL_OK;
  DBuf<uint32_t> slot, sink;
  DBuf<Unit> du;
  DBuf<uint64_t> dwb;
  if (slot.alloc(n) || sink.alloc(1) || du.alloc(units.size()) || dwb.alloc(wb.size()))
    return fail(OVL_ERR_OOM, "probe replay (%llu windows)", (unsigned long long)n);
  HIPC(hipMemcpyAsync(du.p, units.data(), sizeof(Unit) * units.size(), hipMemcpyHostToDevice, s));
  HIPC(hipMemcpyAsync(dwb.p, wb.data(), 8ull * wb.size(), hipMemcpyHostToDevice, s));
  hipLaunchKernelGGL(k_slot_list, dim3(((uint32_t)units.size() + 3) / 4), dim3(256), 0, s,
                     c->reads(), du.p, dwb.p, (uint32_t)units.size(), k,
                     (1ull << (2 * k)) - 1, c->tab_bits, slot.p);
  const uint32_t blocks = 8u * (uint32_t)c->n_cu;
  hipLaunchKernelGGL(k_slot_replay, dim3(blocks), dim3(256), 0, s, (const uint4 *)c->d_tab.p,
                     slot.p, n, sink.p);                                       // warm
  HIPC(hipEventRecord(c->ev[6], s));
  const int reps = 3;
  for (int r = 0; r < reps; r++)
    hipLaunchKernelGGL(k_slot_replay, dim3(blocks), dim3(256), 0, s, (const uint4 *)c->d_tab.p,
                       slot.p, n, sink.p);
  HIPC(hipGetLastError());
  HIPC(hipEventRecord(c->ev[7], s));
  HIPC(hipEventSynchronize(c->ev[7]));
  float ms = 0;
  HIPC(hipEventElapsedTime(&ms, c->ev[6], c->ev[7]));
  *gloads_per_s = ms > 0 ? (double)reps * (double)n / (ms * 1e-3) / 1e9 : 0.0;
  return OVL_OK;
}

// ---- index export / import (ABI 7) ----------------------------------------------------
int ovl_export_index(ovl_ctx *c, ovl_index_desc *o) {
  if (!c || !o) return fail(OVL_ERR_STATE, "null argument");
  if (!c->have_index) return fail(OVL_ERR_STATE, "no index built");
  memset(o, 0, sizeof(*o));
  o->bgn_iid = c->hash_bgn_iid;
  o->end_iid = c->hash_end_iid;
  o->first_iid = c->first_iid;
  o->nreads = c->nreads;
  o->kmer_len = c->P.kmer_len;
  o->tab_bits = c->tab_bits;
  o->slice_bits = c->slice_bits;
  o->hash_lib_lo = c->stats_hash_lib_lo;
  o->hash_lib_hi = c->stats_hash_lib_hi;
  o->records = c->index_records;
  o->table = c->d_tab.p;
  o->table_bytes = sizeof(TabEntry) << c->tab_bits;
  o->occ = c->d_occ.p;
  o->occ_bytes = 8ull * c->index_records;
  if (c->bloom_ok) {
    o->bloom_w = c->bloom_w;
    o->bloom = c->d_bloom.p;
    o->bloom_bytes = 8ull * ((1ull << (c->tab_bits - c->slice_bits)) << c->bloom_w);
  }
  o->read_flags = c->d_flags.p;
  o->read_flags_bytes = 4ull * c->nreads;
  return OVL_OK;
}

int ovl_import_index(ovl_ctx *c, const ovl_index_desc *in) {
  if (!c || !in) return fail(OVL_ERR_STATE, "null argument");
  if (c->nreads == 0) return fail(OVL_ERR_STATE, "no reads loaded");
  if (in->first_iid != c->first_iid || in->nreads != c->nreads)
    return fail(OVL_ERR_BAD_PARAM, "index of reads %u+%u, this context holds %u+%u",
                in->first_iid, in->nreads, c->first_iid, c->nreads);
  if (in->kmer_len != c->P.kmer_len)
    return fail(OVL_ERR_BAD_PARAM, "index of %u-mers, this context uses -k %u", in->kmer_len,
                c->P.kmer_len);
  if (in->tab_bits > 40 || in->slice_bits > in->tab_bits ||
      in->table_bytes != (sizeof(TabEntry) << in->tab_bits) || in->occ_bytes != 8ull * in->records ||
      in->read_flags_bytes != 4ull * in->nreads || !in->table || (in->records && !in->occ) ||
      !in->read_flags || (in->bloom_bytes && (!in->bloom ||
      in->bloom_w > 6 ||
      in->bloom_bytes != 8ull * ((1ull << (in->tab_bits - in->slice_bits)) << in->bloom_w))))
    return fail(OVL_ERR_BAD_PARAM, "inconsistent index descriptor");
  // the limits build_index keeps (and the table / probe kernels assume): 32-bit run offsets,
  // a slice (and, with the filter, its filter region) within one wave's 64 KB of LDS
  if (in->records >= 0xFFFFFFF0ull || in->slice_bits < 1 || (16ull << in->slice_bits) > 65536 ||
      (in->bloom_bytes && (16ull << in->slice_bits) + (8ull << in->bloom_w) > 65536))
    return fail(OVL_ERR_BAD_PARAM, "index descriptor past the build's limits (records %llu, "
                "slice 2^%u, filter 2^%u words)", (unsigned long long)in->records,
                in->slice_bits, in->bloom_w);
  if (in->end_iid < in->bgn_iid || in->bgn_iid < c->first_iid ||
      in->end_iid > c->first_iid + c->nreads - 1)
    return fail(OVL_ERR_BAD_PARAM, "index of hash reads %u-%u outside the loaded reads",
                in->bgn_iid, in->end_iid);
  HIPC(hipSetDevice(c->device));
  hipStream_t s = c->stream;
  c->have_index = false;
  if (c->d_tab.alloc(1ull << in->tab_bits) || c->d_occ.alloc(std::max<uint64_t>(in->records, 1)) ||
      (in->bloom_bytes && c->d_bloom.alloc(in->bloom_bytes / 8)))
    return fail(OVL_ERR_OOM, "imported index (%.1f GB)",
                (in->table_bytes + in->occ_bytes + in->bloom_bytes) / 1e9);
  HIPC(hipEventRecord(c->ev[0], s));
  HIPC(hipMemcpyAsync(c->d_tab.p, in->table, in->table_bytes, hipMemcpyDefault, s));
  if (in->records)
    HIPC(hipMemcpyAsync(c->d_occ.p, in->occ, in->occ_bytes, hipMemcpyDefault, s));
  if (in->bloom_bytes)
    HIPC(hipMemcpyAsync(c->d_bloom.p, in->bloom, in->bloom_bytes, hipMemcpyDefault, s));
  HIPC(hipMemcpyAsync(c->d_flags.p, in->read_flags, in->read_flags_bytes, hipMemcpyDefault, s));
  HIPC(hipEventRecord(c->ev[1], s));
  HIPC(hipStreamSynchronize(s));
  float ms = 0;
  (void)hipEventElapsedTime(&ms, c->ev[0], c->ev[1]);
  c->stats.ms_index = ms;                      // the copy stands in for the build
  c->hash_bgn_iid = in->bgn_iid;
  c->hash_end_iid = in->end_iid;
  c->tab_bits = in->tab_bits;
  c->slice_bits = in->slice_bits;
  c->bloom_w = in->bloom_bytes ? in->bloom_w : 0;
  c->bloom_ok = in->bloom_bytes != 0;
  c->index_records = in->records;
  c->stats_hash_lib_lo = in->hash_lib_lo;
  c->stats_hash_lib_hi = in->hash_lib_hi;
  // the copied flags carry the exporter's NOHASH bits (-H): a later build re-derives them
  if (in->hash_lib_lo != 0 || in->hash_lib_hi != UINT32_MAX) c->nohash_set = true;
  c->have_index = true;
  return OVL_OK;
}

int ovl_ctx_create(const ovl_params *p, int device, ovl_ctx **out) {
  *out = nullptr;
  if (p->kmer_len == 0) return fail(OVL_ERR_BAD_PARAM, "kmer length (-k) needed");
  if (p->kmer_len > 31) return fail(OVL_ERR_BAD_PARAM, "kmer length must be <= 31");
  if (!(p->max_erate > 0.0) || p->max_erate >= 1.0)
    return fail(OVL_ERR_BAD_PARAM, "maxErate out of range");
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
    return fail(OVL_ERR_NO_DEVICE, "no HIP device");
  if (device < 0 || device >= ndev) return fail(OVL_ERR_NO_DEVICE, "bad device ordinal %d", device);
  hipDeviceProp_t prop;
  HIPC(hipGetDeviceProperties(&prop, device));
  if (strncmp(prop.gcnArchName, "gfx950", 6) != 0)
    return fail(OVL_ERR_NO_DEVICE, "device %d is %s, not gfx950", device, prop.gcnArchName);
  HIPC(hipSetDevice(device));

  ovl_ctx *c = new ovl_ctx();
  c->P = *p;
  ovl_params_finalize(&c->P);
  c->device = device;
  c->n_cu = prop.multiProcessorCount;
  memset(&c->stats, 0, sizeof(c->stats));
  if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
      hipStreamCreateWithFlags(&c->xstream, hipStreamNonBlocking) != hipSuccess) {
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
    return fail(OVL_ERR_HIP, "stream create failed");
  }
  for (int i = 0; i < 8; i++) (void)hipEventCreate(&c->ev[i]);
  for (int i = 0; i < 4; i++) (void)hipEventCreate(&c->xev[i]);

  double er = c->P.max_erate;
  c->max_errors = 1 + (int32_t)ceil(er * AS_MAX_READLEN);
  c->branch_match_value = er / (1 + er);
  c->min_branch_tail_slope = (er > 0.06) ? 1.0 : 0.20;
  c->h_error_bound.resize(AS_MAX_READLEN + 1);
  for (uint32_t i = 0; i <= AS_MAX_READLEN; i++)
    c->h_error_bound[i] = (int32_t)ceil(i * er);
  std::vector<int32_t> ml;
  init_match_limit(ml, er, c->max_errors);
  // padded past max_errors: the staged kernel may read its rows' limits straight from here
  // (OVL_GML), where a block's LDS copy held 0x7fffffff beyond max_errors
  ml.resize(ml.size() + 64, 0x7fffffff);
  if (c->d_error_bound.alloc(AS_MAX_READLEN + 1) != hipSuccess ||
      c->d_match_limit.alloc(ml.size()) != hipSuccess) {
    ovl_ctx_destroy(c);
    return fail(OVL_ERR_OOM, "table alloc");
  }
  (void)hipMemcpy(c->d_error_bound.p, c->h_error_bound.data(), 4ull * (AS_MAX_READLEN + 1),
                  hipMemcpyHostToDevice);
  (void)hipMemcpy(c->d_match_limit.p, ml.data(), 4ull * ml.size(), hipMemcpyHostToDevice);
  *out = c;
  return OVL_OK;
}

void ovl_ctx_destroy(ovl_ctx *c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  if (c->xstream) (void)hipStreamSynchronize(c->xstream);
  for (int i = 0; i < 8; i++)
    if (c->ev[i]) (void)hipEventDestroy(c->ev[i]);
  for (int i = 0; i < 4; i++)
    if (c->xev[i]) (void)hipEventDestroy(c->xev[i]);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  if (c->xstream) (void)hipStreamDestroy(c->xstream);
  delete c;
}

static int load_common(ovl_ctx *c, uint32_t first_iid, uint32_t nreads, const uint8_t *d_bases,
                       const uint64_t *d_offsets, const uint32_t *h_lengths) {
  // Until every check and allocation has passed the context holds no reads, so a failed
  // load leaves nothing for a later build / find to run over (they return OVL_ERR_STATE).
  c->nreads = 0;
  c->have_index = false;
  c->have_qual = false;
  c->h_lib.clear();
  c->nohash_set = false;
  if (first_iid == 0 && nreads) return fail(OVL_ERR_BAD_PARAM, "read IDs start at 1");
  if ((uint64_t)first_iid + nreads > 0xFFFFFFFFull)
    return fail(OVL_ERR_BAD_PARAM, "read IDs past 2^32");
  std::vector<uint64_t> wofs(nreads + 1);
  uint64_t w = 0;
  uint32_t max_len = 0;
  for (uint32_t i = 0; i < nreads; i++) {
    if (h_lengths[i] > AS_MAX_READLEN)
      return fail(OVL_ERR_BAD_INPUT, "read %u longer than AS_MAX_READLEN", first_iid + i);
    wofs[i] = w;
    w += (h_lengths[i] + 31) / 32 + 1;
    max_len = std::max(max_len, h_lengths[i]);
  }
  wofs[nreads] = w;
  w += 2;
  if (c->d_fwd.alloc(w) || c->d_rc.alloc(w) || c->d_fwdN.alloc(w) || c->d_rcNul.alloc(w) ||
      c->d_wofs.alloc(nreads + 1) || c->d_len.alloc(nreads) || c->d_flags.alloc(nreads) ||
      c->d_rcFirstNul.alloc(nreads))
    return fail(OVL_ERR_OOM, "read buffers (%llu words)", (unsigned long long)w);
  c->h_len.assign(h_lengths, h_lengths + nreads);
  c->h_wofs.swap(wofs);
  c->max_len = max_len;
  HIPC(hipMemsetAsync(c->d_fwd.p, 0, 8 * w, c->stream));
  HIPC(hipMemsetAsync(c->d_rc.p, 0, 8 * w, c->stream));
  HIPC(hipMemsetAsync(c->d_fwdN.p, 0, 4 * w, c->stream));
  HIPC(hipMemsetAsync(c->d_rcNul.p, 0, 4 * w, c->stream));
  HIPC(hipMemcpyAsync(c->d_wofs.p, c->h_wofs.data(), 8ull * (nreads + 1), hipMemcpyHostToDevice,
                      c->stream));
  HIPC(hipMemcpyAsync(c->d_len.p, h_lengths, 4ull * nreads, hipMemcpyHostToDevice, c->stream));
  DBuf<uint32_t> err;
  if (err.alloc(1)) return fail(OVL_ERR_OOM, "err flag");
  HIPC(hipMemsetAsync(err.p, 0, 4, c->stream));
  if (nreads)
    hipLaunchKernelGGL(k_pack, dim3(nreads), dim3(128), 0, c->stream, d_bases, d_offsets,
                       c->d_len.p, c->d_wofs.p, c->d_fwd.p, c->d_rc.p, c->d_fwdN.p,
                       c->d_rcNul.p, c->d_flags.p, c->d_rcFirstNul.p, err.p,
                       c->P.kmer_len);
  HIPC(hipGetLastError());
  uint32_t h_err = 0;
  HIPC(hipMemcpyAsync(&h_err, err.p, 4, hipMemcpyDeviceToHost, c->stream));
  HIPC(hipStreamSynchronize(c->stream));
  if (h_err)
    return fail(OVL_ERR_BAD_INPUT,
                "reads hold characters other than ACGTN; the GPU path cannot represent them");
  c->first_iid = first_iid;
  c->nreads = nreads;
  return OVL_OK;
}

// Work-order keys for the extension queue: a pair's match-node count (its extension work
// grows with it), so the longest pairs start first and the kernel's tail is short.
__global__ void k_pair_order_keys(const PairRec *pairs, uint32_t n, uint32_t *keys,
                                  uint32_t *idx) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    keys[i] = pairs[i].node_cnt;
    idx[i] = i;
  }
}

// ---- -l (Frag_Olap_Limit): the reference's per-unit pair orders -----------------------
// Process_String_Olaps (Process_String_Overlaps.C:687) walks a query's targets in
// String_Olap_Space order -- Add_Ref (Find_Overlaps.C:158) gives a new target its hash
// slot (StrNum ^ StrNum >> 8) & 255 when that slot is free, else the next overflow entry
// (256, 257, .. in first-hit order) -- and, past the limit, sorted by average diagonal
// (qsort By_Diag_Sum, glibc's stable merge sort: ties keep String_Olap_Space order).
// A target's first hit is its smallest window (diag_bgn); targets first hit in the same
// window come in the occurrence list's order, iid-descending.

// per pair: first-hit keys, the unit's pair count, and the average diagonal (the
// reference sums diagonals in a double: exact for integers, so the sum over nodes is the
// same number; each node of length Len holds Len - k + 1 hits on its diagonal)
__global__ void k_olim_keys(const PairRec *pairs, const Node *pnodes, uint32_t n, int32_t k,
                            uint32_t *ktgt, uint64_t *kfirst, uint32_t *idx, uint64_t *dkey,
                            uint32_t *ucnt) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const PairRec P = pairs[i];
    ktgt[i] = ~P.tgt;
    kfirst[i] = ((uint64_t)P.unit << 24) | (uint32_t)P.diag_bgn;
    idx[i] = i;
    int64_t sum = 0;
    for (uint32_t j = 0; j < P.node_cnt; j++) {
      const Node nd = pnodes[P.node_off + j];
      sum += (int64_t)(nd.Len - k + 1) * (int64_t)(nd.Offset - nd.Start);
    }
    const double avg = (double)sum / (double)P.diag_ct;
    const uint64_t b = __builtin_bit_cast(uint64_t, avg);
    dkey[i] = (b >> 63) ? ~b : (b | (1ull << 63));     // order-preserving
    atomicAdd(&ucnt[P.unit], 1u);
  }
}

__global__ void k_gather_u64(const uint64_t *src, const uint32_t *idx, uint32_t n, uint64_t *dst) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
    dst[i] = src[idx[i]];
}

// A chunk's pairs appended to the pending-extension accumulator: their unit and node indices
// move by where the chunk's units and nodes land there.
__global__ void k_append_pairs(const PairRec *src, uint32_t n, uint32_t unit_base,
                               uint32_t node_base, PairRec *dst) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    PairRec p = src[i];
    p.unit += unit_base;
    p.node_off += node_base;
    dst[i] = p;
  }
}

__global__ void k_gather_unit(const PairRec *pairs, const uint32_t *idx, uint32_t n, uint32_t *dst) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
    dst[i] = pairs[idx[i]].unit;
}

// One wave per unit over its pairs in first-hit order: String_Olap_Space index per pair,
// written as the sort key unit << 32 | index (ks) next to the pair index (ki).
__global__ void __launch_bounds__(256) k_olim_slots(const PairRec *pairs, const uint32_t *first,
                                                    const uint32_t *useg, uint32_t nunits,
                                                    uint32_t str_off, uint64_t *ks, uint32_t *ki) {
  __shared__ uint32_t s_first[4][256];
  __shared__ uint8_t s_taken[4][256];
  const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  uint32_t *fst = s_first[wave];
  uint8_t *taken = s_taken[wave];
  for (uint32_t i = lane; i < 256; i += 64) { fst[i] = 64; taken[i] = 0; }
  __builtin_amdgcn_wave_barrier();
  for (uint32_t u = blockIdx.x * 4 + wave; u < nunits; u += gridDim.x * 4) {
    const uint32_t b = useg[u], e = useg[u + 1];
    uint32_t novf = 0;
    for (uint32_t c0 = b; c0 < e; c0 += 64) {
      const uint32_t i = c0 + lane;
      const bool valid = i < e;
      uint32_t pi = 0, h = 0;
      if (valid) {
        pi = first[i];
        const uint32_t sn = pairs[pi].tgt + str_off;   // StrNum: index in the hash batch
        h = (sn ^ (sn >> 8)) & 255u;
        atomicMin(&fst[h], lane);
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      const bool own = valid && fst[h] == lane && !taken[h];
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      if (valid) fst[h] = 64;
      if (own) taken[h] = 1;
      const uint64_t om = __ballot(valid && !own);
      const uint32_t slot = own ? h : 256u + novf + (uint32_t)__builtin_popcountll(om & ((1ull << lane) - 1));
      novf += (uint32_t)__builtin_popcountll(om);
      if (valid) {
        ks[i] = ((uint64_t)u << 32) | slot;
        ki[i] = pi;
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    for (uint32_t i = lane; i < 256; i += 64) taken[i] = 0;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
}

// Qualities (-w) into the packed layout: read r base i at wofs[r] * 32 + i.
__global__ void k_pack_quals(const uint8_t *q, const uint64_t *offs, const uint32_t *lens,
                             const uint64_t *wofs, uint8_t *out) {
  const uint32_t r = blockIdx.x;
  const uint64_t o = offs[r], w = wofs[r] * 32;
  for (uint32_t i = threadIdx.x; i < lens[r]; i += blockDim.x) out[w + i] = q[o + i];
}

static int load_quals(ovl_ctx *c, const uint8_t *d_quals, const uint64_t *d_offsets) {
  c->have_qual = false;
  if (!d_quals) return OVL_OK;
  uint64_t words = c->h_wofs.empty() ? 0 : c->h_wofs.back() + (c->h_len.back() + 31) / 32 + 1;
  if (c->d_qual.alloc(words * 32 + 64)) return fail(OVL_ERR_OOM, "qualities");
  hipLaunchKernelGGL(k_pack_quals, dim3(c->nreads), dim3(256), 0, c->stream, d_quals, d_offsets,
                     c->d_len.p, c->d_wofs.p, c->d_qual.p);
  HIPC(hipGetLastError());
  HIPC(hipStreamSynchronize(c->stream));
  c->have_qual = true;
  return OVL_OK;
}

int ovl_load_reads(ovl_ctx *c, uint32_t first_iid, uint32_t nreads, const uint8_t *bases,
                   const uint64_t *offsets, const uint32_t *lengths, const uint8_t *quals) {
  if (!c) return fail(OVL_ERR_STATE, "null context");
  HIPC(hipSetDevice(c->device));
  uint64_t total = 0;
  for (uint32_t i = 0; i < nreads; i++) total = std::max(total, offsets[i] + lengths[i]);
  DBuf<uint8_t> db, dq;
  DBuf<uint64_t> doff;
  if (db.alloc(total + 64) || doff.alloc(nreads + 1)) return fail(OVL_ERR_OOM, "staging");
  HIPC(hipMemcpyAsync(db.p, bases, total, hipMemcpyHostToDevice, c->stream));
  HIPC(hipMemcpyAsync(doff.p, offsets, 8ull * nreads, hipMemcpyHostToDevice, c->stream));
  int rc = load_common(c, first_iid, nreads, db.p, doff.p, lengths);
  if (rc == OVL_OK && quals) {
    if (dq.alloc(total + 64)) return fail(OVL_ERR_OOM, "quality staging");
    HIPC(hipMemcpyAsync(dq.p, quals, total, hipMemcpyHostToDevice, c->stream));
    rc = load_quals(c, dq.p, doff.p);
  } else if (rc == OVL_OK) {
    c->have_qual = false;
  }
  (void)hipStreamSynchronize(c->stream);
  return rc;
}

int ovl_load_reads_device(ovl_ctx *c, uint32_t first_iid, uint32_t nreads,
                          const uint8_t *d_bases, const uint64_t *d_offsets,
                          const uint32_t *h_lengths, const uint8_t *d_quals) {
  if (!c) return fail(OVL_ERR_STATE, "null context");
  HIPC(hipSetDevice(c->device));
  int rc = load_common(c, first_iid, nreads, d_bases, d_offsets, h_lengths);
  if (rc == OVL_OK) rc = load_quals(c, d_quals, d_offsets);
  return rc;
}

static uint64_t kmer_code(const char *s, uint32_t k, bool *ok) {
  uint64_t key = 0;
  *ok = true;
  for (uint32_t j = 0; j < k; j++) {
    int v;
    switch (s[j] | 0x20) {
      case 'a': v = 0; break;
      case 'c': v = 1; break;
      case 'g': v = 2; break;
      case 't': v = 3; break;
      default: v = 0; *ok = false;
    }
    key |= (uint64_t)v << (2 * j);
  }
  return key;
}

int ovl_set_skip_kmers(ovl_ctx *c, const char *kmers, uint64_t n) {
  if (!c) return fail(OVL_ERR_STATE, "null context");
  uint32_t k = c->P.kmer_len;
  c->h_skip.clear();
  std::vector<char> rc(k);
  for (uint64_t i = 0; i < n; i++) {
    const char *s = kmers + i * k;
    bool ok;
    uint64_t f = kmer_code(s, k, &ok);
    if (!ok) return fail(OVL_ERR_BAD_INPUT, "skip k-mer %llu is not ACGT", (unsigned long long)i);
    c->h_skip.push_back(f);
    uint64_t r = 0;                                // reverse complement code
    for (uint32_t j = 0; j < k; j++) {
      uint64_t b = (f >> (2 * j)) & 3;
      r |= (3 - b) << (2 * (k - 1 - j));
    }
    c->h_skip.push_back(r);
  }
  std::sort(c->h_skip.begin(), c->h_skip.end());
  c->h_skip.erase(std::unique(c->h_skip.begin(), c->h_skip.end()), c->h_skip.end());
  c->have_index = false;
  return OVL_OK;
}

static __global__ void k_clear_screen(uint32_t *flags, uint32_t n) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) flags[i] &= ~6u;                 // the screened-end bits of the last index
}

// OVL_RFLAG_NOHASH from a per-read byte (1 = not hashed); nohash == null clears it.
static __global__ void k_set_nohash(uint32_t *flags, const uint8_t *nohash, uint32_t n) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    uint32_t f = flags[i] & ~OVL_RFLAG_NOHASH;
    if (nohash && nohash[i]) f |= OVL_RFLAG_NOHASH;
    flags[i] = f;
  }
}

static uint32_t ceil_log2(uint64_t x) {
  uint32_t b = 0;
  while ((1ull << b) < x) b++;
  return b;
}

static uint32_t read_lib(const ovl_ctx *c, uint32_t r) { return c->h_lib.empty() ? 0 : c->h_lib[r]; }

// Mark the reads outside [lo, hi] as not hashed (device flag), or clear every mark.
static int apply_hash_libs(ovl_ctx *c, uint32_t lo, uint32_t hi) {
  bool any = false;
  std::vector<uint8_t> nh;
  if (!c->h_lib.empty() && (lo > 0 || hi < UINT32_MAX)) {
    nh.resize(c->nreads);
    for (uint32_t r = 0; r < c->nreads; r++) {
      nh[r] = (c->h_lib[r] < lo || c->h_lib[r] > hi) ? 1 : 0;
      any |= nh[r] != 0;
    }
  }
  if (!any && !c->nohash_set) return OVL_OK;
  DBuf<uint8_t> d;
  if (any) {
    if (d.alloc(c->nreads)) return fail(OVL_ERR_OOM, "library flags");
    HIPC(hipMemcpyAsync(d.p, nh.data(), c->nreads, hipMemcpyHostToDevice, c->stream));
  }
  hipLaunchKernelGGL(k_set_nohash, dim3((c->nreads + 255) / 256), dim3(256), 0, c->stream,
                     c->d_flags.p, any ? d.p : nullptr, c->nreads);
  HIPC(hipGetLastError());
  HIPC(hipStreamSynchronize(c->stream));
  c->nohash_set = any;
  return OVL_OK;
}

// The index over hash reads bgn..end (clipped to the loaded reads by the callers).
// bloom: also build the batch's Bloom filter (OverlapDriver batches, whose searches are
// mostly by reads outside the hash range; see use_bloom)
// table = false: the records grouped into k-mer runs only (what the driver's first-read
// histogram reads to find a load cut), no table, filter or screened-end flags: the index is
// not searchable (have_index stays false)
static int build_index(ovl_ctx *c, uint32_t bgn, uint32_t end, bool bloom = false,
                       bool table = true) {
  hipStream_t s = c->stream;
  uint32_t k = c->P.kmer_len;
  c->hash_bgn_iid = bgn;
  c->hash_end_iid = end;
  c->have_index = false;
  c->bloom_ok = false;
  HIPC(hipEventRecord(c->ev[0], s));
  hipLaunchKernelGGL(k_clear_screen, dim3((c->nreads + 255) / 256), dim3(256), 0, s,
                     c->d_flags.p, c->nreads);

  uint32_t h0 = bgn - c->first_iid, h1 = (end >= bgn) ? end - c->first_iid + 1 : h0;
  uint64_t P = 0;
  for (uint32_t r = h0; r < h1; r++)
    if ((int32_t)c->h_len[r] >= c->P.min_olap_len && c->h_len[r] >= k && !(c->nohash_set &&
        (read_lib(c, r) < c->stats_hash_lib_lo || read_lib(c, r) > c->stats_hash_lib_hi)))
      P += c->h_len[r] - k + 1;
  uint32_t n_skip = (uint32_t)c->h_skip.size();
  P += n_skip;
  if (P >= 0xFFFFFFF0ull)
    return fail(OVL_ERR_UNSUPPORTED, "hash batch with %llu k-mers; use a smaller -h range",
                (unsigned long long)P);
  if (n_skip) {
    if (c->d_skip.alloc(n_skip)) return fail(OVL_ERR_OOM, "skip");
    HIPC(hipMemcpyAsync(c->d_skip.p, c->h_skip.data(), 8ull * n_skip, hipMemcpyHostToDevice, s));
  }

  uint32_t cb = std::min<uint32_t>(12, std::max<uint32_t>(4, ceil_log2(P / 2048 + 1)));
  uint64_t per_cb = (P >> cb) + 1;
  uint32_t fb = std::min<uint32_t>(11, ceil_log2((per_cb + 127) / 128));   // ~128 per fine bucket
  uint32_t ncb = 1u << cb, nfb = 1u << fb, nfine = ncb * nfb;

  auto rec_alloc = [&](uint64_t n) {
    return c->d_tmpR.alloc(n) || c->d_midR.alloc(n) || c->d_tmpM2.alloc(n) || c->d_occ.alloc(n);
  };
  if (!(c->index_reserve > P && !rec_alloc(c->index_reserve)) && rec_alloc(P))
    return fail(OVL_ERR_OOM, "index records (%llu)", (unsigned long long)P);
  DBuf<uint32_t> &hist = c->b_hist, &cstart = c->b_cstart, &cursor = c->b_cursor,
                 &fstart = c->b_fstart, &fcnt = c->b_fcnt, &misc = c->b_misc, &big = c->b_big;
  if (hist.alloc(ncb) || cstart.alloc(ncb) || cursor.alloc(ncb) || fstart.alloc(nfine) ||
      fcnt.alloc(nfine) || misc.alloc(8) || big.alloc(2 * (size_t)nfine))
    return fail(OVL_ERR_OOM, "index scratch");
  HIPC(hipMemsetAsync(hist.p, 0, 4 * ncb, s));
  HIPC(hipMemsetAsync(misc.p, 0, 32, s));

  BuildArgs A;
  A.R = c->reads();
  A.h0 = h0;
  A.h1 = h1;
  // coarse passes: 2 blocks of 16 waves per CU (32 waves: the coarse scatter is latency-
  // bound -- a dependent packed-base load, LDS atomic and 16-B store per window -- and its
  // 32 KB of LDS histograms per block would cap 4-wave blocks at 20 waves per CU).
  // Measured on 50k x 10 kb: 256 threads x 4 per CU 35.7 ms index, 512 x 4 34.0, 1024 x 2
  // 32.4 (with the parallel fine-bucket scan)
#ifndef OVL_COARSE_BPCU
#define OVL_COARSE_BPCU 2
#endif
#ifndef OVL_COARSE_THREADS
#define OVL_COARSE_THREADS 1024
#endif
  uint32_t nblk = std::max<uint32_t>(1, std::min<uint32_t>(h1 - h0, OVL_COARSE_BPCU * c->n_cu));
  A.reads_per_block = (h1 - h0 + nblk - 1) / nblk;
  if (A.reads_per_block == 0) A.reads_per_block = 1;
  A.k = k;
  A.min_len = c->P.min_olap_len;
  A.kmask = (1ull << (2 * k)) - 1;
  A.skip = n_skip ? c->d_skip.p : nullptr;
  A.n_skip = n_skip;
  A.cb_bits = cb;
  A.fb_bits = fb;
  hipLaunchKernelGGL(k_coarse_hist, dim3(nblk), dim3(OVL_COARSE_THREADS), 0, s, A, hist.p);
  hipLaunchKernelGGL(k_scan_u32, dim3(1), dim3(1024), 0, s, hist.p, cstart.p, ncb, misc.p + 0);
  HIPC(hipMemcpyAsync(cursor.p, cstart.p, 4 * ncb, hipMemcpyDeviceToDevice, s));
  hipLaunchKernelGGL(k_coarse_scatter, dim3(nblk), dim3(OVL_COARSE_THREADS), 0, s, A, cursor.p, c->d_tmpR.p);
  FineArgs F;
  F.inR = c->d_tmpR.p;
  F.midR = c->d_midR.p;
  F.outM = c->d_tmpM2.p;
  F.outP = c->d_occ.p;
  F.cstart = cstart.p;
  F.ccnt = hist.p;
  F.fstart = fstart.p;
  F.fcnt = fcnt.p;
  F.big_list = big.p;
  F.big_n = misc.p + 1;
  F.max_distinct = misc.p + 2;
  F.cb_bits = cb;
  F.fb_bits = fb;
  {
    // per-wave sort buffer: twice the mean fine bucket, power of 2, 64..1024 records
    uint64_t mean = per_cb / nfb + 1;
    uint32_t cap = 64;
    while (cap < 2 * mean && cap < 1024) cap <<= 1;
    F.cap = cap;
  }
  {
    // the sort phase: runs grouped in an LDS hash table, records in registers (cap / 64 per
    // lane); bitonic sorts when the grouped layout would not fit a CU's LDS (cap 1024)
    const bool group = fine_lds_bytes(true, nfb, F.cap) + 256 <= 160 * 1024;
    const size_t fine_lds = fine_lds_bytes(group, nfb, F.cap);
    const void *kf =
        !group           ? reinterpret_cast<const void *>(k_fine<1, false>)
        : F.cap <= 64    ? reinterpret_cast<const void *>(k_fine<1, true>)
        : F.cap <= 128   ? reinterpret_cast<const void *>(k_fine<2, true>)
        : F.cap <= 256   ? reinterpret_cast<const void *>(k_fine<4, true>)
                         : reinterpret_cast<const void *>(k_fine<8, true>);
    if (fine_lds > 65536)
      HIPC(hipFuncSetAttribute(kf, hipFuncAttributeMaxDynamicSharedMemorySize, (int)fine_lds));
    void *kargs[] = {&F};
    HIPC(hipLaunchKernel(kf, dim3(ncb), dim3(OVL_FINE_WAVES * 64), kargs, fine_lds, s));
  }
  HIPC(hipGetLastError());
  uint32_t hm[4];
  HIPC(hipMemcpyAsync(hm, misc.p, 16, hipMemcpyDeviceToHost, s));
  HIPC(hipStreamSynchronize(s));
  // P counted every window; windows holding an 'n' are not hashed (key_is_bad)
  if (hm[0] > P) return fail(OVL_ERR_HIP, "index count %u exceeds bound %llu", hm[0],
                             (unsigned long long)P);
  uint32_t nbig = hm[1];
  if (nbig) {
    std::vector<uint32_t> bl(2 * nbig);
    HIPC(hipMemcpy(bl.data(), big.p, 8ull * nbig, hipMemcpyDeviceToHost));
    uint32_t mx = 0;
    for (uint32_t i = 0; i < nbig; i++) mx = std::max(mx, bl[2 * i + 1]);
    uint32_t n2 = 1;
    while (n2 < mx) n2 <<= 1;
    DBuf<uint64_t> sM, sP;
    if (sM.alloc((size_t)n2 * nbig) || sP.alloc((size_t)n2 * nbig))
      return fail(OVL_ERR_OOM, "big fine buckets");
    hipLaunchKernelGGL(k_fine_big, dim3(nbig), dim3(1024), 0, s, c->d_tmpM2.p, c->d_occ.p,
                       big.p, sM.p, sP.p, n2, misc.p + 2);
    HIPC(hipMemcpyAsync(hm, misc.p, 16, hipMemcpyDeviceToHost, s));
    HIPC(hipStreamSynchronize(s));
  }
  if (!table) {
    HIPC(hipEventRecord(c->ev[1], s));
    HIPC(hipStreamSynchronize(s));
    float ms = 0;
    (void)hipEventElapsedTime(&ms, c->ev[0], c->ev[1]);
    c->stats.ms_index += ms;
    c->index_records = hm[0];
    return OVL_OK;
  }
  uint32_t maxd = std::max<uint32_t>(hm[2], 1);
#ifndef OVL_SLICE_Q
#define OVL_SLICE_Q 8
#endif
  // slots per slice >= OVL_SLICE_Q / 4 x the largest fine bucket's distinct k-mers (and
  // always more than it, so every probe sequence meets an empty slot).  2x: a denser table
  // (1.25x / 1.5x: 16 -> 8 GB at 50k x 10 kb) builds 1.5 ms faster but lengthens the probe
  // sequences, +2.7 ms in k_probe.  Slices sized to their OWN bucket (2 x distinct + 1,
  // ~6 GB) were measured in round 3 too: k_probe 12.4 -> 22.2 ms per launch, since the
  // per-slice {base, size} lookup is a second dependent random access per window
  // (profiles/r03d_bench_perslice.json); not kept
  const uint64_t slice_q = c->dense_tables ? 4 : OVL_SLICE_Q;
  c->slice_bits = std::max<uint32_t>(1, ceil_log2(slice_q * maxd / 4 + 1));
  c->tab_bits = cb + fb + c->slice_bits;
  if (c->d_tab.alloc(1ull << c->tab_bits)) return fail(OVL_ERR_OOM, "table 2^%u", c->tab_bits);
  TableArgs T;
  T.M = c->d_tmpM2.p;
  T.P = c->d_occ.p;
  T.fstart = fstart.p;
  T.fcnt = fcnt.p;
  T.tab = c->d_tab.p;
  T.nfine = nfine;
  T.slice_bits = c->slice_bits;
  T.tab_bits = c->tab_bits;
  T.len = c->d_len.p;
  T.rflags = c->d_flags.p;
  T.first_iid = c->first_iid;
  T.k = k;
  T.bloom = nullptr;
  T.bloom_w = 0;
  if (bloom) {
    // ~8 filter bits per indexed window (>= distinct k-mers) in every fine bucket's region,
    // a power of two of 64-bit words, at most 64: ~130 MB for a batch of canu's
    // --hashbits 23 --hashload 0.75
    uint64_t words = (8ull * hm[0] + 64ull * nfine - 1) / (64ull * nfine);
    uint32_t w = 0;
    while (w < 6 && (1ull << w) < words) w++;
    if (c->d_bloom.alloc((size_t)nfine << w)) return fail(OVL_ERR_OOM, "bloom filter");
    T.bloom = c->d_bloom.p;
    T.bloom_w = w;
    c->bloom_w = w;
  }
  uint32_t S = 1u << c->slice_bits;
  // LDS per wave: its slice and, with the filter, its fine bucket's filter region.  A slice
  // whose wave does not fit 64 KB with the filter is built without it (the filter is only a
  // shortcut in front of the table); without it, it is refused
  if (bloom && 16ull * S + (8ull << T.bloom_w) > 65536) {
    bloom = false;
    T.bloom = nullptr;
    T.bloom_w = 0;
  }
  const uint64_t per_wave = 16ull * S + (bloom ? 8ull << T.bloom_w : 0ull);
  if (per_wave > 65536) return fail(OVL_ERR_UNSUPPORTED, "k-mer slice too large (%u)", S);
  uint32_t wpb = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(4, 65536ull / per_wave));
  size_t lds = (size_t)wpb * per_wave;
  hipLaunchKernelGGL(k_table, dim3((nfine + wpb - 1) / wpb), dim3(64 * wpb), lds, s, T);
  HIPC(hipGetLastError());
  HIPC(hipEventRecord(c->ev[1], s));
  HIPC(hipStreamSynchronize(s));
  float ms = 0;
  (void)hipEventElapsedTime(&ms, c->ev[0], c->ev[1]);
  c->stats.ms_index += ms;
  c->index_records = hm[0];
  // the build scratch (2 x 16 B per window) stays allocated for the next build: freeing and
  // re-allocating gigabytes per job costs tens of ms on some hosts (and HBM is plentiful)
  c->have_index = true;
  c->bloom_ok = bloom;
  return OVL_OK;
}

static int clip_hash_range(ovl_ctx *c, uint32_t &bgn, uint32_t &end) {
  if (!c) return fail(OVL_ERR_STATE, "null context");
  if (c->nreads == 0) return fail(OVL_ERR_STATE, "no reads loaded");
  HIPC(hipSetDevice(c->device));
  if (bgn < 1) bgn = 1;
  if (bgn < c->first_iid) bgn = c->first_iid;
  uint32_t last = c->first_iid + c->nreads - 1;
  if (end > last) end = last;
  return OVL_OK;
}

int ovl_build_hash_index(ovl_ctx *c, uint32_t bgn, uint32_t end) {
  int rc = clip_hash_range(c, bgn, end);
  if (rc) return rc;
  c->stats_hash_lib_lo = 0;
  c->stats_hash_lib_hi = UINT32_MAX;
  if ((rc = apply_hash_libs(c, 0, UINT32_MAX))) return rc;
  c->stats.ms_index = 0;
  return build_index(c, bgn, end);
}

int ovl_set_read_libraries(ovl_ctx *c, const uint32_t *lib_ids) {
  if (!c) return fail(OVL_ERR_STATE, "null context");
  if (c->nreads == 0) return fail(OVL_ERR_STATE, "no reads loaded");
  if (!lib_ids) { c->h_lib.clear(); return OVL_OK; }
  c->h_lib.assign(lib_ids, lib_ids + c->nreads);
  c->have_index = false;
  return OVL_OK;
}

void ovl_hash_limits_init(ovl_hash_limits *l) {
  l->max_hash_strings = 10000;
  l->max_hash_data_len = 100000000ull;
  l->hash_mask_bits = 22;
  l->max_hash_load = 0.6;
  l->min_lib_hash = 0;
  l->max_lib_hash = UINT32_MAX;
}

void ovl_driver_params_init(ovl_driver_params *d) {
  d->bgn_hash_iid = 1;
  d->end_hash_iid = UINT32_MAX;
  d->bgn_ref_iid = 1;
  d->end_ref_iid = UINT32_MAX;
  d->min_lib_ref = 0;
  d->max_lib_ref = UINT32_MAX;
  d->num_threads = 1;
  d->store_num_reads = 0;
  ovl_hash_limits_init(&d->limits);
}

static const uint32_t ENTRIES_PER_BUCKET = 21;          // overlapInCore.H:102
static const uint64_t MAX_STRING_NUM = (1ull << 31) - 1; // overlapInCore.C:57-63

// The most windows one index build may take: its records are 32-bit indexed, and its build
// needs ~112 B per window (two 16-B record arrays, keys and positions, a table of up to 4
// slots per window) out of the HBM that is free now plus what the current index and the
// previous search hold (released when a build needs it), less 64 GB kept for the seed and
// extension buffers (whose budgets shrink to fit).  OVL_TEST_INDEX_WINDOW_CAP lowers
// it (tests of the capped path).
static void sq_release(ovl_ctx *c, bool free_mem = true);
// the sorted-window probe checks the batch's Bloom filter before the table (OVL_SQ_BLOOM=0:
// it reads the table for every window, and the batch is built without the filter)
static bool sq_bloom() {
  static const bool on = !getenv("OVL_SQ_BLOOM") || atoi(getenv("OVL_SQ_BLOOM")) != 0;
  return on;
}
static size_t sq_held_bytes(const ovl_ctx *c);
static void release_find_buffers(ovl_ctx *c) {
  auto &f = c->fb;
  for (int i = 0; i < 2; i++) {
    f.units[i].release(); f.pnodes[i].release(); f.pairs[i].release();
  }
  f.rbase.release(); f.probe.release(); f.uhits.release();
  f.uflags.release(); f.done.release(); f.dset.release(); f.big.release(); f.live.release();
  f.defer.release(); f.defer2.release(); f.okey.release(); f.oidx.release();
  f.okey2.release(); f.oidx2.release(); f.otmp.release(); f.pool.release();
  f.ok64a.release(); f.ok64b.release(); f.dkey.release(); f.oa.release(); f.ob.release();
  f.ucnt.release(); f.useg.release(); f.hcnt.release(); f.hbase.release(); f.hbuf.release();
  f.rows.release(); f.rowdir.release(); f.deltas.release();
  sq_release(c);
  // the extension accumulator's buffers, once nothing waits in them
  if (c->acc.np == 0) {
    c->acc.units.release(); c->acc.pnodes.release(); c->acc.pairs.release();
    c->acc.nu = c->acc.nn = 0;
  }
}

// HBM figures of the last index_window_cap call, for error messages
static thread_local uint64_t g_cap_free = 0, g_cap_reserve = 0;

static uint64_t index_window_cap(ovl_ctx *c) {
  uint64_t cap = 0xFFFFFFF0ull - 64 - c->h_skip.size();
  size_t fr = 0, tot = 0;
  g_cap_free = g_cap_reserve = 0;
  if (hipMemGetInfo(&fr, &tot) == hipSuccess) {
    const auto &f = c->fb;
    const uint64_t held = 2ull * c->d_tmpR.n * sizeof(Rec2) + 2ull * c->d_occ.n * 8 +
                          (uint64_t)c->d_tab.n * sizeof(TabEntry) + f.probe.n * sizeof(Probe) +
                          (f.pool.n + f.pnodes[0].n + f.pnodes[1].n) * sizeof(Node) +
                          (f.pairs[0].n + f.pairs[1].n) * sizeof(PairRec) +
                          4ull * (f.rows.n + f.rowdir.n + f.deltas.n) +
                          c->acc.units.n * sizeof(Unit) + c->acc.pnodes.n * sizeof(Node) +
                          c->acc.pairs.n * sizeof(PairRec) +
                          (c->sq.on ? 0 : sq_held_bytes(c));   // an earlier job's sorted windows
    // the search and extension buffers of the batch are sized by budget (up to ~64 GB on a
    // 288 GB part): keep that much aside, or a fifth of a smaller device
    const uint64_t avail = fr + held;
    const uint64_t reserve = std::min<uint64_t>(64ull << 30, (uint64_t)tot / 5);
    g_cap_free = avail;
    g_cap_reserve = reserve;
    cap = std::min<uint64_t>(cap, avail > reserve ? (avail - reserve) / 112 : 0);
  }
  if (const char *e = getenv("OVL_TEST_INDEX_WINDOW_CAP"))
    cap = std::min<uint64_t>(cap, strtoull(e, nullptr, 10));
  return std::max<uint64_t>(cap, 1);
}

// Build_Hash_Index's loading loop (overlapInCore-Build_Hash_Index.C:495-541): before each
// read it requires String_Ct < Max_Hash_Strings, total_len < Max_Hash_Data_Len and
// Hash_Entries < hash_entry_limit.  String_Ct counts every ID (skipped reads too);
// total_len grows by len + 1 per loaded read; Hash_Entries by the k-mers a read brings
// that no earlier read of the batch holds.  The first two are known from the lengths; the
// third needs the batch's k-mers, so the index is built over the first two's range and its
// first-occurrence histogram decides -- rebuilding the shorter batch when the table load
// stops it earlier.
// boundaries_only: the batch's end alone (the driver's first phase, super-batches): no
// build unless the table load may cut the batch, and then no table and no cut index
static int build_batch_impl(ovl_ctx *c, uint32_t bgn, uint32_t end, const ovl_hash_limits *L,
                            uint32_t *last_iid, bool boundaries_only = false) {
  int rc = clip_hash_range(c, bgn, end);
  if (rc) return rc;
  if (!L) return fail(OVL_ERR_BAD_PARAM, "null limits");
  if (L->max_hash_strings == 0) return fail(OVL_ERR_BAD_PARAM, "no memory model (--hashstrings 0)");
  if (L->hash_mask_bits == 0 || L->hash_mask_bits > 40)
    return fail(OVL_ERR_BAD_PARAM, "--hashbits %u", L->hash_mask_bits);
  if (end < bgn) return fail(OVL_ERR_BAD_PARAM, "empty hash range %u-%u", bgn, end);
  const uint32_t k = c->P.kmer_len;
  auto loadable = [&](uint32_t r) {
    uint32_t lib = read_lib(c, r);
    return lib >= L->min_lib_hash && lib <= L->max_lib_hash &&
           (int64_t)c->h_len[r] >= (int64_t)c->P.min_olap_len;
  };
  // :495-523 -- the allocation pass counts every loadable read up to endID; the reference
  // asserts when that exceeds the data limit by more than one maximal read
  uint64_t max_alloc = 0;
  for (uint32_t id = bgn; id <= end && id >= bgn; id++)
    if (loadable(id - c->first_iid)) max_alloc += c->h_len[id - c->first_iid] + 1;
  if (max_alloc >= L->max_hash_data_len + AS_MAX_READLEN)
    return fail(OVL_ERR_BAD_PARAM,
                "hash range %u-%u holds %llu bases, more than --hashdatalen %llu + "
                "AS_MAX_READLEN (Build_Hash_Index.C:523 asserts)", bgn, end,
                (unsigned long long)max_alloc, (unsigned long long)L->max_hash_data_len);
  // strings and bases
  uint32_t e = end;
  uint64_t total = 0, windows = 0;
  for (uint32_t id = bgn;; id++) {
    uint32_t r = id - c->first_iid;
    if (loadable(r)) {
      total += c->h_len[r] + 1;
      if (c->h_len[r] >= k) windows += c->h_len[r] - k + 1;
    }
    if (id == end) break;
    if ((uint64_t)(id + 1 - bgn) >= L->max_hash_strings || total >= L->max_hash_data_len) {
      e = id;
      break;
    }
  }
  c->stats_hash_lib_lo = L->min_lib_hash;
  c->stats_hash_lib_hi = L->max_lib_hash;
  if ((rc = apply_hash_libs(c, L->min_lib_hash, L->max_lib_hash))) return rc;
  // table load: at most one entry per window, so only a batch with more windows than the
  // limit can be stopped by it
  const uint64_t entry_limit =
      (uint64_t)(L->max_hash_load * (double)(1ull << L->hash_mask_bits) * (double)ENTRIES_PER_BUCKET);
  const bool load_may_cut = windows >= entry_limit && e > bgn;
  auto too_big = [&](uint64_t wcap) {
    return fail(OVL_ERR_UNSUPPORTED, "hash batch %u-%u holds %llu k-mers, more than one index "
                "on this GPU (%llu: %.1f GB free or held by this context, %.1f GB kept for "
                "the search buffers); lower --hashstrings", bgn, e,
                (unsigned long long)windows, (unsigned long long)wcap, g_cap_free / 1e9,
                g_cap_reserve / 1e9);
  };
  if (boundaries_only && !load_may_cut) {
    // the driver's first phase builds nothing here, but a batch no index can hold would
    // become a super-batch of its own and fail later with a bare out-of-memory
    const uint64_t wcap = index_window_cap(c);
    if (windows > wcap) return too_big(wcap);
    *last_iid = e;
    return OVL_OK;
  }
  // When the load may cut the batch, the first build covers only a prefix of about twice
  // the limit's windows (a read's new k-mers are at most its windows, so the cut lies past
  // the limit's windows; typical reads bring 0.3-0.7 new k-mers per window).  A prefix the
  // load does not stop inside is doubled.  One index holds at most wcap windows (32-bit
  // records; this GPU's free HBM): the previous batch's search buffers are released only
  // when the build needs their memory, since every (re)allocation costs ~30 GB/s of
  // clearing.
  // Consecutive batches of one job cut at about the same number of windows, so after the
  // first cut the prefix is the previous cut's windows + 1/8 (a prefix the cut does not fall
  // inside is doubled, as above): one build of ~1.1x instead of ~2x the batch before the
  // rebuild of the cut range
  uint64_t target = load_may_cut ? std::min<uint64_t>(windows, std::max<uint64_t>(2 * entry_limit, 1u << 20))
                                 : windows;
  if (load_may_cut && c->cut_windows_hint)
    target = std::min<uint64_t>(windows, std::max<uint64_t>(c->cut_windows_hint + c->cut_windows_hint / 8,
                                                            1u << 20));
  for (;;) {
    const uint64_t wcap = index_window_cap(c);
    if (!load_may_cut && windows > wcap) return too_big(wcap);
    const uint64_t tw = std::min(target, wcap);
    uint32_t eb = e;
    if (tw < windows) {
      uint64_t w = 0;
      eb = bgn;
      for (uint32_t id = bgn; id <= e; id++) {
        uint32_t r = id - c->first_iid;
        uint64_t add = (loadable(r) && c->h_len[r] >= k) ? c->h_len[r] - k + 1 : 0;
        if (w + add > tw && id > bgn) break;
        w += add;
        eb = id;
      }
    }
    const bool bloom = !boundaries_only && (!c->sq.on || sq_bloom());
    if ((rc = build_index(c, bgn, eb, bloom, !boundaries_only)) == OVL_ERR_OOM) {
      // the previous batch's search buffers make room (the next search grows them again)
      release_find_buffers(c);
      c->stats.find_releases++;
      rc = build_index(c, bgn, eb, bloom, !boundaries_only);
    }
    if (rc) return rc;
    if (!load_may_cut) break;
    hipStream_t s = c->stream;
    uint32_t nr = eb - bgn + 1;
    DBuf<uint32_t> &hist = c->b_first;
    if (hist.alloc(nr)) return fail(OVL_ERR_OOM, "first-read histogram");
    HIPC(hipMemsetAsync(hist.p, 0, 4ull * nr, s));
    uint32_t n = (uint32_t)c->index_records;
    if (n && nr <= 2u * OVL_FR_WORDS)
      hipLaunchKernelGGL(k_first_reads_lds, dim3((n + OVL_FR_CHUNK - 1) / OVL_FR_CHUNK), dim3(1024),
                         0, s, c->d_tmpM2.p, c->d_occ.p, n, bgn, nr, hist.p);
    else if (n)
      hipLaunchKernelGGL(k_first_reads, dim3(std::min<uint32_t>((n + 255) / 256, 16384)), dim3(256),
                         0, s, c->d_tmpM2.p, c->d_occ.p, n, bgn, hist.p);
    HIPC(hipGetLastError());
    std::vector<uint32_t> h(nr);
    HIPC(hipMemcpyAsync(h.data(), hist.p, 4ull * nr, hipMemcpyDeviceToHost, s));
    HIPC(hipStreamSynchronize(s));
    uint64_t entries = 0;
    uint32_t el = eb;
    bool reached = false;
    for (uint32_t i = 0; i < nr; i++) {
      entries += h[i];
      if (entries >= entry_limit) { el = bgn + i; reached = true; break; }
    }
    if (reached) {
      if (el < eb && !boundaries_only) {
        // the prefix's index cut down to the batch (k_cut_index), or built again over it
        // (OVL_CUT_FILTER=0; read per build, so a test can compare the two in one process).
        // After a cut, index_records stays the prefix's count on purpose: the occurrence array
        // is the prefix's, and the cut table's runs point into it (an export copies all of it).
        // Reads in (el, eb] keep the screened-end bits the prefix build set; they are no
        // target of this batch, and the next build clears every read's bits (k_clear_screen)
        const bool cut = !getenv("OVL_CUT_FILTER") || atoi(getenv("OVL_CUT_FILTER")) != 0;
        if (cut) {
          HIPC(hipEventRecord(c->ev[0], s));
          hipLaunchKernelGGL(k_cut_index, dim3(8 * c->n_cu), dim3(256), 0, s, c->d_tab.p,
                             1ull << c->tab_bits, (const uint64_t *)c->d_occ.p, el);
          HIPC(hipGetLastError());
          HIPC(hipEventRecord(c->ev[1], s));
          HIPC(hipStreamSynchronize(s));
          float ms = 0;
          (void)hipEventElapsedTime(&ms, c->ev[0], c->ev[1]);
          c->stats.ms_index += ms;
          c->hash_end_iid = el;
        } else if ((rc = build_index(c, bgn, el, bloom))) {
          return rc;
        }
      }
      e = el;
      uint64_t cw = 0;
      for (uint32_t id = bgn; id <= el; id++) {
        const uint32_t r = id - c->first_iid;
        if (loadable(r) && c->h_len[r] >= k) cw += c->h_len[r] - k + 1;
      }
      c->cut_windows_hint = cw;
      break;
    }
    if (eb == e) break;                           // the whole range, under the load limit
    if (tw >= wcap)
      return fail(OVL_ERR_UNSUPPORTED, "hash batch from %u: the table load limit (%llu entries, "
                  "--hashbits %u --hashload %g) is not reached within %llu k-mers, the most one "
                  "index holds on this GPU; lower --hashbits or --hashload", bgn,
                  (unsigned long long)entry_limit, L->hash_mask_bits, L->max_hash_load,
                  (unsigned long long)wcap);
    target = std::min<uint64_t>(windows, 2 * tw);
  }
  *last_iid = e;
  return OVL_OK;
}

int ovl_build_hash_batch(ovl_ctx *c, uint32_t bgn, uint32_t end, const ovl_hash_limits *L,
                         uint32_t *last_iid) {
  if (c) c->stats.ms_index = 0;
  return build_batch_impl(c, bgn, end, L, last_iid);
}

IndexDev index_dev(const ovl_ctx *c) {
  IndexDev X;
  X.tab = c->d_tab.p;
  X.occ = c->d_occ.p;
  X.tab_bits = c->tab_bits;
  X.slice_bits = c->slice_bits;
  X.k = c->P.kmer_len;
  X.kmask = (1ull << (2 * c->P.kmer_len)) - 1;
  X.bloom = nullptr;
  X.bloom_w = 0;
  return X;
}

// Whether a search of ref reads bgn..end should probe through the Bloom filter: when at
// least 3/4 of them lie outside the hash range (OverlapDriver's later batches, probed by
// every earlier query), most of their windows miss the table.  OVL_BLOOM=0/1 forces it.
static bool use_bloom(const ovl_ctx *c, uint32_t bgn, uint32_t end) {
  if (!c->bloom_ok) return false;                 // only driver batches build one
  if (const char *e = getenv("OVL_BLOOM")) return atoi(e) != 0;
  if (end < bgn) return false;
  const uint64_t q = (uint64_t)end - bgn + 1;
  const uint32_t lo = std::max(bgn, c->hash_bgn_iid), hi = std::min(end, c->hash_end_iid);
  const uint64_t inside = hi >= lo ? (uint64_t)hi - lo + 1 : 0;
  return 4 * (q - inside) >= 3 * q;
}

// The sorted query windows of an OverlapDriver job (k_sq_keys / k_probe_sorted): the units
// find_impl searches (ref reads bgn..end of libraries [lib_lo, lib_hi] at least --minlength
// and k long, both orientations, read order), their windows keyed by mix64(k-mer) and
// radix-sorted once, in runs of <= 2^29 windows.  A batch searches the units of the reads
// below its last hash read: a prefix of them, so per run a window-id bound.  Off (and the
// random-lookup probe used) when the keys would take more than half the free HBM.
//
// The device arrays outlive the job (free_mem false at a job's end): they are grow-only like
// the search buffers, since hipMalloc of the ~58 GB a configs[4] rank job sorts takes ~1.7 s
// here (profiles/r04s_chain_occ_c4_sq.txt) -- the keys themselves are recomputed and sorted by
// every job.
static size_t sq_held_bytes(const ovl_ctx *c) {
  const auto &Q = c->sq;
  return 8 * (Q.key.n + Q.key2.n + Q.dwbase.n) + 4 * (Q.wid.n + Q.wid2.n + Q.ublk.n + Q.uhits.n +
         Q.uflags.n) + Q.tmp.n + sizeof(Unit) * Q.dunits.n;
}
static void sq_release(ovl_ctx *c, bool free_mem) {
  auto &Q = c->sq;
  Q.on = false;
  if (free_mem) {
    Q.key.release(); Q.key2.release(); Q.wid.release(); Q.wid2.release(); Q.ublk.release();
    Q.dwbase.release(); Q.dunits.release(); Q.tmp.release(); Q.uhits.release(); Q.uflags.release();
    Q.sig.release();
  }
  Q.units.clear(); Q.ureadiid.clear(); Q.uwin.clear(); Q.wb.clear(); Q.runs.clear();
  Q.probed = -1;
}

static int sq_prepare(ovl_ctx *c, uint32_t bgn, uint32_t end, uint32_t lib_lo, uint32_t lib_hi) {
  auto &Q = c->sq;
  if (Q.on && Q.ref_bgn == bgn && Q.ref_end == end && Q.lib_lo == lib_lo && Q.lib_hi == lib_hi)
    return OVL_OK;
  sq_release(c, false);
  const uint32_t k = c->P.kmer_len;
  for (uint32_t a = bgn; a <= end && a >= bgn; a++) {         // find_impl's unit rule
    const uint32_t r = a - c->first_iid;
    const int32_t L = (int32_t)c->h_len[r];
    const uint32_t lib = read_lib(c, r);
    if (lib < lib_lo || lib > lib_hi || L < c->P.min_olap_len || L < (int32_t)k) continue;
    for (uint32_t dir = 0; dir < 2; dir++) {
      Q.units.push_back(Unit{r, dir});
      Q.ureadiid.push_back(a);
      Q.uwin.push_back((uint64_t)(L - (int32_t)k + 1));
    }
  }
  const uint32_t nu = (uint32_t)Q.units.size();
  if (nu == 0) return OVL_OK;
  // runs of <= RUN windows (hipcub sorts index with int)
  // 2^29 windows per run: a run's sort needs ~24 B per window beside the 12 B it keeps (the
  // configs[4] rank-0 job at 1/8 scale: 3.8 G windows, 58 GB with 2^29-window runs, 71 GB
  // with 2^30 -- past half of the ~133 GB free when its second batch starts)
  const uint64_t RUN = 1ull << 29;
  uint64_t total = 0, maxrun = 0;
  for (uint32_t u = 0; u < nu;) {
    ovl_ctx::SqRun R;
    R.u0 = u;
    R.e0 = total;
    R.n = 0;
    while (u < nu && (R.n + Q.uwin[u] <= RUN || u == R.u0)) R.n += Q.uwin[u++];
    R.u1 = u;
    R.wb0 = Q.wb.size();
    uint64_t acc = 0;
    for (uint32_t x = R.u0; x < R.u1; x++) { Q.wb.push_back(acc); acc += Q.uwin[x]; }
    Q.wb.push_back(acc);
    total += R.n;
    maxrun = std::max(maxrun, R.n);
    Q.runs.push_back(R);
  }
  size_t fr = 0, tot = 0;
  if (hipMemGetInfo(&fr, &tot) != hipSuccess) return OVL_OK;
  const uint64_t need = 12ull * total + 24ull * maxrun + 8ull * (maxrun >> 9) + 64ull * nu;
  Q.resorted = 0;
  if (getenv("OVL_TIMING"))
    fprintf(stderr, "OVL_TIMING sorted query windows: %u units, %llu windows in %zu runs, "
            "%.1f GB needed, %.1f GB free\n", nu, (unsigned long long)total, Q.runs.size(),
            need / 1e9, fr / 1e9);
  // up to half the free HBM (the configs[4] rank-0 job at 1/8 scale: 3.8 G windows, 67 GB),
  // counting what an earlier job's arrays hold as free.  A driver job's query chunks were
  // planned against that rule before its search buffers existed (plan_query_chunks); from
  // then on those buffers keep their size (sticky_budgets), so a later chunk needs only fit
  // what is free beside them -- under the half rule the full-size configs[4] job sorted its
  // first chunk only and probed the other five by random lookups (r05g: 120 launches)
  const uint64_t avail = fr + sq_held_bytes(c);
  if (c->sticky_budgets ? need + (4ull << 30) > avail : need > avail / 2) {
    sq_release(c);
    c->stats.sq_declined++;
    if (getenv("OVL_TIMING"))
      fprintf(stderr, "OVL_TIMING sorted query windows declined: %.1f GB needed, %.1f GB "
              "available -> random-lookup probes\n", need / 1e9, avail / 1e9);
    return OVL_OK;
  }
  hipStream_t s = c->stream;
  const auto t0 = std::chrono::steady_clock::now();
  size_t tmpb = 0;
  // Windows need only be ordered by the key's top 24 bits (a table slot is its top
  // tab_bits): 3 radix passes instead of 8.  This ROCm's hipcub / rocPRIM radix sort over a
  // partial bit range of 64-bit keys returned duplicated ids and an unsorted order below
  // ~1.4 M items (tools/sortcheck.hip: 100 k and 882,524 items wrong for [32|40|48, 64),
  // 1.44 M to 2^27 right; profiles/r04n_sortcheck.log), so runs under PART_MIN windows sort
  // all 64 bits, and a partially sorted run is checked on both properties that broke
  // (k_sq_sorted_check: key order, and the (key, wid) multiset against k_sq_keys' signature)
  // and sorted again over all bits if either fails.  OVL_TEST_SQ_CORRUPT=1 (tests) checks
  // every run and duplicates a window id in the first run's sorted output, so the fallback
  // path runs.
  const uint64_t PART_MIN = 1ull << 22;
  const int PART_LO = 40;
  {
    size_t t64 = 0;
    HIPC(hipcub::DeviceRadixSort::SortPairs(nullptr, tmpb, Q.key2.p, Q.key.p, Q.wid2.p, Q.wid.p,
                                            (int)std::min<uint64_t>(maxrun, RUN), PART_LO, 64, s));
    HIPC(hipcub::DeviceRadixSort::SortPairs(nullptr, t64, Q.key2.p, Q.key.p, Q.wid2.p, Q.wid.p,
                                            (int)std::min<uint64_t>(maxrun, RUN), 0, 64, s));
    tmpb = std::max(tmpb, t64);
  }
  std::vector<uint32_t> ublk;
  for (auto &R : Q.runs) {
    R.ub0 = ublk.size();
    uint32_t x = 0;
    for (uint64_t w = 0; w < R.n; w += 512) {
      while (Q.wb[R.wb0 + x + 1] <= w) x++;
      ublk.push_back(x);
    }
  }
  // a driver job's chunks differ by a few windows: the first one takes the largest chunk's
  // size (ovl_ctx::sq_reserve), or the next would free and reallocate ~57 GB (~1.7 s here)
  if (c->sq_reserve > total && (Q.key.n < c->sq_reserve || Q.wid.n < c->sq_reserve))
    if (Q.key.alloc(c->sq_reserve) || Q.wid.alloc(c->sq_reserve)) { /* exact sizes below */ }
  if (Q.key.alloc(total) || Q.wid.alloc(total) || Q.key2.alloc(maxrun) || Q.wid2.alloc(maxrun) ||
      Q.tmp.alloc(std::max<size_t>(tmpb, 1)) || Q.dwbase.alloc(Q.wb.size()) ||
      Q.dunits.alloc(nu) || Q.ublk.alloc(std::max<size_t>(ublk.size(), 1)) ||
      Q.uhits.alloc(nu) || Q.uflags.alloc(nu) || Q.sig.alloc(5)) {
    sq_release(c);
    return OVL_OK;                                 // no room: the random-lookup probe
  }
  const bool test_corrupt = getenv("OVL_TEST_SQ_CORRUPT") && atoi(getenv("OVL_TEST_SQ_CORRUPT"));
  HIPC(hipMemcpyAsync(Q.dwbase.p, Q.wb.data(), 8ull * Q.wb.size(), hipMemcpyHostToDevice, s));
  HIPC(hipMemcpyAsync(Q.dunits.p, Q.units.data(), sizeof(Unit) * nu, hipMemcpyHostToDevice, s));
  if (!ublk.empty())
    HIPC(hipMemcpyAsync(Q.ublk.p, ublk.data(), 4ull * ublk.size(), hipMemcpyHostToDevice, s));
  for (const auto &R : Q.runs) {
    SqKeyArgs KA;
    KA.R = c->reads();
    KA.units = Q.dunits.p + R.u0;
    KA.wbase = Q.dwbase.p + R.wb0;
    KA.nunits = R.u1 - R.u0;
    KA.k = k;
    KA.kmask = (1ull << (2 * k)) - 1;
    KA.key = Q.key2.p;
    KA.wid = Q.wid2.p;
    KA.sig = Q.sig.p;
    // keys, sort, and (partial-range runs) the check; with `bits_lo` 0 the sort is over all bits
    auto sort_run = [&](int bits_lo, bool corrupt) -> int {
      HIPC(hipMemsetAsync(Q.sig.p, 0, 5 * sizeof(unsigned long long), s));
      hipLaunchKernelGGL(k_sq_keys, dim3((KA.nunits + 3) / 4), dim3(256), 0, s, KA);
      HIPC(hipGetLastError());
      size_t tb = tmpb;
      HIPC(hipcub::DeviceRadixSort::SortPairs(Q.tmp.p, tb, Q.key2.p, Q.key.p + R.e0, Q.wid2.p,
                                              Q.wid.p + R.e0, (int)R.n, bits_lo, 64, s));
      if (corrupt && R.n >= 2)
        HIPC(hipMemcpyAsync(Q.wid.p + R.e0 + 1, Q.wid.p + R.e0, 4, hipMemcpyDeviceToDevice, s));
      return OVL_OK;
    };
    auto check_run = [&](int bits_lo, bool *broken) -> int {
      hipLaunchKernelGGL(k_sq_sorted_check, dim3(4 * c->n_cu), dim3(256), 0, s,
                         (const uint64_t *)(Q.key.p + R.e0), (const uint32_t *)(Q.wid.p + R.e0),
                         R.n, (uint32_t)bits_lo, Q.sig.p, (uint32_t *)(Q.sig.p + 4));
      HIPC(hipGetLastError());
      unsigned long long h[5] = {0, 0, 0, 0, 0};
      HIPC(hipMemcpyAsync(h, Q.sig.p, sizeof(h), hipMemcpyDeviceToHost, s));
      HIPC(hipStreamSynchronize(s));
      *broken = (uint32_t)h[4] != 0 || h[0] != h[2] || h[1] != h[3];
      return OVL_OK;
    };
    const int lo = R.n >= PART_MIN ? PART_LO : 0;
    const bool corrupt = test_corrupt && &R == &Q.runs[0];
    if (int rc = sort_run(lo, corrupt)) return rc;
    if (lo || test_corrupt) {
      bool broken = false;
      if (int rc = check_run(lo, &broken)) return rc;
      if (broken) {                                  // the keys again, every bit sorted
        if (int rc = sort_run(0, false)) return rc;
        if (int rc = check_run(0, &broken)) return rc;
        if (broken)
          return fail(OVL_ERR_HIP, "sorted query windows: run of %llu windows failed its check "
                      "after a full-range sort", (unsigned long long)R.n);
        Q.resorted++;
      }
    }
  }
  c->stats.sq_resorted += Q.resorted;
  HIPC(hipStreamSynchronize(s));
  Q.ms_sort = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  if (getenv("OVL_TIMING"))
    fprintf(stderr, "OVL_TIMING sorted query windows: sorted in %.1f ms (%u runs sorted again "
            "over all bits)\n", Q.ms_sort, Q.resorted);
  c->stats.ms_seed += Q.ms_sort;
  Q.ref_bgn = bgn; Q.ref_end = end; Q.lib_lo = lib_lo; Q.lib_hi = lib_hi;
  Q.on = true;
  Q.probed = -1;
  return OVL_OK;
}

// Process_Overlaps (overlapInCore-Process_Overlaps.C:101-137) over ref reads bgn..end of
// libraries [lib_lo, lib_hi] against the current index.  append: keep the records and
// counters already held (the driver's later hash batches).
static int find_impl(ovl_ctx *c, uint32_t bgn, uint32_t end, uint32_t lib_lo, uint32_t lib_hi,
                     bool append, uint64_t *n_out, bool flush = true) {
  if (!c) return fail(OVL_ERR_STATE, "null context");
  if (!c->have_index) return fail(OVL_ERR_STATE, "ovl_build_hash_index() first");
  HIPC(hipSetDevice(c->device));
  hipStream_t s = c->stream;
  const uint32_t k = c->P.kmer_len;
  if (bgn < 1) bgn = 1;
  if (bgn < c->first_iid) bgn = c->first_iid;
  uint32_t last = c->first_iid + c->nreads - 1;
  if (end > last) end = last;

  // units: (query, FORWARD), (query, REVERSE) -- Process_Overlaps.C:124-128
  std::vector<Unit> units;
  std::vector<uint64_t> uwin;
  uint64_t nref = 0;
  for (uint32_t a = bgn; a <= end && a >= bgn; a++) {
    uint32_t r = a - c->first_iid;
    int32_t L = (int32_t)c->h_len[r];
    uint32_t lib = read_lib(c, r);
    if (lib < lib_lo || lib > lib_hi) continue;  // -R (Process_Overlaps.C:108)
    if (L < c->P.min_olap_len) continue;         // :114
    nref++;
    if (L < (int32_t)k) continue;
    if (a >= c->hash_end_iid) continue;          // no hash read with a larger ID
    units.push_back(Unit{r, 0});
    units.push_back(Unit{r, 1});
    uwin.push_back((uint64_t)(L - (int32_t)k + 1));
    uwin.push_back((uint64_t)(L - (int32_t)k + 1));
  }
  if (!append) {
    c->acc.nu = c->acc.nn = c->acc.np = 0;          // a new job: nothing pending
    ovl_stats keep_idx = c->stats;
    memset(&c->stats, 0, sizeof(c->stats));
    c->stats.ms_index = keep_idx.ms_index;
    c->stats.hash_batches = 1;
    c->nout = 0;
  }
  c->stats.ref_reads += nref;

  // OverlapDriver batches: the job's query windows sorted once (sq_prepare); this batch's
  // units are the first nu of the job's (the reads below its last hash read)
  if (c->sq_request && !units.empty())
    if (int rc = sq_prepare(c, bgn, end, lib_lo, lib_hi)) return rc;
  const bool sqm = c->sq_request && c->sq.on && !units.empty();
  if (sqm) {
    auto &Q = c->sq;
    if (units.size() > Q.units.size() ||
        memcmp(units.data(), Q.units.data(), sizeof(Unit) * units.size()) != 0)
      return fail(OVL_ERR_HIP, "sorted query windows: unit list mismatch");
    Q.probed = -1;                                  // a new index: no run probed against it
  }
  std::vector<uint32_t> sq_uh;                      // the probed run's unit hit counts
  size_t sq_run = 0;

  // per-context device buffers, sized per batch
  // A batch is sized by seed hits (node pool + list-ordered copy: 32 B per hit); the probe
  // window budget adapts to the hits-per-window ratio seen so far so that a batch's probe
  // results are all consumed (units beyond the hit budget would otherwise be re-probed).
  // seed hits per batch; halved while the chain buffers do not fit the HBM the index
  // leaves, as the probe-slot cap is for the probe records
  // 3.5 G: the 50k x 10 kb job in 2 chunks (1.27 s per step) rather than 4 (1.29 s) or 8
  // (1.34 s) -- fewer re-probed windows and extension tails; node indices stay < 2^32
  uint64_t HIT_BUDGET = 3584ull << 20;
  {
    // within the HBM left beside the index: the node pool and its list-ordered copy take
    // ~33 B per hit; keep them under 60 % of what is free now plus what they already hold
    size_t fr = 0, tot = 0;
    if (hipMemGetInfo(&fr, &tot) == hipSuccess) {
      const uint64_t held = (c->fb.pool.n + c->fb.pnodes[0].n + c->fb.pnodes[1].n) * sizeof(Node);
      HIT_BUDGET = std::min<uint64_t>(HIT_BUDGET, (uint64_t)((fr + held) * 0.6) / 33);
    }
    // a driver job's later searches chain within the buffers its first one sized (more hit
    // chunks per run instead of a regrow of the pool and its copy)
    if (c->sticky_budgets && c->fb.pnodes[0].n > (16ull << 20))
      HIT_BUDGET = std::min<uint64_t>(HIT_BUDGET, c->fb.pnodes[0].n - 1);
  }
  if (const char *e = getenv("OVL_HIT_BUDGET_M"))             // experiments: millions of hits
    HIT_BUDGET = std::max<uint64_t>(16, strtoull(e, nullptr, 10)) << 20;
  HIT_BUDGET = std::max<uint64_t>(HIT_BUDGET, 16ull << 20);
  uint64_t win_cap = 1536ull << 20;
  uint64_t WIN_BUDGET = 512ull << 20;           // probe slots per batch (8 B each)
  auto &d_rbase = c->fb.rbase;
  auto &d_probe = c->fb.probe;
  auto &d_uhits = c->fb.uhits;
  auto &d_uflags = c->fb.uflags;
  auto &d_ctr = c->fb.ctr;
  auto &d_defer = c->fb.defer;
  auto &d_pool = c->fb.pool;
  auto &d_stats = c->fb.stats;
  // OVL_PIPELINE=1 runs chunk i's extension on a second stream while chunk i+1 is probed and
  // chained (two buffer slots).  Measured slower (50k x 10 kb: 1.37-1.41 s vs 1.31 s per
  // job): the extension keeps every CU's issue slots busy, so the co-running probe and chain
  // only take them from it.  Default: one stream, one slot.
  // -l: every pair through the ordered generic kernel (a unit's pairs one after another)
  const bool ordered = c->P.frag_olap_limit != UINT64_MAX;
  const bool pipe = getenv("OVL_PIPELINE") != nullptr && !ordered;
  hipStream_t xs = pipe ? c->xstream : s;
  const bool window = c->P.use_window_filter && c->P.max_erate <= 0.06;
  if (window && !c->have_qual)
    return fail(OVL_ERR_BAD_PARAM, "-w (window filter) needs the reads' qualities");
  if (d_ctr.alloc(16) || d_stats.alloc(16) || c->fb.xctr[0].alloc(16) ||
      c->fb.xctr[1].alloc(16) || c->fb.xnout.alloc(1))
    return fail(OVL_ERR_OOM, "counters");
  HIPC(hipMemsetAsync(d_stats.p, 0, 128, s));

  // ---- extension configuration --------------------------------------------------------
  // Pairs go through up to three launches: the staged kernel at full occupancy (8 waves per
  // <= 64 KB block) for pairs whose reads are both <= len1, the staged kernel with more LDS
  // per wave for reads <= len2, and the generic kernel for the rest (reads with an 'n',
  // bands wider than the register window, longer reads).  Each launch's scratch and LDS are
  // sized for its own length class, so one long read in a job does not shrink the others.
  auto ecap_of = [&](uint64_t L) {
    return c->h_error_bound[std::min<uint64_t>(L, AS_MAX_READLEN)] + 2;
  };
  auto sw_of = [](uint64_t L) { return (int32_t)(((L + 31) / 32 + 2) & ~1ull); };
  auto stg_lds_of = [&](uint64_t L) { return 4ull * (4ull * (uint64_t)sw_of(L) + OVL_SCR_STAGE); };
  auto ml_of = [](int32_t ec) { return 4ull * (((uint64_t)(ec + 2) + 3) & ~3ull); };
  // the staged kernel's block-shared Edit_Match_Limit table
  auto sml_of = [&](int32_t ec) { return ml_of(ec); };
  auto fits = [&](uint64_t L, uint32_t wpb, size_t cap) {
    return stg_lds_of(L) * wpb + sml_of(ecap_of(L)) <= cap;
  };
  auto longest_fitting = [&](uint32_t wpb, size_t cap) -> uint32_t {
    uint64_t lo = 0, hi = c->max_len;
    if (fits(hi, wpb, cap)) return (uint32_t)hi;
    while (lo + 1 < hi) {
      const uint64_t mid = (lo + hi) / 2;
      if (fits(mid, wpb, cap)) lo = mid; else hi = mid;
    }
    return (uint32_t)lo;
  };
  struct ExtClass {
    uint32_t len = 0, wpb = 1, waves = 0;
    int32_t ecap = 0, sw = 0;
    size_t lds = 0;
    bool l16 = false;
    uint64_t stride = 0;
    bool wide = false;             // the 2 x OVL_RJ-chunk register window (wide bands)
  };
  // the staged kernel instance of a class
  auto stage_kernel = [](bool l16, bool wide) -> const void * {
    if (wide) return l16 ? reinterpret_cast<const void *>(k_extend<true, true, false, 2 * OVL_RJ>)
                         : reinterpret_cast<const void *>(k_extend<true, false, false, 2 * OVL_RJ>);
    return l16 ? reinterpret_cast<const void *>(k_extend<true, true>)
               : reinterpret_cast<const void *>(k_extend<true, false>);
  };
  const uint64_t SCRATCH_BUDGET = 24ull << 30;
  std::vector<ExtClass> ext_stage;
  auto per_wave_bytes = [](const ExtClass &g) {
    return g.stride * 4 + 16ull * (g.ecap + 2) + 28ull * (g.ecap + 8);
  };
  auto make_stage = [&](uint32_t L, size_t cap, bool allow_knob, bool wide = false) -> int {
    ExtClass g;
    g.len = L;
    g.wide = wide;
    g.ecap = ecap_of(L);
    g.sw = sw_of(L);
    g.l16 = L < 16384;
    g.wpb = (uint32_t)std::min<uint64_t>(8, (cap - std::min<uint64_t>(cap, sml_of(g.ecap))) / stg_lds_of(L));
    if (g.wpb < 1) return -1;
    g.lds = stg_lds_of(L) * g.wpb + sml_of(g.ecap);
    // experiment knob: OVL_EXT_BLOCKS_PER_CU pads the LDS so that at most that many blocks
    // fit on a CU (occupancy studies); unset = natural occupancy
    if (allow_knob)
      if (const char *bp = getenv("OVL_EXT_BLOCKS_PER_CU")) {
        int nb = atoi(bp);
        if (nb > 0) g.lds = std::max<size_t>(g.lds, (160 * 1024) / nb - 256);
      }
    const uint64_t lw = wide ? std::max<uint64_t>(OVL_LOGW, 128 * OVL_RJ) : OVL_LOGW;
    uint64_t st = (uint64_t)(g.ecap + 2) * lw / (g.l16 ? 2 : 1);   // the row log
    if (window) st = std::max<uint64_t>(st, 3ull * (g.ecap + 9) + 2ull * L + 64);
    g.stride = (st + 63) & ~63ull;
    const void *kfn = stage_kernel(g.l16, wide);
    if (g.lds > 64 * 1024)
      if (hipFuncSetAttribute(kfn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)g.lds) != hipSuccess)
        return -1;
    // persistent grid: as many blocks as are resident at once (registers and LDS), so no
    // block starts only after the work queue has drained; within the scratch budget
    uint32_t waves = 4u * OVL_EXT_OCC * c->n_cu;
    int bpc = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&bpc, kfn, 64 * g.wpb, g.lds) == hipSuccess &&
        bpc > 0)
      waves = std::min<uint32_t>(waves, (uint32_t)bpc * g.wpb * c->n_cu);
    while (waves > g.wpb && (uint64_t)waves * per_wave_bytes(g) > SCRATCH_BUDGET) waves /= 2;
    g.waves = std::max<uint32_t>(g.wpb, (waves / g.wpb) * g.wpb);
    if (!wide) c->ext_classes.push_back(g.len);
    ext_stage.push_back(g);
    return 0;
  };
  c->ext_classes.clear();
  // occupancy tiers of the staged kernel: 3 blocks of 8 waves per CU (the register limit),
  // 3 blocks of 6, then blocks of up to 8 waves within 160 KB (as many as fit a CU).  A
  // class's length is the span it stages (k_extend stages a pair's overlap span, not its
  // whole reads): the tier's limit, or the longest loaded read when that is shorter, so a
  // short-read job's launch is exactly what it was and a long-read job's pairs with shorter
  // spans run at the higher occupancy.
  {
    uint32_t prev = 0;
    const size_t tier_cap[3] = {52 * 1024, 52 * 1024, 160 * 1024};
    const uint32_t tier_wpb[3] = {8, 6, 1};
    for (int t = 0; t < 3; t++) {
      const uint32_t T = longest_fitting(tier_wpb[t], tier_cap[t]);
      const uint32_t L = std::min<uint32_t>(T, c->max_len);
      if (L < 64 || L <= prev) continue;
      if (make_stage(L, tier_cap[t], t == 0)) return fail(OVL_ERR_HIP, "staged kernel setup");
      prev = L;
    }
    // the wide class: the pairs of every staged class whose band outgrew the register window
    // (the rest of their deferrals -- 'n' bases -- pass on to the generic kernel)
    if (!ext_stage.empty() && !getenv("OVL_NO_WIDE") &&
        make_stage(ext_stage.back().len, 160 * 1024, false, true))
      return fail(OVL_ERR_HIP, "wide staged kernel setup");
  }
  // the generic kernel: every read length; rows in LDS while two row buffers and the
  // Edit_Match_Limit table fit a CU, else in global memory (GR)
  ExtClass gen;
  gen.len = c->max_len;
  gen.ecap = ecap_of(c->max_len);
  {
    const size_t ml = ml_of(gen.ecap);
    size_t w = 4ull * ((2ull * (2 * gen.ecap + 8) + TB_ROWS * TB_W + OVL_LDCAP + 3) & ~3ull);
    gen.l16 = w + ml > 160 * 1024;                       // GR
    if (gen.l16) w = 4ull * ((TB_ROWS * TB_W + OVL_LDCAP + 3) & ~3ull);
    gen.wpb = (4 * w <= 80 * 1024) ? 4 : (2 * w <= 80 * 1024) ? 2 : 1;
    gen.lds = w * gen.wpb + (gen.l16 ? 0 : ml);
    uint64_t st = (uint64_t)(gen.ecap + 2) * (gen.ecap + 2) + 4ull * (gen.ecap + 2) + 64;
    if (window) st = std::max<uint64_t>(st, 3ull * (gen.ecap + 9) + 2ull * c->max_len + 64);
    // a wave's band-compact row log holds every row of one extension (quadratic in the
    // error limit); past 2^28 ints the GR kernel checks its cursor and fails loudly
    if (gen.l16) st = std::min<uint64_t>(st, 1ull << 28);
    gen.stride = (st + 63) & ~63ull;
    uint32_t waves = 24u * c->n_cu;
    while (waves > gen.wpb && (uint64_t)waves * per_wave_bytes(gen) > (16ull << 30)) waves /= 2;
    gen.waves = std::max<uint32_t>(gen.wpb, (waves / gen.wpb) * gen.wpb);
    const void *kfn = gen.l16 ? reinterpret_cast<const void *>(k_extend<false, true>)
                              : reinterpret_cast<const void *>(k_extend<false, false>);
    if (ordered)
      kfn = gen.l16 ? reinterpret_cast<const void *>(k_extend<false, true, true>)
                    : reinterpret_cast<const void *>(k_extend<false, false, true>);
    if (gen.lds > 64 * 1024)
      HIPC(hipFuncSetAttribute(kfn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)gen.lds));
  }
  uint64_t rows_n = gen.stride * gen.waves, rowdir_n = 4ull * (gen.ecap + 2) * gen.waves,
           deltas_n = 7ull * (gen.ecap + 8) * gen.waves;
  for (const ExtClass &g : ext_stage) {
    rows_n = std::max<uint64_t>(rows_n, g.stride * g.waves);
    rowdir_n = std::max<uint64_t>(rowdir_n, 4ull * (g.ecap + 2) * g.waves);
    deltas_n = std::max<uint64_t>(deltas_n, 7ull * (g.ecap + 8) * g.waves);
  }
  auto &d_rows = c->fb.rows;
  auto &d_rowdir = c->fb.rowdir;
  auto &d_deltas = c->fb.deltas;
  if (d_rows.alloc(rows_n) || d_rowdir.alloc(rowdir_n) || d_deltas.alloc(deltas_n))
    return fail(OVL_ERR_OOM, "extension scratch");
  c->stats_ext_waves = ext_stage.empty() ? 0 : ext_stage[0].waves;
  c->stats_gen_waves = gen.waves;
  uint32_t chain_waves = 4u * OVL_CHAIN_OCC * c->n_cu;   // OVL_CHAIN_OCC blocks of 4 waves per CU

  // With OVL_PIPELINE, chunk i's extension runs on xs while chunk i+1 is probed and chained
  // on s.  Any return from here on first drains xs (its kernels use this context's buffers).
  struct Drain {
    hipStream_t x;
    ~Drain() { (void)hipStreamSynchronize(x); }
  } drain{xs};
  // records: the device counter xnout continues from the records already held (the
  // driver's earlier hash batches); the host tracks an upper bound (<= 3 per pair)
  uint32_t nout32 = (uint32_t)c->nout;
  HIPC(hipMemcpyAsync(c->fb.xnout.p, &nout32, 4, hipMemcpyHostToDevice, s));
  HIPC(hipStreamSynchronize(s));
  uint64_t nout_ub = c->nout;
  auto ensure_out = [&](uint64_t need) -> int {
    if (need <= c->d_out.n && c->d_out.p) return OVL_OK;
    HIPC(hipStreamSynchronize(xs));
    uint32_t cur = 0;
    HIPC(hipMemcpy(&cur, c->fb.xnout.p, 4, hipMemcpyDeviceToHost));
    DBuf<Rec> bigger;
    if (bigger.alloc(need + (need >> 2))) return fail(OVL_ERR_OOM, "output grow");
    if (cur)
      HIPC(hipMemcpyAsync(bigger.p, c->d_out.p, sizeof(Rec) * cur, hipMemcpyDeviceToDevice, s));
    HIPC(hipStreamSynchronize(s));
    std::swap(bigger.p, c->d_out.p);
    std::swap(bigger.n, c->d_out.n);
    return OVL_OK;
  };
  if (int rc = ensure_out(std::max<uint64_t>(c->nout + (1u << 20), c->nout + units.size() * 8)))
    return rc;

  float ms_probe = 0, ms_chain = 0, ms_ext = 0;
  float ms_probe_rest = 0;        // the sorted-window probe step's work beside its kernel
  uint64_t npairs_tot = 0, probe_bytes = 0, seed_hits_tot = 0, n_big_units = 0, nodes_tot = 0;
  uint64_t staged_pairs = 0, long_pairs = 0, generic_pairs = 0;
  uint32_t chain_retries = 0;
  uint32_t n_probe_launch = 0, n_ext_launch = 0, n_probe_sorted = 0;
  uint32_t nu = (uint32_t)units.size();
  uint32_t u0 = 0;
  const uint32_t ctr_next[4] = {5, 11, 13, 15}, ctr_defer[4] = {8, 12, 14, 10};
  bool pending[2] = {false, false};
  uint32_t slot_pairs[2] = {0, 0};
  // chunk i's extension has finished: its counters, class split and time
  auto collect = [&](int sl) -> int {
    if (!pending[sl]) return OVL_OK;
    pending[sl] = false;
    HIPC(hipEventSynchronize(c->xev[2 + sl]));
    uint32_t hx[16];
    HIPC(hipMemcpy(hx, c->fb.xctr[sl].p, 64, hipMemcpyDeviceToHost));
    float t = 0;
    (void)hipEventElapsedTime(&t, c->xev[sl], c->xev[2 + sl]);
    ms_ext += t;
    if (hx[7] & 32u)
      return fail(OVL_ERR_UNSUPPORTED, "an extension needs more than 2^28 row cells (error limit "
                  "%d of a %u-base read): past the generic kernel's per-wave row log",
                  ecap_of(c->max_len), c->max_len);
    if (hx[7]) return fail(OVL_ERR_HIP, "extension capacity exceeded (flags %u)", hx[7]);
    uint32_t left = slot_pairs[sl];
    for (size_t ci = 0; ci < ext_stage.size() && !ordered; ci++) {
      const uint32_t nd = hx[ctr_defer[ci]];
      if (getenv("OVL_DEBUG"))
        fprintf(stderr, "OVL_DEBUG class %zu (reads <= %u): deferred %u of %u pairs\n", ci,
                ext_stage[ci].len, nd, left);
      if (ci == 0) staged_pairs += left - nd;
      else long_pairs += left - nd;
      left = nd;
    }
    generic_pairs += left;
    return OVL_OK;
  };
  // One chunk's (or the accumulator's) pairs through the extension kernels on xs, the host
  // not waiting: work order, the staged classes, the generic kernel; collect(slot) reads
  // its counters back.
  auto launch_ext = [&](int slot, const Unit *ext_units, PairRec *ext_pairs, Node *ext_pnodes,
                        uint32_t npairs, uint32_t nc) -> int {
    auto &x_ctr = c->fb.xctr[slot];
      nout_ub += 3ull * npairs;
      if (int rc = ensure_out(nout_ub)) return rc;
      ExtendArgs EA;
      EA.R = c->reads();
      EA.units = ext_units;
      EA.pairs = ext_pairs;
      EA.npairs = npairs;
      EA.npairs_dev = nullptr;
      EA.restore = 0;
      EA.pnodes = ext_pnodes;
      EA.pair_next = x_ctr.p + 5;
      EA.error_bound = c->d_error_bound.p;
      EA.match_limit = c->d_match_limit.p;
      EA.max_errors = c->max_errors;
      EA.branch_match_value = c->branch_match_value;
      EA.min_branch_tail_slope = c->min_branch_tail_slope;
      EA.min_branch_end_dist = 20;
      EA.partial = c->P.partial;
      EA.unique = c->P.unique_olap_per_pair;
      EA.min_olap_len = c->P.min_olap_len;
      EA.use_hopeless = c->P.use_hopeless_check;
      EA.k = (int32_t)k;
      EA.filter_by_kmer_count = c->P.filter_by_kmer_count;
      EA.minkmer_exp = exp(-1.0 * (double)k * c->P.max_erate);
      EA.rows = d_rows.p;
      EA.rowdir = d_rowdir.p;
      EA.deltas = d_deltas.p;
      EA.out = c->d_out.p;
      EA.nout = c->fb.xnout.p;
      EA.out_cap = (uint32_t)std::min<uint64_t>(c->d_out.n, 0xFFFFFFF0ull);
      EA.stats = d_stats.p;
      EA.window = window ? 1 : 0;
      EA.overflow = x_ctr.p + 7;
      EA.dbg = nullptr;
      if (getenv("OVL_DEBUG")) {
        if (!c->dbg.p) {
          HIPC(hipStreamSynchronize(xs));
          if (c->dbg.alloc(32)) return fail(OVL_ERR_OOM, "debug counters");
          HIPC(hipMemsetAsync(c->dbg.p, 0, 256, xs));
        }
        EA.dbg = c->dbg.p;
      }
      EA.list = nullptr;
      EA.defer = nullptr;
      EA.ndefer = nullptr;
      EA.olim = c->P.frag_olap_limit;
      EA.nunits = nc;
      EA.useg = nullptr;
      EA.ord_slot = nullptr;
      EA.ord_diag = nullptr;
      EA.dkey = nullptr;
      slot_pairs[slot] = npairs;
      HIPC(hipMemsetAsync(x_ctr.p, 0, 64, xs));
      if (npairs && ordered) {
        // the reference's two pair orders per unit (see k_olim_keys): String_Olap_Space
        // order and By_Diag_Sum order, by stable radix sorts
        auto &fb = c->fb;
        const int n = (int)npairs;
        size_t t1 = 0, t2 = 0, t3 = 0;
        HIPC(hipcub::DeviceRadixSort::SortPairs(nullptr, t1, fb.okey.p, fb.okey2.p, fb.oa.p,
                                                fb.ob.p, n, 0, 32, xs));
        HIPC(hipcub::DeviceRadixSort::SortPairs(nullptr, t2, fb.ok64a.p, fb.ok64b.p, fb.oa.p,
                                                fb.ob.p, n, 0, 64, xs));
        HIPC(hipcub::DeviceScan::ExclusiveSum(nullptr, t3, fb.ucnt.p, fb.useg.p, (int)nc + 1, xs));
        const size_t tmp = std::max(std::max(t1, t2), t3);
        HIPC(hipStreamSynchronize(xs));
        if (fb.okey.grow(npairs) || fb.okey2.grow(npairs) || fb.oa.grow(npairs) ||
            fb.ob.grow(npairs) || fb.oidx.grow(npairs) || fb.oidx2.grow(npairs) ||
            fb.ok64a.grow(npairs) || fb.ok64b.grow(npairs) || fb.dkey.grow(npairs) ||
            fb.ucnt.grow((size_t)nc + 1) || fb.useg.grow((size_t)nc + 1) ||
            fb.otmp.grow(std::max<size_t>(tmp, 1)))
          return fail(OVL_ERR_OOM, "-l pair orders");
        const dim3 grid(std::min<uint32_t>((npairs + 255) / 256, 4096)), blk(256);
        HIPC(hipMemsetAsync(fb.ucnt.p, 0, 4ull * (nc + 1), xs));
        // first-hit order: by ~tgt, then (stably) by (unit, diag_bgn)
        hipLaunchKernelGGL(k_olim_keys, grid, blk, 0, xs, ext_pairs, ext_pnodes, npairs, (int32_t)k,
                           fb.okey.p, fb.ok64a.p, fb.oa.p, fb.dkey.p, fb.ucnt.p);
        HIPC(hipGetLastError());
        HIPC(hipcub::DeviceScan::ExclusiveSum(fb.otmp.p, t3, fb.ucnt.p, fb.useg.p, (int)nc + 1, xs));
        size_t tt = t1;
        HIPC(hipcub::DeviceRadixSort::SortPairs(fb.otmp.p, tt, fb.okey.p, fb.okey2.p, fb.oa.p,
                                                fb.ob.p, n, 0, 32, xs));
        hipLaunchKernelGGL(k_gather_u64, grid, blk, 0, xs, fb.ok64a.p, fb.ob.p, npairs, fb.ok64b.p);
        tt = t2;
        HIPC(hipcub::DeviceRadixSort::SortPairs(fb.otmp.p, tt, fb.ok64b.p, fb.ok64a.p, fb.ob.p,
                                                fb.oa.p, n, 0, 64, xs));
        // String_Olap_Space indices, then the order by (unit, index)
        hipLaunchKernelGGL(k_olim_slots, dim3(std::min<uint32_t>((nc + 3) / 4, 8192)), blk, 0, xs,
                           ext_pairs, fb.oa.p, fb.useg.p, nc,
                           c->first_iid - c->hash_bgn_iid, fb.ok64b.p, fb.ob.p);
        HIPC(hipGetLastError());
        tt = t2;
        HIPC(hipcub::DeviceRadixSort::SortPairs(fb.otmp.p, tt, fb.ok64b.p, fb.ok64a.p, fb.ob.p,
                                                fb.oidx.p, n, 0, 64, xs));       // oidx: ord_slot
        // By_Diag_Sum: stably by the diagonal key, then stably by unit
        hipLaunchKernelGGL(k_gather_u64, grid, blk, 0, xs, fb.dkey.p, fb.oidx.p, npairs, fb.ok64a.p);
        tt = t2;
        HIPC(hipcub::DeviceRadixSort::SortPairs(fb.otmp.p, tt, fb.ok64a.p, fb.ok64b.p, fb.oidx.p,
                                                fb.oa.p, n, 0, 64, xs));
        hipLaunchKernelGGL(k_gather_unit, grid, blk, 0, xs, ext_pairs, fb.oa.p, npairs, fb.okey.p);
        tt = t1;
        HIPC(hipcub::DeviceRadixSort::SortPairs(fb.otmp.p, tt, fb.okey.p, fb.okey2.p, fb.oa.p,
                                                fb.oidx2.p, n, 0, 32, xs));      // oidx2: ord_diag
        HIPC(hipGetLastError());
        EA.useg = fb.useg.p;
        EA.ord_slot = fb.oidx.p;
        EA.ord_diag = fb.oidx2.p;
        EA.dkey = fb.dkey.p;
      }
      if (npairs && !ordered) {
        // the extension-only buffers are shared by the slots: regrowing one waits for xs
        auto &fb = c->fb;
        size_t tmp = 0;
        HIPC(hipcub::DeviceRadixSort::SortPairsDescending(nullptr, tmp, fb.okey.p, fb.okey2.p,
                                                          fb.oidx.p, fb.oidx2.p, (int)npairs, 0,
                                                          32, xs));
        if (fb.okey.n < npairs || fb.oidx.n < npairs || fb.okey2.n < npairs || fb.oidx2.n < npairs ||
            d_defer.n < npairs || fb.defer2.n < npairs || fb.otmp.n < tmp || !fb.otmp.p) {
          HIPC(hipStreamSynchronize(xs));
          if (fb.okey.grow(npairs) || fb.oidx.grow(npairs) || fb.okey2.grow(npairs) ||
              fb.oidx2.grow(npairs) || d_defer.grow(npairs) || fb.defer2.grow(npairs) ||
              fb.otmp.grow(std::max<size_t>(tmp, 1)))
            return fail(OVL_ERR_OOM, "work order");
        }
        if (npairs > 1) {
          // longest-first work order (node count descending; ties keep pair order)
          hipLaunchKernelGGL(k_pair_order_keys, dim3(std::min<uint32_t>((npairs + 255) / 256, 4096)),
                             dim3(256), 0, xs, ext_pairs, npairs, fb.okey.p, fb.oidx.p);
          HIPC(hipGetLastError());
          HIPC(hipcub::DeviceRadixSort::SortPairsDescending(fb.otmp.p, tmp, fb.okey.p, fb.okey2.p,
                                                            fb.oidx.p, fb.oidx2.p, (int)npairs, 0,
                                                            32, xs));
          EA.list = fb.oidx2.p;
        }
      }
      HIPC(hipEventRecord(c->xev[slot], xs));
      if (npairs && ordered) {
        EA.e_cap = gen.ecap;
        EA.rows_cap = gen.stride;
        EA.sw_words = 0;
        EA.pair_next = x_ctr.p + 9;
        n_ext_launch++;
        if (gen.l16)
          hipLaunchKernelGGL((k_extend<false, true, true>), dim3(gen.waves / gen.wpb),
                             dim3(64 * gen.wpb), gen.lds, xs, EA);
        else
          hipLaunchKernelGGL((k_extend<false, false, true>), dim3(gen.waves / gen.wpb),
                             dim3(64 * gen.wpb), gen.lds, xs, EA);
        HIPC(hipGetLastError());
      } else if (npairs) {
        // the staged classes in turn, each deferring what it cannot take to the next list
        // (whose length the next launch reads from the device counter); the generic kernel
        // takes the last list, or every pair when no class exists
        uint32_t *defer_buf[2] = {d_defer.p, c->fb.defer2.p};
        for (size_t ci = 0; ci < ext_stage.size(); ci++) {
          const ExtClass &g = ext_stage[ci];
          EA.e_cap = g.ecap;
          EA.rows_cap = g.stride;
          EA.sw_words = g.sw;
          EA.pair_next = x_ctr.p + ctr_next[ci];
          EA.defer = defer_buf[ci & 1];
          EA.ndefer = x_ctr.p + ctr_defer[ci];
          // without the pipeline, a later class whose input list is empty is not launched
          // (the host reads the previous class's defer count, as for the generic kernel
          // below): the bench job's one staged launch then is the extension's only launch
          bool launch = true;
          if (!pipe && ci > 0) {
            uint32_t nd = 0;
            HIPC(hipMemcpyAsync(&nd, x_ctr.p + ctr_defer[ci - 1], 4, hipMemcpyDeviceToHost, xs));
            HIPC(hipStreamSynchronize(xs));
            launch = nd > 0;
          }
          if (!launch) {
            // an empty class defers nothing: its counter stays 0 for the next one
          } else {
          n_ext_launch++;
          if (g.wide && g.l16)
            hipLaunchKernelGGL((k_extend<true, true, false, 2 * OVL_RJ>), dim3(g.waves / g.wpb),
                               dim3(64 * g.wpb), g.lds, xs, EA);
          else if (g.wide)
            hipLaunchKernelGGL((k_extend<true, false, false, 2 * OVL_RJ>), dim3(g.waves / g.wpb),
                               dim3(64 * g.wpb), g.lds, xs, EA);
          else if (g.l16)
            hipLaunchKernelGGL((k_extend<true, true>), dim3(g.waves / g.wpb), dim3(64 * g.wpb), g.lds, xs, EA);
          else
            hipLaunchKernelGGL((k_extend<true, false>), dim3(g.waves / g.wpb), dim3(64 * g.wpb), g.lds, xs, EA);
          HIPC(hipGetLastError());
          }
          EA.list = defer_buf[ci & 1];
          EA.npairs_dev = x_ctr.p + ctr_defer[ci];
          EA.restore = 1;          // a deferred pair may have had nodes removed (~Len)
        }
        EA.e_cap = gen.ecap;
        EA.rows_cap = gen.stride;
        EA.sw_words = 0;
        EA.pair_next = x_ctr.p + 9;
        EA.defer = nullptr;
        EA.ndefer = nullptr;
        // without the pipeline the host waits for this chunk next anyway: read the last
        // class's defer count and skip an empty generic launch
        bool gen_needed = true;
        if (!pipe && !ext_stage.empty()) {
          uint32_t nd = 0;
          HIPC(hipMemcpyAsync(&nd, x_ctr.p + ctr_defer[ext_stage.size() - 1], 4,
                              hipMemcpyDeviceToHost, xs));
          HIPC(hipStreamSynchronize(xs));
          gen_needed = nd > 0;
        }
        if (gen_needed) {
          n_ext_launch++;
          if (gen.l16)
            hipLaunchKernelGGL((k_extend<false, true>), dim3(gen.waves / gen.wpb), dim3(64 * gen.wpb),
                               gen.lds, xs, EA);
          else
            hipLaunchKernelGGL((k_extend<false, false>), dim3(gen.waves / gen.wpb), dim3(64 * gen.wpb),
                               gen.lds, xs, EA);
          HIPC(hipGetLastError());
        }
      }
    HIPC(hipEventRecord(c->xev[2 + slot], xs));
    pending[slot] = true;
    return OVL_OK;
  };
  // Extend everything the accumulator holds; it is empty again for the next chunk (the
  // stream orders the next appends after this launch's reads).
  auto flush_acc = [&]() -> int {
    if (int rc = collect(0)) return rc;
    auto &A = c->acc;
    const uint32_t np = (uint32_t)A.np;
    slot_pairs[0] = np;
    int rc = launch_ext(0, A.units.p, A.pairs.p, A.pnodes.p, np, (uint32_t)A.nu);
    A.nu = A.nn = A.np = 0;
    return rc;
  };
  // Append a chunk's units, list nodes and pairs to the accumulator (device copies on s,
  // which the extension also runs on without OVL_PIPELINE: nothing is overwritten early).
  const uint64_t ACC_PAIRS = 4ull << 20, ACC_NODES = 1ull << 30;
  auto acc_append = [&](const Unit *u, uint32_t nu_c, const Node *nodes, uint64_t nn_c,
                        const PairRec *pairs, uint32_t np_c) -> int {
    auto &A = c->acc;
    if (A.nu + nu_c >= 0xFFFFFFF0ull || A.nn + nn_c >= 0xFFFFFFF0ull)
      return fail(OVL_ERR_UNSUPPORTED, "extension accumulator past 2^32 entries");
    auto acc_fits = [&]() {
      return A.units.n >= A.nu + nu_c && A.pnodes.n >= A.nn + nn_c && A.pairs.n >= A.np + np_c;
    };
    // once it holds a launch's worth (a quarter of the flush thresholds), what the
    // accumulator holds is extended rather than moved into bigger buffers: a regrow on a full
    // device costs ~1 s (the full-size configs[4] job, r05e), while smaller launches lose to
    // their tails (one launch per search: extension 8.4 -> 23 s, r05f)
    if (!acc_fits() && (A.np >= ACC_PAIRS / 4 || A.nn >= ACC_NODES / 4))
      if (int rc = flush_acc()) return rc;
    if (!acc_fits()) {
      // growing moves the buffers: the pending extension (which reads them) must be done,
      // and what the accumulator holds is carried over
      HIPC(hipStreamSynchronize(xs));
      HIPC(hipStreamSynchronize(s));
      auto regrow = [&](auto &buf, uint64_t used, uint64_t need) -> int {
        if (buf.n >= need && buf.p) return OVL_OK;
        typename std::remove_reference<decltype(buf)>::type bigger;
        if (bigger.alloc(std::max<uint64_t>(need, buf.n + buf.n / 2))) return -1;
        if (used) HIPC(hipMemcpy(bigger.p, buf.p, used * sizeof(*buf.p), hipMemcpyDeviceToDevice));
        std::swap(bigger.p, buf.p);
        std::swap(bigger.n, buf.n);
        return OVL_OK;
      };
      if (regrow(A.units, A.nu, A.nu + nu_c) || regrow(A.pnodes, A.nn, A.nn + nn_c) ||
          regrow(A.pairs, A.np, A.np + np_c)) {
        // no room for bigger buffers beside the ones being copied (a device nearly full of
        // sorted windows, index and search buffers): what the accumulator holds is extended
        // now, and the emptied buffers are freed before this chunk's own are allocated
        if (A.nu || A.nn || A.np) {
          if (int rc = flush_acc()) return rc;
          HIPC(hipStreamSynchronize(xs));
          HIPC(hipStreamSynchronize(s));
        }
        if ((A.units.n < nu_c && A.units.alloc(nu_c)) ||
            (A.pnodes.n < nn_c && A.pnodes.alloc(nn_c)) || (A.pairs.n < np_c && A.pairs.alloc(np_c)))
          return fail(OVL_ERR_OOM, "extension accumulator (%llu nodes)", (unsigned long long)nn_c);
      }
    }
    if (nu_c)
      HIPC(hipMemcpyAsync(A.units.p + A.nu, u, sizeof(Unit) * nu_c, hipMemcpyDeviceToDevice, s));
    if (nn_c)
      HIPC(hipMemcpyAsync(A.pnodes.p + A.nn, nodes, sizeof(Node) * nn_c, hipMemcpyDeviceToDevice, s));
    if (np_c) {
      hipLaunchKernelGGL(k_append_pairs, dim3(std::min<uint32_t>((np_c + 255) / 256, 4096)),
                         dim3(256), 0, s, pairs, np_c, (uint32_t)A.nu, (uint32_t)A.nn,
                         A.pairs.p + A.np);
      HIPC(hipGetLastError());
    }
    A.nu += nu_c;
    A.nn += nn_c;
    A.np += np_c;
    return OVL_OK;
  };
  const bool bloom = nu > 0 && use_bloom(c, bgn, end);
  uint64_t chunk = 0;
  while (u0 < nu) {
    const int slot = pipe ? (int)(chunk & 1) : 0;
    // this slot's buffers are free once the extension of chunk i-2 has finished
    if (int rc = collect(slot)) return rc;
    auto &d_units = c->fb.units[slot];
    auto &d_pnodes = c->fb.pnodes[slot];
    auto &d_pairs = c->fb.pairs[slot];
    uint32_t nb = 0;
    std::vector<uint64_t> rbase;
    std::vector<uint32_t> uh;
    uint32_t *chain_uflags = nullptr;
    if (sqm) {
      // the run of sorted windows holding unit u0: probed once per batch (k_probe_sorted),
      // its records then chained in hit-budget chunks
      auto &Q = c->sq;
      while (Q.runs[sq_run].u1 <= u0) sq_run++;
      const auto &R = Q.runs[sq_run];
      const uint32_t ue = std::min<uint32_t>(R.u1, nu);
      if (Q.probed != (int)sq_run) {
        const uint64_t wlim = Q.wb[R.wb0 + (ue - R.u0)];
        if (d_probe.grow(R.n)) return fail(OVL_ERR_OOM, "probe records (%llu)", (unsigned long long)R.n);
        HIPC(hipEventRecord(c->ev[4], s));           // the probe step: seed-phase time
        HIPC(hipMemsetAsync(d_probe.p, 0, 8ull * wlim, s));
        HIPC(hipMemsetAsync(Q.uflags.p + R.u0, 0, 4ull * (ue - R.u0), s));
        HIPC(hipMemsetAsync(Q.uhits.p + R.u0, 0, 4ull * (ue - R.u0), s));
        SqProbeArgs SA;
        SA.X = index_dev(c);
        if (c->bloom_ok && sq_bloom()) {        // the filter in front of the table
          SA.X.bloom = c->d_bloom.p;
          SA.X.bloom_w = c->bloom_w;
        }
        SA.R = c->reads();
        SA.key = Q.key.p + R.e0;
        SA.wid = Q.wid.p + R.e0;
        SA.n = R.n;
        SA.wlim = (uint32_t)wlim;
        SA.units = Q.dunits.p + R.u0;
        SA.wbase = Q.dwbase.p + R.wb0;
        SA.ublk = Q.ublk.p + R.ub0;
        SA.k = k;
        SA.out = d_probe.p;
        SA.unit_flags = Q.uflags.p + R.u0;
        SA.unit_hits = Q.uhits.p + R.u0;
        // the kernel alone is timed (the records' zeroing and the unit hit counts around it
        // are not the probe's bytes)
        HIPC(hipEventRecord(c->ev[2], s));
        hipLaunchKernelGGL(k_probe_sorted, dim3(8 * c->n_cu), dim3(256), 0, s, SA);
        HIPC(hipEventRecord(c->ev[3], s));
        n_probe_launch++;
        n_probe_sorted++;
        HIPC(hipGetLastError());
        HIPC(hipEventRecord(c->ev[5], s));
        sq_uh.resize(ue - R.u0);
        HIPC(hipMemcpyAsync(sq_uh.data(), Q.uhits.p + R.u0, 4ull * (ue - R.u0),
                            hipMemcpyDeviceToHost, s));
        HIPC(hipStreamSynchronize(s));
        float t = 0, tstep = 0;
        (void)hipEventElapsedTime(&t, c->ev[2], c->ev[3]);
        (void)hipEventElapsedTime(&tstep, c->ev[4], c->ev[5]);
        ms_probe += t;
        ms_probe_rest += tstep > t ? tstep - t : 0.f;  // the records' zeroing
        // algorithmic bytes: the sorted windows (8-B key + 4-B id), and the table and its
        // filter read once each -- or, when they are larger than the run (a full-size
        // configs[4] super-batch's 68.7 GB table against a run of 2^29 windows), at most one
        // entry and one filter word per window (the hits' 8-B records are not counted)
        const uint64_t tab_b = 16ull << c->tab_bits;
        const uint64_t flt_b = SA.X.bloom ? 8ull * ((1ull << (c->tab_bits - c->slice_bits)) << c->bloom_w) : 0ull;
        probe_bytes += 12ull * R.n + std::min<uint64_t>(tab_b, 16ull * R.n) +
                       std::min<uint64_t>(flt_b, 8ull * R.n);
        Q.probed = (int)sq_run;
      }
      nb = ue - u0;
      rbase.assign(Q.wb.begin() + R.wb0 + (u0 - R.u0), Q.wb.begin() + R.wb0 + (ue - R.u0) + 1);
      uh.assign(sq_uh.begin() + (u0 - R.u0), sq_uh.begin() + (ue - R.u0));
      chain_uflags = Q.uflags.p + u0;
      if (d_units.grow(nb) || d_rbase.grow(nb + 1))
        return fail(OVL_ERR_OOM, "unit buffers");
      HIPC(hipMemcpyAsync(d_units.p, units.data() + u0, sizeof(Unit) * nb, hipMemcpyHostToDevice, s));
      HIPC(hipMemcpyAsync(d_rbase.p, rbase.data(), 8ull * (nb + 1), hipMemcpyHostToDevice, s));
    } else {
    // batch by probe slots
    uint32_t u1 = u0;
    uint64_t wsum = 0;
    while (u1 < nu && (wsum + uwin[u1] <= WIN_BUDGET || u1 == u0)) wsum += uwin[u1++];
    nb = u1 - u0;
    rbase.resize(nb + 1);
    uint64_t acc = 0;
    for (uint32_t i = 0; i < nb; i++) { rbase[i] = acc; acc += uwin[u0 + i]; }
    rbase[nb] = acc;
    if (d_units.grow(nb) || d_rbase.grow(nb + 1) || d_probe.grow(acc) ||
        d_uhits.grow(nb) || d_uflags.grow(nb)) {
      if (nb == 1 || WIN_BUDGET <= (16ull << 20)) return fail(OVL_ERR_OOM, "probe buffers");
      win_cap = WIN_BUDGET = WIN_BUDGET / 2;
      continue;
    }
    HIPC(hipMemcpyAsync(d_units.p, units.data() + u0, sizeof(Unit) * nb, hipMemcpyHostToDevice, s));
    HIPC(hipMemcpyAsync(d_rbase.p, rbase.data(), 8ull * (nb + 1), hipMemcpyHostToDevice, s));
    ProbeArgs PA;
    PA.R = c->reads();
    PA.X = index_dev(c);
    if (bloom) {
      PA.X.bloom = c->d_bloom.p;
      PA.X.bloom_w = c->bloom_w;
    }
    PA.units = d_units.p;
    PA.rbase = d_rbase.p;
    PA.nunits = nb;
    PA.out = d_probe.p;
    PA.unit_hits = d_uhits.p;
    PA.unit_flags = d_uflags.p;
    PA.k = k;
    HIPC(hipEventRecord(c->ev[2], s));
    if (bloom) hipLaunchKernelGGL(k_probe<true>, dim3((nb + 3) / 4), dim3(256), 0, s, PA);
    else       hipLaunchKernelGGL(k_probe<false>, dim3((nb + 3) / 4), dim3(256), 0, s, PA);
    n_probe_launch++;
    HIPC(hipGetLastError());
    HIPC(hipEventRecord(c->ev[3], s));
    uh.resize(nb);
    HIPC(hipMemcpyAsync(uh.data(), d_uhits.p, 4ull * nb, hipMemcpyDeviceToHost, s));
    HIPC(hipStreamSynchronize(s));
    float t = 0;
    (void)hipEventElapsedTime(&t, c->ev[2], c->ev[3]);
    ms_probe += t;
    if (getenv("OVL_TIMING"))
      fprintf(stderr, "OVL_TIMING probe launch: %u units, %llu windows, %.3f ms\n", nb,
              (unsigned long long)acc, t);
    // algorithmic bytes: per window one 16-B table entry and one 8-B Probe record, plus the
    // packed query (2 bits per base); see DESIGN.md
    probe_bytes += acc * 24 + acc / 4;
    chain_uflags = d_uflags.p;
    }
    // shrink the batch to the hit budget (probe results stay valid for the prefix)
    uint64_t hsum = 0;
    uint32_t nc = 0;
    auto fit_hits = [&]() {
      hsum = 0;
      nc = 0;
      while (nc < nb && (hsum + uh[nc] <= HIT_BUDGET || nc == 0)) hsum += uh[nc++];
      double ratio = (double)hsum / (double)std::max<uint64_t>(1, rbase[nc]);
      double wb = (double)HIT_BUDGET / std::max(ratio, 1e-3) * 1.05;
      WIN_BUDGET = (uint64_t)std::min(std::max(wb, 16.0 * (1 << 20)), (double)win_cap);
    };
    fit_hits();

    // Chaining.  The first launch chains every unit whose targets fit one pass of the
    // 128-target table and lists the others; the second chains the listed units over
    // several passes with a done set sized for their targets.  Capacities come from the
    // probe's hit counts; a batch that still overflows one (the counters say by how much)
    // is chained again with bigger buffers -- never dropped.
    uint64_t per_unit = 256;                           // test knob: force the regrow path
    if (const char *e = getenv("OVL_TEST_PAIRS_PER_UNIT")) per_unit = std::max(1, atoi(e));
    uint64_t pool_cap = 0, pairs_cap = 0, pnodes_cap = 0;
    // nodes <= hits; a wave claims OVL_NODE_BLOCK nodes at a time for at most 64 lanes per
    // claim, so a block wastes < 64 / 4096 of itself, and each wave ends holding one block
    auto pool_for = [&](uint64_t h) {
      return h + h / 32 + (uint64_t)(chain_waves + 2) * OVL_NODE_BLOCK + 8;
    };
    auto set_caps = [&]() {
      pool_cap = pool_for(hsum);
      pairs_cap = std::min<uint64_t>(hsum + 1, (uint64_t)nc * per_unit + 1024);
      pnodes_cap = hsum + 1;
    };
    set_caps();
    // only units with hits are chained: a unit without one adds no pair, node, counter or
    // flag, yet its wave would read every window's record (a full-size configs[4] search
    // against a super-batch of ~2 % of the reads: about half its units)
    std::vector<uint32_t> live;
    live.reserve(nc);
    for (uint32_t i = 0; i < nc; i++)
      if (uh[i]) live.push_back(i);
    const bool all_live = live.size() == nc;
    if (!all_live && !live.empty()) {
      if (c->fb.live.grow(live.size())) return fail(OVL_ERR_OOM, "unit list");
      HIPC(hipMemcpyAsync(c->fb.live.p, live.data(), 4ull * live.size(), hipMemcpyHostToDevice, s));
    }
    const uint32_t hash_reads = c->hash_end_iid - c->hash_bgn_iid + 1;
    uint32_t hc[16];
    unsigned long long chain_hits = 0;
    for (int attempt = 0;; attempt++) {
      if (pool_cap >= 0xFFFFFFF0ull || pairs_cap >= 0xFFFFFFF0ull || pnodes_cap >= 0xFFFFFFF0ull)
        return fail(OVL_ERR_UNSUPPORTED, "chain buffers past 2^32 entries (%llu hits)",
                    (unsigned long long)hsum);
      // sized for the hit budget, not this batch's hits: the next batch reuses them as they are
      if (d_pool.grow(std::max(pool_cap, pool_for(HIT_BUDGET))) ||
          d_pnodes.grow(std::max<uint64_t>(pnodes_cap, HIT_BUDGET + 1)) || d_pairs.grow(pairs_cap) ||
          c->fb.big.grow(nc) || c->fb.chits.grow(1)) {
        if (nc == 1 || hsum <= (16ull << 20))
          return fail(OVL_ERR_OOM, "chain buffers (%llu hits)", (unsigned long long)hsum);
        HIT_BUDGET = hsum / 2;                         // fewer units per chain launch
        // the buffers that did fit were sized for the larger budget: drop them too
        d_pool.release();
        d_pnodes.release();
        d_pairs.release();
        fit_hits();
        set_caps();
        attempt--;
        continue;
      }
      uint32_t ctr_init[16] = {0};
      ctr_init[1] = 1;                                 // pool_next: node 0 is null
      HIPC(hipMemcpyAsync(d_ctr.p, ctr_init, 64, hipMemcpyHostToDevice, s));
      HIPC(hipMemsetAsync(c->fb.chits.p, 0, 8, s));
      ChainArgs CA;
      CA.R = c->reads();
      CA.occ = c->d_occ.p;
      CA.units = d_units.p;
      CA.rbase = d_rbase.p;
      CA.probes = d_probe.p;
      CA.unit_flags = chain_uflags;
      CA.nunits = all_live ? nc : (uint32_t)live.size();
      CA.k = k;
      CA.unit_next = d_ctr.p + 0;
      CA.pool = d_pool.p;
      CA.pool_next = d_ctr.p + 1;
      CA.pool_cap = (uint32_t)pool_cap;
      CA.pnodes = d_pnodes.p;
      CA.pnodes_next = d_ctr.p + 2;
      CA.pnodes_cap = (uint32_t)pnodes_cap;
      CA.pairs = d_pairs.p;
      CA.npairs = d_ctr.p + 3;
      CA.pairs_cap = (uint32_t)pairs_cap;
      CA.overflow = d_ctr.p + 4;
      CA.unit_list = all_live ? nullptr : c->fb.live.p;
      CA.big_units = c->fb.big.p;
      CA.n_big = d_ctr.p + 10;
      CA.done_slots = nullptr;
      CA.done_set = nullptr;
      CA.done_cap = 0;
      CA.set_mask = 0;
      CA.seed_hits = c->fb.chits.p;
      CA.prof = nullptr;
#ifdef OVL_CHAIN_PROF
      if (!c->dbg.p) {
        if (c->dbg.alloc(32)) return fail(OVL_ERR_OOM, "debug counters");
        HIPC(hipMemsetAsync(c->dbg.p, 0, 256, s));
      }
      CA.prof = c->dbg.p + 24;
#endif
      HIPC(hipEventRecord(c->ev[4], s));
      hipLaunchKernelGGL(k_chain, dim3(chain_waves / 4), dim3(256), 0, s, CA);
      HIPC(hipGetLastError());
      HIPC(hipMemcpyAsync(hc, d_ctr.p, 64, hipMemcpyDeviceToHost, s));
      HIPC(hipStreamSynchronize(s));
      const uint32_t n_big = hc[10];
      if (n_big && !hc[4]) {
        std::vector<uint32_t> big(n_big);
        HIPC(hipMemcpy(big.data(), c->fb.big.p, 4ull * n_big, hipMemcpyDeviceToHost));
        uint32_t cap = 1;                              // distinct targets of any listed unit
        for (uint32_t b : big) cap = std::max<uint32_t>(cap, std::min<uint32_t>(uh[b], hash_reads));
        uint32_t smask = 1;
        while (smask + 1 < 2ull * cap) smask = 2 * smask + 1;
        uint32_t w2 = std::min<uint32_t>(chain_waves, (n_big + 3) & ~3u);
        while (w2 > 4 && (uint64_t)w2 * (cap + smask + 1) * 4 > (4ull << 30)) w2 = (w2 / 2 + 3) & ~3u;
        if (c->fb.done.grow((size_t)w2 * cap) || c->fb.dset.grow((size_t)w2 * (smask + 1)))
          return fail(OVL_ERR_OOM, "done sets (%u targets x %u waves)", cap, w2);
        HIPC(hipMemsetAsync(c->fb.dset.p, 0, 4ull * w2 * (smask + 1), s));
        HIPC(hipMemsetAsync(d_ctr.p, 0, 4, s));      // unit_next
        CA.unit_list = c->fb.big.p;
        CA.nunits = n_big;
        CA.big_units = nullptr;
        CA.n_big = nullptr;
        CA.done_slots = c->fb.done.p;
        CA.done_set = c->fb.dset.p;
        CA.done_cap = cap;
        CA.set_mask = smask;
        hipLaunchKernelGGL(k_chain, dim3(w2 / 4), dim3(256), 0, s, CA);
        HIPC(hipGetLastError());
        HIPC(hipMemcpyAsync(hc, d_ctr.p, 64, hipMemcpyDeviceToHost, s));
        HIPC(hipStreamSynchronize(s));
        n_big_units += n_big;
      }
      HIPC(hipEventRecord(c->ev[5], s));
      HIPC(hipStreamSynchronize(s));
      if (!hc[4]) break;
      if ((hc[4] & 4u) || attempt >= 3)
        return fail(OVL_ERR_HIP, "chain capacity still exceeded after %d attempts (flags %u)",
                    attempt + 1, hc[4]);
      // grow what overflowed from what the counters asked for, then chain the batch again
      if (hc[4] & 1u) pool_cap = (uint64_t)hc[1] + (uint64_t)(chain_waves + 2) * OVL_NODE_BLOCK;
      if (hc[4] & 2u) {
        pairs_cap = std::max<uint64_t>(pairs_cap, (uint64_t)hc[3] + 1024);
        pnodes_cap = std::max<uint64_t>(pnodes_cap, (uint64_t)hc[2] + 1024);
      }
      chain_retries++;
    }
    {
      float t = 0;
      (void)hipEventElapsedTime(&t, c->ev[4], c->ev[5]);
      ms_chain += t;
    }
    {
      unsigned long long h = 0;
      HIPC(hipMemcpy(&h, c->fb.chits.p, 8, hipMemcpyDeviceToHost));
      chain_hits += h;
      seed_hits_tot += chain_hits;
    }
    uint32_t npairs = hc[3];
    npairs_tot += npairs;
    nodes_tot += hc[2];                                  // pnodes_next: the lists' nodes

    // ---- the extension ----------------------------------------------------------------
    // Default path: the chunk's chains go to the accumulator (c->acc) and are extended
    // together once ACC_PAIRS pairs have gathered or the job ends, so a launch's tail (its
    // last, longest pairs on few waves) is paid once per job rather than once per probe
    // chunk and per hash batch (canu's small --hashbits batches made that tail most of a
    // configs[4] rank's extension time).  -l (a unit's pairs in the reference's order) and
    // OVL_PIPELINE extend each chunk as it comes, from the slot's own buffers.
    if (!ordered && !pipe) {
      if (int rc = acc_append(d_units.p, nc, d_pnodes.p, hc[2], d_pairs.p, npairs)) return rc;
      if (c->acc.np >= ACC_PAIRS || c->acc.nn >= ACC_NODES)
        if (int rc = flush_acc()) return rc;
    } else {
      if (int rc = launch_ext(slot, d_units.p, d_pairs.p, d_pnodes.p, npairs, nc)) return rc;
    }
    chunk++;
    u0 += nc;
  }
  if (flush && c->acc.np)
    if (int rc = flush_acc()) return rc;
  for (int sl = 0; sl < 2; sl++)
    if (int rc = collect(sl)) return rc;
  {
    uint32_t n = 0;
    HIPC(hipMemcpy(&n, c->fb.xnout.p, 4, hipMemcpyDeviceToHost));
    c->nout = n;
  }
  unsigned long long hs[16];
  HIPC(hipMemcpy(hs, d_stats.p, 128, hipMemcpyDeviceToHost));
#ifdef OVL_CHAIN_PROF
  if (c->dbg.p) {
    unsigned long long cp[8];
    (void)hipMemcpy(cp, c->dbg.p + 24, 64, hipMemcpyDeviceToHost);
    const double tot = (double)(cp[0] + cp[1] + cp[2] + cp[3] + cp[4] + cp[5]) + 1e-9;
    fprintf(stderr, "OVL_CHAIN_PROF wave-cycles (cumulative): probe+qualify %.3f stage %.3f "
            "discover %.3f scatter %.3f replay %.3f emit %.3f (shares); %llu chunks, %llu "
            "staged occurrences, %.0f cycles per chunk\n", cp[0] / tot, cp[1] / tot,
            cp[2] / tot, cp[3] / tot, cp[4] / tot, cp[5] / tot, cp[6], cp[7],
            tot / (double)(cp[6] ? cp[6] : 1));
  }
#endif
  if (c->dbg.p) {
    unsigned long long dd[32];
    (void)hipMemcpy(dd, c->dbg.p, 256, hipMemcpyDeviceToHost);
    fprintf(stderr, "OVL_DEBUG cyc_A=%llu cyc_B=%llu cyc_cont=%llu cyc_C=%llu cyc_argmax=%llu "
            "cyc_remove=%llu nodes=%llu\n", dd[16], dd[17], dd[18], dd[19], dd[20], dd[21],
            dd[22]);
    fprintf(stderr, "OVL_DEBUG ped=%llu rows=%llu chunks=%llu slide_iters=%llu tb=%llu iters=%llu "
            "cyc_chunks=%llu cyc_tb=%llu pairs=%llu maxrows=%llu cyc_rest=%llu cyc_ped=%llu "
            "cyc_calls=%llu cyc_pair=%llu cyc_stage=%llu cyc_extend=%llu\n",
            dd[0], dd[1], dd[2], dd[3], dd[4], dd[5], dd[6], dd[7], dd[8], dd[9], dd[10], dd[11],
            dd[12], dd[13], dd[14], dd[15]);
  }
  // counters add up over the driver's hash batches (the reference sums its per-thread
  // counters into globals, Process_Overlaps.C:156-163)
  c->stats.kmer_hits_without_olap += hs[0];
  c->stats.kmer_hits_with_olap += hs[1];
  c->stats.kmer_hits_skipped += hs[2];
  c->stats.multi_overlaps += hs[3];
  c->stats.total_overlaps += hs[4];
  c->stats.contained_overlaps += hs[5];
  c->stats.dovetail_overlaps += hs[6];
  c->stats.seed_hits += seed_hits_tot;
  c->stats.multi_pass_units += n_big_units;
  c->stats.chain_retries += chain_retries;
  c->stats.staged_pairs += staged_pairs;
  c->stats.long_pairs += long_pairs;
  c->stats.generic_pairs += generic_pairs;
  c->stats.ext_waves = c->stats_ext_waves;
  c->stats.generic_waves = c->stats_gen_waves;
  c->stats.stage_len = c->ext_classes.empty() ? 0 : c->ext_classes[0];
  c->stats.long_stage_len = c->ext_classes.size() > 1 ? c->ext_classes.back() : 0;
  c->stats.bad_short_window += hs[8];
  c->stats.bad_long_window += hs[9];
  c->stats.pairs += npairs_tot;
  c->stats.seed_nodes += nodes_tot;
  c->stats.ms_seed += ms_probe + ms_probe_rest + ms_chain;
  c->stats.ms_extend += ms_ext;
  c->stats.ms_probe_kernel += ms_probe;
  c->stats.probe_bytes += probe_bytes;
  c->stats.probe_launches += n_probe_launch;
  c->stats.probe_sorted_launches += n_probe_sorted;
  c->stats.extend_launches += n_ext_launch;
  *n_out = c->nout;
  return OVL_OK;
}

int ovl_seed_hits(ovl_ctx *c, uint32_t bgn, uint32_t end, ovl_seed_hit *out, uint64_t max_hits,
                  uint64_t *n_hits) {
  if (!c || !n_hits) return fail(OVL_ERR_STATE, "null argument");
  if (!c->have_index) return fail(OVL_ERR_STATE, "ovl_build_hash_index() first");
  HIPC(hipSetDevice(c->device));
  hipStream_t s = c->stream;
  const uint32_t k = c->P.kmer_len;
  if (bgn < 1) bgn = 1;
  if (bgn < c->first_iid) bgn = c->first_iid;
  uint32_t last = c->first_iid + c->nreads - 1;
  if (end > last) end = last;
  std::vector<Unit> units;
  std::vector<uint64_t> uwin;
  for (uint32_t a = bgn; a <= end && a >= bgn; a++) {
    uint32_t r = a - c->first_iid;
    int32_t L = (int32_t)c->h_len[r];
    if (L < c->P.min_olap_len || L < (int32_t)k) continue;
    units.push_back(Unit{r, 0});
    units.push_back(Unit{r, 1});
    uwin.push_back((uint64_t)(L - (int32_t)k + 1));
    uwin.push_back((uint64_t)(L - (int32_t)k + 1));
  }
  // units in batches of <= 512 M probe slots; each batch's hits are written to a device
  // buffer of at most 256 M hits (4 GB), in pieces of whole units
  const uint64_t WIN_BUDGET = 512ull << 20, HIT_BUF = 256ull << 20;
  auto &fb = c->fb;
  // kept in the context (grow-only): a repeated call allocates nothing
  DBuf<uint64_t> &ucnt = fb.hcnt, &ubase = fb.hbase;
  DBuf<uint4> &hbuf = fb.hbuf;
  uint64_t total = 0, copied = 0;
  float ms_tot = 0;
  const uint32_t nu = (uint32_t)units.size();
  for (uint32_t u0 = 0; u0 < nu;) {
    uint32_t u1 = u0;
    uint64_t acc = 0;
    while (u1 < nu && (acc + uwin[u1] <= WIN_BUDGET || u1 == u0)) acc += uwin[u1++];
    const uint32_t nb = u1 - u0;
    std::vector<uint64_t> rbase(nb + 1);
    acc = 0;
    for (uint32_t i = 0; i < nb; i++) { rbase[i] = acc; acc += uwin[u0 + i]; }
    rbase[nb] = acc;
    if (fb.units[0].grow(nb) || fb.rbase.grow(nb + 1) || fb.probe.grow(acc) ||
        fb.uhits.grow(nb) || fb.uflags.grow(nb) || ucnt.grow(nb) || ubase.grow(nb))
      return fail(OVL_ERR_OOM, "seed-hit buffers");
    HIPC(hipMemcpyAsync(fb.units[0].p, units.data() + u0, sizeof(Unit) * nb, hipMemcpyHostToDevice, s));
    HIPC(hipMemcpyAsync(fb.rbase.p, rbase.data(), 8ull * (nb + 1), hipMemcpyHostToDevice, s));
    HIPC(hipEventRecord(c->ev[2], s));
    ProbeArgs PA;
    PA.R = c->reads();
    PA.X = index_dev(c);
    PA.units = fb.units[0].p;
    PA.rbase = fb.rbase.p;
    PA.nunits = nb;
    PA.out = fb.probe.p;
    PA.unit_hits = fb.uhits.p;
    PA.unit_flags = fb.uflags.p;
    PA.k = k;
    hipLaunchKernelGGL(k_probe<false>, dim3((nb + 3) / 4), dim3(256), 0, s, PA);
    HitArgs HA;
    HA.R = c->reads();
    HA.occ = c->d_occ.p;
    HA.units = fb.units[0].p;
    HA.rbase = fb.rbase.p;
    HA.probes = fb.probe.p;
    HA.nunits = nb;
    HA.k = k;
    HA.unit_hits = ucnt.p;
    HA.unit_base = nullptr;
    HA.out = nullptr;
    hipLaunchKernelGGL(k_hitlist, dim3((nb + 3) / 4), dim3(256), 0, s, HA);
    HIPC(hipGetLastError());
    HIPC(hipEventRecord(c->ev[3], s));
    std::vector<uint64_t> cnt(nb);
    HIPC(hipMemcpyAsync(cnt.data(), ucnt.p, 8ull * nb, hipMemcpyDeviceToHost, s));
    HIPC(hipStreamSynchronize(s));
    // ms_seed_hits is device time of the kernels alone: the probe + count pass here, each
    // write pass below; the host's piece cuts, buffer growth, uploads, the hit copies to
    // the host and the syncs between pieces are outside every event pair
    {
      float t = 0;
      (void)hipEventElapsedTime(&t, c->ev[2], c->ev[3]);
      ms_tot += t;
    }
    // write pass, in pieces of whole units that fit the hit buffer: every unit's base
    // within its piece is computed once (one host pass over the batch) and uploaded once;
    // the hit buffer only grows (one allocation at the largest piece)
    std::vector<uint64_t> base(nb, 0);
    std::vector<uint32_t> cuts{0};
    uint64_t hmax = 1;
    for (uint32_t p0 = 0; p0 < nb;) {
      uint32_t p1 = p0;
      uint64_t h = 0;
      while (p1 < nb && (h + cnt[p1] <= HIT_BUF || p1 == p0)) { base[p1] = h; h += cnt[p1++]; }
      hmax = std::max<uint64_t>(hmax, h);
      cuts.push_back(p1);
      p0 = p1;
    }
    if (hbuf.grow(hmax))
      return fail(OVL_ERR_OOM, "seed-hit list (%llu hits)", (unsigned long long)hmax);
    HIPC(hipMemcpyAsync(ubase.p, base.data(), 8ull * nb, hipMemcpyHostToDevice, s));
    for (size_t pc = 0; pc + 1 < cuts.size(); pc++) {
      const uint32_t p0 = cuts[pc], p1 = cuts[pc + 1];
      const uint64_t a2 = base[p1 - 1] + cnt[p1 - 1];
      HA.out = hbuf.p;
      HA.units = fb.units[0].p + p0;
      HA.rbase = fb.rbase.p + p0;
      HA.unit_base = ubase.p + p0;
      HA.nunits = p1 - p0;
      HIPC(hipEventRecord(c->ev[4], s));
      hipLaunchKernelGGL(k_hitlist, dim3((p1 - p0 + 3) / 4), dim3(256), 0, s, HA);
      HIPC(hipGetLastError());
      HIPC(hipEventRecord(c->ev[5], s));
      if (out && copied < max_hits && a2) {
        uint64_t n = std::min<uint64_t>(a2, max_hits - copied);
        HIPC(hipMemcpyAsync(out + copied, hbuf.p, 16ull * n, hipMemcpyDeviceToHost, s));
        copied += n;
      }
      HIPC(hipStreamSynchronize(s));
      float t = 0;
      (void)hipEventElapsedTime(&t, c->ev[4], c->ev[5]);
      ms_tot += t;
      total += a2;
    }
    u0 = u1;
  }
  c->stats.ms_seed_hits = ms_tot;
  *n_hits = total;
  return OVL_OK;
}

int ovl_find_overlaps(ovl_ctx *c, uint32_t bgn, uint32_t end, uint64_t *n_out) {
  return find_impl(c, bgn, end, 0, UINT32_MAX, false, n_out);
}

// OverlapDriver (overlapInCore.C:190-300).
// Query chunks of an OverlapDriver job whose sorted query windows (sq_prepare) would not fit
// the HBM all at once (configs[4]'s full-size rank jobs: ~28 G windows, 330 GB of keys and
// ids).  The ref range bgn..end is cut into consecutive chunks whose windows fit the budget
// sq_prepare checks against (half the HBM free now and held by sorted windows, less a margin
// for the next builds), counted with sq_prepare's unit rule.  One chunk: the whole range.
// OVL_SQ_CHUNK_WINDOWS (tests) caps a chunk's windows.
static std::vector<std::pair<uint32_t, uint32_t>> plan_query_chunks(ovl_ctx *c, uint32_t bgn,
                                                                    uint32_t end, uint32_t lib_lo,
                                                                    uint32_t lib_hi,
                                                                    uint64_t *max_windows) {
  std::vector<std::pair<uint32_t, uint32_t>> out;
  const uint32_t k = c->P.kmer_len;
  size_t fr = 0, tot = 0;
  uint64_t budget = UINT64_MAX;
  if (hipMemGetInfo(&fr, &tot) == hipSuccess) {
    const uint64_t half = (fr + sq_held_bytes(c)) / 2;
    const uint64_t fixed = 24ull * (1ull << 29) + 8ull * (1ull << 20);   // one run's sort scratch
    budget = half > fixed ? (half - fixed) * 9 / 10 : 0;
  }
  uint64_t wcap = budget / 13;                       // 12 B per window + the unit arrays
  if (const char *e = getenv("OVL_SQ_CHUNK_WINDOWS")) wcap = std::min<uint64_t>(wcap, strtoull(e, nullptr, 10));
  wcap = std::max<uint64_t>(wcap, 1);
  uint32_t lo = bgn;
  uint64_t w = 0;
  for (uint32_t a = bgn; a <= end && a >= bgn; a++) {
    const uint32_t r = a - c->first_iid;
    const int32_t L = (int32_t)c->h_len[r];
    const uint32_t lib = read_lib(c, r);
    uint64_t add = 0;
    if (!(lib < lib_lo || lib > lib_hi || L < c->P.min_olap_len || L < (int32_t)k))
      add = 2ull * (uint64_t)(L - (int32_t)k + 1);
    if (w + add > wcap && a > lo) {
      out.push_back({lo, a - 1});
      *max_windows = std::max(*max_windows, w);
      lo = a;
      w = 0;
    }
    w += add;
  }
  if (end >= bgn) out.push_back({lo, end});
  *max_windows = std::max(*max_windows, w);
  return out;
}

// ref reads of bgn..end that find_impl counts in ref_reads (Process_Overlaps.C:108-114)
static uint64_t count_ref_reads(const ovl_ctx *c, uint32_t bgn, uint32_t end, uint32_t lib_lo,
                                uint32_t lib_hi) {
  uint64_t n = 0;
  for (uint32_t a = bgn; a <= end && a >= bgn; a++) {
    const uint32_t r = a - c->first_iid;
    const uint32_t lib = read_lib(c, r);
    if (lib < lib_lo || lib > lib_hi || (int32_t)c->h_len[r] < c->P.min_olap_len) continue;
    n++;
  }
  return n;
}

int ovl_overlap_driver(ovl_ctx *c, const ovl_driver_params *d, uint64_t *n_out) {
  if (!c || !d || !n_out) return fail(OVL_ERR_STATE, "null argument");
  if (c->nreads == 0) return fail(OVL_ERR_STATE, "no reads loaded");
  const ovl_hash_limits &L = d->limits;
  if (L.max_hash_strings == 0)                                    // main() :423
    return fail(OVL_ERR_BAD_PARAM, "No memory model supplied; -M needed!");
  if (L.max_hash_strings > MAX_STRING_NUM)                        // :429
    return fail(OVL_ERR_BAD_PARAM, "Too many strings (--hashstrings), must be less than %llu",
                (unsigned long long)MAX_STRING_NUM);
  HIPC(hipSetDevice(c->device));
  const uint32_t last_loaded = c->first_iid + c->nreads - 1;
  const uint32_t num_reads = d->store_num_reads ? d->store_num_reads : last_loaded;
  uint32_t g_bgn_hash = std::max<uint32_t>(d->bgn_hash_iid, 1);          // :208-212
  uint32_t g_end_hash = std::min<uint32_t>(d->end_hash_iid, num_reads);
  uint32_t g_bgn_ref = std::max<uint32_t>(d->bgn_ref_iid, 1);            // :237-241
  uint32_t g_end_ref = std::min<uint32_t>(d->end_ref_iid, num_reads);
  // every read the job touches must be loaded
  if ((g_bgn_hash < g_end_hash && (g_bgn_hash < c->first_iid || g_end_hash > last_loaded)) ||
      (g_bgn_ref < g_end_ref && (g_bgn_ref < c->first_iid || g_end_ref > last_loaded)))
    return fail(OVL_ERR_BAD_PARAM, "-h %u-%u / -r %u-%u reach past the loaded reads %u-%u",
                g_bgn_hash, g_end_hash, g_bgn_ref, g_end_ref, c->first_iid, last_loaded);
  // Process_Overlaps' block schedule (:249-269, Process_Overlaps.C:86-171): blocks of
  // perThread reads from bgnRefID on, each searched only while it starts below endRefID --
  // the reads before endRefID always, endRefID itself unless a block starts on it.
  uint32_t ref_last = 0;
  bool any_ref = false;
  if (g_bgn_ref < g_end_ref) {
    uint32_t T = std::max<uint32_t>(d->num_threads, 1);
    uint32_t per = 1 + (g_end_ref - g_bgn_ref) / T / 8;
    ref_last = ((g_end_ref - g_bgn_ref) % per == 0) ? g_end_ref - 1 : g_end_ref;
    any_ref = true;
  }
  memset(&c->stats, 0, sizeof(c->stats));
  c->nout = 0;
  c->acc.nu = c->acc.nn = c->acc.np = 0;
  c->cut_windows_hint = 0;
  c->have_index = false;                    // a job builds its own indexes (none is reused)
  uint32_t bgn = g_bgn_hash;
  uint32_t end = g_bgn_hash + L.max_hash_strings - 1;                    // inclusive
  uint64_t batches = 0;
  // the query windows sorted once per query chunk (sq_prepare): OVL_SQ=1 always, 0 never,
  // 2 from a job's second search on, 3 (the default) when a query chunk is searched by
  // SQ_AUTO_SEARCHES indexes or more.  The sort costs about one random-lookup probe of the
  // same windows (the configs[4] rank-0 job at 1/8 scale, 14 batches: sort 134 ms, seed 847
  // against 892 ms; profiles/r04y_c4_*.log).
  const uint64_t SQ_AUTO_SEARCHES = 3;
  int sq_mode = 3;
  if (const char *e = getenv("OVL_SQ")) sq_mode = atoi(e);
  struct SqOff {
    ovl_ctx *c;
    ~SqOff() { c->sq_request = false; sq_release(c, false); }
  } sq_off{c};
  auto timing_line = [&](const char *what, double build_ms, double find_ms) {
    if (!getenv("OVL_TIMING")) return;
    fprintf(stderr, "OVL_TIMING %s: wall build %.1f ms, find %.1f ms; device index %.1f seed %.1f "
            "extend %.1f ms, alloc/free %.1f ms (%llu allocs, %.1f GB) so far\n", what, build_ms,
            find_ms, c->stats.ms_index, c->stats.ms_seed, c->stats.ms_extend, g_alloc_ms,
            (unsigned long long)g_alloc_n, g_alloc_bytes / 1e9);
  };
  using clk = std::chrono::steady_clock;
  auto ms_since = [](clk::time_point a, clk::time_point b) {
    return std::chrono::duration<double, std::milli>(b - a).count();
  };
  // -l (Frag_Olap_Limit) counts a query's overlaps per Find_Overlaps call, i.e. per hash
  // batch (A_/B_Olaps_For_Frag, Find_Overlaps.C:306), and orders its targets by their first
  // hit in the batch: those jobs search batch by batch, as the reference does.
  const bool ordered = c->P.frag_olap_limit != UINT64_MAX;
  int sb_mode = 1;
  if (const char *e = getenv("OVL_SUPERBATCH")) sb_mode = atoi(e);
  if (!any_ref || ordered || sb_mode == 0) {
    while (bgn < g_end_hash) {                                           // :222
      if (end > g_end_hash) end = g_end_hash;
      uint32_t loaded = 0;
      const auto t0 = clk::now();
      int rc = build_batch_impl(c, bgn, end, &L, &loaded);
      if (rc) return rc;
      const auto t1 = clk::now();
      end = loaded;
      batches++;
      if (any_ref) {
        // the batches' pairs are extended together: the last batch flushes what is pending
        uint64_t n = 0;
        const bool last_batch = !(end + 1 < g_end_hash);
        c->sq_request = sq_mode == 1 || (sq_mode == 2 && batches >= 2);
        if ((rc = find_impl(c, g_bgn_ref, ref_last, d->min_lib_ref, d->max_lib_ref, true, &n,
                            last_batch)))
          return rc;
      }
      char what[96];
      snprintf(what, sizeof(what), "batch %llu: hash %u-%u", (unsigned long long)batches, bgn, end);
      timing_line(what, ms_since(t0, t1), ms_since(t1, clk::now()));
      bgn = end + 1;
      end = bgn + L.max_hash_strings - 1;
    }
    c->stats.hash_batches = batches;
    c->stats.query_chunks = any_ref ? 1 : 0;
    *n_out = c->nout;
    return OVL_OK;
  }

  // ---- super-batches (the default without -l) -----------------------------------------
  // A query read meets, in every batch it searches, exactly the hashed reads with larger IDs
  // (Find_Overlaps.C:328), and everything Process_String_Olaps reads of a (query, target)
  // pair -- its seed hits in window and chain order, its Add_Match list, the target's
  // screened ends (Mark_Screened_Ends_Chain, Build_Hash_Index.C:147-170: per read), the
  // query's hi_hits flags (skip k-mers are in every batch's table) -- depends on the pair
  // alone.  So searching the UNION of consecutive batches' hashed reads gives every pair,
  // record and -s counter the batches give one by one; only the batches' ends (the table-load
  // cuts, the one-read tail that is never hashed, :222) need the reference's loading loop.
  // Phase 1 runs that loop (Build_Hash_Index's stop rules, build_batch_impl) and records the
  // batches; phase 2 groups consecutive batches into super-batches of up to sb_cap windows;
  // phase 3 searches every (query chunk, super-batch) pair whose reads can meet: a canu job
  // of ~100 batches is then ~10 searches of each query instead of ~100.
  std::vector<std::pair<uint32_t, uint32_t>> bat;            // the reference's batches
  double phase1_ms = 0;
  {
    const auto t0 = clk::now();
    while (bgn < g_end_hash) {                                           // :222
      if (end > g_end_hash) end = g_end_hash;
      uint32_t loaded = 0;
      int rc = build_batch_impl(c, bgn, end, &L, &loaded, true);
      if (rc) return rc;
      end = loaded;
      batches++;
      bat.push_back({bgn, end});
      bgn = end + 1;
      end = bgn + L.max_hash_strings - 1;
    }
    phase1_ms = ms_since(t0, clk::now());
  }
  c->stats.hash_batches = batches;
  if (bat.empty()) {
    c->stats.query_chunks = 0;
    *n_out = c->nout;
    return OVL_OK;
  }
  // phase 2: super-batches of up to sb_cap windows -- a share of what one index may take
  // (index_window_cap, with this context's current index counted as free), leaving the rest
  // of the HBM to the sorted query windows and the search buffers.  OVL_SB_WINDOWS caps it.
  const uint32_t k = c->P.kmer_len;
  auto batch_windows = [&](uint32_t b, uint32_t e) {
    uint64_t w = 0;
    for (uint32_t id = b; id <= e; id++) {
      const uint32_t r = id - c->first_iid;
      const uint32_t lib = read_lib(c, r);
      if (lib >= L.min_lib_hash && lib <= L.max_lib_hash &&
          (int64_t)c->h_len[r] >= (int64_t)c->P.min_olap_len && c->h_len[r] >= k)
        w += c->h_len[r] - k + 1;
    }
    return w;
  };
  uint64_t sb_pct = 55;
  if (const char *e = getenv("OVL_SB_PCT")) sb_pct = std::min<uint64_t>(95, std::max(5, atoi(e)));
  uint64_t sb_cap = index_window_cap(c) * sb_pct / 100;
  if (const char *e = getenv("OVL_SB_WINDOWS")) sb_cap = std::min<uint64_t>(sb_cap, strtoull(e, nullptr, 10));
  sb_cap = std::max<uint64_t>(sb_cap, 1);
  std::vector<std::pair<uint32_t, uint32_t>> sbs;
  uint64_t sb_max = 0;                                         // the largest one's windows
  {
    uint64_t w = 0;
    for (const auto &b : bat) {
      const uint64_t bw = batch_windows(b.first, b.second);
      if (!sbs.empty() && w + bw <= sb_cap) {
        sbs.back().second = b.second;
        w += bw;
      } else {
        sbs.push_back(b);
        w = bw;
      }
      sb_max = std::max(sb_max, w);
    }
  }
  // the index buffers for the largest super-batch from the first build on, and search buffers
  // that keep their first size (ovl_ctx::index_reserve / sticky_budgets), for this job only
  struct Reserve {
    ovl_ctx *c;
    ~Reserve() {
      c->index_reserve = 0; c->sq_reserve = 0; c->sticky_budgets = false; c->dense_tables = false;
    }
  } reserve_guard{c};
  c->index_reserve = sb_max + c->h_skip.size();
  c->sticky_budgets = true;
  // phase 3: the searches.  The first super-batch is built, then the query chunks are planned
  // with its index resident (plan_query_chunks: what the sorted windows may take).
  auto build_sb = [&](size_t si) -> int {
    uint32_t hb = sbs[si].first, he = sbs[si].second;
    if (c->have_index && c->hash_bgn_iid == hb && c->hash_end_iid == he) return OVL_OK;
    int rc = clip_hash_range(c, hb, he);
    if (rc) return rc;
    const bool bloom = !c->sq.on || sq_bloom();
    if ((rc = build_index(c, hb, he, bloom)) == OVL_ERR_OOM) {
      release_find_buffers(c);
      c->stats.find_releases++;
      rc = build_index(c, hb, he, bloom);
    }
    return rc;
  };
  // searches of one query chunk: the super-batches whose reads reach past its first read
  auto searches_of = [&](uint32_t qlo) {
    uint64_t n = 0;
    for (const auto &sb : sbs) n += qlo < sb.second ? 1 : 0;
    return n;
  };
  const bool sq_on = sq_mode == 1 || (sq_mode == 2 && sbs.size() >= 2) ||
                     (sq_mode == 3 && searches_of(g_bgn_ref) >= SQ_AUTO_SEARCHES);
  if (sq_on) {
    // sorted windows (12 B + unit arrays) past a quarter of the device will need chunks: the
    // full-size configs[4] rank job (13.7 G windows, ~180 GB) does, its 1/8-scale side line
    // (3.8 G, ~50 GB) does not.  OVL_DENSE_TABLES=0|1 overrides.
    uint64_t qw = 0;
    for (uint32_t a = g_bgn_ref; a <= ref_last && a >= g_bgn_ref; a++) {
      const uint32_t r = a - c->first_iid;
      const int32_t Lr = (int32_t)c->h_len[r];
      const uint32_t lib = read_lib(c, r);
      if (!(lib < d->min_lib_ref || lib > d->max_lib_ref || Lr < c->P.min_olap_len || Lr < (int32_t)k))
        qw += 2ull * (uint64_t)(Lr - (int32_t)k + 1);
    }
    size_t fr = 0, tot = 0;
    if (hipMemGetInfo(&fr, &tot) == hipSuccess) c->dense_tables = 13 * qw > tot / 4;
    if (const char *e = getenv("OVL_DENSE_TABLES")) c->dense_tables = atoi(e) != 0;
  }
  const auto t_sb0 = clk::now();
  if (int rc = build_sb(0)) return rc;
  const double sb0_ms = ms_since(t_sb0, clk::now());
  std::vector<std::pair<uint32_t, uint32_t>> qchunks;
  if (sq_on) qchunks = plan_query_chunks(c, g_bgn_ref, ref_last, d->min_lib_ref, d->max_lib_ref,
                                         &c->sq_reserve);
  if (qchunks.empty()) qchunks.push_back({g_bgn_ref, ref_last});
  // (chunk, super-batch), the super-batches of every other chunk in reverse order: a chunk
  // then starts with the index its predecessor ended on when both reach the last super-batch
  std::vector<std::pair<size_t, size_t>> plan;
  for (size_t qi = 0; qi < qchunks.size(); qi++)
    for (size_t i = 0; i < sbs.size(); i++) {
      const size_t si = (qi & 1) ? sbs.size() - 1 - i : i;
      if (qchunks[qi].first < sbs[si].second) plan.push_back({qi, si});
    }
  if (getenv("OVL_TIMING"))
    fprintf(stderr, "OVL_TIMING super-batches: %llu batches (phase 1 %.1f ms) -> %zu super-batches "
            "of <= %llu windows, %zu query chunks over refs %u-%u, %zu searches, sorted windows %s%s\n",
            (unsigned long long)batches, phase1_ms, sbs.size(), (unsigned long long)sb_cap,
            qchunks.size(), g_bgn_ref, ref_last, plan.size(), sq_on ? "on" : "off", c->dense_tables ? ", dense tables" : "");
  c->sq_request = sq_on;
  for (size_t pi = 0; pi < plan.size(); pi++) {
    const auto [qi, si] = plan[pi];
    const auto t0 = clk::now();
    if (int rc = build_sb(si)) return rc;
    const auto t1 = clk::now();
    uint64_t n = 0;
    if (int rc = find_impl(c, qchunks[qi].first, qchunks[qi].second, d->min_lib_ref,
                           d->max_lib_ref, true, &n, pi + 1 == plan.size()))
      return rc;
    char what[128];
    snprintf(what, sizeof(what), "query chunk %zu (refs %u-%u) x super-batch %zu (hash %u-%u)", qi,
             qchunks[qi].first, qchunks[qi].second, si, sbs[si].first, sbs[si].second);
    timing_line(what, pi == 0 ? sb0_ms : ms_since(t0, t1), ms_since(t1, clk::now()));
  }
  // ref_reads as the reference counts them: every batch's search over the whole -r range
  c->stats.ref_reads = batches * count_ref_reads(c, g_bgn_ref, ref_last, d->min_lib_ref,
                                                 d->max_lib_ref);
  c->stats.query_chunks = (uint32_t)qchunks.size();
  c->stats.super_batches = (uint32_t)sbs.size();
  *n_out = c->nout;
  return OVL_OK;
}

int ovl_fetch_overlaps(ovl_ctx *c, ovl_record *out, uint64_t max_records, uint64_t *n_copied) {
  if (!c) return fail(OVL_ERR_STATE, "null context");
  HIPC(hipSetDevice(c->device));
  std::vector<Rec> h(c->nout);
  if (c->nout)
    HIPC(hipMemcpy(h.data(), c->d_out.p, sizeof(Rec) * c->nout, hipMemcpyDeviceToHost));
  std::sort(h.begin(), h.end(), [](const Rec &x, const Rec &y) {
    if (x.a_iid != y.a_iid) return x.a_iid < y.a_iid;
    if (x.b_iid != y.b_iid) return x.b_iid < y.b_iid;
    if (x.w0 != y.w0) return x.w0 < y.w0;
    return x.w1 < y.w1;
  });
  uint64_t n = std::min<uint64_t>(max_records, h.size());
  for (uint64_t i = 0; i < n; i++) {
    out[i].a_iid = h[i].a_iid;
    out[i].b_iid = h[i].b_iid;
    out[i].dat[0] = h[i].w0;
    out[i].dat[1] = h[i].w1;
  }
  *n_copied = n;
  return OVL_OK;
}

int ovl_write_ovb(const ovl_record *recs, uint64_t n, const char *path, int with_counts) {
  if (!path || (n && !recs)) return fail(OVL_ERR_BAD_PARAM, "null argument");
  if (write_ovb_file(recs, n, path, with_counts != 0))
    return fail(OVL_ERR_BAD_INPUT, "writing '%s': %s", path, strerror(errno));
  return OVL_OK;
}

int ovl_ctx_write_ovb(ovl_ctx *c, const char *path) {
  if (!c) return fail(OVL_ERR_STATE, "null context");
  std::vector<ovl_record> h(c->nout);
  uint64_t got = 0;
  int rc = ovl_fetch_overlaps(c, h.data(), h.size(), &got);
  if (rc) return rc;
  return ovl_write_ovb(h.data(), got, path, 1);
}

int ovl_ctx_write_stats(ovl_ctx *c, const char *path) {
  if (!c || !path) return fail(OVL_ERR_STATE, "null argument");
  if (write_stats_file(c->stats, path))
    return fail(OVL_ERR_BAD_INPUT, "writing '%s': %s", path, strerror(errno));
  return OVL_OK;
}

int ovl_get_stats(ovl_ctx *c, ovl_stats *out) {
  if (!c) return fail(OVL_ERR_STATE, "null context");
  *out = c->stats;
  return OVL_OK;
}

}  // extern "C"
