/*
 * canu_mhap.h -- C-ABI of the MI355X-native MHAP MinHash sketch / filter stage.
 *
 * Replaces the MHAP jar canu runs for overlapper=mhap (src/mhap/mhap-2.1.2.tar, invoked by
 * src/pipelines/canu/OverlapMhap.pm:374-498: "precompute" = sketch a block, then one job per
 * query block = compare against the hash blocks).  The output keeps MHAP's text format, the
 * one src/mhap/mhapConvert.C:114-150 turns into ovOverlap records (.ovb), so canu's
 * mhapConvert step runs unchanged on it.
 *
 *   reference (OverlapMhap.pm option)          here
 *   -----------------------------------------  -------------------------------------------
 *   -k <MhapMerSize>              (:381)       mhap_params.k
 *   --num-hashes                  (:386)       mhap_params.num_hashes
 *   --num-min-matches             (:387)       mhap_params.min_matches
 *   --ordered-sketch-size         (:388)       mhap_params.ordered_sketch
 *   --ordered-kmer-size           (:389)       mhap_params.ordered_k
 *   --threshold                   (:390)       mhap_params.threshold
 *   --min-olap-length             (:392)       mhap_params.min_olap
 *   -f frequentMers.ignore        (:394)       mhap_set_filter_kmers()
 *   -p block.fasta (precompute)   (:395)       mhap_load_reads*() + mhap_sketch()
 *   -s hash blocks / -q queries   (:494-495)   mhap_build_index() + mhap_compare()
 *   stdout  *.mhap                (:496)       mhap_fetch() / mhap_write_text()
 *
 * The algorithm is the published MinHash sketch + ordered-sketch filter, restated in
 * oracle/mhap_oracle.py (PARITY UNPINNED against the jar, which is never run).
 * All functions return 0 or a negative status (same codes as canu_ovl.h); mhap_last_error()
 * gives a message.  No CPU fallback: without a gfx950 device mhap_ctx_create() fails.
 */
#ifndef CANU_MHAP_H
#define CANU_MHAP_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MHAP_ABI_VERSION 5

typedef struct {
  uint32_t k;               /* -k                      MinHash k-mer size, 1..32        */
  uint32_t num_hashes;      /* --num-hashes            1..1024                          */
  uint32_t min_matches;     /* --num-min-matches                                        */
  uint32_t ordered_sketch;  /* --ordered-sketch-size   1..1984                          */
  uint32_t ordered_k;       /* --ordered-kmer-size     1..32                            */
  int32_t  min_olap;        /* --min-olap-length                                        */
  double   threshold;       /* --threshold (identity of the second-stage filter)        */
} mhap_params;

/* canu's correction defaults at 'normal' sensitivity (OverlapMhap.pm:116-121,
 * Defaults.pm:704-705): k 16, 512 hashes, 3 min matches, threshold 0.78, ordered sketch
 * 1536 of 12-mers, min overlap 500. */
void        mhap_params_init(mhap_params *p);

/* One MHAP output line (mhapConvert.C:117-120 column order). */
typedef struct {
  uint32_t a_iid, b_iid;    /* query read, hash read (gkStore IDs)                      */
  double   erate;           /* estimated error (Mash distance of the 2nd-stage Jaccard) */
  uint32_t count;           /* shared min-mers (first stage)                            */
  int32_t  a_bgn, a_end, a_len;
  uint32_t b_rc;            /* 1: b coordinates are on b's reverse complement           */
  int32_t  b_bgn, b_end, b_len;
} mhap_record;

typedef struct {
  uint64_t sketched_reads;
  uint64_t candidates;      /* pairs passing the first stage                            */
  uint64_t overlaps;        /* pairs passing the second stage                           */
  double   ms_sketch;       /* device time: MinHash + ordered sketches                  */
  double   ms_index;        /* device time: MinHash index sort                          */
  double   ms_candidates;   /* device time: first-stage lookups                         */
  double   ms_compare;      /* device time: second-stage filter                         */
  uint64_t sketch_kmers;    /* k-mers hashed by the MinHash kernel                      */
  double   ms_sketch_kernel; /* device time of the MinHash kernel launches alone (ABI 5:
                                the dominant kernel's live launch time, bench_mhap.py)   */
  uint64_t sketch_launches; /* its launches                                              */
} mhap_stats;

typedef struct mhap_ctx mhap_ctx;

int         mhap_ctx_create(const mhap_params *p, int device, mhap_ctx **out);
void        mhap_ctx_destroy(mhap_ctx *ctx);
const char *mhap_last_error(void);
int         mhap_abi_version(void);

/* Reads first_iid .. first_iid+nreads-1; bases concatenated (any case; non-ACGT breaks
 * k-mers), read i at offsets[i] for lengths[i] bytes.  Copied to the device once. */
int         mhap_load_reads(mhap_ctx *ctx, uint32_t first_iid, uint32_t nreads,
                            const uint8_t *bases, const uint64_t *offsets,
                            const uint32_t *lengths);
/* Same with device-resident bases/offsets (HBM), host lengths. */
int         mhap_load_reads_device(mhap_ctx *ctx, uint32_t first_iid, uint32_t nreads,
                                   const uint8_t *d_bases, const uint64_t *d_offsets,
                                   const uint32_t *h_lengths);

/* -f: k-mers (n * k ACGT bytes, back to back) that never enter a MinHash sketch. */
int         mhap_set_filter_kmers(mhap_ctx *ctx, const char *kmers, uint64_t n);

/* The jar's repeat weighting (MHAP 2.x tf-idf; options canu always passes,
 * OverlapMhap.pm:382, :390).  Restated from the published algorithm -- parity with the jar
 * is unpinned: each distinct k-mer c of a read enters the MinHash sketch with
 * an integer weight w(c) >= 1, i.e. w(c) consecutive draws of its xorshift64 chain per
 * hash function instead of one:
 *   tf(c)   occurrences of c in the read (1 with no_tf)
 *   idf(c)  ln(1 / fraction(c)) for -f k-mers with fraction >= filter_threshold, else
 *           ln(1 / filter_threshold); scaled linearly onto [1, repeat_idf_scale] between
 *           the most frequent -f k-mer (1) and ln(1 / filter_threshold) (repeat_idf_scale)
 *   w(c)    max(1, floor(tf(c) * m(c) + 0.5)), m(c) = r + (1 - r) * scaled idf(c), where
 *           r = repeat_weight; r >= 1 or no -f k-mers: m = 1 (tf only)
 * repeat_weight < 0 is MHAP 1.x's unweighted sketch: -f k-mers with a fraction >=
 * filter_threshold are dropped, every other k-mer counts once.
 * supress_noise (--supress-noise, OverlapMhap.pm:383 / :483, passed when
 * mhapFilterUnique is set; the -f file then lists every k-mer at or above the unique-k-mer
 * count, Meryl.pm:678-714) -- restated from MHAP 2.x's option text ("1) completely removes
 * any k-mers not specified in the filter file, 2) supresses k-mers not specified in the
 * filter file, similar to repeats"), parity unpinned:
 *   0  as above;
 *   1  k-mers not in the -f file never enter a sketch (weighted sketches only);
 *   2  k-mers not in the -f file get the multiplier of the most frequent -f k-mer
 *      (scaled idf 1, m = 1 for canu's r = 0.9); -f k-mers below filter_threshold keep the
 *      top multiplier (scaled idf repeat_idf_scale) as before. */
typedef struct {
  double  repeat_weight;      /* --repeat-weight     (canu: 0.9; < 0 unweighted)         */
  double  repeat_idf_scale;   /* --repeat-idf-scale  (canu: 10)                          */
  double  filter_threshold;   /* --filter-threshold  (canu: mhapFilterThreshold 5e-6)    */
  int32_t no_tf;              /* --no-tf                                                 */
  int32_t supress_noise;      /* --supress-noise 0 / 1 / 2 (ABI 4)                       */
} mhap_weighting;

/* Unweighted defaults: repeat_weight -1, repeat_idf_scale 10, filter_threshold 1e-5, tf on,
 * supress_noise 0. */
void        mhap_weighting_init(mhap_weighting *w);

/* -f with its second column: n k-mers (n * k bytes) and the fraction of all k-mers each
 * one is (Meryl.pm:699-716 writes "kmer<TAB>fraction" lines, both strands), with the
 * weighting options.  n = 0 sets the weighting alone (tf weighting, no idf). */
int         mhap_set_kmer_frequencies(mhap_ctx *ctx, const char *kmers, const double *fractions,
                                      uint64_t n, const mhap_weighting *w);

/* Sketch reads bgn_iid..end_iid (inclusive): MinHash sketch + ordered sketch. */
int         mhap_sketch(mhap_ctx *ctx, uint32_t bgn_iid, uint32_t end_iid);

/* Device arrays holding every loaded read's sketches, for an all-gather across ranks:
 *   minhash  int32 [nreads][num_hashes]
 *   ordered  uint64 [nreads][ordered_sketch]  (hash << 32 | pos << 1 | strand)
 *   ocount   uint32 [nreads]                  (entries used in each ordered row)
 * Valid after mhap_load_reads*(); rows of reads this rank did not sketch are filled by the
 * caller (e.g. RCCL all-gather) before mhap_build_index(). */
int         mhap_sketch_buffers(mhap_ctx *ctx, void **d_minhash, void **d_ordered,
                                void **d_ocount);

/* Copy the sketch rows of reads first_iid .. first_iid+n-1 between the context and caller
 * device buffers laid out like mhap_sketch_buffers() (rows of those reads only):
 * to_ctx = 0 exports the context's rows, to_ctx = 1 imports the caller's (e.g. after an
 * RCCL all-gather of every rank's exported slice).  Device-to-device, on the context's
 * stream; returns after it completes. */
int         mhap_copy_sketches(mhap_ctx *ctx, uint32_t first_iid, uint32_t n, void *d_minhash,
                               void *d_ordered, void *d_ocount, int to_ctx);

/* The same rows to / from host memory (the executable's .dat files).  A context loaded
 * with mhap_load_reads_device(ctx, first, n, NULL, NULL, lengths) holds lengths only: it can
 * import sketches and compare, not sketch. */
int         mhap_copy_sketches_host(mhap_ctx *ctx, uint32_t first_iid, uint32_t n,
                                    void *h_minhash, void *h_ordered, void *h_ocount,
                                    int to_ctx);

/* Build the MinHash index over all loaded reads' sketches. */
int         mhap_build_index(mhap_ctx *ctx);

/* Build the MinHash index over the sketches of reads bgn_iid..end_iid only: the jar's
 * hash block (-s block.dat) when the query blocks are loaded beside it. */
int         mhap_build_index_range(mhap_ctx *ctx, uint32_t bgn_iid, uint32_t end_iid);

/* Compare queries bgn_iid..end_iid against every indexed read with a larger ID (each pair
 * once: the all-vs-all, and the jar's hash block against itself); results stay on the
 * device; *n_out = records found. */
int         mhap_compare(mhap_ctx *ctx, uint32_t bgn_iid, uint32_t end_iid, uint64_t *n_out);

/* Compare queries bgn_iid..end_iid against every indexed read but themselves: the jar's
 * query blocks (-q) against its hash block, a_iid = the query, b_iid = the hash read. */
int         mhap_compare_all(mhap_ctx *ctx, uint32_t bgn_iid, uint32_t end_iid,
                             uint64_t *n_out);

/* Records of the last compare, sorted by (a_iid, b_iid). */
int         mhap_fetch(mhap_ctx *ctx, mhap_record *out, uint64_t max_records,
                       uint64_t *n_copied);

/* MHAP's text output of the last compare, numbered the way mhapConvert -h/-q expects:
 * hash read b_iid is written as b_iid - (hash_base - 1); query a_iid as
 * a_iid - (query_base - 1) + num_hash (mhapConvert.C:122-123). */
int         mhap_write_text(mhap_ctx *ctx, const char *path, uint32_t hash_base,
                            uint32_t num_hash, uint32_t query_base);

int         mhap_get_stats(mhap_ctx *ctx, mhap_stats *out);

#ifdef __cplusplus
}
#endif

#endif
