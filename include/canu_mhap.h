/*
 * canu_mhap.h -- C-ABI of the MI355X-native MHAP stage (sketch, index, two-stage filter).
 *
 * Replaces the MHAP 2.1.2 jar canu runs for overlapper=mhap (src/mhap/mhap-2.1.2.tar,
 * invoked by src/pipelines/canu/OverlapMhap.pm:374-498: "precompute" = sketch a block, then
 * one job per query block = compare against the hash block).  The output keeps MHAP's text
 * line, the one src/mhap/mhapConvert.C:114-150 turns into ovOverlap records (.ovb), so
 * canu's mhapConvert step runs unchanged on it.
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
 *   --max-shift / --min-store-length / --no-rc  mhap_params (jar defaults 0.2 / 0 / off)
 *   --repeat-weight --repeat-idf-scale --filter-threshold --no-tf   mhap_weighting
 *   -f frequentMers.ignore        (:394)       mhap_set_kmer_frequencies()
 *   -p block.fasta (precompute)   (:395)       mhap_load_reads*() + mhap_sketch()
 *   -s hash block / -q queries    (:494-495)   mhap_build_index() + mhap_compare*()
 *   stdout  *.mhap                (:496)       mhap_fetch() / mhap_write_text()
 *
 * The algorithm is the jar's own, read from its bytecode (the jar is never run: no JVM, and
 * prebuilt reference binaries are not executed) and restated in oracle/mhap_jar.py, which
 * names the class, method and bytecode offsets of every step.  In short:
 *   - a read is used when it has >= min_olap bases (and a k-mer); both strands of every
 *     used read are sketched and indexed, queries are forward strands;
 *   - MinHash sketch (MinHashSketch.computeNgramMinHashesWeighted): per distinct k-mer
 *     key = Murmur3_x64_128 h1 of its UTF-16 chars (Guava), weight w (tf-idf, below); per
 *     hash function j the key's xorshift64 chain (<<21, >>>35, <<4) is drawn w times; the
 *     signed-smallest draw wins (first k-mer occurrence on ties) and stores the key's low
 *     (even j) or high (odd j) 32 bits;
 *   - ordered sketch (BottomOverlapSketch): the ordered_sketch smallest Murmur3_x86_32
 *     k'-mer hashes with their positions, duplicates kept;
 *   - first stage: >= min_matches equal sketch entries; self jobs compare each query with
 *     the stored reads of smaller ID (MinHashSearch.findMatches);
 *   - second stage: the ordered sketches' shared k'-mers -> median shift -> overlap edges ->
 *     bottom-sketch Jaccard in the overlap -> identity = (2J / (1 + J))^(1/k'); kept when
 *     >= threshold; erate = 1 - identity.
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

#define MHAP_ABI_VERSION 7

typedef struct {
  uint32_t k;               /* -k                      MinHash k-mer size, 1..32        */
  uint32_t num_hashes;      /* --num-hashes            1..1024                          */
  uint32_t min_matches;     /* --num-min-matches                                        */
  uint32_t ordered_sketch;  /* --ordered-sketch-size   1..2048                          */
  uint32_t ordered_k;       /* --ordered-kmer-size     1..32                            */
  int32_t  min_olap;        /* --min-olap-length       reads shorter are not used       */
  double   threshold;       /* --threshold             identity of the second stage     */
  double   max_shift;       /* --max-shift             (jar default 0.2)                */
  int32_t  min_store;       /* --min-store-length      (jar default 0)                  */
  int32_t  no_rc;           /* --no-rc                 store forward strands only        */
} mhap_params;

/* canu's correction defaults at 'normal' sensitivity (OverlapMhap.pm:116-121,
 * Defaults.pm:704-705): k 16, 512 hashes, 3 min matches, threshold 0.78, ordered sketch
 * 1536 of 12-mers, min overlap 500; the jar's max shift 0.2, min store 0, both strands. */
void        mhap_params_init(mhap_params *p);

/* One MHAP output line (MatchResult.toString, mhapConvert.C:117-120 column order):
 *   a b erate raw 0 a_bgn a_end a_len b_rc b_bgn b_end b_len */
typedef struct {
  uint32_t a_iid, b_iid;    /* query read, stored read (gkStore IDs)                    */
  double   erate;           /* 1 - min(identity, 1)                                     */
  double   raw;             /* rawScore: shared k'-mers inside the overlap               */
  int32_t  a_bgn, a_end, a_len;
  uint32_t b_rc;            /* 1: b coordinates are on b's reverse complement           */
  int32_t  b_bgn, b_end, b_len;
  uint32_t count;           /* shared MinHash entries (first stage; not printed)        */
} mhap_record;

typedef struct {
  uint64_t sketched_reads;  /* reads used (>= min_olap) in the last mhap_sketch()       */
  uint64_t candidates;      /* pairs passing the first stage                            */
  uint64_t overlaps;        /* pairs passing the second stage                           */
  double   ms_sketch;       /* device time: MinHash + ordered sketches                  */
  double   ms_index;        /* device time: MinHash index sort                          */
  double   ms_candidates;   /* device time: first-stage lookups                         */
  double   ms_compare;      /* device time: second-stage filter                         */
  uint64_t sketch_kmers;    /* distinct k-mers entering MinHash sketches                */
  double   ms_sketch_kernel; /* device time of the MinHash draw kernel launches alone    */
  uint64_t sketch_launches; /* its launches                                              */
  uint64_t sketch_draws;    /* xorshift64 draws made (sum over k-mers of w x num_hashes) */
} mhap_stats;

typedef struct mhap_ctx mhap_ctx;

int         mhap_ctx_create(const mhap_params *p, int device, mhap_ctx **out);
void        mhap_ctx_destroy(mhap_ctx *ctx);
const char *mhap_last_error(void);
int         mhap_abi_version(void);

/* Reads first_iid .. first_iid+nreads-1; bases concatenated (read as the jar's FASTA reader
 * gives them: upper-cased, every other byte kept), read i at offsets[i] for lengths[i]
 * bytes.  Copied to the device once. */
int         mhap_load_reads(mhap_ctx *ctx, uint32_t first_iid, uint32_t nreads,
                            const uint8_t *bases, const uint64_t *offsets,
                            const uint32_t *lengths);
/* Same with device-resident bases/offsets (HBM), host lengths. */
int         mhap_load_reads_device(mhap_ctx *ctx, uint32_t first_iid, uint32_t nreads,
                                   const uint8_t *d_bases, const uint64_t *d_offsets,
                                   const uint32_t *h_lengths);

/* The weighting options (MhapMain's defaults: repeat_weight 0.9, repeat_idf_scale 3,
 * filter_threshold 1e-5; canu passes --repeat-idf-scale 10).  Without a -f table
 * (mhap_set_weighting alone) a k-mer's weight is its count in the read (repeat_weight >= 0)
 * or 1 (repeat_weight < 0). */
typedef struct {
  double  repeat_weight;      /* --repeat-weight                                         */
  double  repeat_idf_scale;   /* --repeat-idf-scale                                      */
  double  filter_threshold;   /* --filter-threshold                                      */
  int32_t no_tf;              /* --no-tf                                                 */
  int32_t supress_noise;      /* --supress-noise 0 / 1 / 2 (FrequencyCounts.removeUnique):
                                 with a -f table, 1 drops every k-mer a Guava 19 Bloom
                                 filter of the file's keys rejects (keepKmer); 2 builds
                                 the filter and never reads it (= 0); without -f no effect */
} mhap_weighting;

void        mhap_weighting_init(mhap_weighting *w);
int         mhap_set_weighting(mhap_ctx *ctx, const mhap_weighting *w);

/* -f (FrequencyCounts): n k-mers (n * k bytes, back to back) with their fractions, in file
 * order.  A k-mer's key is the hash of the smaller of it and its reverse complement (both
 * strands unless no_rc); entries with fraction >= filter_threshold form the table.  With
 * the table, a read's k-mer of count c gets weight
 *   repeat_weight < 0:       0 when in the table (never sketched), else 1
 *   0 <= repeat_weight < 1:  max(1, round(tf * scaled_idf)), tf = c (1 with no_tf),
 *                            scaled_idf = repeat_idf_scale for k-mers not in the table,
 *                            else 1 + (idf(f) - idf(max f)) / ((idf(threshold) -
 *                            idf(max f)) / (scale - 1)), idf(x) = ln(max f / x - r)
 *   repeat_weight >= 1:      c */
int         mhap_set_kmer_frequencies(mhap_ctx *ctx, const char *kmers, const double *fractions,
                                      uint64_t n, const mhap_weighting *w);
/* (ABI 7) the same with the file's first line, the k-mer count the jar sizes its Bloom
 * filter by (FrequencyCounts.<init> @149-207: BloomFilter.create(funnel, count, 1e-5), a
 * count of 0 read as 1); mhap_set_kmer_frequencies passes n.  Every line's key enters the
 * filter whatever its fraction. */
int         mhap_set_kmer_frequencies_ex(mhap_ctx *ctx, const char *kmers,
                                         const double *fractions, uint64_t n,
                                         uint64_t expected, const mhap_weighting *w);

/* Sketch reads bgn_iid..end_iid (inclusive): both strands' MinHash + ordered sketches. */
int         mhap_sketch(mhap_ctx *ctx, uint32_t bgn_iid, uint32_t end_iid);

/* Device arrays holding every loaded read's sketches (row 2r: read r forward, 2r+1: its
 * reverse complement), for an all-gather across ranks:
 *   minhash  int32  [nreads][2][num_hashes]
 *   ordered  uint64 [nreads][2][ordered_sketch]   ((hash ^ 0x80000000) << 32 | position)
 *   ocount   uint32 [nreads][2]                   (entries used; 0: strand not stored)
 * Valid after mhap_load_reads*(); rows of reads this rank did not sketch are filled by the
 * caller (e.g. RCCL all-gather) before mhap_build_index(). */
int         mhap_sketch_buffers(mhap_ctx *ctx, void **d_minhash, void **d_ordered,
                                void **d_ocount);

/* Copy the sketch rows of reads first_iid .. first_iid+n-1 between the context and caller
 * device buffers laid out like mhap_sketch_buffers() (rows of those reads only):
 * to_ctx = 0 exports the context's rows, to_ctx = 1 imports the caller's.  Device-to-device,
 * on the context's stream; returns after it completes. */
int         mhap_copy_sketches(mhap_ctx *ctx, uint32_t first_iid, uint32_t n, void *d_minhash,
                               void *d_ordered, void *d_ocount, int to_ctx);

/* The same rows to / from host memory (the executable's .dat files).  A context loaded
 * with mhap_load_reads_device(ctx, first, n, NULL, NULL, lengths) holds lengths only: it can
 * import sketches and compare, not sketch. */
int         mhap_copy_sketches_host(mhap_ctx *ctx, uint32_t first_iid, uint32_t n,
                                    void *h_minhash, void *h_ordered, void *h_ocount,
                                    int to_ctx);

/* Build the MinHash index over all loaded reads' stored strands. */
int         mhap_build_index(mhap_ctx *ctx);

/* ... over the strands of reads bgn_iid..end_iid only: the jar's hash block (-s block.dat)
 * when the query blocks are loaded beside it. */
int         mhap_build_index_range(mhap_ctx *ctx, uint32_t bgn_iid, uint32_t end_iid);

/* The jar's self search (-s without --no-self): queries bgn_iid..end_iid (forward strands)
 * against the indexed strands of reads with a smaller ID (MinHashSearch.findMatches,
 * toSelf); results stay on the device; *n_out = records found. */
int         mhap_compare(mhap_ctx *ctx, uint32_t bgn_iid, uint32_t end_iid, uint64_t *n_out);

/* The jar's query search (-q): queries bgn_iid..end_iid against every indexed read but
 * themselves (toSelf false), a_iid = the query, b_iid = the stored read. */
int         mhap_compare_all(mhap_ctx *ctx, uint32_t bgn_iid, uint32_t end_iid,
                             uint64_t *n_out);

/* Records of the last compare, sorted by (a_iid, b_iid, b_rc). */
int         mhap_fetch(mhap_ctx *ctx, mhap_record *out, uint64_t max_records,
                       uint64_t *n_copied);

/* MHAP's text output of the last compare ("%s %s %.6f %.6f %d ..." as Java formats it:
 * the shortest decimal of each double rounded half-up), numbered the way mhapConvert -h/-q
 * expects: stored read b_iid is written as b_iid - (hash_base - 1); query a_iid as
 * a_iid - (query_base - 1) + num_hash (mhapConvert.C:122-123). */
int         mhap_write_text(mhap_ctx *ctx, const char *path, uint32_t hash_base,
                            uint32_t num_hash, uint32_t query_base);

/* One record as that text line (no newline) into buf[cap]. */
int         mhap_format_line(const mhap_record *r, uint32_t hash_base, uint32_t num_hash,
                             uint32_t query_base, char *buf, size_t cap);

int         mhap_get_stats(mhap_ctx *ctx, mhap_stats *out);

#ifdef __cplusplus
}
#endif

#endif
