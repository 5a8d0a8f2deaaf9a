/*
 * canu_ovl.h -- C-ABI of the MI355X-native overlapInCore seed-and-extend path.
 *
 * This is the drop-in boundary: plain pointers and sizes, no torch / HIP types.
 * It replaces the compute inside canu's overlapInCore driver:
 *
 *   reference                                               replaced by
 *   -----------------------------------------------------   -------------------------------
 *   src/overlapInCore/overlapInCore.C:190 OverlapDriver()    ovl_ctx_* lifecycle below
 *   src/overlapInCore/overlapInCore.C:306 main() (options)   ovl_params + ovl_params_init()
 *   src/overlapInCore/overlapInCore.C:487-529 (HSF/Bit_Eq.)  done inside ovl_ctx_create()
 *   src/overlapInCore/overlapInCore-Build_Hash_Index.C:443   ovl_build_hash_index()
 *     Build_Hash_Index(gkStore*, bgnID, endID)
 *   src/overlapInCore/overlapInCore-Build_Hash_Index.C:235   ovl_set_skip_kmers()
 *     Mark_Skip_Kmers() (-k <frequentMers.fasta>)
 *   src/overlapInCore/overlapInCore-Process_Overlaps.C:78    ovl_find_overlaps()
 *     Process_Overlaps() -> Find_Overlaps(FORWARD/REVERSE)
 *     -> Process_String_Olaps -> Process_Matches
 *     -> prefixEditDistance::Extend_Alignment
 *     -> Output_Overlap / Output_Partial_Overlap
 *   src/stores/ovStoreFile.C:198 ovFile::writeOverlap()      ovl_fetch_overlaps() returns the
 *                                                            records; the caller keeps writing
 *                                                            them with its own ovFile.
 *
 * Records are returned in ovOverlap's in-memory layout for AS_MAX_READLEN_BITS == 21
 * (src/stores/ovOverlap.H:93-116): a_iid, b_iid, then the two 64-bit bitfield words
 * (ahg5:21 ahg3:21 evalue:12 flipped:1 forOBT:1 forDUP:1 forUTG:1 extra1:6 |
 *  bhg5:21 bhg3:21 span:21 extra2:1).
 *
 * Reads are handed over as the gkStore hands them to overlapInCore
 * (gkStore::gkStore_loadReadData -> char* sequence, char* qualities): bases in any case
 * (the library lowercases, as Process_Overlaps.C:122 does), qualities as small integers
 * (already minus '!'), or NULL when the window filter is not used.
 *
 * All functions return 0 on success and a negative ovl_status on error; ovl_last_error()
 * gives a message.  There is no CPU fallback: without a usable gfx950 device
 * ovl_ctx_create() fails with OVL_ERR_NO_DEVICE.
 */
#ifndef CANU_OVL_H
#define CANU_OVL_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define OVL_ABI_VERSION 8

typedef enum {
  OVL_OK               =  0,
  OVL_ERR_NO_DEVICE    = -1,   /* no HIP device / not gfx950                          */
  OVL_ERR_BAD_PARAM    = -2,   /* parameter outside what the reference accepts        */
  OVL_ERR_UNSUPPORTED  = -3,   /* reference option this build does not implement      */
  OVL_ERR_BAD_INPUT    = -4,   /* read data the GPU path cannot represent             */
  OVL_ERR_HIP          = -5,   /* a HIP runtime call failed                           */
  OVL_ERR_OOM          = -6,   /* device or host allocation failed                    */
  OVL_ERR_STATE        = -7    /* call order violated (e.g. find before build)        */
} ovl_status;

/* One overlap, ovOverlap (src/stores/ovOverlap.H:285) without the gkStore pointer. */
typedef struct {
  uint32_t a_iid;
  uint32_t b_iid;
  uint64_t dat[2];
} ovl_record;

/* overlapInCore options (oicParameters, src/overlapInCore/overlapInCore.H:418). */
typedef struct {
  uint32_t kmer_len;              /* -k <n>              G.Kmer_Len                      */
  double   max_erate;             /* --maxerate          G.maxErate (host mirror parses  */
                                  /*                     with strtof, as main() does)    */
  int32_t  min_olap_len;          /* --minlength         G.Min_Olap_Len                  */
  int32_t  partial;               /* -G                  G.Doing_Partial_Overlaps        */
  int32_t  unique_olap_per_pair;  /* -u / -m             G.Unique_Olap_Per_Pair          */
  int32_t  use_window_filter;     /* -w                  G.Use_Window_Filter             */
  int32_t  use_hopeless_check;    /* -z clears it        G.Use_Hopeless_Check            */
  uint64_t frag_olap_limit;       /* -l                  G.Frag_Olap_Limit (UINT64_MAX)  */
  uint64_t filter_by_kmer_count;  /* --minkmers          G.Filter_By_Kmer_Count          */
} ovl_params;

/* Defaults of oicParameters::initialize() (overlapInCore.H:425). kmer_len is left 0, as
 * there; ovl_ctx_create() rejects 0 like main() does (overlapInCore.C:426). */
void        ovl_params_init(ovl_params *p);

/* The fix-ups main() applies after option parsing (overlapInCore.C:416-421):
 * maxErate > 0.06 turns the window filter and the hopeless check off. */
void        ovl_params_finalize(ovl_params *p);

typedef struct ovl_ctx ovl_ctx;

/* Create a context on HIP device `device` (ordinal; one process per GPU). */
int         ovl_ctx_create(const ovl_params *p, int device, ovl_ctx **out);
void        ovl_ctx_destroy(ovl_ctx *ctx);
const char *ovl_last_error(void);
int         ovl_abi_version(void);

/* Load reads first_iid .. first_iid+nreads-1 (gkStore IDs, 1-based in canu).
 *   bases    concatenated sequence bytes, read i at bases[offsets[i]] for lengths[i] bytes
 *   quals    same layout, or NULL (required only when use_window_filter is set); quality
 *            values as gkStore hands them out (numeric QVs)
 * The data are copied to device memory (2-bit packed + exception masks) once; every
 * later call works on the resident copy. */
int         ovl_load_reads(ovl_ctx *ctx, uint32_t first_iid, uint32_t nreads,
                           const uint8_t *bases, const uint64_t *offsets,
                           const uint32_t *lengths, const uint8_t *quals);

/* The same, but the caller's buffers are already device pointers (HBM resident). */
int         ovl_load_reads_device(ovl_ctx *ctx, uint32_t first_iid, uint32_t nreads,
                                  const uint8_t *d_bases, const uint64_t *d_offsets,
                                  const uint32_t *h_lengths, const uint8_t *d_quals);

/* Frequent k-mers that must not seed overlaps (-k <fasta>, Mark_Skip_Kmers).
 * kmers: n_kmers * kmer_len bytes of ACGT text, back to back. Both orientations are
 * screened, as the reference does. Must be called before ovl_build_hash_index(). */
int         ovl_set_skip_kmers(ovl_ctx *ctx, const char *kmers, uint64_t n_kmers);

/* Build the k-mer index over hash reads bgn_iid..end_iid (inclusive, like -h), all of them
 * in one index (no batch limits). */
int         ovl_build_hash_index(ovl_ctx *ctx, uint32_t bgn_iid, uint32_t end_iid);

/* Library IDs of the loaded reads (gkRead_libraryID), for the -H / -R filters of the
 * driver below.  Without this call every read is in library 0.  lib_ids: one per loaded
 * read, in load order. */
int         ovl_set_read_libraries(ovl_ctx *ctx, const uint32_t *lib_ids);

/* How much of the -h range one hash batch holds: the loading rules of Build_Hash_Index
 * (overlapInCore-Build_Hash_Index.C:495-541, defaults oicParameters::initialize(),
 * overlapInCore.H:447-450). */
typedef struct {
  uint32_t max_hash_strings;      /* --hashstrings  G.Max_Hash_Strings  (10000)          */
  uint64_t max_hash_data_len;     /* --hashdatalen  G.Max_Hash_Data_Len (100000000)      */
  uint32_t hash_mask_bits;        /* --hashbits     G.Hash_Mask_Bits    (22)             */
  double   max_hash_load;         /* --hashload     G.Max_Hash_Load     (0.6)            */
  uint32_t min_lib_hash;          /* -H             G.minLibToHash      (0)              */
  uint32_t max_lib_hash;          /*                G.maxLibToHash      (UINT32_MAX)     */
} ovl_hash_limits;

void        ovl_hash_limits_init(ovl_hash_limits *l);

/* Build_Hash_Index(gkpStore, bgnID, endID) (overlapInCore-Build_Hash_Index.C:443): index
 * hash reads from bgn_iid on, stopping where the reference stops loading -- after
 * max_hash_strings IDs, once max_hash_data_len bases (+1 per read) are in, or once the
 * distinct k-mers reach max_hash_load * 2^hash_mask_bits * 21 table entries -- and return
 * the last ID loaded in *last_iid.  Reads outside [min_lib_hash, max_lib_hash] or shorter
 * than min_olap_len are not hashed (they still count as strings).  Fails with
 * OVL_ERR_BAD_PARAM where the reference asserts (:523: more than max_hash_data_len +
 * AS_MAX_READLEN bases in bgn..end). */
int         ovl_build_hash_batch(ovl_ctx *ctx, uint32_t bgn_iid, uint32_t end_iid,
                                 const ovl_hash_limits *lim, uint32_t *last_iid);

/* OverlapDriver() (overlapInCore.C:190-300): the whole job.  Hash batches over the -h range
 * (ovl_build_hash_batch; a batch starts only while its first ID is below the range end,
 * :222), each searched by the -r reads (Process_Overlaps, both orientations) as the
 * reference's -t threads would take them in blocks (:249-269, Process_Overlaps.C:86: a
 * block that starts at the range end is not searched).  -h / -r ends are clipped to
 * store_num_reads (0 = the last loaded ID).  Records and counters of all batches
 * accumulate: ovl_fetch_overlaps / ovl_get_stats / ovl_ctx_write_* then see the job. */
typedef struct {
  uint32_t bgn_hash_iid, end_hash_iid;   /* -h  (1, UINT32_MAX)                         */
  uint32_t bgn_ref_iid, end_ref_iid;     /* -r  (1, UINT32_MAX)                         */
  uint32_t min_lib_ref, max_lib_ref;     /* -R  (0, UINT32_MAX)                         */
  uint32_t num_threads;                  /* -t  (1): only the ref block schedule uses it */
  uint32_t store_num_reads;              /* gkStore_getNumReads(), 0 = last loaded ID   */
  ovl_hash_limits limits;
} ovl_driver_params;

void        ovl_driver_params_init(ovl_driver_params *d);
int         ovl_overlap_driver(ovl_ctx *ctx, const ovl_driver_params *d, uint64_t *n_out);

/* Search ref reads bgn_iid..end_iid (inclusive, like -r) against the index, both
 * orientations, and keep the resulting records on the device. Returns the number of
 * records found in *n_out. Work is done on the context's stream; the call returns
 * after the stream is synchronized. */
int         ovl_find_overlaps(ovl_ctx *ctx, uint32_t bgn_iid, uint32_t end_iid,
                              uint64_t *n_out);

/* One seed hit: an Add_Ref call of Find_Overlaps (overlapInCore-Find_Overlaps.C:328-370)
 * -- query read, target (hash) read, the query window's offset in the searched
 * orientation with the orientation in bit 31 (1 = REVERSE), the k-mer's offset in the
 * target. */
typedef struct {
  uint32_t a_iid;
  uint32_t b_iid;
  uint32_t a_pos_dir;
  uint32_t b_pos;
} ovl_seed_hit;

/* The seed-hit list of ref reads bgn_iid..end_iid against the current index (the k-mer
 * lookup alone: no chaining, no extension), in the reference's order: query ascending,
 * FORWARD then REVERSE, window ascending, then the k-mer's chain order (target, offset
 * descending).  *n_hits = the total; min(max_hits, total) hits are copied to out (host
 * memory).  out == NULL counts only (the lookup still runs in full on the device). */
int         ovl_seed_hits(ovl_ctx *ctx, uint32_t bgn_iid, uint32_t end_iid,
                          ovl_seed_hit *out, uint64_t max_hits, uint64_t *n_hits);

/* Copy the records of the last ovl_find_overlaps() to host memory, sorted by
 * ovOverlap::operator< (a_iid, b_iid, dat[0], dat[1]).  max_records bounds the copy. */
int         ovl_fetch_overlaps(ovl_ctx *ctx, ovl_record *out, uint64_t max_records,
                               uint64_t *n_copied);

/* Statistics of the last find (the counters overlapInCore prints with -s). */
typedef struct {
  uint64_t kmer_hits_without_olap;
  uint64_t kmer_hits_with_olap;
  uint64_t kmer_hits_skipped;
  uint64_t multi_overlaps;
  uint64_t total_overlaps;
  uint64_t contained_overlaps;
  uint64_t dovetail_overlaps;
  uint64_t seed_hits;              /* kmer hits (Add_Ref calls)                        */
  uint64_t pairs;                  /* (query, orientation, target) pairs with hits     */
  double   ms_index;               /* device time of the index build                   */
  double   ms_seed;                /* device time of seed lookup + chaining            */
  double   ms_extend;              /* device time of extension + output                */
  double   ms_probe_kernel;        /* device time of the hash-probe kernel alone       */
  uint64_t probe_bytes;            /* algorithmic bytes of the hash-probe kernel       */
  uint32_t probe_launches;         /* k_probe launches of the last find                */
  uint32_t extend_launches;        /* k_extend launches (staged + generic)             */
  uint64_t bad_short_window;       /* -w rejections, Bad_Short_Window_Ct               */
  uint64_t bad_long_window;        /* -w rejections, Bad_Long_Window_Ct                */
  uint64_t hash_batches;           /* hash batches of the last driver run (1 otherwise) */
  uint64_t ref_reads;              /* query reads searched (both orientations each)    */
  uint64_t multi_pass_units;       /* (query, orientation) units with > 128 targets     */
  uint64_t chain_retries;          /* chain launches repeated with grown buffers        */
  double   ms_seed_hits;           /* device time of the last ovl_seed_hits (probe + list) */
  uint64_t staged_pairs;           /* pairs the full-occupancy staged kernel extended    */
  uint64_t long_pairs;             /* pairs of the long-read staged class               */
  uint64_t generic_pairs;          /* pairs of the generic kernel ('n', wide bands, ...) */
  uint32_t ext_waves;              /* waves of the full-occupancy staged launch          */
  uint32_t generic_waves;          /* waves of the generic launch                        */
  uint32_t stage_len;              /* longest read of the full-occupancy class           */
  uint32_t long_stage_len;         /* longest read of the long-read class (0: none)      */
  uint64_t seed_nodes;             /* match nodes (Add_Match lists) handed to the extension
                                      (ABI 3) */
  uint32_t probe_sorted_launches;  /* of probe_launches: the sorted-window probe
                                      (k_probe_sorted, ABI 6); its ms_probe_kernel and
                                      probe_bytes are that kernel's alone */
  uint32_t sq_resorted;            /* sorted-window runs whose partial-range radix sort failed
                                      its order / permutation check and were sorted again
                                      over all key bits (ABI 7) */
  uint32_t query_chunks;           /* query chunks of the last driver run whose sorted
                                      windows were searched one after another (1: the
                                      whole -r range at once; ABI 7) */
  uint32_t super_batches;          /* indexes the last driver run searched: consecutive hash
                                      batches joined (0: batch by batch, as with -l; ABI 7) */
  uint32_t sq_declined;            /* searches that asked for sorted query windows and fell
                                      back to random-lookup probes: the windows did not fit
                                      beside the buffers (ABI 8) */
  uint32_t find_releases;          /* search buffers released because an index build ran out
                                      of memory (the next search allocates them again; a
                                      chunk's sorted windows go with them; ABI 8) */
} ovl_stats;

int         ovl_get_stats(ovl_ctx *ctx, ovl_stats *out);

/* overlapInCore's output files (host code, no device needed):
 *   ovl_write_ovb      records, in the given order, as the .ovb that
 *                      ovFile(gkp, name, ovFileFullWrite) writes (src/stores/ovStoreFile.C:198:
 *                      a_iid, b_iid, dat words as hi32/lo32, in 43,680-record blocks, each
 *                      framed as size_t length + a snappy stream the reference reader
 *                      decodes -- literal-only, see canu_amd/csrc/ovl_ovb.h) and,
 *                      when with_counts, the "<base>.counts" overlaps-per-read file the
 *                      ovFile destructor saves (src/stores/ovStoreHistogram.C:226/:322)
 *   ovl_ctx_write_ovb  the last find's records (ovl_fetch_overlaps order) + .counts, i.e.
 *                      overlapInCore's -o output (overlapInCore.C:197)
 *   ovl_ctx_write_stats  the -s statistics text (overlapInCore.C:580-588) */
int         ovl_write_ovb(const ovl_record *recs, uint64_t n, const char *path,
                          int with_counts);
int         ovl_ctx_write_ovb(ovl_ctx *ctx, const char *path);
int         ovl_ctx_write_stats(ovl_ctx *ctx, const char *path);

/* HIP stream the context runs on (as void*, a hipStream_t), for callers that time or
 * order work around it. */
void       *ovl_ctx_stream(ovl_ctx *ctx);

/* Measurement only (bench.py's probe roofline; no reference counterpart, ABI 4): the rate
 * of independent random 16-B loads over the CURRENT index table's own allocation
 * (2^tab_bits slots, the table the hash probe looks each query window up in), in G loads/s,
 * and the table's bytes -- the memory system's ceiling for one random lookup per window on
 * this device at this table size.  Reads the table only; needs an index. */
int         ovl_probe_ceiling(ovl_ctx *ctx, double *gloads_per_s, uint64_t *table_bytes);

/* Measurement only (ABI 5): the table lookups k_probe makes for the query windows of reads
 * bgn..end (both orientations, the search's window rule; the first 2^28 windows), replayed
 * as pure 16-B loads with nothing else in the loop, in G loads/s -- the memory system's rate
 * for that exact lookup stream (the uniform ceiling above ignores that overlapping reads
 * share k-mers, so the probe can beat it).  Reads the table only; needs an index. */
int         ovl_probe_replay(ovl_ctx *ctx, uint32_t bgn, uint32_t end, double *gloads_per_s,
                             uint64_t *n_windows);

/* A built k-mer index as device buffers (ABI 7): what Build_Hash_Index leaves for
 * Find_Overlaps (overlapInCore-Build_Hash_Index.C:443 -- the hash table, the occurrence
 * lists, and the reads' screened-end flags Mark_Skip_Kmers sets), so that one process can
 * build it and others search it: the north star's "all-gather / share the k-mer index over
 * xGMI" (INTEGRATION.md).
 *   ovl_export_index  fills `out` with this context's device pointers and byte counts; they
 *                     stay valid until its next index build or ovl_ctx_destroy.
 *   ovl_import_index  copies an exported index -- device memory of this GPU, a peer's, or
 *                     buffers a collective filled -- into this context (hipMemcpy), which then
 *                     searches it as if it had built it.  The context must hold the same reads
 *                     (first_iid, read count) and k-mer length as the exporter. */
typedef struct {
  uint32_t bgn_iid, end_iid;       /* hashed reads (-h)                                    */
  uint32_t first_iid, nreads;      /* the read store the index was built over              */
  uint32_t kmer_len;
  uint32_t tab_bits, slice_bits;   /* table: 2^tab_bits 16-B slots in 2^slice_bits slices  */
  uint32_t bloom_w;                /* Bloom filter: 2^bloom_w 8-B words per slice          */
  uint32_t hash_lib_lo, hash_lib_hi;   /* -H libraries the index was built from            */
  uint64_t records;                /* occurrence records                                   */
  const void *table;      uint64_t table_bytes;
  const void *occ;        uint64_t occ_bytes;
  const void *bloom;      uint64_t bloom_bytes;    /* 0 bytes: no filter                   */
  const void *read_flags; uint64_t read_flags_bytes;   /* 4 B per loaded read              */
} ovl_index_desc;

int         ovl_export_index(ovl_ctx *ctx, ovl_index_desc *out);
int         ovl_import_index(ovl_ctx *ctx, const ovl_index_desc *in);

#ifdef __cplusplus
}
#endif

#endif
