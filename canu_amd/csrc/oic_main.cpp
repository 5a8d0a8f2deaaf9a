// oic_main.cpp -- an `overlapInCore` executable over libcanu_ovl.so (the MI355X path).
//
// Drop-in for canu's overlapper job: it accepts main()'s command line
// (src/overlapInCore/overlapInCore.C:306-483), including the line canu's pipeline writes
// into overlap.sh (src/pipelines/canu/OverlapInCore.pm:207-226):
//
//   overlapInCore [-G] -t N -k K -k <frequentMers.fasta> --hashbits B --hashload F
//                 --maxerate E --minlength L [--minkmers]
//                 -h a-b -r c-d [--hashstrings N --hashdatalen M]
//                 -o <job>.ovb.WORKING -s <job>.stats <gkpStore>
//
// reads the gkpStore with its own read-only reader (gkp_store.h), runs OverlapDriver()
// (hash batches, both orientations of every ref read) on the GPU through the C-ABI
// (ovl_overlap_driver), and writes what the reference writes: the -o .ovb (ovFile full
// format) with its <base>.counts, and the -s statistics (to stderr without -s).
// Records are written sorted by ovOverlap::operator<; the reference writes them in its
// threads' completion order, which no reader depends on (ovStoreBuild sorts).
//
// There is no CPU path: without a gfx950 device the job fails (exit 1).
#include <algorithm>
#include <cctype>
#include <cerrno>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/canu_ovl.h"
#include "gkp_store.h"

namespace {

// AS_UTL_decodeRange (src/AS_UTL/AS_UTL_decodeRange.C): "a-b" or "a".
void decode_range(const char *s, uint32_t &lo, uint32_t &hi) {
  char *e = nullptr;
  unsigned long a = strtoul(s, &e, 10), b = a;
  if (*e == '-') b = strtoul(e + 1, &e, 10);
  lo = (uint32_t)a;
  hi = (uint32_t)b;
}

// Mark_Skip_Kmers (overlapInCore-Build_Hash_Index.C:235-286): pairs of lines, '>' header
// then exactly Kmer_Len bases.  A malformed line ends the job, as there.  K-mers holding
// anything but ACGT cannot equal a hashed window (windows with such a base are not
// hashed), so they are dropped here.
bool read_skip_kmers(FILE *F, uint32_t k, std::string &out, uint64_t &n) {
  char line[1024];
  int ct = 0;
  n = 0;
  out.clear();
  while (fgets(line, sizeof(line), F)) {
    ct++;
    size_t len = strlen(line) - 1;
    if (line[0] != '>' || line[len] != '\n') {
      fprintf(stderr, "ERROR:  Bad line %d in kmer skip file\n", ct);
      fputs(line, stderr);
      return false;
    }
    if (!fgets(line, sizeof(line), F)) {
      fprintf(stderr, "ERROR:  Bad line after %d in kmer skip file\n", ct);
      return false;
    }
    ct++;
    len = strlen(line) - 1;
    if (len != k || line[len] != '\n') {
      fprintf(stderr, "ERROR:  Bad line %d in kmer skip file\n", ct);
      fputs(line, stderr);
      return false;
    }
    bool acgt = true;
    for (size_t i = 0; i < len; i++) {
      char c = (char)tolower(line[i]);
      acgt &= c == 'a' || c == 'c' || c == 'g' || c == 't';
      line[i] = c;
    }
    if (acgt) {
      out.append(line, len);
      n++;
    }
  }
  fprintf(stderr, "Read %d kmers to mark to skip\n", ct / 2);
  return true;
}

void usage(const char *prog) {
  fprintf(stderr, "USAGE:  %s [options] <gkpStorePath>\n", prog);
  fprintf(stderr, "\n");
  fprintf(stderr, "-G          do partial overlaps\n");
  fprintf(stderr, "-h <range>  to specify fragments to put in hash table\n");
  fprintf(stderr, "-H <range>  libraries to put in the hash table\n");
  fprintf(stderr, "-k          if one or two digits, the length of a kmer, otherwise\n");
  fprintf(stderr, "            the filename containing a list of kmers to ignore in\n");
  fprintf(stderr, "            the hash table\n");
  fprintf(stderr, "-l          specify the maximum number of overlaps per\n");
  fprintf(stderr, "            fragment-end per batch of fragments (not supported on the GPU path)\n");
  fprintf(stderr, "-m          allow multiple overlaps per oriented fragment pair\n");
  fprintf(stderr, "-o          specify output file name\n");
  fprintf(stderr, "-r <range>  specify old fragments to overlap\n");
  fprintf(stderr, "-R <range>  libraries of the old fragments\n");
  fprintf(stderr, "-s <file>   write statistics here (default stderr)\n");
  fprintf(stderr, "-t <n>      threads of the reference job (sets its read-block schedule)\n");
  fprintf(stderr, "-u          allow only 1 overlap per oriented fragment pair\n");
  fprintf(stderr, "-w          filter out overlaps with too many errors in a window\n");
  fprintf(stderr, "-z          skip the hopeless check\n");
  fprintf(stderr, "\n");
  fprintf(stderr, "--maxerate <n>     only output overlaps with fraction <n> or less error (e.g., 0.06 == 6%%)\n");
  fprintf(stderr, "--minlength <n>    only output overlaps of <n> or more bases\n");
  fprintf(stderr, "--minkmers         filter pairs by the expected number of shared kmers\n");
  fprintf(stderr, "\n");
  fprintf(stderr, "--hashbits n       Use n bits for the hash mask.\n");
  fprintf(stderr, "--hashstrings n    Load at most n strings into the hash table at one time.\n");
  fprintf(stderr, "--hashdatalen n    Load at most n bytes into the hash table at one time.\n");
  fprintf(stderr, "--hashload f       Load to at most 0.0 < f < 1.0 capacity (default 0.6).\n");
  fprintf(stderr, "--maxreadlen n     all reads must be shorter than n; --hashstrings limited to 2^(30-m)\n");
  fprintf(stderr, "\n");
  fprintf(stderr, "CANU_OVL_DEVICE    environment: HIP device ordinal (default 0)\n");
}

int die_ovl(const char *what, int rc) {
  fprintf(stderr, "ERROR: %s failed (%d): %s\n", what, rc, ovl_last_error());
  return 1;
}

}  // namespace

int main(int argc, char **argv) {
  ovl_params P;
  ovl_params_init(&P);
  ovl_driver_params D;
  ovl_driver_params_init(&D);
  const char *store_path = nullptr, *out_name = nullptr, *stat_name = nullptr;
  const char *dump_path = nullptr;                // --dump-store (test hook, no GPU)
  FILE *skip_file = nullptr;
  uint64_t max_string_num = (1ull << 31) - 1;     // MAX_STRING_NUM (overlapInCore.C:57-63)
  uint32_t max_read_len = UINT32_MAX;             // --maxreadlen
  bool minkmers_seen = false;

  int err = 0;
  for (int arg = 1; arg < argc; arg++) {
    const char *a = argv[arg];
    auto next = [&]() -> const char * {
      if (arg + 1 >= argc) { err++; return "0"; }
      return argv[++arg];
    };
    if (!strcmp(a, "-G")) {
      P.partial = 1;
    } else if (!strcmp(a, "-h")) {
      decode_range(next(), D.bgn_hash_iid, D.end_hash_iid);
    } else if (!strcmp(a, "-H")) {
      decode_range(next(), D.limits.min_lib_hash, D.limits.max_lib_hash);
    } else if (!strcmp(a, "-r")) {
      decode_range(next(), D.bgn_ref_iid, D.end_ref_iid);
    } else if (!strcmp(a, "-R")) {
      decode_range(next(), D.min_lib_ref, D.max_lib_ref);
    } else if (!strcmp(a, "-k")) {
      const char *v = next();
      if ((isdigit((unsigned char)v[0]) && v[1] == 0) ||
          (isdigit((unsigned char)v[0]) && isdigit((unsigned char)v[1]) && v[2] == 0)) {
        P.kmer_len = (uint32_t)strtoull(v, nullptr, 10);
      } else {
        errno = 0;
        skip_file = fopen(v, "r");
        if (errno || !skip_file) {
          fprintf(stderr, "ERROR: Failed to open -k '%s': %s\n", v, strerror(errno));
          return 1;
        }
      }
    } else if (!strcmp(a, "-l")) {
      long v = strtol(next(), nullptr, 10);
      P.frag_olap_limit = v < 1 ? UINT64_MAX : (uint64_t)v;
    } else if (!strcmp(a, "-m")) {
      P.unique_olap_per_pair = 0;
    } else if (!strcmp(a, "-u")) {
      P.unique_olap_per_pair = 1;
    } else if (!strcmp(a, "--hashbits")) {
      D.limits.hash_mask_bits = (uint32_t)strtoull(next(), nullptr, 10);
    } else if (!strcmp(a, "--hashstrings")) {
      D.limits.max_hash_strings = (uint32_t)strtoull(next(), nullptr, 10);
    } else if (!strcmp(a, "--hashdatalen")) {
      D.limits.max_hash_data_len = strtoull(next(), nullptr, 10);
    } else if (!strcmp(a, "--hashload")) {
      D.limits.max_hash_load = atof(next());
    } else if (!strcmp(a, "--maxreadlen")) {
      // the CPU table packs (read, offset) into 30 bits (overlapInCore.C:366-378)
      uint32_t desired = (uint32_t)strtoul(next(), nullptr, 10);
      uint32_t offset_bits = 1;
      while (((uint32_t)1 << offset_bits) < desired) offset_bits++;
      max_string_num = (1ull << (30 - offset_bits)) - 1;
      max_read_len = (1u << offset_bits) - 1;
    } else if (!strcmp(a, "-o")) {
      out_name = next();
    } else if (!strcmp(a, "-s")) {
      stat_name = next();
    } else if (!strcmp(a, "-t")) {
      D.num_threads = (uint32_t)strtoull(next(), nullptr, 10);
    } else if (!strcmp(a, "--minlength")) {
      P.min_olap_len = (int32_t)strtol(next(), nullptr, 10);
    } else if (!strcmp(a, "--minkmers")) {
      // evaluated where it appears, with the -k / --maxerate / --minlength seen so far
      P.filter_by_kmer_count = (uint64_t)(int)floor(
          exp(-1.0 * (double)P.kmer_len * P.max_erate) * (P.min_olap_len - (int)P.kmer_len + 1));
      minkmers_seen = true;
    } else if (!strcmp(a, "--maxerate")) {
      P.max_erate = strtof(next(), nullptr);
    } else if (!strcmp(a, "--dump-store")) {
      dump_path = next();
    } else if (!strcmp(a, "-w")) {
      P.use_window_filter = 1;
    } else if (!strcmp(a, "-z")) {
      P.use_hopeless_check = 0;
    } else if (store_path == nullptr) {
      store_path = a;
    } else {
      fprintf(stderr, "Unknown option '%s'\n", a);
      err++;
    }
  }
  (void)minkmers_seen;

  if (P.max_erate > 0.06) {                                   // :416-421
    if (P.use_window_filter)
      fprintf(stderr, "High error rates requested -- window-filter turned off despite -w flag!\n");
    ovl_params_finalize(&P);
  }
  if (D.limits.max_hash_strings == 0) fprintf(stderr, "* No memory model supplied; -M needed!\n"), err++;
  if (P.kmer_len == 0) fprintf(stderr, "* No kmer length supplied; -k needed!\n"), err++;
  if (D.limits.max_hash_strings > max_string_num)
    fprintf(stderr, "Too many strings (--hashstrings), must be less than %llu\n",
            (unsigned long long)max_string_num), err++;
  if (out_name == nullptr && dump_path == nullptr)
    fprintf(stderr, "ERROR:  No output file name specified\n"), err++;
  if (err || store_path == nullptr) {
    usage(argv[0]);
    return 1;
  }

  // ---- the store ----------------------------------------------------------------------
  gkp::Store store;
  std::string msg;
  if (!store.open(store_path, msg)) {
    fprintf(stderr, "gkStore()--  failed to open '%s' for read-only access: %s\n", store_path,
            msg.c_str());
    return 1;
  }
  const uint32_t nstore = store.num_reads();
  // the reads the job touches: the -h and -r ranges, clipped as OverlapDriver clips them
  uint32_t hb = std::max<uint32_t>(D.bgn_hash_iid, 1), he = std::min<uint32_t>(D.end_hash_iid, nstore);
  uint32_t rb = std::max<uint32_t>(D.bgn_ref_iid, 1), re = std::min<uint32_t>(D.end_ref_iid, nstore);
  uint32_t lo = UINT32_MAX, hi = 0;
  if (hb <= he) { lo = std::min(lo, hb); hi = std::max(hi, he); }
  if (rb <= re) { lo = std::min(lo, rb); hi = std::max(hi, re); }
  if (lo > hi) { lo = 1; hi = nstore ? 1 : 0; }

  std::vector<uint8_t> bases, quals;
  std::vector<uint64_t> offs;
  std::vector<uint32_t> lens, libs;
  const bool need_q = P.use_window_filter != 0;
  uint64_t total = 0;
  for (uint32_t id = lo; id <= hi && id >= lo && hi; id++) total += store.length(id);
  bases.reserve(total);
  if (need_q) quals.reserve(total);
  std::string seq, qlt;
  for (uint32_t id = lo; id <= hi && id >= lo && hi; id++) {
    if (store.read_id(id) != id) {
      fprintf(stderr, "ERROR: read %u of '%s' carries ID %u\n", id, store_path, store.read_id(id));
      return 1;
    }
    if (store.length(id) > max_read_len) {
      fprintf(stderr, "ERROR: read %u is %u bases, --maxreadlen allows %u\n", id, store.length(id),
              max_read_len);
      return 1;
    }
    offs.push_back(bases.size());
    lens.push_back(store.length(id));
    libs.push_back(store.library(id));
    if (!store.load(id, seq, qlt, msg)) {
      fprintf(stderr, "ERROR: %s\n", msg.c_str());
      return 1;
    }
    bases.insert(bases.end(), seq.begin(), seq.end());
    if (need_q) quals.insert(quals.end(), qlt.begin(), qlt.end());
  }
  const uint32_t nload = (uint32_t)lens.size();
  if (dump_path) {
    // the loaded reads as: u32 first_id, u32 n, then per read u32 library, u32 length,
    // then all bases, then all QVs -- what the store reader decoded (tests/test_cli.py)
    if (!need_q) {
      quals.clear();
      for (uint32_t id = lo; id <= hi && id >= lo && hi; id++) {
        if (!store.load(id, seq, qlt, msg)) { fprintf(stderr, "ERROR: %s\n", msg.c_str()); return 1; }
        quals.insert(quals.end(), qlt.begin(), qlt.end());
      }
    }
    FILE *F = fopen(dump_path, "wb");
    if (!F) { fprintf(stderr, "ERROR: can't write '%s'\n", dump_path); return 1; }
    uint32_t hdr[2] = {lo, nload};
    fwrite(hdr, 4, 2, F);
    for (uint32_t i = 0; i < nload; i++) { fwrite(&libs[i], 4, 1, F); fwrite(&lens[i], 4, 1, F); }
    fwrite(bases.data(), 1, bases.size(), F);
    fwrite(quals.data(), 1, quals.size(), F);
    fclose(F);
    return 0;
  }
  fprintf(stderr, "Loaded reads %u-%u of %u from '%s' (%llu bases)\n", lo, hi, nstore, store_path,
          (unsigned long long)bases.size());

  // ---- the GPU job ----------------------------------------------------------------------
  int device = 0;
  if (const char *dv = getenv("CANU_OVL_DEVICE")) device = atoi(dv);
  ovl_ctx *ctx = nullptr;
  int rc = ovl_ctx_create(&P, device, &ctx);
  if (rc) return die_ovl("ovl_ctx_create", rc);
  if (nload) {
    rc = ovl_load_reads(ctx, lo, nload, bases.data(), offs.data(), lens.data(),
                        need_q ? quals.data() : nullptr);
    if (rc) return die_ovl("ovl_load_reads", rc);
    if ((rc = ovl_set_read_libraries(ctx, libs.data()))) return die_ovl("ovl_set_read_libraries", rc);
  }
  std::vector<uint8_t>().swap(bases);
  std::vector<uint8_t>().swap(quals);
  if (skip_file) {
    std::string km;
    uint64_t nk = 0;
    if (!read_skip_kmers(skip_file, P.kmer_len, km, nk)) return 1;
    fclose(skip_file);
    if ((rc = ovl_set_skip_kmers(ctx, km.data(), nk))) return die_ovl("ovl_set_skip_kmers", rc);
  }
  D.store_num_reads = nstore;
  uint64_t nrec = 0;
  if (nload && (rc = ovl_overlap_driver(ctx, &D, &nrec))) return die_ovl("ovl_overlap_driver", rc);
  ovl_stats st;
  memset(&st, 0, sizeof(st));
  if (nload) ovl_get_stats(ctx, &st);
  fprintf(stderr, "%llu hash batches, %llu ref reads, %llu overlaps (index %.1f ms, seed %.1f ms, "
          "extend %.1f ms on the GPU)\n", (unsigned long long)st.hash_batches,
          (unsigned long long)st.ref_reads, (unsigned long long)nrec, st.ms_index, st.ms_seed,
          st.ms_extend);

  // ---- outputs: -o .ovb + .counts, -s statistics (overlapInCore.C:197, :569-591) -------
  if (nload) rc = ovl_ctx_write_ovb(ctx, out_name);
  else rc = ovl_write_ovb(nullptr, 0, out_name, 1);
  if (rc) return die_ovl("writing the .ovb", rc);
  if (stat_name) {
    rc = ovl_ctx_write_stats(ctx, stat_name);
    if (rc) {
      fprintf(stderr, "WARNING: failed to open '%s' for writing: %s\n", stat_name, ovl_last_error());
      stat_name = nullptr;
    }
  }
  if (!stat_name) {
    fprintf(stderr, " Kmer hits without olaps = %lld\n", (long long)st.kmer_hits_without_olap);
    fprintf(stderr, "    Kmer hits with olaps = %lld\n", (long long)st.kmer_hits_with_olap);
    fprintf(stderr, "  Multiple overlaps/pair = %lld\n", (long long)st.multi_overlaps);
    fprintf(stderr, " Total overlaps produced = %lld\n", (long long)st.total_overlaps);
    fprintf(stderr, "      Contained overlaps = %lld\n", (long long)st.contained_overlaps);
    fprintf(stderr, "       Dovetail overlaps = %lld\n", (long long)st.dovetail_overlaps);
    fprintf(stderr, "Rejected by short window = %lld\n", (long long)st.bad_short_window);
    fprintf(stderr, " Rejected by long window = %lld\n", (long long)st.bad_long_window);
  }
  ovl_ctx_destroy(ctx);
  fprintf(stderr, "Bye.\n");
  return 0;
}
