/*
 * ref_harness.cpp -- drives the REFERENCE overlapInCore, compiled from its own sources
 * under /root/reference/src by oracle/Makefile (outputs into oracle/_ref/ only).
 *
 *   TEST INFRASTRUCTURE ONLY: used to pin oracle/oic_oracle.c, to generate the golden
 *   fixtures in tests/golden/, and as bench.py's cpu_baseline ("kind": "reference").
 *
 * What it does, with the reference's own code doing all the work:
 *   1. builds a real gkpStore from a reads file, with the calls gatekeeperCreate makes
 *      (gatekeeperCreate.C:438-441: gkStore_addEmptyRead, gkRead_encodeSeqQlt,
 *      gkStore_stashReadData);
 *   2. sets the overlapInCore globals exactly as main() does after option parsing
 *      (overlapInCore.C:416-552: error-rate fix-ups, hash-function shifts, Bit_Equivalent,
 *      Char_Is_Bad, table allocation) -- main() itself is not called because it starts
 *      with AS_configure(), which lives in AS_global.C next to a build-generated header;
 *   3. calls the reference's OverlapDriver() (overlapInCore.C:190), which writes a real
 *      snappy-compressed .ovb with the reference's ovFile;
 *   4. reads that .ovb back with the reference's ovFile::readOverlap and dumps every record
 *      as {uint32 a_iid, uint32 b_iid, uint64 dat[2]} (24 bytes) to the output file.
 *
 * Reads file format (written by canu_amd/readsfile.py):
 *   "OICR" u32 version=1, u32 nreads, u32 has_quals,
 *   u32 len[nreads], then all bases back to back, then (if has_quals) all quals (0..60).
 *
 * usage: oic_ref <reads.bin> <workdir> <out.bin> [options]
 *        oic_ref --read-ovb <in.ovb> <out.bin>
 *        oic_ref <reads.bin> <workdir> - --gkp-only   (gkpStore for mhapConvert -G)
 *   -k N  --maxerate F  --minlength N  -G  -m|-u  -w  -z  -l N  --minkmers
 *   --hashbits N  --hashload F  --hashstrings N  --hashdatalen N  -t N
 *   -h a-b  -r a-b  --skip <kmers.fasta>  --time (print wall seconds of OverlapDriver)
 *   -s <file> (the statistics text main() prints)
 */

#include "overlapInCore.H"
#include "AS_UTL_decodeRange.H"

#include <sys/stat.h>
#include <sys/time.h>
#include <vector>
#include <string>

int OverlapDriver(void);

static double now_s(void) {
  struct timeval tv;
  gettimeofday(&tv, NULL);
  return tv.tv_sec + tv.tv_usec * 1e-6;
}

static void die(const char *m) {
  fprintf(stderr, "oic_ref: %s\n", m);
  exit(1);
}

//  oic_ref --read-ovb <in.ovb> <out.bin>: read any .ovb with the reference's
//  ovFile(NULL, name, ovFileFull)::readOverlap (ovStoreFile.C) and dump its records in file
//  order, 24 bytes each -- the checker for the library's own .ovb writer.
static int read_ovb(const char *inPath, const char *outPath) {
  ovFile   *in = new ovFile(NULL, inPath, ovFileFull);
  ovOverlap ov(NULL);
  FILE *O = fopen(outPath, "wb");
  if (!O) die("can't open output");
  uint64_t n = 0;
  while (in->readOverlap(&ov)) {
    uint32_t ids[2] = { ov.a_iid, ov.b_iid };
    uint64_t w[2]   = { ov.dat.dat[0], ov.dat.dat[1] };
    fwrite(ids, 4, 2, O);
    fwrite(w, 8, 2, O);
    n++;
  }
  fclose(O);
  delete in;
  fprintf(stdout, "RECORDS %lu\n", (unsigned long)n);
  return 0;
}

int main(int argc, char **argv) {
  if (argc == 4 && strcmp(argv[1], "--read-ovb") == 0)
    return read_ovb(argv[2], argv[3]);
  if (argc < 4)
    die("usage: oic_ref <reads.bin> <workdir> <out.bin> [options]");

  const char *readsPath = argv[1];
  std::string work      = argv[2];
  const char *outPath   = argv[3];

  G.initialize();
  bool        minkmers = false;
  bool        timeIt   = false;
  bool        gkpOnly  = false;   //  build <workdir>/ref.gkpStore and stop (mhapConvert's -G)
  const char *skipPath = NULL;
  const char *statPath = NULL;    //  -s: main()'s statistics text (overlapInCore.C:569-591)
  const char *libsPath = NULL;    //  --libs: one uint32 library number (1..) per read

  for (int arg = 4; arg < argc; arg++) {
    const char *a = argv[arg];
    if      (!strcmp(a, "-k"))            G.Kmer_Len = strtoull(argv[++arg], NULL, 10);
    else if (!strcmp(a, "--maxerate"))    G.maxErate = strtof(argv[++arg], NULL);
    else if (!strcmp(a, "--minlength"))   G.Min_Olap_Len = strtol(argv[++arg], NULL, 10);
    else if (!strcmp(a, "-G"))            G.Doing_Partial_Overlaps = true;
    else if (!strcmp(a, "-m"))            G.Unique_Olap_Per_Pair = false;
    else if (!strcmp(a, "-u"))            G.Unique_Olap_Per_Pair = true;
    else if (!strcmp(a, "-w"))            G.Use_Window_Filter = true;
    else if (!strcmp(a, "-z"))            G.Use_Hopeless_Check = false;
    else if (!strcmp(a, "-l")) {
      G.Frag_Olap_Limit = strtol(argv[++arg], NULL, 10);
      if (G.Frag_Olap_Limit < 1) G.Frag_Olap_Limit = UINT64_MAX;
    }
    else if (!strcmp(a, "--minkmers"))    minkmers = true;
    else if (!strcmp(a, "--hashbits"))    G.Hash_Mask_Bits = strtoull(argv[++arg], NULL, 10);
    else if (!strcmp(a, "--hashload"))    G.Max_Hash_Load = atof(argv[++arg]);
    else if (!strcmp(a, "--hashstrings")) G.Max_Hash_Strings = strtoull(argv[++arg], NULL, 10);
    else if (!strcmp(a, "--hashdatalen")) G.Max_Hash_Data_Len = strtoull(argv[++arg], NULL, 10);
    else if (!strcmp(a, "-t"))            G.Num_PThreads = strtoull(argv[++arg], NULL, 10);
    else if (!strcmp(a, "-h"))            AS_UTL_decodeRange(argv[++arg], G.bgnHashID, G.endHashID);
    else if (!strcmp(a, "-r"))            AS_UTL_decodeRange(argv[++arg], G.bgnRefID, G.endRefID);
    else if (!strcmp(a, "-H"))            AS_UTL_decodeRange(argv[++arg], G.minLibToHash, G.maxLibToHash);
    else if (!strcmp(a, "-R"))            AS_UTL_decodeRange(argv[++arg], G.minLibToRef, G.maxLibToRef);
    else if (!strcmp(a, "--libs"))        libsPath = argv[++arg];
    else if (!strcmp(a, "--skip"))        skipPath = argv[++arg];
    else if (!strcmp(a, "--time"))        timeIt = true;
    else if (!strcmp(a, "--gkp-only"))    gkpOnly = true;
    else if (!strcmp(a, "-s"))            statPath = argv[++arg];
    else { fprintf(stderr, "unknown option '%s'\n", a); exit(1); }
  }

  //  --minkmers is evaluated where it appears in main(); canu passes it after -k,
  //  --maxerate and --minlength, so evaluating it last is the same.
  if (minkmers)
    G.Filter_By_Kmer_Count = int(floor(exp(-1.0 * (double)G.Kmer_Len * G.maxErate) *
                                       (G.Min_Olap_Len - G.Kmer_Len + 1)));

  //  ---- 1. gkpStore ------------------------------------------------------------------
  FILE *R = fopen(readsPath, "rb");
  if (!R) die("can't open reads file");
  char     magic[4];
  uint32_t hdr[3];
  if (fread(magic, 1, 4, R) != 4 || memcmp(magic, "OICR", 4) != 0) die("bad reads magic");
  if (fread(hdr, 4, 3, R) != 3 || hdr[0] != 1) die("bad reads header");
  uint32_t nreads = hdr[1], hasq = hdr[2];
  std::vector<uint32_t> lens(nreads);
  if (nreads && fread(lens.data(), 4, nreads, R) != nreads) die("short lengths");
  uint64_t total = 0;
  for (uint32_t i = 0; i < nreads; i++) total += lens[i];
  //  quals only when the file has them (a 2 M x 12 kb read set would otherwise hold 24 GB
  //  of zeros beside its bases)
  std::vector<char> bases(total + 1), quals(hasq ? total + 1 : 1);
  if (total && fread(bases.data(), 1, total, R) != total) die("short bases");
  if (hasq && total && fread(quals.data(), 1, total, R) != total) die("short quals");
  fclose(R);

  mkdir(work.c_str(), 0755);
  std::string gkp = work + "/ref.gkpStore";

  //  reads may be spread over several libraries (-H / -R filter on gkRead_libraryID())
  std::vector<uint32_t> rlib(nreads, 1);
  if (libsPath) {
    FILE *L = fopen(libsPath, "rb");
    if (!L || (nreads && fread(rlib.data(), 4, nreads, L) != nreads)) die("bad --libs file");
    fclose(L);
  }
  uint32_t nlibs = 1;
  for (uint32_t i = 0; i < nreads; i++) {
    if (rlib[i] < 1) die("library numbers start at 1");
    nlibs = rlib[i] > nlibs ? rlib[i] : nlibs;
  }

  {
    gkStore   *store = gkStore::gkStore_open(gkp.c_str(), gkStore_create);
    std::vector<gkLibrary *> libs(nlibs + 1, NULL);
    for (uint32_t l = 1; l <= nlibs; l++) {
      char ln[32];
      snprintf(ln, sizeof(ln), l == 1 ? "synthetic" : "synthetic%u", l);
      libs[l] = store->gkStore_addEmptyLibrary(ln);
    }
    uint32_t   maxl  = 0;
    for (uint32_t i = 0; i < nreads; i++) maxl = lens[i] > maxl ? lens[i] : maxl;
    std::vector<char> S(maxl + 1), Q(maxl + 1);
    char H[64];
    uint64_t off = 0;
    for (uint32_t i = 0; i < nreads; i++) {
      memcpy(S.data(), bases.data() + off, lens[i]);
      S[lens[i]] = 0;
      if (hasq) {
        for (uint32_t j = 0; j < lens[i]; j++) Q[j] = (char)(quals[off + j] + '!');
        Q[lens[i]] = 0;
      } else {
        Q[0] = 0;
      }
      snprintf(H, sizeof(H), "read%u", i + 1);
      gkLibrary  *lib = libs[rlib[i]];
      gkRead     *nr = store->gkStore_addEmptyRead(lib);
      gkReadData *nd = nr->gkRead_encodeSeqQlt(H, S.data(), Q.data(), lib->gkLibrary_defaultQV());
      store->gkStore_stashReadData(nr, nd);
      delete nd;
      off += lens[i];
    }
    store->gkStore_close();
  }

  if (gkpOnly) {
    fprintf(stdout, "GKPSTORE %s\n", gkp.c_str());
    return 0;
  }

  //  ---- 2. globals, as overlapInCore.C main() sets them ---------------------------------
  std::string ovb = work + "/ref.ovb";
  G.Frag_Store_Path = (char *)gkp.c_str();
  G.Outfile_Name    = (char *)ovb.c_str();

  if (skipPath) {
    G.Kmer_Skip_File = fopen(skipPath, "r");
    if (!G.Kmer_Skip_File) die("can't open skip kmers");
  }

  if (G.maxErate > 0.06) {
    G.Use_Window_Filter  = FALSE;
    G.Use_Hopeless_Check = FALSE;
  }
  if (G.Kmer_Len == 0) die("-k needed");

  HSF1 = G.Kmer_Len - (G.Hash_Mask_Bits / 2);
  HSF2 = 2 * G.Kmer_Len - G.Hash_Mask_Bits;
  SV1  = HSF1 + 2;
  SV2  = (HSF1 + HSF2) / 2;
  SV3  = HSF2 - 2;

  omp_set_num_threads(G.Num_PThreads);

  Bit_Equivalent['a'] = Bit_Equivalent['A'] = 0;
  Bit_Equivalent['c'] = Bit_Equivalent['C'] = 1;
  Bit_Equivalent['g'] = Bit_Equivalent['G'] = 2;
  Bit_Equivalent['t'] = Bit_Equivalent['T'] = 3;
  for (int i = 0; i < 256; i++) {
    char ch = tolower((char)i);
    Char_Is_Bad[i] = (ch == 'a' || ch == 'c' || ch == 'g' || ch == 't') ? 0 : 1;
  }

  Hash_Table       = new Hash_Bucket_t [HASH_TABLE_SIZE];
  Hash_Check_Array = new Check_Vector_t [HASH_TABLE_SIZE];
  String_Info      = new Hash_Frag_Info_t [G.Max_Hash_Strings];
  String_Start     = new int64 [G.Max_Hash_Strings];
  String_Start_Size = G.Max_Hash_Strings;
  memset(Hash_Check_Array, 0, sizeof(Check_Vector_t)   * HASH_TABLE_SIZE);
  memset(String_Info,      0, sizeof(Hash_Frag_Info_t) * G.Max_Hash_Strings);
  memset(String_Start,     0, sizeof(int64)            * G.Max_Hash_Strings);

  //  ---- 3. the reference driver ---------------------------------------------------------
  double t0 = now_s();
  OverlapDriver();
  double t1 = now_s();
  if (timeIt)
    fprintf(stdout, "OVERLAPDRIVER_SECONDS %.6f\n", t1 - t0);
  fprintf(stdout, "STATS kmer_hits_without_olap=%lu kmer_hits_with_olap=%lu multi=%lu total=%lu contained=%lu dovetail=%lu\n",
          (unsigned long)Kmer_Hits_Without_Olap_Ct, (unsigned long)Kmer_Hits_With_Olap_Ct,
          (unsigned long)Multi_Overlap_Ct, (unsigned long)Total_Overlaps,
          (unsigned long)Contained_Overlap_Ct, (unsigned long)Dovetail_Overlap_Ct);

  //  the -s file, in the reference's own format (overlapInCore.C:580-588)
  if (statPath) {
    FILE *S = fopen(statPath, "w");
    if (!S) die("can't open -s file");
    fprintf(S, " Kmer hits without olaps = " F_S64 "\n", Kmer_Hits_Without_Olap_Ct);
    fprintf(S, "    Kmer hits with olaps = " F_S64 "\n", Kmer_Hits_With_Olap_Ct);
    fprintf(S, "  Multiple overlaps/pair = " F_S64 "\n", Multi_Overlap_Ct);
    fprintf(S, " Total overlaps produced = " F_S64 "\n", Total_Overlaps);
    fprintf(S, "      Contained overlaps = " F_S64 "\n", Contained_Overlap_Ct);
    fprintf(S, "       Dovetail overlaps = " F_S64 "\n", Dovetail_Overlap_Ct);
    fprintf(S, "Rejected by short window = " F_S64 "\n", Bad_Short_Window_Ct);
    fprintf(S, " Rejected by long window = " F_S64 "\n", Bad_Long_Window_Ct);
    fclose(S);
  }

  //  ---- 4. read the .ovb back with the reference reader ---------------------------------
  gkStore *store = gkStore::gkStore_open(gkp.c_str());
  ovFile  *in    = new ovFile(store, ovb.c_str(), ovFileFull);
  ovOverlap ov(store);
  FILE *O = fopen(outPath, "wb");
  if (!O) die("can't open output");
  uint64_t n = 0;
  while (in->readOverlap(&ov)) {
    uint32_t ids[2] = { ov.a_iid, ov.b_iid };
    uint64_t w[2]   = { ov.dat.dat[0], ov.dat.dat[1] };
    fwrite(ids, 4, 2, O);
    fwrite(w, 8, 2, O);
    n++;
  }
  fclose(O);
  delete in;
  store->gkStore_close();
  fprintf(stdout, "RECORDS %lu\n", (unsigned long)n);
  return 0;
}
