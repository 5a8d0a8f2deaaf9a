/*
 * store_harness.cpp -- the REFERENCE ovStore build, compiled from its own sources under
 * /root/reference/src/stores by oracle/Makefile (outputs into oracle/_ref/ only).
 *
 *   TEST INFRASTRUCTURE ONLY: the checker for the configs[4] host merge (per-rank .ovb
 *   files -> one ovStore), tests/test_store_merge.py.
 *
 *   ovs_ref --build <gkpStore> <store> <in.ovb>...
 *       restates ovStoreBuild.C main() (:473-655) with every overlap in one bucket: the
 *       reference's ovStoreFilter (-e 1.0, :494) makes each input overlap's forward and
 *       reverse copies and its for-UTG/OBT/DUP flags (:522-538), the kept copies are sorted
 *       with ovOverlap::operator< (__gnu_sequential::sort, :637) and written in that order by
 *       the reference's ovStoreWriter (:644-652).  One bucket instead of ovStoreBuild's
 *       IID-range buckets changes nothing in the store: its buckets are IID ranges written in
 *       increasing order, each sorted the same way.  main() itself is not called because it
 *       starts with AS_configure() (AS_global.C, next to a build-generated header).
 *   ovs_ref --dump <gkpStore> <store> <out.bin>
 *       reads the store back with the reference's ovStore::readOverlap in store order and
 *       dumps {uint32 a_iid, uint32 b_iid, uint64 dat[2]} (24 B) per overlap.
 */

#include "AS_global.H"
#include "gkStore.H"
#include "ovStore.H"

#include <algorithm>
#include <parallel/algorithm>
#include <vector>

static void die(const char *m) {
  fprintf(stderr, "ovs_ref: %s\n", m);
  exit(1);
}

static int build_store(const char *gkpName, const char *ovlName, int nin, char **inputs) {
  gkStore       *gkp    = gkStore::gkStore_open(gkpName);
  const uint32   maxIID = gkp->gkStore_getNumReads() + 1;
  ovStoreFilter *filter = new ovStoreFilter(gkp, 1.0);
  std::vector<ovOverlap> kept;
  for (int i = 0; i < nin; i++) {
    ovOverlap foverlap(gkp), roverlap(gkp);
    ovFile   *in = new ovFile(gkp, inputs[i], ovFileFull);
    while (in->readOverlap(&foverlap)) {
      filter->filterOverlap(foverlap, roverlap);      //  copies f into r
      if (foverlap.dat.ovl.forUTG || foverlap.dat.ovl.forOBT || foverlap.dat.ovl.forDUP)
        kept.push_back(foverlap);
      if (roverlap.dat.ovl.forUTG || roverlap.dat.ovl.forOBT || roverlap.dat.ovl.forDUP)
        kept.push_back(roverlap);
    }
    delete in;
  }
  delete filter;
  for (const ovOverlap &o : kept)
    if (o.a_iid == 0 || o.b_iid == 0 || o.a_iid >= maxIID || o.b_iid >= maxIID)
      die("overlap IDs out of range");
  __gnu_sequential::sort(kept.begin(), kept.end());
  ovStoreWriter *store = new ovStoreWriter(ovlName, gkp);
  for (ovOverlap &o : kept)
    store->writeOverlap(&o);
  delete store;
  gkp->gkStore_close();
  fprintf(stdout, "STORED %lu\n", (unsigned long)kept.size());
  return 0;
}

static int dump_store(const char *gkpName, const char *ovlName, const char *outPath) {
  gkStore  *gkp = gkStore::gkStore_open(gkpName);
  ovStore  *ovs = new ovStore(ovlName, gkp);
  ovOverlap ov(gkp);
  FILE     *O = fopen(outPath, "wb");
  if (!O) die("can't open output");
  uint64_t n = 0;
  while (ovs->readOverlap(&ov)) {
    uint32_t ids[2] = { ov.a_iid, ov.b_iid };
    uint64_t w[2]   = { ov.dat.dat[0], ov.dat.dat[1] };
    fwrite(ids, 4, 2, O);
    fwrite(w, 8, 2, O);
    n++;
  }
  fclose(O);
  delete ovs;
  gkp->gkStore_close();
  fprintf(stdout, "RECORDS %lu\n", (unsigned long)n);
  return 0;
}

int main(int argc, char **argv) {
  if (argc >= 5 && strcmp(argv[1], "--build") == 0)
    return build_store(argv[2], argv[3], argc - 4, argv + 4);
  if (argc == 5 && strcmp(argv[1], "--dump") == 0)
    return dump_store(argv[2], argv[3], argv[4]);
  die("usage: ovs_ref --build <gkpStore> <store> <in.ovb>... | --dump <gkpStore> <store> <out.bin>");
  return 1;
}
