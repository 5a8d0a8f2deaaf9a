// ovl_ovb.h -- overlapInCore's output files, written from ovOverlap records (host code).
//
// Reference:
//   src/overlapInCore/overlapInCore.C:197   Out_BOF = new ovFile(gkpStore, Outfile_Name,
//                                            ovFileFullWrite)
//   src/stores/ovStoreFile.C:198            ovFile::writeOverlap: full format = a_iid, b_iid,
//                                            then each 64-bit dat word as (hi32, lo32)
//                                            (ovOverlapWORDSZ == 64), uint32 words
//   src/stores/ovStoreFile.C:160            writeBuffer: 1 MiB blocks, each snappy-framed
//                                            (ovStore.H:40 defines SNAPPY)
//   src/stores/ovStoreHistogram.C:226       addOverlap: _opr[a]++, _opr[b]++ (FullWrite only)
//   src/stores/ovStoreHistogram.C:322       saveData: "<base>.counts" = uint32 oprLen,
//                                            uint32 opr[oprLen], oprLen = max id seen + 1
//   src/AS_UTL/AS_UTL_fileIO.C:56           AS_UTL_findBaseFileName: cut at the first '.'
//                                            after the last '/'
//   src/overlapInCore/overlapInCore.C:569   the -s statistics text
#pragma once

#include <cinttypes>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

namespace ovl {

// "<base>.counts" for an output path, as createDataName(name, prefix, "counts") builds it
// for a prefix that is not an existing directory.
inline std::string counts_path(const char *ovb_path) {
  std::string b = ovb_path;
  size_t slash = b.rfind('/');
  size_t dot = b.find('.', slash == std::string::npos ? 0 : slash);
  if (dot != std::string::npos) b.resize(dot);
  return b + ".counts";
}

// ovFile's buffer: bufferSize 1 MiB rounded down to a multiple of lcm = 20 * 24 words
// (ovStoreFile.C:66-76) = 262,080 uint32 = 43,680 full records per block.
constexpr uint64_t OVB_BLOCK_RECORDS = 43680;

// One snappy-framed block as ovFile::writeBuffer writes it when SNAPPY is defined
// (ovStore.H:40, ovStoreFile.C:171-182): size_t compressed length, then a raw snappy
// stream.  The stream written here is the format's plain form -- the uncompressed length
// as a varint, then ONE literal element holding every byte -- which snappy::RawUncompress
// (the reference reader, ovStoreFile.C:297) decodes to the same words.  (Google's
// compressor would also emit copy elements; those bytes are an encoder choice, not part of
// what the reader needs.)
inline bool put_snappy_block(FILE *F, const uint32_t *words, size_t nw) {
  const uint64_t n = (uint64_t)nw * 4;
  uint8_t hdr[16];
  size_t h = 0;
  uint64_t v = n;                                      // preamble: varint32 length
  do {
    uint8_t b = v & 0x7f;
    v >>= 7;
    hdr[h++] = b | (v ? 0x80 : 0);
  } while (v);
  const uint64_t m = n - 1;                            // literal tag: length - 1
  if (m < 60) {
    hdr[h++] = (uint8_t)(m << 2);
  } else {
    int nb = m < (1ull << 8) ? 1 : m < (1ull << 16) ? 2 : m < (1ull << 24) ? 3 : 4;
    hdr[h++] = (uint8_t)((59 + nb) << 2);
    for (int i = 0; i < nb; i++) hdr[h++] = (uint8_t)(m >> (8 * i));
  }
  const uint64_t cl = h + n;                           // size_t, little-endian host
  size_t cls = (size_t)cl;
  return fwrite(&cls, sizeof(size_t), 1, F) == 1 && fwrite(hdr, 1, h, F) == h &&
         fwrite(words, 4, nw, F) == nw;
}

// Write records (in the given order) as an ovFileFullWrite .ovb plus its .counts file.
// Returns 0, or -1 with errno set by the failing stdio call.
inline int write_ovb_file(const ovl_record *r, uint64_t n, const char *path, bool counts) {
  FILE *F = fopen(path, "wb");
  if (!F) return -1;
  std::vector<uint32_t> buf;
  buf.reserve(6 * OVB_BLOCK_RECORDS);
  uint32_t max_id = 0;
  bool any = false;
  std::vector<uint32_t> opr;
  for (uint64_t i = 0; i < n; i++) {
    // ovFile::writeOverlap (ovStoreFile.C:198): a_iid, b_iid, dat words hi32 then lo32
    buf.push_back(r[i].a_iid);
    buf.push_back(r[i].b_iid);
    for (int w = 0; w < 2; w++) {
      buf.push_back((uint32_t)(r[i].dat[w] >> 32));
      buf.push_back((uint32_t)(r[i].dat[w] & 0xffffffffu));
    }
    if (buf.size() == 6 * OVB_BLOCK_RECORDS) {
      if (!put_snappy_block(F, buf.data(), buf.size())) { fclose(F); return -1; }
      buf.clear();
    }
    if (counts) {
      uint32_t m = r[i].a_iid > r[i].b_iid ? r[i].a_iid : r[i].b_iid;
      if (opr.size() < (size_t)m + 1) opr.resize((size_t)m + 1 + m / 2, 0);
      if (m > max_id) max_id = m;
      any = true;
      opr[r[i].a_iid]++;
      opr[r[i].b_iid]++;
    }
  }
  if (!buf.empty() && !put_snappy_block(F, buf.data(), buf.size())) { fclose(F); return -1; }
  if (fclose(F) != 0) return -1;
  if (!counts) return 0;
  FILE *C = fopen(counts_path(path).c_str(), "wb");
  if (!C) return -1;
  uint32_t len = any ? max_id + 1 : 0;
  bool ok = fwrite(&len, 4, 1, C) == 1;
  if (ok && len) ok = fwrite(opr.data(), 4, len, C) == len;
  if (fclose(C) != 0) ok = false;
  return ok ? 0 : -1;
}

// The -s statistics file (overlapInCore.C:580-588), counters of one job.
inline int write_stats_file(const ovl_stats &s, const char *path) {
  FILE *F = fopen(path, "w");
  if (!F) return -1;
  // F_S64 = "%" PRId64 (AS_global.H:180)
  fprintf(F, " Kmer hits without olaps = %" PRId64 "\n", (int64_t)s.kmer_hits_without_olap);
  fprintf(F, "    Kmer hits with olaps = %" PRId64 "\n", (int64_t)s.kmer_hits_with_olap);
  fprintf(F, "  Multiple overlaps/pair = %" PRId64 "\n", (int64_t)s.multi_overlaps);
  fprintf(F, " Total overlaps produced = %" PRId64 "\n", (int64_t)s.total_overlaps);
  fprintf(F, "      Contained overlaps = %" PRId64 "\n", (int64_t)s.contained_overlaps);
  fprintf(F, "       Dovetail overlaps = %" PRId64 "\n", (int64_t)s.dovetail_overlaps);
  fprintf(F, "Rejected by short window = %" PRId64 "\n", (int64_t)s.bad_short_window);
  fprintf(F, " Rejected by long window = %" PRId64 "\n", (int64_t)s.bad_long_window);
  return fclose(F) == 0 ? 0 : -1;
}

}  // namespace ovl
