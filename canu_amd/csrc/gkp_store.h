// gkp_store.h -- read-only access to a canu gkpStore directory (host code, no HIP).
//
// overlapInCore opens the store with gkStore::gkStore_open(path) (overlapInCore.C:195) and
// pulls every read through gkStore_getRead / gkStore_loadReadData.  This is a from-scratch
// reader of the same on-disk layout (it does not link the reference's gkStore.C):
//
//   <store>/info       gkStoreInfo (src/stores/gkStore.H:350-401): u64 magic "canu:GKP",
//                      u64 version, u32 sizeof(gkLibrary), sizeof(gkRead), library-ID bits,
//                      library-name size, read-ID bits, read-length bits, unused,
//                      numLibraries, numReads (56 bytes with padding)
//   <store>/reads      gkRead[numReads + 1] indexed by read ID (gkStore.H:333-338):
//                      word 0 = readID:37 | libraryID:6 | seqLen:21 (low bits first),
//                      word 1 = mPtr:48 | pID:16  (mPtr = byte offset into blobs)
//   <store>/blobs      per read at mPtr: "BLOB" u32 len, then chunks (tag, u32 padded len,
//                      data) until "STOP" (gkStore.C:50-156, encoder gkStore.C:285-430):
//                      VERS, NAME, 2SEQ (2-bit ACGT, 4 bases per byte, first base in the
//                      high bits; gkStoreEncode.C:81), USEQ (raw bases), UQLT (QV - '!'),
//                      QVAL (one QV for every base)
//
// The store is opened read-only, as the reference does (gkStore.C:694-727).
#pragma once

#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

namespace gkp {

struct Info {                      // gkStoreInfo as it lies in <store>/info
  uint64_t magic, version;
  uint32_t library_size, read_size, max_libraries_bits, library_name_size;
  uint32_t max_read_bits, max_readlen_bits, unused;
  uint32_t num_libraries, num_reads;
};
static_assert(sizeof(Info) == 56, "gkStoreInfo is 56 bytes on disk");

constexpr uint64_t GK_MAGIC = 0x504b473a756e6163ull;   // "canu:GKP"
constexpr uint32_t LIB_BITS = 6, READLEN_BITS = 21, READ_BITS = 64 - 21 - 6;
constexpr uint32_t LIBRARY_SIZE = 128 + 10 * 4;        // gkLibrary: name[128] + 10 uint32
constexpr uint32_t READ_SIZE = 16;

class Store {
 public:
  ~Store() { close(); }

  // Opens <path>; false with a message in err when the store is missing or was written
  // with parameters this reader (and overlapInCore) cannot use (gkStore.C:612-641).
  bool open(const std::string &path, std::string &err) {
    close();
    path_ = path;
    FILE *I = fopen((path + "/info").c_str(), "rb");
    if (!I) { err = "can't open '" + path + "/info'"; return false; }
    bool ok = fread(&info_, sizeof(Info), 1, I) == 1;
    fclose(I);
    if (!ok) { err = "short read of '" + path + "/info'"; return false; }
    if (info_.magic != GK_MAGIC) { err = "'" + path + "' is not a canu gkpStore"; return false; }
    if (info_.library_size != LIBRARY_SIZE || info_.read_size != READ_SIZE ||
        info_.max_libraries_bits != LIB_BITS || info_.library_name_size != 128 ||
        info_.max_read_bits != READ_BITS || info_.max_readlen_bits != READLEN_BITS) {
      err = "store parameters are incompatible (gkLibrary / gkRead sizes or bit widths)";
      return false;
    }
    FILE *R = fopen((path + "/reads").c_str(), "rb");
    if (!R) { err = "can't open '" + path + "/reads'"; return false; }
    reads_.resize(2ull * (info_.num_reads + 1));
    ok = fread(reads_.data(), 16, info_.num_reads + 1, R) == info_.num_reads + 1;
    fclose(R);
    if (!ok) { err = "short read of '" + path + "/reads'"; return false; }
    blobs_ = fopen((path + "/blobs").c_str(), "rb");
    if (!blobs_) { err = "can't open '" + path + "/blobs'"; return false; }
    return true;
  }

  void close() {
    if (blobs_) fclose(blobs_);
    blobs_ = nullptr;
  }

  uint32_t num_reads() const { return info_.num_reads; }
  uint32_t num_libraries() const { return info_.num_libraries; }

  uint32_t read_id(uint32_t id) const { return (uint32_t)(reads_[2 * id] & ((1ull << READ_BITS) - 1)); }
  uint32_t library(uint32_t id) const {
    return (uint32_t)((reads_[2 * id] >> READ_BITS) & ((1u << LIB_BITS) - 1));
  }
  uint32_t length(uint32_t id) const { return (uint32_t)(reads_[2 * id] >> (READ_BITS + LIB_BITS)); }
  uint64_t mptr(uint32_t id) const { return reads_[2 * id + 1] & ((1ull << 48) - 1); }

  // gkStore_loadReadData: the read's bases (as stored: 2SEQ decodes to upper case) and
  // QVs (integers, '!' already removed).  Returns false with a message on a malformed blob.
  bool load(uint32_t id, std::string &seq, std::string &qlt, std::string &err) {
    const uint32_t L = length(id);
    seq.assign(L, 0);
    qlt.assign(L, 0);
    if (fseeko(blobs_, (off_t)mptr(id), SEEK_SET) != 0) { err = "seek in blobs"; return false; }
    uint8_t hdr[8];
    if (fread(hdr, 1, 8, blobs_) != 8 || memcmp(hdr, "BLOB", 4) != 0) {
      err = "read " + std::to_string(id) + ": no BLOB at its offset";
      return false;
    }
    uint32_t blen;
    memcpy(&blen, hdr + 4, 4);
    buf_.resize(blen);
    if (blen && fread(buf_.data(), 1, blen, blobs_) != blen) { err = "short blob"; return false; }
    size_t p = 0;
    bool have_seq = false;
    while (true) {
      if (p + 8 > buf_.size()) { err = "read " + std::to_string(id) + ": blob without STOP"; return false; }
      const uint8_t *tag = buf_.data() + p;
      uint32_t clen;
      memcpy(&clen, tag + 4, 4);
      const uint8_t *dat = tag + 8;
      if (!memcmp(tag, "STOP", 4)) break;
      if (p + 8 + clen > buf_.size()) { err = "chunk past the blob"; return false; }
      if (!memcmp(tag, "VERS", 4) || !memcmp(tag, "NAME", 4) || !memcmp(tag, "QSEQ", 4)) {
        // not needed for overlaps
      } else if (!memcmp(tag, "USEQ", 4)) {
        if (clen < L) { err = "USEQ shorter than the read"; return false; }
        memcpy(&seq[0], dat, L);
        have_seq = true;
      } else if (!memcmp(tag, "UQLT", 4)) {
        if (clen < L) { err = "UQLT shorter than the read"; return false; }
        memcpy(&qlt[0], dat, L);
      } else if (!memcmp(tag, "2SEQ", 4)) {
        static const char acgt[4] = {'A', 'C', 'G', 'T'};
        if ((uint64_t)clen * 4 < L) { err = "2SEQ shorter than the read"; return false; }
        for (uint32_t i = 0; i < L; i++) seq[i] = acgt[(dat[i >> 2] >> (6 - 2 * (i & 3))) & 3];
        have_seq = true;
      } else if (!memcmp(tag, "QVAL", 4)) {
        uint32_t qv;
        memcpy(&qv, dat, 4);
        memset(&qlt[0], (int)(char)qv, L);
      } else {
        // 3SEQ / 4QLT / 5QLT have no encoder in this canu (gkStoreEncode.C:120-165) and
        // the reference's decoders leave the buffers untouched; anything else it asserts on
        err = "read " + std::to_string(id) + ": unsupported blob chunk '" +
              std::string((const char *)tag, 4) + "'";
        return false;
      }
      p += 8 + clen;
    }
    if (!have_seq && L) { err = "read " + std::to_string(id) + " has no sequence chunk"; return false; }
    return true;
  }

 private:
  std::string path_;
  Info info_{};
  std::vector<uint64_t> reads_;
  std::vector<uint8_t> buf_;
  FILE *blobs_ = nullptr;
};

}  // namespace gkp
