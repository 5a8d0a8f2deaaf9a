"""CPU restatement of MHAP 2.1.2 as the jar canu runs executes it (TEST INFRASTRUCTURE ONLY).

Only tests/, __graft_entry__.smoke() and bench_mhap.py's cpu_baseline leg use this module.

The reference ships MHAP only as compiled classes (src/mhap/mhap-2.1.2.tar ->
mhap-2.1.2.jar; third party: MHAP 2.1.2, Berlin et al. 2015).  The jar is never run or loaded
here and no JVM exists; its class files were READ as data with tools/classfile.py (a
constant-pool + bytecode disassembler) and the methods below restate what that bytecode
does, method by method.  Each function names the class, method and bytecode offsets it
follows ("MinHashSketch.computeNgramMinHashesWeighted @243-328").  The two library hashes
the jar calls are Guava's published Murmur3 functions (com.google.common.hash.Hashing
.murmur3_128(0) / murmur3_32(0), Hasher.putUnencodedChars: each char as 2 little-endian
bytes), restated here from MurmurHash3 (x64_128 / x86_32).  PARITY IS PINNED TO THE
BYTECODE'S MEANING, NOT TO JAR OUTPUTS: no output of the jar exists in the reference and the
jar cannot be run, so a misreading would not be caught by a fixture.

Pipeline (MhapMain -> MinHashSearch), canu's options (OverlapMhap.pm:381-392):
  * every read of at least --min-olap-length bases (SequenceSketchStreamer.enqueue @16-30)
    is sketched forward AND reverse-complemented (enqueue @67-95; Utils.rc is the IUPAC
    complement); a read with no k-mer is skipped (enqueueUntilFound's catch)
  * MinHash sketch of a sequence string (SequenceSketch.<init> @20-39: doRC false):
    MinHashSketch.computeNgramMinHashesWeighted
  * ordered sketch: BottomOverlapSketch.<init>(seq, k', S, false)
  * the index stores both strands of every read (MinHashSearch.<init> @97-175 -> addData:
    dequeue(fwdOnly = !doRC)); queries are forward sketches
  * MinHashSearch.findMatches: shared min-mer count per stored sketch >= --num-min-matches,
    then BottomOverlapSketch.getOverlapInfo >= --threshold -> MatchResult
  * MatchResult.toString: "%s %s %.6f %.6f %d %d %d %d %d %d %d %d"
"""
from __future__ import annotations

import math

import numpy as np

M64 = (1 << 64) - 1
M32 = (1 << 32) - 1
LONG_MAX = (1 << 63) - 1

# Utils$Translate.<clinit>: the complement table Utils.rc uses (IUPAC)
_COMP = {ord(a): ord(b) for a, b in zip("ABCDGHKMNRSTVWY", "TVGHCDMKNYSABWR")}
_COMP_TAB = np.zeros(256, dtype=np.uint8)
for _a, _b in _COMP.items():
    _COMP_TAB[_a] = _b


def default_params(**kw) -> dict:
    """MhapMain's option defaults (<init> option table @100-271) with canu's 'normal'
    correction settings where canu passes them (OverlapMhap.pm:109-150, :381-392)."""
    p = dict(k=16, num_hashes=512, min_matches=3, threshold=0.78, ordered_sketch=1536,
             ordered_k=12, min_olap=500, max_shift=0.2, min_store=0, repeat_weight=0.9,
             repeat_idf_scale=10.0, filter_threshold=1e-5, no_tf=False, no_rc=False)
    p.update(kw)
    return p


# ---- Guava Murmur3 (Hashing.murmur3_128(0) / murmur3_32(0)) ---------------------------
def _rotl64(x, r):
    return ((x << r) | (x >> (64 - r))) & M64


def _fmix64(k):
    k ^= k >> 33
    k = (k * 0xFF51AFD7ED558CCD) & M64
    k ^= k >> 33
    k = (k * 0xC4CEB9FE1A85EC53) & M64
    k ^= k >> 33
    return k


def murmur3_128(data: bytes, seed: int = 0) -> tuple[int, int]:
    """MurmurHash3_x64_128: (h1, h2) as unsigned 64-bit values (Guava's HashCode bytes are h1
    then h2, each little-endian)."""
    c1, c2 = 0x87C37B91114253D5, 0x4CF5AD432745937F
    h1 = h2 = seed & M64
    n = len(data)
    nb = n // 16
    for i in range(nb):
        k1 = int.from_bytes(data[16 * i:16 * i + 8], "little")
        k2 = int.from_bytes(data[16 * i + 8:16 * i + 16], "little")
        k1 = (k1 * c1) & M64
        k1 = _rotl64(k1, 31)
        k1 = (k1 * c2) & M64
        h1 ^= k1
        h1 = _rotl64(h1, 27)
        h1 = (h1 + h2) & M64
        h1 = (h1 * 5 + 0x52DCE729) & M64
        k2 = (k2 * c2) & M64
        k2 = _rotl64(k2, 33)
        k2 = (k2 * c1) & M64
        h2 ^= k2
        h2 = _rotl64(h2, 31)
        h2 = (h2 + h1) & M64
        h2 = (h2 * 5 + 0x38495AB5) & M64
    tail = data[16 * nb:]
    k1 = k2 = 0
    t = len(tail)
    if t > 8:
        k2 = int.from_bytes(tail[8:], "little")
        k2 = (k2 * c2) & M64
        k2 = _rotl64(k2, 33)
        k2 = (k2 * c1) & M64
        h2 ^= k2
    if t > 0:
        k1 = int.from_bytes(tail[:8], "little")
        k1 = (k1 * c1) & M64
        k1 = _rotl64(k1, 31)
        k1 = (k1 * c2) & M64
        h1 ^= k1
    h1 ^= n
    h2 ^= n
    h1 = (h1 + h2) & M64
    h2 = (h2 + h1) & M64
    h1 = _fmix64(h1)
    h2 = _fmix64(h2)
    h1 = (h1 + h2) & M64
    h2 = (h2 + h1) & M64
    return h1, h2


def murmur3_128_h1(data: bytes, seed: int = 0) -> int:
    """MurmurHash3_x64_128's first 64 bits (Guava HashCode.asLong: the first 8 bytes of the
    hash, little-endian = h1), as a signed Java long."""
    h1 = murmur3_128(data, seed)[0]
    return h1 - (1 << 64) if h1 >> 63 else h1


def murmur3_32(data: bytes, seed: int = 0) -> int:
    """MurmurHash3_x86_32 (Guava HashCode.asInt), as a signed Java int."""
    c1, c2 = 0xCC9E2D51, 0x1B873593
    h = seed & M32
    n = len(data)
    nb = n // 4
    for i in range(nb):
        k = int.from_bytes(data[4 * i:4 * i + 4], "little")
        k = (k * c1) & M32
        k = ((k << 15) | (k >> 17)) & M32
        k = (k * c2) & M32
        h ^= k
        h = ((h << 13) | (h >> 19)) & M32
        h = (h * 5 + 0xE6546B64) & M32
    tail = data[4 * nb:]
    if tail:
        k = int.from_bytes(tail, "little")
        k = (k * c1) & M32
        k = ((k << 15) | (k >> 17)) & M32
        k = (k * c2) & M32
        h ^= k
    h ^= n
    h ^= h >> 16
    h = (h * 0x85EBCA6B) & M32
    h ^= h >> 13
    h = (h * 0xC2B2AE35) & M32
    h ^= h >> 16
    return h - (1 << 32) if h >> 31 else h


def _chars(s: bytes) -> bytes:
    """putUnencodedChars: every char as 2 little-endian bytes (ASCII: the byte, then 0)."""
    out = bytearray(2 * len(s))
    out[0::2] = s
    return bytes(out)


def rc(s: bytes) -> bytes:
    """Utils.rc @0-54: reverse, upper case, IUPAC complement (Utils$Translate)."""
    return bytes(_COMP_TAB[np.frombuffer(s.upper()[::-1], dtype=np.uint8)])


def seq_hashes_long(s: bytes, k: int, do_rc: bool = False) -> list[int]:
    """HashUtils.computeSequenceHashesLong(s, k, seed 0, doRC) @0-108: per k-mer the
    murmur3_128 h1 of its chars; with doRC the lexicographically smaller of the k-mer and
    its reverse complement (String.compareTo) is hashed."""
    out = []
    for i in range(len(s) - k + 1):
        km = s[i:i + k]
        if do_rc:
            r = rc(km)
            if r < km:
                km = r
        out.append(murmur3_128_h1(_chars(km)))
    return out


def seq_hashes_int(s: bytes, k: int) -> np.ndarray:
    """HashUtils.computeSequenceHashes(s, k, false) @0-106: murmur3_32 of each k-mer."""
    return np.array([murmur3_32(_chars(s[i:i + k])) for i in range(len(s) - k + 1)],
                    dtype=np.int32)


# ---- the same two hashes over every window of a sequence at once (numpy) ----------------
# Equal, element for element, to seq_hashes_long(s, k, False) / seq_hashes_int(s, k) above
# (tests/test_mhap.py checks both against each other); used by the sketches below for speed.
def _windows(s: bytes, k: int) -> np.ndarray:
    a = np.frombuffer(s, dtype=np.uint8).astype(np.uint64)
    return np.lib.stride_tricks.sliding_window_view(a, k)


def _u64(v: int) -> np.uint64:
    return np.uint64(v & M64)


def _rotl64_np(x, r):
    return (x << np.uint64(r)) | (x >> np.uint64(64 - r))


def _fmix64_np(k):
    k = k ^ (k >> np.uint64(33))
    k = k * _u64(0xFF51AFD7ED558CCD)
    k = k ^ (k >> np.uint64(33))
    k = k * _u64(0xC4CEB9FE1A85EC53)
    return k ^ (k >> np.uint64(33))


def _lanes64(w: np.ndarray, c0: int, n: int) -> np.ndarray:
    """Chars c0 .. c0+n-1 (n <= 4) of every window as little-endian UTF-16 in one u64."""
    v = np.zeros(w.shape[0], dtype=np.uint64)
    for j in range(n):
        v |= w[:, c0 + j] << np.uint64(16 * j)
    return v


def murmur128_h1_windows(s: bytes, k: int) -> np.ndarray:
    """murmur3_128_h1(_chars(window)) of every k-window of s, int64."""
    n = len(s) - k + 1
    if n <= 0:
        return np.zeros(0, dtype=np.int64)
    w = _windows(s, k)
    c1, c2 = _u64(0x87C37B91114253D5), _u64(0x4CF5AD432745937F)
    h1 = np.zeros(n, dtype=np.uint64)
    h2 = np.zeros(n, dtype=np.uint64)
    with np.errstate(over="ignore"):
        nb = k // 8                                   # 16-byte blocks = 8 chars
        for b in range(nb):
            k1 = _lanes64(w, 8 * b, 4)
            k2 = _lanes64(w, 8 * b + 4, 4)
            k1 = _rotl64_np(k1 * c1, 31) * c2
            h1 ^= k1
            h1 = _rotl64_np(h1, 27) + h2
            h1 = h1 * np.uint64(5) + np.uint64(0x52DCE729)
            k2 = _rotl64_np(k2 * c2, 33) * c1
            h2 ^= k2
            h2 = _rotl64_np(h2, 31) + h1
            h2 = h2 * np.uint64(5) + np.uint64(0x38495AB5)
        t = k - 8 * nb                                # tail chars
        if t > 4:
            k2 = _lanes64(w, 8 * nb + 4, t - 4)
            h2 ^= _rotl64_np(k2 * c2, 33) * c1
        if t > 0:
            k1 = _lanes64(w, 8 * nb, min(t, 4))
            h1 ^= _rotl64_np(k1 * c1, 31) * c2
        h1 ^= np.uint64(2 * k)
        h2 ^= np.uint64(2 * k)
        h1 = h1 + h2
        h2 = h2 + h1
        h1 = _fmix64_np(h1)
        h2 = _fmix64_np(h2)
        h1 = h1 + h2
    return h1.view(np.int64)


def murmur32_windows(s: bytes, k: int) -> np.ndarray:
    """murmur3_32(_chars(window)) of every k-window of s, int32."""
    n = len(s) - k + 1
    if n <= 0:
        return np.zeros(0, dtype=np.int32)
    w = _windows(s, k).astype(np.uint32)
    c1, c2 = np.uint32(0xCC9E2D51), np.uint32(0x1B873593)
    h = np.zeros(n, dtype=np.uint32)

    def rotl(x, r):
        return (x << np.uint32(r)) | (x >> np.uint32(32 - r))

    with np.errstate(over="ignore"):
        for b in range(k // 2):                       # 4-byte blocks = 2 chars
            kk = w[:, 2 * b] | (w[:, 2 * b + 1] << np.uint32(16))
            h ^= rotl(kk * c1, 15) * c2
            h = rotl(h, 13) * np.uint32(5) + np.uint32(0xE6546B64)
        if k % 2:
            h ^= rotl(w[:, k - 1] * c1, 15) * c2
        h ^= np.uint32(2 * k)
        h ^= h >> np.uint32(16)
        h = h * np.uint32(0x85EBCA6B)
        h ^= h >> np.uint32(13)
        h = h * np.uint32(0xC2B2AE35)
        h ^= h >> np.uint32(16)
    return h.view(np.int32)


# ---- Guava 19.0 BloomFilter (bundled in the jar: META-INF/maven/com.google.guava) ----------
class GuavaBloom:
    """com.google.common.hash.BloomFilter as the jar's bundled Guava 19.0 builds it, restated
    from its bytecode: create(funnel, n, fpp) @0-136 -> MURMUR128_MITZ_64 with
      numBits = (long) (-n * ln(fpp) / (ln 2 * ln 2))          optimalNumOfBits @0-33
      k = max(1, (int) Math.round((double) numBits / n * ln 2))  optimalNumOfHashFunctions
      BitArray: ceil(numBits / 64) longs, bitSize = 64 x that   BitArray.<init>, bitSize
    put / mightContain (BloomFilterStrategies$2): the murmur3_128 of the funnel's bytes (the
    Long funnel, FrequencyCounts.lambda$0: putLong = 8 little-endian bytes), hash1 = h1
    (lowerEight), hash2 = h2 (upperEight); for i < k the bit (hash1 + i * hash2 (wrapping) &
    Long.MAX_VALUE) % bitSize, word bit >>> 6, bit (int) bit & 63 (Java's << takes 6 bits)."""

    def __init__(self, n: int, fpp: float):
        if n == 0:
            n = 1
        bits = int(float(-n) * math.log(fpp) / (math.log(2.0) * math.log(2.0)))
        self.k = max(1, java_round(bits / float(n) * math.log(2.0)))
        self.words = np.zeros(-(-bits // 64), dtype=np.uint64)
        self.bit_size = 64 * self.words.shape[0]

    def _bits(self, key: int):
        h1, h2 = murmur3_128((key & M64).to_bytes(8, "little"))
        c = h1
        for _ in range(self.k):
            yield (c & LONG_MAX) % self.bit_size
            c = (c + h2) & M64

    def put(self, key: int) -> None:
        for b in self._bits(key):
            self.words[b >> 6] |= np.uint64(1 << (b & 63))

    def might_contain(self, key: int) -> bool:
        return all((int(self.words[b >> 6]) >> (b & 63)) & 1 for b in self._bits(key))


# ---- FrequencyCounts (-f) ----------------------------------------------------------------
class FrequencyCounts:
    """FrequencyCounts.<init>(reader, filterCutoff, offset, removeUnique, noTf, threads,
    range, doRC) @0-429 and its lambda$1 @0-206: line 1 the k-mer count, then "kmer frac"
    lines; a k-mer's key is computeSequenceHashesLong(kmer, len, 0, doRC)[0]; lines with
    frac >= filterCutoff enter fractionCounts (key -> frac) and raise maxValue.
    MhapMain passes offset = --repeat-weight when it lies in [0, 1) (else 0), range =
    --repeat-idf-scale, doRC = !--no-rc.  removeUnique (--supress-noise) > 0 (@189-207): a
    Guava BloomFilter.create(Long funnel, expected = line 1's count (0 -> 1, @171-187),
    1e-5) into which lambda$1 @162-185 puts EVERY line's key, whatever its fraction;
    keepKmer @0-21 asks it only when removeUnique == 1 (2 builds it and never reads it).
    expected: line 1's count (None: the number of lines)."""

    def __init__(self, kmers, fractions, p: dict, expected=None):
        self.remove_unique = int(p.get("supress_noise", 0))
        if self.remove_unique not in (0, 1, 2):
            raise ValueError("Unknown removeUnique option")
        self.valid = None
        if self.remove_unique > 0:
            n = len(kmers) if expected is None else int(expected)
            self.valid = GuavaBloom(n if n > 0 else 1, 1e-5)
        rw = float(p["repeat_weight"])
        self.offset = rw if 0.0 <= rw < 1.0 else 0.0
        self.range = float(p["repeat_idf_scale"])
        self.filter_cutoff = float(p["filter_threshold"])
        self.no_tf = bool(p.get("no_tf", False))
        do_rc = not p.get("no_rc", False)
        self.counts = {}
        self.max_value = -math.inf
        for km, f in zip(kmers, fractions):
            km = km.encode() if isinstance(km, str) else bytes(km)
            key = seq_hashes_long(km, len(km), do_rc)[0]
            if self.valid is not None:
                self.valid.put(key)
            f = float(f)
            if f >= self.filter_cutoff:
                self.max_value = max(self.max_value, f)
                self.counts[key] = f
        self.min_value = self.filter_cutoff
        self.min_idf = self.idf(self.max_value)
        self.max_idf = self.idf(self.min_value)

    def idf(self, x: float) -> float:               # idf(D) @0-14
        v = self.max_value / x - self.offset         # Math.log: NaN below 0 (no -f line
        if v != v or v < 0.0:                         # over the cutoff: maxValue -inf)
            return math.nan
        return math.log(v) if v > 0.0 else -math.inf

    def keep_kmer(self, key: int) -> bool:           # keepKmer @0-21
        return self.valid.might_contain(key) if self.remove_unique == 1 else True

    def is_popular(self, key: int) -> bool:          # isPopular @0-13
        return key in self.counts

    def tf_weight(self, c: int) -> float:            # tfWeight @0-11
        return 1.0 if self.no_tf else float(c)

    def scaled_idf(self, key: int) -> float:         # scaledIdf(J, D) @31-94
        f = self.counts.get(key)
        if f is None:
            return self.range
        idf = self.idf(f)
        scale = (self.max_idf - self.min_idf) / (self.range - 1.0)
        return 1.0 + (idf - self.min_idf) / scale


def i32(x: int) -> int:
    """Java int arithmetic: wrap to a signed 32-bit value."""
    x &= M32
    return x - (1 << 32) if x >> 31 else x


def java_round(x: float) -> int:
    """Math.round(double): the closest long, ties toward positive infinity."""
    r = math.floor(x)
    return int(r + 1) if x - r >= 0.5 else int(r)


# ---- MinHashSketch.computeNgramMinHashesWeighted -----------------------------------------
def minhash(s: bytes, p: dict, fc: FrequencyCounts | None):
    """MinHashSketch.computeNgramMinHashesWeighted(s, k, H, filter, false, repeatWeight)
    @0-476: None when the sequence has no k-mer (@10-26 / @142-160 / @458-473: the read is
    skipped).  Otherwise int32[H]:
      keys = computeSequenceHashesLong(s, k, 0, false); a LinkedOpenHashMap counts each key
        (insertion order = first occurrence)                                  @27-139
      weight: repeatWeight < 0 -> 1 (0 for a popular -f key); a -f table and
        0 <= repeatWeight < 1 -> max(1, round(tfWeight(count) * scaledIdf(key))); else
        the count                                                             @241-324
      per key with weight > 0, x = key; for word 0..H-1, weight times:
        x ^= x << 21; x ^= x >>> 35; x ^= x << 4 (longs); if x < best[word] (signed):
        best[word] = x, hash[word] = (int) key (even word) or (int) (key >>> 32) (odd)
                                                                              @334-445"""
    k, H = p["k"], p["num_hashes"]
    if len(s) - k + 1 < 1:
        return None
    keys = murmur128_h1_windows(s, k)                # = seq_hashes_long(s, k, False)
    if fc is not None and fc.remove_unique == 1:      # keepKmer @70-83: never counted
        keep = np.array([fc.keep_kmer(int(x)) for x in np.unique(keys)], dtype=bool)
        keys = keys[keep[np.searchsorted(np.unique(keys), keys)]] if keys.size else keys
    uk, first, cnt = np.unique(keys, return_index=True, return_counts=True)
    order = np.argsort(first, kind="stable")          # LinkedOpenHashMap: insertion order
    counts = dict(zip(uk[order].tolist(), cnt[order].tolist()))
    if not counts:
        return None
    rw = float(p["repeat_weight"])
    ks, ws = [], []
    for key, c in counts.items():
        w = c
        if rw < 0.0:
            w = 1
            if fc is not None and fc.is_popular(key):
                w = 0
        elif fc is not None and 0.0 <= rw < 1.0:
            w = java_round(fc.tf_weight(w) * fc.scaled_idf(key))
            if w < 1:
                w = 1
        if w <= 0:
            continue
        ks.append(key)
        ws.append(w)
    if not ks:
        return None
    key_u = np.array([kk & M64 for kk in ks], dtype=np.uint64)
    w = np.array(ws, dtype=np.int64)
    out = np.zeros(max(1, H), dtype=np.int32)
    lo = (key_u & np.uint64(M32)).astype(np.uint32).view(np.int32)
    hi = (key_u >> np.uint64(32)).astype(np.uint32).view(np.int32)
    # the keys' chains advance independently, so keys of equal weight are stepped together
    # (a class), each class's minimum scattered back into insertion order per word
    classes = [(int(c), np.flatnonzero(w == c)) for c in np.unique(w)]
    xs = [key_u[idx].copy() for _, idx in classes]
    best = np.empty(key_u.shape[0], dtype=np.int64)
    with np.errstate(over="ignore"):
        for j in range(H):
            for ci, (wc, idx) in enumerate(classes):
                x = xs[ci]
                b = None
                for _ in range(wc):
                    x ^= x << np.uint64(21)
                    x ^= x >> np.uint64(35)
                    x ^= x << np.uint64(4)
                    v = x.view(np.int64)
                    b = v.copy() if b is None else np.minimum(b, v)
                best[idx] = b
            # strictly smaller wins: the first key (insertion order) among equal minima
            i = int(np.argmin(best))
            if best[i] < LONG_MAX:
                out[j] = lo[i] if j % 2 == 0 else hi[i]
    return out


# ---- BottomOverlapSketch ----------------------------------------------------------------
def ordered_sketch(s: bytes, p: dict):
    """BottomOverlapSketch.<init>(s, k', S, false) @0-177: (hashes int32, positions int32) of
    the S smallest k'-mer murmur3_32 hashes, in signed order; equal hashes keep position
    order (IntArrays.radixSortIndirect(perm, hashes, stable)); duplicates stay.  Its
    seqLength = len - k' + 1 (None when < 1)."""
    kk, S = p["ordered_k"], p["ordered_sketch"]
    n = len(s) - kk + 1
    if n <= 0:
        return None
    h = murmur32_windows(s, kk)                      # = seq_hashes_int(s, kk)
    perm = np.argsort(h, kind="stable")[:min(S, n)]
    return h[perm].astype(np.int32), perm.astype(np.int32), n


class _MatchData:
    """BottomOverlapSketch$MatchData: the recorded (pos1, pos2, shift) matches."""

    def __init__(self, sl1: int, sl2: int, max_shift: float):
        self.sl1, self.sl2, self.msp = sl1, sl2, max_shift
        self.p1, self.p2, self.sh = [], [], []
        self._upd = True
        self.median = 0
        self.absmax = 0

    def reset(self):                                 # reset @0-10
        self.p1, self.p2, self.sh = [], [], []
        self._upd = True

    def record(self, a, b, s):                       # recordMatch @66-111
        self.p1.append(a)
        self.p2.append(b)
        self.sh.append(s)
        self._upd = True

    def update(self):                                # performUpdate @0-134
        if not self._upd:
            return
        n = len(self.sh)
        if n > 0:
            # Utils.quickSelect(copy, n / 2, n): the (n/2)-th smallest
            self.median = sorted(self.sh)[n // 2]
            lo = max(0, -self.median)
            hi = min(self.sl1, self.sl2 - self.median)
            olap = max(10, hi - lo)
            self.absmax = min(max(self.sl1, self.sl2), int(olap * self.msp))
        else:
            self.median = 0
            self.absmax = max(self.sl1, self.sl2) + 1
        self._upd = False

    def valid(self):                                 # valid1/2 Lower/Upper
        self.update()
        m, a = self.median, self.absmax
        return (max(0, -m - a), max(0, m - a),
                min(self.sl1, self.sl2 - m + a), min(self.sl2, self.sl1 + m + a))

    def optimize(self):                              # optimizeShifts @0-165
        if not self.sh:
            return
        self.update()
        m = self.median
        p1, p2, sh = self.p1, self.p2, self.sh
        prev = -1
        for i in range(len(sh)):
            if prev >= 0 and p1[prev] == p1[i]:
                if abs(sh[prev] - m) > abs(sh[i] - m):
                    p1[prev], p2[prev], sh[prev] = p1[i], p2[i], sh[i]
            else:
                prev += 1
                p1[prev], p2[prev], sh[prev] = p1[i], p2[i], sh[i]
        del p1[prev + 1:], p2[prev + 1:], sh[prev + 1:]
        self._upd = True

    def edges(self):                                 # computeEdges @0-255
        self.update()
        m, a = self.median, self.absmax
        l1 = l2 = 0x7FFFFFFF
        r1 = r2 = -0x80000000
        c = 0
        for x1, x2, s in zip(self.p1, self.p2, self.sh):
            if abs(s - m) > a:
                continue
            l1, l2, r1, r2 = min(l1, x1), min(l2, x2), max(r1, x1), max(r2, x2)
            c += 1
        if c < 3:
            return None
        # imul / isub (wrapping), i2d, ddiv, Math.round, l2i
        def edge(x, y):
            return i32(java_round(i32(i32(c * x) - y) / float(c - 1)))
        a1 = max(0, edge(l1, r1))
        a2 = min(self.sl1, edge(r1, l1))
        b1 = max(0, edge(l2, r2))
        b2 = min(self.sl2, edge(r2, l2))
        return a1, a2, b1, b2, c


def _record_matching(md: _MatchData, s1, s2):
    """BottomOverlapSketch.recordMatchingKmers @0-450: a merge of the two sorted sketches
    within the valid windows of the current median shift; of a run of equal hashes on both
    sides the first and the last pairs are recorded."""
    v1lo, v2lo, v1hi, v2hi = md.valid()
    m, amax = md.median, md.absmax
    h1s, p1s = s1
    h2s, p2s = s2
    n1, n2 = len(h1s), len(h2s)
    i1 = i2 = 0
    md.reset()
    while i1 < n1 and i2 < n2:
        h1, p1 = int(h1s[i1]), int(p1s[i1])
        h2, p2 = int(h2s[i2]), int(p2s[i2])
        if h1 < h2 or p1 < v1lo or p1 >= v1hi:
            i1 += 1
            continue
        if h2 < h1 or p2 < v2lo or p2 >= v2hi:
            i2 += 1
            continue
        s = p2 - p1
        d = s - m
        if d > amax:
            i1 += 1
            continue
        if d < -amax:
            i2 += 1
            continue
        md.record(p1, p2, s)
        l1 = i1
        j = i1 + 1
        while j < n1 and int(h1s[j]) == h1 and v1lo <= int(p1s[j]) < v1hi:
            l1 = j
            j += 1
        l2 = i2
        j = i2 + 1
        while j < n2 and int(h2s[j]) == h2 and v2lo <= int(p2s[j]) < v2hi:
            l2 = j
            j += 1
        if i1 == l1 and i2 == l2:
            i1 += 1
            i2 += 1
        else:
            a, b = int(p1s[l1]), int(p2s[l2])
            md.record(a, b, b - a)
            i1, i2 = l1 + 1, l2 + 1


def _groups(h1s, h2s):
    """The hashes present in both sorted sketches: [(a0, a1, b0, b1)] index ranges, in
    hash order."""
    u1, i1, c1 = np.unique(h1s, return_index=True, return_counts=True)
    u2, i2, c2 = np.unique(h2s, return_index=True, return_counts=True)
    _, x1, x2 = np.intersect1d(u1, u2, assume_unique=True, return_indices=True)
    return [(int(i1[a]), int(i1[a] + c1[a]), int(i2[b]), int(i2[b] + c2[b]))
            for a, b in zip(x1, x2)]


def _record_matching_groups(md: _MatchData, groups, p1s, p2s):
    """_record_matching, one group of equal hashes at a time: the merge records only
    entries of equal hash and enters every group at the group's first entries on both sides
    (a smaller hash on either side is stepped over, whatever the windows), so the groups are
    independent and their records come out in hash order (tests/test_mhap.py checks this
    form against the merge itself)."""
    v1lo, v2lo, v1hi, v2hi = md.valid()
    m, amax = md.median, md.absmax
    md.reset()
    for a0, a1, b0, b1 in groups:
        i1, i2 = a0, b0
        while i1 < a1 and i2 < b1:
            p1 = p1s[i1]
            if p1 < v1lo or p1 >= v1hi:
                i1 += 1
                continue
            p2 = p2s[i2]
            if p2 < v2lo or p2 >= v2hi:
                i2 += 1
                continue
            d = p2 - p1 - m
            if d > amax:
                i1 += 1
                continue
            if d < -amax:
                i2 += 1
                continue
            md.record(p1, p2, p2 - p1)
            l1 = i1
            while l1 + 1 < a1 and v1lo <= p1s[l1 + 1] < v1hi:
                l1 += 1
            l2 = i2
            while l2 + 1 < b1 and v2lo <= p2s[l2 + 1] < v2hi:
                l2 += 1
            if i1 == l1 and i2 == l2:
                i1 += 1
                i2 += 1
            else:
                md.record(p1s[l1], p2s[l2], p2s[l2] - p1s[l1])
                i1, i2 = l1 + 1, l2 + 1


def overlap_info(A, B, max_shift: float, kk: int, literal: bool = False):
    """BottomOverlapSketch.getOverlapInfo(other, maxShift) @0-211: None (EMPTY) or
    (score, raw, a1, a2, b1, b2).  A, B = (hashes, positions, seqLength).  literal: run the
    jar's merge itself instead of its group form (same records)."""
    md = _MatchData(A[2], B[2], max_shift)
    if literal:
        def rec():
            _record_matching(md, A[:2], B[:2])
    else:
        groups = _groups(A[0], B[0])
        p1s, p2s = A[1].tolist(), B[1].tolist()

        def rec():
            _record_matching_groups(md, groups, p1s, p2s)
    rec()
    if not md.sh:
        return None
    rec()
    if not md.sh:
        return None
    md.optimize()
    if not md.sh:
        return None
    e = md.edges()
    if e is None:
        return None
    a1, a2, b1, b2, c = e
    # computeKBottomSketchJaccard @0-227 (entries of each sketch inside its edge range, in
    # sketch order)
    sel1 = A[0][(A[1] >= a1) & (A[1] <= a2)].tolist()
    sel2 = B[0][(B[1] >= b1) & (B[1] <= b2)].tolist()
    n = min(len(sel1), len(sel2))
    if n == 0:
        J = 0.0
    else:
        i = j = inter = 0
        for _ in range(n):
            if sel1[i] < sel2[j]:
                i += 1
            elif sel1[i] > sel2[j]:
                j += 1
            else:
                inter += 1
                i += 1
                j += 1
        J = inter / float(n)
    # jaccardToIdentity @0-25: exp(-(-1/k * ln(2J / (1 + J))))
    if J > 0.0:
        d = (-1.0 / kk) * math.log(2.0 * J / (1.0 + J))
        score = math.exp(-d)
    else:
        score = 0.0
    return score, float(c), a1, a2, b1, b2


MHAP_DTYPE = np.dtype([("a", "<u4"), ("b", "<u4"), ("erate", "<f8"), ("raw", "<f8"),
                       ("a_bgn", "<i4"), ("a_end", "<i4"), ("a_len", "<i4"), ("o", "<u4"),
                       ("b_bgn", "<i4"), ("b_end", "<i4"), ("b_len", "<i4"),
                       ("count", "<u4")])


def frequency_counts(freq, p: dict):
    """freq: None, (k-mers, fractions) or (k-mers, fractions, line 1's count)."""
    if freq is None:
        return None
    return FrequencyCounts(freq[0], freq[1], p, freq[2] if len(freq) > 2 else None)


def sketch_read(s: bytes, p: dict, fc):
    """SequenceSketch.<init> for one strand: (minhash, ordered) or None (skipped read)."""
    mh = minhash(s, p, fc)
    if mh is None:
        return None
    osk = ordered_sketch(s, p)
    if osk is None:
        return None
    return mh, osk


def read_bytes(rs, i: int) -> bytes:
    o, L = int(rs.offsets[i]), int(rs.lengths[i])
    return rs.bases[o:o + L].tobytes().upper()


def sketches(rs, p: dict, fc=None, reads=None):
    """{(read index, strand 0 fwd / 1 rc): (minhash, ordered, length)} for the reads the
    streamer keeps (>= min_olap bases, sketchable)."""
    out = {}
    for i in (range(rs.nreads) if reads is None else reads):
        L = int(rs.lengths[i])
        if L < p["min_olap"]:
            continue
        s = read_bytes(rs, i)
        f = sketch_read(s, p, fc)
        if f is None:
            continue
        out[(i, 0)] = (f[0], f[1], L)
        if not p.get("no_rc", False):
            r = sketch_read(rc(s), p, fc)
            if r is not None:
                out[(i, 1)] = (r[0], r[1], L)
    return out


def sketch_rows(rs, p: dict, freq=None, reads=None):
    """The sketches in the library's layout (canu_mhap.h mhap_sketch_buffers): minhash
    int32 [n][2][H], ordered uint64 [n][2][S] ((hash ^ 0x80000000) << 32 | position),
    ocount uint32 [n][2] (0: strand not stored); rows of reads not sketched stay zero."""
    fc = frequency_counts(freq, p)
    n, H, S = rs.nreads, p["num_hashes"], p["ordered_sketch"]
    mh = np.zeros((n, 2, H), dtype=np.int32)
    od = np.zeros((n, 2, S), dtype=np.uint64)
    oc = np.zeros((n, 2), dtype=np.uint32)
    for (i, st), (m, (h, pos, _), _) in sketches(rs, p, fc, reads).items():
        mh[i, st] = m
        oc[i, st] = h.shape[0]
        od[i, st, :h.shape[0]] = ((h.view(np.uint32) ^ np.uint32(0x80000000)).astype(np.uint64)
                                  << np.uint64(32)) | pos.astype(np.uint64)
    return mh, od, oc


def find_matches(q_id, q, store: dict, p: dict, to_self: bool):
    """MinHashSearch.findMatches(query, toSelf) @0-610: the stored sketches sharing at
    least --num-min-matches min-mers with the query (per hash function j: query[j] equal
    to the stored sketch's [j]), then the length / self rules and the second stage.
    Returns [(target id, shared count, overlap info)] for accepted targets."""
    out = []
    qmh, qosk, qlen = q
    ms = p.get("min_store", 0)
    for t_id, (tmh, tosk, tlen) in store.items():
        if t_id[0] == q_id[0]:
            continue
        cnt = int((qmh == tmh).sum())
        if cnt < p["min_matches"]:
            continue
        if tlen < ms and qlen < ms:                          # @393-416
            continue
        if to_self and t_id[0] > q_id[0] and tlen >= ms and qlen >= ms:   # @419-462
            continue
        if to_self and tlen < ms and qlen >= ms:             # @465-492
            continue
        oi = overlap_info(qosk, tosk, p.get("max_shift", 0.2), p["ordered_k"])
        if oi is None:
            continue
        if oi[0] >= p["threshold"]:
            out.append((t_id, cnt, oi))
    return out


def match_record(q_id, t_id, cnt, oi, qlen: int, tlen: int, first_iid: int):
    """MatchResult.<init> @0-179: reverse-strand coordinates mirrored as len - x - 1, the
    score capped at 1; the row of MatchResult.toString (+ the first-stage count)."""
    score, raw, a1, a2, b1, b2 = oi
    if q_id[1]:
        a1, a2 = qlen - a2 - 1, qlen - a1 - 1
    if t_id[1]:
        b1, b2 = tlen - b2 - 1, tlen - b1 - 1
    score = min(score, 1.0)
    return (first_iid + q_id[0], first_iid + t_id[0], 1.0 - score, raw, a1, a2, qlen,
            t_id[1], b1, b2, tlen, cnt)


def run(rs, p: dict, freq=None, q_range=None, t_range=None, to_self: bool = True) -> np.ndarray:
    """The jar's compute step over rs: the stored reads t_range (0-based [lo, hi), default
    all; both strands, AbstractMatchSearch's store) searched by the forward sketches of the
    query reads q_range (default: the stored reads, the -s self search).  to_self: the self
    search (MinHashSearch.findMatches toSelf: only stored reads of smaller ID); False: the -q
    search.  Rows sorted by (a, b, o)."""
    fc = frequency_counts(freq, p)
    t_lo, t_hi = t_range if t_range is not None else (0, rs.nreads)
    q_lo, q_hi = q_range if q_range is not None else (t_lo, t_hi)
    store = sketches(rs, p, fc, range(t_lo, t_hi))
    qs = [i for i in range(q_lo, q_hi) if not t_lo <= i < t_hi]
    queries = {k: v for k, v in store.items() if k[1] == 0 and q_lo <= k[0] < q_hi}
    queries.update(sketches(rs, dict(p, no_rc=True), fc, qs))
    rows = []
    for q_id in sorted(queries):
        for t_id, cnt, oi in find_matches(q_id, queries[q_id], store, p, to_self):
            rows.append(match_record(q_id, t_id, cnt, oi, queries[q_id][2], store[t_id][2],
                                     rs.first_iid))
    a = np.array(rows, dtype=MHAP_DTYPE)
    return a[np.lexsort((a["o"], a["b"], a["a"]))] if a.size else a


def run_self(rs, p: dict, freq=None) -> np.ndarray:
    """The jar's -s block against itself."""
    return run(rs, p, freq=freq)
