"""The MHAP stage (include/canu_mhap.h, canu_amd/csrc/mhap.hip) against the jar's semantics.

The reference ships MHAP 2.1.2 only as a jar (src/mhap/mhap-2.1.2.tar): class files, no
sources, no fixtures, and no JVM here.  Its bytecode was read as data (tools/classfile.py)
and restated method by method in oracle/mhap_jar.py.  What pins what:
  * the two library hashes the jar calls (Guava Murmur3_x64_128 / Murmur3_x86_32), by the
    published test vectors of MurmurHash3;
  * the restatement's faster forms (numpy window hashes, the group form of the ordered-
    sketch merge), against the literal restatement of the bytecode;
  * the output format, by the reference's own consumer: every line goes through
    mhapConvert (src/mhap/mhapConvert.C, compiled from the reference source into
    oracle/_ref/) and comes out as the ovOverlap records the line describes;
  * the GPU path, against the restatement: integers bit-exact, erate bit-exact (the
    identity is computed on the host with the same libm calls as the oracle).
PARITY PINNED TO THE BYTECODE'S MEANING, NOT TO JAR OUTPUTS (none exist in the reference).
CPU tests run here; @gpu tests on the MI355X box."""
import os
import re

import numpy as np
import pytest

import mhap_jar as M
import oracle
from canu_amd import mhap
from canu_amd.synth import ReadSet, synth_reads

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "canu_mhap.h")
FIELDS = ("a", "b", "erate", "raw", "a_bgn", "a_end", "a_len", "o", "b_bgn", "b_end",
          "b_len", "count")


def _reads(n=60, L=3000, cov=12, err=0.04, seed=3, **kw):
    return synth_reads(n_reads=n, read_len=L, genome_len=int(n * L / cov), error_rate=err,
                       seed=seed, **kw)


@pytest.fixture(scope="module")
def small():
    return _reads()


@pytest.fixture(scope="module")
def small_oracle(small):
    return M.run(small, M.default_params())


# ------------------------------------------------------------------------------- CPU ----

def test_header_declares_the_python_exports():
    src = re.sub(r"/\*.*?\*/", "", open(HEADER).read(), flags=re.S)
    assert sorted(set(re.findall(r"\b(mhap_[a-z_]+)\s*\(", src))) == sorted(mhap.EXPORTS)


def test_library_exports_every_declared_symbol(built):
    lib = mhap.load_library()
    assert [f for f in mhap.EXPORTS if not hasattr(lib, f)] == []
    assert lib.mhap_abi_version() == mhap.ABI_VERSION == 7


def test_record_layout_matches_the_header(built):
    """mhap_record: 56 bytes, the fields at the C offsets."""
    dt = mhap.MHAP_DTYPE
    assert dt.itemsize == 56
    assert [dt.fields[f][1] for f in ("a", "b", "erate", "raw", "a_bgn", "o", "b_len", "count")] \
        == [0, 4, 8, 16, 24, 36, 48, 52]


def test_params_init_is_canu_normal_and_jar_defaults(built):
    lib = mhap.load_library()
    p = mhap._Params()
    lib.mhap_params_init(p)
    d = mhap.MhapParameters()
    assert (p.k, p.num_hashes, p.min_matches, p.ordered_sketch, p.ordered_k, p.min_olap) == \
        (d.k, d.num_hashes, d.num_min_matches, d.ordered_sketch_size, d.ordered_kmer_size,
         d.min_olap_length) == (16, 512, 3, 1536, 12, 500)
    assert abs(p.threshold - 0.78) < 1e-12
    assert (p.max_shift, p.min_store, p.no_rc) == (d.max_shift, d.min_store_length, 0) == \
        (0.2, 0, 0)
    w = mhap._Weighting()
    lib.mhap_weighting_init(w)
    # MhapMain's option table: --repeat-weight 0.9, --repeat-idf-scale 3, --filter-threshold 1e-5
    assert (w.repeat_weight, w.repeat_idf_scale, w.filter_threshold, w.no_tf, w.supress_noise) \
        == (0.9, 3.0, 1e-5, 0, 0)
    assert (d.repeat_weight, d.repeat_idf_scale, d.filter_threshold) == (0.9, 3.0, 1e-5)


def test_sensitivity_presets():
    """OverlapMhap.pm:109-150."""
    lo = mhap.MhapParameters.sensitivity("low")
    assert (lo.num_hashes, lo.num_min_matches, lo.ordered_sketch_size, lo.ordered_kmer_size) == \
        (256, 3, 1000, 14)
    hi = mhap.MhapParameters.sensitivity("high", nanopore=True)
    assert hi.num_hashes == 768 and hi.num_min_matches == 2 and abs(hi.threshold - 0.78) < 1e-12
    utg = mhap.MhapParameters.sensitivity("normal", tag="utg")
    assert (utg.num_hashes, utg.num_min_matches, utg.ordered_kmer_size) == (128, 5, 18)
    with pytest.raises(ValueError):
        mhap.MhapParameters.sensitivity("fast")


def test_parse_canu_command_line():
    """The jar's options as canu writes them (OverlapMhap.pm:380-395), weighting included."""
    argv = ("--repeat-weight 0.9 --repeat-idf-scale 10 -k 16 --num-hashes 768 "
            "--num-min-matches 2 --threshold 0.73 --filter-threshold 0.000005 "
            "--ordered-sketch-size 1536 --ordered-kmer-size 12 --min-olap-length 500 "
            "--num-threads 8 -s ./blocks/000001.dat -q queries/000001").split()
    p, io = mhap.parse_mhap_args(argv)
    assert (p.k, p.num_hashes, p.num_min_matches, p.ordered_sketch_size) == (16, 768, 2, 1536)
    assert abs(p.threshold - 0.73) < 1e-12 and p.min_olap_length == 500
    assert (p.repeat_weight, p.repeat_idf_scale, p.filter_threshold) == (0.9, 10.0, 0.000005)
    assert not p.no_tf and not p.no_rc and p.max_shift == 0.2
    assert io["-s"] == "./blocks/000001.dat" and io["--num-threads"] == "8"
    assert mhap.parse_mhap_args(["--no-tf"])[0].no_tf
    q = mhap.parse_mhap_args(["--max-shift", "0.3", "--min-store-length", "900", "--no-rc"])[0]
    assert (q.max_shift, q.min_store_length, q.no_rc) == (0.3, 900, True)
    assert mhap.parse_mhap_args(["--supress-noise", "2"])[0].supress_noise == 2
    with pytest.raises(mhap.MhapError):
        mhap.parse_mhap_args(["--supress-noise", "3"])
    with pytest.raises(mhap.MhapError):
        mhap.parse_mhap_args(["--bogus"])


def test_frequency_file(tmp_path):
    """The -f file canu writes (Meryl.pm:699-716): gzip, a count line, kmer<TAB>fraction."""
    import gzip
    path = str(tmp_path / "f.ignore.gz")
    with gzip.open(path, "wt") as f:
        f.write("4\nACGTACGTACGTACGT\t1.000000e-03\nACGTACGTACGTACGT\t1.000000e-03\n"
                "AAAAAAAAAAAAAAAA\t5.000000e-06\nTTTTTTTTTTTTTTTT\t5.000000e-06\n")
    km, fr = mhap.read_frequency_file(path, 16)
    assert km[0] == "ACGTACGTACGTACGT" and len(km) == 4 and fr[2] == 5e-6


def test_murmur3_published_vectors():
    """Guava's Murmur3 functions are MurmurHash3_x64_128 / x86_32 (seed 0): the published
    test vectors of both, and Guava's hashUnencodedChars = the chars as UTF-16LE bytes."""
    assert M.murmur3_32(b"") == 0
    assert M.murmur3_32(b"hello") & M.M32 == 0x248BFA47
    assert M.murmur3_32(b"abc") & M.M32 == 0xB3DD93FA
    assert M.murmur3_32(b"The quick brown fox jumps over the lazy dog") & M.M32 == 0x2E4FF723
    assert M.murmur3_128_h1(b"") == 0
    assert M.murmur3_128_h1(b"hello") & M.M64 == 0xCBD8A7B341BD9B02
    # Guava's own test vector: "6c1b07bc7bbc4be347939ac4a93c437a" = bytes of (h1, h2)
    assert M.murmur3_128_h1(b"The quick brown fox jumps over the lazy dog") & M.M64 == \
        0xE34BBC7BBC071B6C
    assert M._chars(b"AC") == b"A\x00C\x00"
    # the whole 128 bits (h1, h2), which Guava's BloomFilter strategy reads
    assert M.murmur3_128(b"hello") == (0xCBD8A7B341BD9B02, 0x5B1E906A48AE1D19)
    assert M.murmur3_128(b"The quick brown fox jumps over the lazy dog") == \
        (0xE34BBC7BBC071B6C, 0x7A433CA9C49A9347)


def test_guava_bloom_filter_restatement():
    """--supress-noise's filter (Guava 19.0 BloomFilter, MURMUR128_MITZ_64, as bundled in the
    jar): sizing by optimalNumOfBits / optimalNumOfHashFunctions, whole 64-bit words; every
    key put is found; ~1e-5 false positives; FrequencyCounts puts every line's key (any
    fraction) and keepKmer asks the filter only for removeUnique 1."""
    b = M.GuavaBloom(1000, 1e-5)
    assert b.bit_size == 24000 and b.words.shape[0] == 375 and b.k == 17   # 23,962 bits
    b0 = M.GuavaBloom(0, 1e-5)                       # a count line of 0 reads as 1
    assert b0.bit_size == 64 and b0.k == 16            # 23 bits, round(15.9)
    rng = np.random.default_rng(3)
    keys = [int(x) for x in rng.integers(-2**63, 2**63 - 1, 1000, dtype=np.int64)]
    for x in keys:
        b.put(x)
    assert all(b.might_contain(x) for x in keys)
    other = [int(x) for x in rng.integers(-2**63, 2**63 - 1, 20000, dtype=np.int64)]
    assert sum(b.might_contain(x) for x in other) <= 3
    p = M.default_params(filter_threshold=1e-5)
    km = ["AAAAAAAAAAAAAAAC", "ACGTACGTACGTACGA", "CCCCCCCCCCCCCCCA"]
    fr = [1e-3, 1e-7, 1e-6]                           # two lines below the cutoff
    keys = [M.seq_hashes_long(x.encode(), 16, True)[0] for x in km]
    for mode in (1, 2):
        fc = M.FrequencyCounts(km, fr, dict(p, supress_noise=mode), expected=3)
        assert len(fc.counts) == 1 and all(fc.valid.might_contain(x) for x in keys)
        assert fc.keep_kmer(keys[2]) and (fc.keep_kmer(12345) == (mode == 2))
    assert M.FrequencyCounts(km, fr, p).keep_kmer(12345)


def test_window_hashes_equal_the_scalar_restatement():
    rng = np.random.default_rng(1)
    for k in list(range(1, 33)):
        s = bytes(rng.choice(list(b"ACGTNacgRY"), size=70).astype(np.uint8))
        assert np.array_equal(M.murmur128_h1_windows(s, k),
                              np.array(M.seq_hashes_long(s, k), dtype=np.int64)), k
        assert np.array_equal(M.murmur32_windows(s, k), M.seq_hashes_int(s, k)), k
    assert M.murmur128_h1_windows(b"ACG", 4).shape == (0,)


def test_reverse_complement_is_utils_rc():
    """Utils.rc: reverse, upper case, IUPAC complement (Utils$Translate); other bytes -> 0."""
    assert M.rc(b"ACGTN") == b"NACGT"
    assert M.rc(b"acgt") == b"ACGT"
    assert M.rc(b"RYKMBDHVSW") == b"WSBDHVKMRY"
    assert M.rc(b"X") == b"\x00"


def test_java_arithmetic():
    assert [M.java_round(x) for x in (0.5, 1.5, 2.4999999, -0.5, -1.5, -2.6)] == \
        [1, 2, 2, 0, -1, -3]
    assert M.i32(2 ** 31) == -2 ** 31 and M.i32(-1) == -1 and M.i32(3 * 2 ** 32 + 5) == 5
    # String.format("%.6f"): the shortest decimal, half up (C's printf rounds the binary value)
    assert mhap.java_fixed6(5e-7) == "0.000001" and "%.6f" % 5e-7 == "0.000000"
    assert mhap.java_fixed6(116.0) == "116.000000"
    assert mhap.java_fixed6(0.0) == "0.000000"
    assert mhap.java_fixed6(0.06954645004) == "0.069546"
    assert mhap.java_fixed6(1.0000005) == "1.000001"


def _random_sketch(rng, n, sl, nh):
    """An ordered sketch with many repeated hashes: (hashes sorted, positions by hash then
    position, seqLength)."""
    h = rng.integers(-nh, nh, n).astype(np.int32)
    pos = rng.choice(sl, n, replace=False).astype(np.int32)
    o = np.lexsort((pos, h))
    return h[o], pos[o], sl


def test_group_form_of_the_merge_equals_the_literal_merge():
    """overlap_info with the jar's merge itself (recordMatchingKmers, literal) and with its
    group form (what the GPU evaluates): the same records, edges and score, over random
    sketches with heavy hash duplication and every shift regime."""
    rng = np.random.default_rng(5)
    diffs = 0
    for trial in range(400):
        nh = int(rng.choice([3, 8, 40, 400]))
        A = _random_sketch(rng, int(rng.integers(1, 120)), int(rng.integers(130, 900)), nh)
        B = _random_sketch(rng, int(rng.integers(1, 120)), int(rng.integers(130, 900)), nh)
        ms = float(rng.choice([0.05, 0.2, 0.5, -0.5]))
        lit = M.overlap_info(A, B, ms, 12, literal=True)
        grp = M.overlap_info(A, B, ms, 12)
        assert lit == grp, trial
        diffs += lit is not None
    assert diffs > 100


def test_bit_plane_draws_equal_the_xorshift_chain():
    """The bit-sliced draws of k_mh_bitslice (mhap.hip), restated on the host: 32 chains in
    64 planes (plane b, bit p = bit b of chain p), a xorshift64 step as plane XORs -- x ^= x <<
    21 is plane b ^= plane b - 21 from the top down, x ^= x >>> 35 plane b ^= plane b + 35 from
    the bottom up, x ^= x << 4 plane b ^= plane b - 4 from the top down -- equals the jar's
    chain (MinHashSketch.computeNgramMinHashesWeighted @334-445) draw for draw, and the
    filter (the top Z = clz(T ^ 2^63) planes of x ^ 2^63 all zero) lets every draw <= T
    through."""
    rng = np.random.default_rng(7)
    x = rng.integers(0, 2**63, size=32, dtype=np.uint64) * np.uint64(2) + np.uint64(1)
    planes = [np.uint32(0)] * 64
    for b in range(64):
        planes[b] = np.uint32(sum(int((int(x[p]) >> b) & 1) << p for p in range(32)))
    M64 = (1 << 64) - 1
    chains = [int(v) for v in x]
    for _ in range(40):
        for b in range(63, 20, -1):
            planes[b] ^= planes[b - 21]
        for b in range(0, 29):
            planes[b] ^= planes[b + 35]
        for b in range(63, 3, -1):
            planes[b] ^= planes[b - 4]
        for p in range(32):
            c = chains[p]
            c ^= (c << 21) & M64
            c ^= c >> 35
            c ^= (c << 4) & M64
            chains[p] = c
        back = [sum(((int(planes[b]) >> p) & 1) << b for b in range(64)) for p in range(32)]
        assert back == chains
        # the filter: for a threshold between the chains' values, every chain <= T passes
        signed = sorted((c - (1 << 64) if c >> 63 else c) for c in chains)
        T = signed[3]
        U = (T & M64) ^ (1 << 63)
        Z = 64 if U == 0 else 64 - U.bit_length()
        z = ~int(planes[63]) & 0xFFFFFFFF
        for i in range(1, Z):
            z |= int(planes[63 - i])
        for p in range(32):
            v = chains[p] - (1 << 64) if chains[p] >> 63 else chains[p]
            if v <= T:
                assert not (z >> p) & 1


def test_frequency_counts_keys_and_scaled_idf():
    """FrequencyCounts: a k-mer and its reverse complement share one key (the smaller
    string's hash); scaled idf runs from 1 (the most frequent k-mer) to the scale (a k-mer
    at the cutoff; also every k-mer not in the table); lines below the cutoff are dropped."""
    p = M.default_params(repeat_idf_scale=10.0, filter_threshold=1e-5)
    km = ["AAAAAAAAAAAAAAAC", "GTTTTTTTTTTTTTTT", "ACGTACGTACGTACGA", "CCCCCCCCCCCCCCCC"]
    fr = [1e-3, 1e-3, 1e-5, 1e-6]
    fc = M.FrequencyCounts(km, fr, p)
    k0 = M.seq_hashes_long(km[0].encode(), 16, True)[0]
    assert k0 == M.seq_hashes_long(km[1].encode(), 16, True)[0]      # reverse complements
    assert k0 == M.seq_hashes_long(b"AAAAAAAAAAAAAAAC", 16, False)[0]   # the smaller string
    assert len(fc.counts) == 2
    assert abs(fc.scaled_idf(k0) - 1.0) < 1e-12
    k2 = M.seq_hashes_long(km[2].encode(), 16, True)[0]
    assert abs(fc.scaled_idf(k2) - 10.0) < 1e-9
    assert fc.scaled_idf(12345) == 10.0


def test_oracle_finds_the_true_overlaps(small, small_oracle):
    """Sanity of the restated algorithm: overlaps it reports are real (genome intervals
    intersect, orientation = strand difference), a is the larger ID (the self search), and
    it finds most true overlaps of >= 1.5 kb."""
    rs, rec = small, small_oracle
    assert len(rec) > 100
    st, sd, L = rs.starts, rs.strands.astype(int), rs.lengths.astype(int)
    for r in rec:
        a, b = int(r["a"]) - 1, int(r["b"]) - 1
        assert b < a
        ov = min(st[a] + L[a], st[b] + L[b]) - max(st[a], st[b])
        assert ov > 0, (a, b)
        assert int(r["o"]) == (sd[a] ^ sd[b])
        assert r["count"] >= 3 and 0.0 <= r["erate"] <= 0.22
    found = {(int(r["a"]) - 1, int(r["b"]) - 1) for r in rec}
    true = [(a, b) for a in range(rs.nreads) for b in range(a)
            if min(st[a] + L[a], st[b] + L[b]) - max(st[a], st[b]) >= 1500]
    hit = sum((a, b) in found for a, b in true)
    assert hit >= 0.9 * len(true), (hit, len(true))


@pytest.mark.skipif(not oracle.mhap_convert_available(), reason="reference mhapConvert not built")
def test_reference_mhapconvert_reads_our_lines(small, small_oracle, tmp_path):
    """The format is the one the reference's mhapConvert consumes: IDs, hangs, flip and
    erate of every converted ovOverlap match the line."""
    rec = small_oracle
    path = str(tmp_path / "q.mhap")
    with open(path, "w") as f:
        for r in rec:
            f.write(mhap.format_line(r, 1, small.nreads, 1) + "\n")
    ov = oracle.mhap_convert(small, path, 1, small.nreads, 1)
    assert len(ov) == len(rec)
    w0, w1 = ov["w0"], ov["w1"]
    ahg5, ahg3 = w0 & 0x1FFFFF, (w0 >> 21) & 0x1FFFFF
    bhg5, bhg3 = w1 & 0x1FFFFF, (w1 >> 21) & 0x1FFFFF
    flipped = (w0 >> 54) & 1
    assert np.array_equal(ov["a"], rec["a"]) and np.array_equal(ov["b"], rec["b"])
    assert np.array_equal(ahg5, rec["a_bgn"]) and np.array_equal(ahg3, rec["a_len"] - rec["a_end"])
    o = rec["o"].astype(bool)
    assert np.array_equal(flipped.astype(bool), o)
    want_b5 = np.where(o, rec["b_len"] - rec["b_end"], rec["b_bgn"])
    want_b3 = np.where(o, rec["b_bgn"], rec["b_len"] - rec["b_end"])
    assert np.array_equal(bhg5, want_b5) and np.array_equal(bhg3, want_b3)
    # for*: forUTG/forOBT/forDUP all set (mhapConvert.C:131-133)
    assert np.all((w0 >> 55) & 7 == 7)


# ------------------------------------------------------------------------------- GPU ----

def _same(got, want):
    assert got.shape == want.shape, (got.shape, want.shape)
    for f in FIELDS:
        assert np.array_equal(got[f], want[f]), f


def _rows(m, n, P):
    """The context's sketch rows (mhap_sketch_buffers) copied to the host."""
    import ctypes
    pmh, pord, pcnt = m.sketch_buffers()
    H, S = P.num_hashes, P.ordered_sketch_size
    mh = np.zeros((n, 2, H), dtype=np.int32)
    od = np.zeros((n, 2, S), dtype=np.uint64)
    oc = np.zeros((n, 2), dtype=np.uint32)
    hip = ctypes.CDLL("libamdhip64.so")        # hipMemcpy D2H (synchronous) of the rows
    hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    for arr, ptr in ((mh, pmh), (od, pord), (oc, pcnt)):
        assert hip.hipMemcpy(arr.ctypes.data, ptr, arr.nbytes, 2) == 0
    return mh, od, oc


def _same_rows(got, want):
    mh, od, oc = got
    wmh, wod, woc = want
    assert np.array_equal(oc, woc)
    used = oc > 0
    assert np.array_equal(mh[used], wmh[used])
    for i, s in zip(*np.nonzero(used)):
        assert np.array_equal(od[i, s, :oc[i, s]], wod[i, s, :woc[i, s]]), (i, s)


CASES = {
    "normal": (dict(), mhap.MhapParameters()),
    "high_ragged_ns": (dict(n=70, L=3000, err=0.05, seed=5, len_jitter=0.5, n_rate=0.002),
                       mhap.MhapParameters.sensitivity("high", min_olap=1500)),
    "low_k14": (dict(n=50, L=5000, err=0.03, seed=6),
                mhap.MhapParameters.sensitivity("low", min_olap=500)),
    # BASELINE configs[3]'s read length: 15 kb reads at 25x, 5 % error, the 'normal' preset
    "configs3_15kb": (dict(n=60, L=15000, cov=25, err=0.05, seed=9), mhap.MhapParameters()),
    "utg_small_k": (dict(n=50, L=2500, err=0.02, seed=7),
                    mhap.MhapParameters(k=12, num_hashes=128, num_min_matches=5,
                                        ordered_kmer_size=18, ordered_sketch_size=700,
                                        min_olap_length=200, threshold=0.8)),
    "max_shift_min_store": (dict(n=60, L=3000, err=0.04, seed=8, len_jitter=0.4),
                            mhap.MhapParameters(num_hashes=256, max_shift=0.05,
                                                min_store_length=2800, min_olap_length=300)),
    "no_rc_odd_k": (dict(n=50, L=3000, err=0.03, seed=10),
                    mhap.MhapParameters(k=13, num_hashes=200, ordered_kmer_size=11,
                                        ordered_sketch_size=900, no_rc=True)),
}


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(CASES))
def test_gpu_matches_oracle(built, name):
    kw, P = CASES[name]
    rs = _reads(**kw)
    m = mhap.Mhap(P, device=0)
    got = m.run(rs)
    st = m.stats()
    rows = _rows(m, rs.nreads, P)
    m.close()
    want = M.run(rs, P.as_oracle())
    assert len(want) > 20
    _same(got, want)
    assert st["overlaps"] == len(want) and st["candidates"] >= len(want)
    _same_rows(rows, M.sketch_rows(rs, P.as_oracle()))


def _freq_for(rs, every=11, span=2400):
    """-f entries for a read set: some of read 0's 16-mers at graded fractions, both
    strands written as canu does (Meryl.pm:699-716)."""
    r0 = rs.read(0).decode()
    comp = str.maketrans("ACGT", "TGCA")
    km, fr = [], []
    for j, i in enumerate(range(0, span, every)):
        m = r0[i:i + 16]
        f = 5e-6 * (1.5 ** (j % 12))
        km += [m, m.translate(comp)[::-1]]
        fr += [f, f]
    return km, np.array(fr)


@pytest.mark.gpu
@pytest.mark.parametrize("variant", ["canu", "no_tf", "tf_only", "count", "unweighted",
                                     "repeat_read", "k20"])
def test_gpu_weighted_sketch_rows_match_oracle(built, variant):
    """The weighted MinHash rows in HBM (distinct k-mers by a segmented radix sort, tf as run
    lengths, the -f table's scaled idf) equal the restatement's, bit for bit; every mode of
    computeNgramMinHashesWeighted's weight: tf-idf (canu), no tf, repeat weight >= 1 (the
    count), no table (the count), repeat weight < 0 (1, table k-mers dropped)."""
    kw = dict(n=24, L=3000, cov=8, seed=19)
    if variant == "repeat_read":
        kw.update(n_repeats=6, repeat_len=400)        # tf > 1 inside reads
    rs = _reads(**kw)
    P = mhap.MhapParameters(num_hashes=48, ordered_sketch_size=600, ordered_kmer_size=14,
                            min_olap_length=300).canu_weighting()
    freq = _freq_for(rs)
    if variant == "no_tf":
        P.no_tf = True
    if variant == "tf_only":
        P.repeat_weight = 1.0
    if variant == "count":
        freq = None
    if variant == "unweighted":
        P.repeat_weight = -1.0
    if variant == "k20":
        P.k = 20
        freq = ([x + "ACGT" for x in freq[0]], freq[1])
    m = mhap.Mhap(P, device=0)
    m.load_reads(rs)
    if freq is None:
        m.set_weighting()
    else:
        m.set_kmer_frequencies(*freq)
    m.sketch()
    st = m.stats()
    got = _rows(m, rs.nreads, P)
    m.close()
    _same_rows(got, M.sketch_rows(rs, P.as_oracle(), freq))
    assert st["sketch_draws"] >= st["sketch_kmers"] * P.num_hashes > 0


@pytest.mark.gpu
def test_gpu_weighted_job_matches_oracle(built):
    """canu's weighting end to end (-f table, --repeat-weight 0.9 --repeat-idf-scale 10):
    records of the self job equal the restatement's."""
    rs = _reads(n=40, L=3000, cov=10, seed=23)
    P = mhap.MhapParameters(num_hashes=96, ordered_sketch_size=1000,
                            min_olap_length=400).canu_weighting()
    freq = _freq_for(rs, every=5)
    m = mhap.Mhap(P, device=0)
    got = m.run(rs, frequencies=freq)
    m.close()
    want = M.run(rs, P.as_oracle(), freq=freq)
    assert len(want) > 20
    _same(got, want)


def _odd_reads():
    """Edge cases of one read set: a read shorter than k (not used), one shorter than
    --min-olap-length (not used), a homopolymer (one hash repeated: the ordered sketch's
    radix select must descend past its first digit), lower case / IUPAC / N bases (the
    complement table), and ordinary reads overlapping them."""
    base = _reads(n=20, L=2500, cov=6, err=0.03, seed=31)
    seqs = [base.read(i) for i in range(base.nreads)]
    g = bytearray(seqs[3])
    g[100:140] = b"acgtacgtacgtRYKMnnnnNNNNswSWbdhv" + b"A" * 8
    seqs[3] = bytes(g)
    seqs += [b"ACGTACGTAC", seqs[5][:400], b"A" * 2600, seqs[7][:1200] + b"T" * 1400]
    lens = np.array([len(s) for s in seqs], dtype=np.uint32)
    offs = np.zeros(len(seqs), dtype=np.uint64)
    offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    return ReadSet(bases=np.frombuffer(b"".join(seqs), dtype=np.uint8).copy(), offsets=offs,
                   lengths=lens, first_iid=1)


@pytest.mark.gpu
def test_gpu_edge_reads_match_oracle(built):
    rs = _odd_reads()
    P = mhap.MhapParameters(num_hashes=128, ordered_sketch_size=800, min_olap_length=500,
                            threshold=0.6)
    m = mhap.Mhap(P, device=0)
    got = m.run(rs)
    st = m.stats()
    rows = _rows(m, rs.nreads, P)
    m.close()
    want_rows = M.sketch_rows(rs, P.as_oracle())
    _same_rows(rows, want_rows)
    assert rows[2][20].tolist() == [0, 0] and rows[2][21].tolist() == [0, 0]   # not used
    assert rows[2][22, 0] == 800                                             # homopolymer
    assert st["sketched_reads"] == rs.nreads - 2
    _same(got, M.run(rs, P.as_oracle()))


@pytest.mark.gpu
def test_gpu_shards_query_search_and_text(built, small, small_oracle, tmp_path):
    """Query-range shards of the self search (the multi-GPU split) union to the whole job;
    the -q search (compare_all: every stored read, toSelf false) equals the restatement's;
    the text the library writes is byte-identical to the oracle records' lines (and, where
    built, goes through the reference mhapConvert)."""
    P = mhap.MhapParameters()
    m = mhap.Mhap(P, device=0)
    m.load_reads(small)
    m.set_weighting()
    m.sketch()
    m.build_index()
    parts = []
    for lo, hi in ((1, 20), (21, 45), (46, small.nreads)):
        m.compare(lo, hi)
        parts.append(m.fetch())
    m.compare()
    path = str(tmp_path / "all.mhap")
    m.write_text(path, 1, small.nreads, 1)
    # the -q search: reads 41.. against the stored reads 1..40
    m.build_index(1, 40)
    m.compare(41, small.nreads, all_targets=True)
    cross = m.fetch()
    m.close()
    _same(np.concatenate(parts), small_oracle)
    want = "".join(mhap.format_line(r, 1, small.nreads, 1) + "\n" for r in small_oracle)
    assert open(path).read() == want
    P0 = P.as_oracle()
    _same(cross, M.run(small, P0, q_range=(40, small.nreads), t_range=(0, 40), to_self=False))
    oracle.require_reference(mhap_convert=True)
    assert len(oracle.mhap_convert(small, path)) == len(small_oracle)


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [1, 2])
def test_gpu_supress_noise_rows_match_oracle(built, mode):
    """--supress-noise with canu's -f table: 1 keeps only the k-mers the jar's Guava Bloom
    filter of the file's keys accepts -- here read 0's k-mers of the table, so every other
    read loses nearly all of its k-mers (those strands skipped, ocount 0) -- and 2 builds
    the filter and never reads it (the rows of --supress-noise 0).  The filter is sized by
    the file's count line (a smaller count: more false positives kept)."""
    rs = _reads(n=24, L=3000, cov=8, seed=19)
    P = mhap.MhapParameters(num_hashes=48, ordered_sketch_size=600, ordered_kmer_size=14,
                            min_olap_length=300, supress_noise=mode).canu_weighting()
    km, fr = _freq_for(rs, every=3)
    for expected in (len(km), 40):
        m = mhap.Mhap(P, device=0)
        m.load_reads(rs)
        m.set_kmer_frequencies(km, fr, expected)
        m.sketch()
        got = _rows(m, rs.nreads, P)
        m.close()
        want = M.sketch_rows(rs, P.as_oracle(), (km, fr, expected))
        _same_rows(got, want)
        if mode == 2:
            _same_rows(got, M.sketch_rows(rs, dict(P.as_oracle(), supress_noise=0), (km, fr)))
        elif expected == len(km):
            assert want[2][0].all() and (want[2][1:] == 0).sum() > 0
    # without a -f table there is no FrequencyCounts and so no filter
    m = mhap.Mhap(P, device=0)
    m.load_reads(rs)
    m.set_weighting()
    m.sketch()
    got = _rows(m, rs.nreads, P)
    m.close()
    _same_rows(got, M.sketch_rows(rs, P.as_oracle()))


@pytest.mark.gpu
def test_gpu_supress_noise_job_matches_oracle(built):
    """--supress-noise 1 end to end (self job) against the restatement; the filter's keys
    are the k-mers of reads 0-9 (every line below --filter-threshold: an empty tf-idf table,
    the filter alone), so the sketches hold only those k-mers."""
    rs = _reads(n=40, L=3000, cov=10, seed=23)
    P = mhap.MhapParameters(num_hashes=96, ordered_sketch_size=1000, min_olap_length=400,
                            supress_noise=1).canu_weighting()
    comp = str.maketrans("ACGT", "TGCA")
    km, fr = [], []
    for r in range(10):
        s = rs.read(r).decode()
        for i in range(0, len(s) - 16, 2):
            km += [s[i:i + 16], s[i:i + 16].translate(comp)[::-1]]
            fr += [1e-7, 1e-7]                       # below the cutoff: filter only
    freq = (km, np.array(fr), len(km))
    m = mhap.Mhap(P, device=0)
    got = m.run(rs, frequencies=freq)
    m.close()
    want = M.run(rs, P.as_oracle(), freq=freq)
    assert len(want) > 5
    # the sketches hold only the filter's k-mers: another set of records than without it
    assert len(want) != len(M.run(rs, dict(P.as_oracle(), supress_noise=0), freq=freq))
    _same(got, want)


def test_library_formats_lines_like_java(built):
    """mhap_format_line (the C library's MatchResult.toString) equals format_line for
    values on both sides of every rounding edge."""
    import ctypes
    lib = mhap.load_library()
    rng = np.random.default_rng(2)
    vals = [5e-7, 1.0000005, 0.0, 1.0, 0.123456499999, 0.1234565, 2.5e-7, 0.9999995]
    vals += list(rng.random(300)) + [round(float(x), 7) for x in rng.random(300)]
    r = np.zeros(1, dtype=mhap.MHAP_DTYPE)
    buf = ctypes.create_string_buffer(256)
    for i, v in enumerate(vals):
        r[0] = (7, 3, v, float(i % 50), 1, 2, 3, i % 2, 4, 5, 6, 9)
        assert lib.mhap_format_line(r.ctypes.data, 1, 0, 1, buf, 256) == 0
        assert buf.value.decode() == mhap.format_line(r[0]), v
