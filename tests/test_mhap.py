"""The MHAP stage (include/canu_mhap.h, canu_amd/csrc/mhap.hip).

PARITY UNPINNED against the MHAP jar (src/mhap/mhap-2.1.2.tar: a prebuilt third-party
archive, never run here).  What IS pinned:
  * the output format, by the reference's own consumer: every line must go through
    mhapConvert (src/mhap/mhapConvert.C, compiled from the reference source into
    oracle/_ref/) and come out as the ovOverlap records the line describes;
  * the GPU path, against the CPU restatement oracle/mhap_oracle.py: integers bit-exact,
    erate within 1e-6 (written with 6 decimals);
  * sanity of the restated algorithm against the synthetic reads' known genome layout.
CPU tests run here; @gpu tests on the MI355X box."""
import os
import re

import numpy as np
import pytest

import mhap_oracle as M
import oracle
from canu_amd import mhap
from canu_amd.synth import synth_reads

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "canu_mhap.h")
FIELDS = ("a", "b", "count", "a_bgn", "a_end", "a_len", "o", "b_bgn", "b_end", "b_len")


def _reads(n=90, L=4000, cov=15, err=0.04, seed=3, **kw):
    return synth_reads(n_reads=n, read_len=L, genome_len=int(n * L / cov), error_rate=err,
                       seed=seed, **kw)


@pytest.fixture(scope="module")
def small():
    return _reads()


@pytest.fixture(scope="module")
def small_oracle(small):
    return M.run(small, M.default_params())


def test_header_declares_the_python_exports():
    src = re.sub(r"/\*.*?\*/", "", open(HEADER).read(), flags=re.S)
    assert sorted(set(re.findall(r"\b(mhap_[a-z_]+)\s*\(", src))) == sorted(mhap.EXPORTS)


def test_library_exports_every_declared_symbol(built):
    lib = mhap.load_library()
    assert [f for f in mhap.EXPORTS if not hasattr(lib, f)] == []
    assert lib.mhap_abi_version() == mhap.ABI_VERSION == 5


def test_params_init_is_canu_normal(built):
    lib = mhap.load_library()
    p = mhap._Params()
    lib.mhap_params_init(p)
    d = mhap.MhapParameters()
    assert (p.k, p.num_hashes, p.min_matches, p.ordered_sketch, p.ordered_k, p.min_olap) == \
        (d.k, d.num_hashes, d.num_min_matches, d.ordered_sketch_size, d.ordered_kmer_size,
         d.min_olap_length) == (16, 512, 3, 1536, 12, 500)
    assert abs(p.threshold - 0.78) < 1e-12


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
    assert not p.no_tf
    assert io["-s"] == "./blocks/000001.dat" and io["--num-threads"] == "8"
    assert mhap.parse_mhap_args(["--no-tf"])[0].no_tf
    assert p.supress_noise == 0
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


def _weighted_params(**kw):
    p = M.default_params(num_hashes=96)
    p.update(repeat_weight=0.9, repeat_idf_scale=10.0, filter_threshold=5e-6)
    p.update(kw)
    return p


def _freq_for(rs, every=11):
    """-f entries for a read set: some of read 0's 16-mers at graded fractions, both
    strands written as canu does."""
    r0 = rs.read(0).decode()
    comp = str.maketrans("ACGT", "TGCA")
    km, fr = [], []
    for j, i in enumerate(range(0, 2400, every)):
        m = r0[i:i + 16]
        f = 5e-6 * (1.5 ** (j % 12))
        km += [m, m.translate(comp)[::-1]]
        fr += [f, f]
    return km, np.array(fr)


def test_oracle_weighting_properties():
    """The restated weighting (canu_mhap.h): with weight 1 everywhere the weighted sketch
    IS the unweighted one; tf weighting changes only reads with repeated k-mers; the -f
    table lowers the weight of listed (frequent) k-mers relative to the rest."""
    rs = _reads(n=6, L=3000, cov=10, seed=17)
    base = M.sketch(rs, M.default_params(num_hashes=96))
    # no -f, no tf: every weight is 1
    w1 = M.sketch_weighted(rs, _weighted_params(no_tf=True), None)
    assert np.array_equal(w1, base)
    # r >= 1: m = 1 for every k-mer (tf only); a read with no repeated k-mer is unchanged
    tfo = M.sketch_weighted(rs, _weighted_params(repeat_weight=1.0), _freq_for(rs))
    assert np.array_equal(tfo, M.sketch_weighted(rs, _weighted_params(repeat_weight=1.0)))
    # the multipliers: frequent k-mers get the smallest, unlisted ones the largest
    km, fr = _freq_for(rs)
    codes, mult, dm = M.kmer_multipliers(km, fr, _weighted_params())
    assert codes.size == np.unique(codes).size and mult.min() >= 1.0 - 1e-12
    assert abs(dm - (0.9 + 0.1 * 10.0)) < 1e-12 and mult.max() <= dm
    assert abs(mult.min() - 1.0) < 1e-12                 # the most frequent: scaled idf 1
    # a read whose k-mers are all listed at one fraction gets a sketch unlike the tf one
    full = M.sketch_weighted(rs, _weighted_params(), (km, fr))
    assert not np.array_equal(full, tfo)


def _noise_freq(rs, every=3):
    """An mhapFilterUnique-style -f list (Meryl.pm:678-714: every k-mer at or above the
    unique-count threshold, with its fraction): some of the reads' k-mers, most of them
    below --filter-threshold, a few repeats above it."""
    km, fr = _freq_for(rs, every=every)
    fr = fr.copy()
    fr[np.arange(fr.size) % 6 >= 2] = 2e-7        # solid but not repeated: below 5e-6
    return km, fr


def test_oracle_supress_noise():
    """--supress-noise (canu_mhap.h, restated from the jar's option text; unpinned): every
    -f k-mer is in the table (those below the threshold at the top multiplier); an unlisted
    k-mer is weighted like the most frequent one (2) or never enters a sketch (1)."""
    rs = _reads(n=6, L=3000, cov=10, seed=17)
    km, fr = _noise_freq(rs)
    p0 = _weighted_params()
    c0, m0, d0 = M.kmer_multipliers(km, fr, p0)
    for mode in (1, 2):
        c, m, d = M.kmer_multipliers(km, fr, dict(p0, supress_noise=mode))
        assert c.size > c0.size                   # the below-threshold k-mers are listed
        assert abs(m.max() - d0) < 1e-12          # ... at the top multiplier
        assert (abs(d - m.min()) < 1e-12) if mode == 2 else d == -1.0
    s0 = M.sketch_weighted(rs, p0, (km, fr))
    s1 = M.sketch_weighted(rs, dict(p0, supress_noise=1), (km, fr))
    s2 = M.sketch_weighted(rs, dict(p0, supress_noise=2), (km, fr))
    assert not np.array_equal(s0, s2) and not np.array_equal(s1, s2)
    # mode 1 keeps only listed k-mers: every read's sketch values are >= mode 0's
    assert (s1 >= s0).all() and (s1 != s0).any()
    # nothing listed: with mode 1 no k-mer is left (empty sketches)
    none = ([km[0]], np.array([fr[0]]))
    c, m, d = M.kmer_multipliers(none[0], none[1], dict(p0, supress_noise=1))
    assert c.size == 1 and d == -1.0


def test_oracle_kmer_codes():
    """Canonical 2-bit codes, first base most significant; non-ACGT breaks k-mers."""
    c = M._CODE[np.frombuffer(b"ACGTNACGTA", dtype=np.uint8)]
    pos, can, s = M.kmers(c, 4)
    # ACGT is its own reverse complement; CGTA/ACGT after the N
    assert pos.tolist() == [0, 5, 6]
    assert int(can[0]) == 0b00011011 == int(can[1])      # ACGT = its own reverse complement
    assert int(can[2]) == 0b01101100                      # CGTA < rc TACG (0b11000110)
    assert s.tolist() == [0, 0, 0]
    pos, can, s = M.kmers(M._CODE[np.frombuffer(b"TTTT", dtype=np.uint8)], 4)
    assert int(can[0]) == 0 and s.tolist() == [1]        # AAAA on the other strand


def test_oracle_finds_the_true_overlaps(small, small_oracle):
    """Sanity of the restated algorithm: overlaps it reports are real (genome intervals
    intersect, orientation = strand difference, offset close to the truth) and it finds
    most true overlaps of >= 1.5 kb."""
    rs, rec = small, small_oracle
    assert len(rec) > 100
    st, sd, L = rs.starts, rs.strands.astype(int), rs.lengths.astype(int)
    for r in rec:
        a, b = int(r["a"]) - 1, int(r["b"]) - 1
        ov = min(st[a] + L[a], st[b] + L[b]) - max(st[a], st[b])
        assert ov > 0, (a, b)
        assert int(r["o"]) == (sd[a] ^ sd[b])
    found = {(int(r["a"]) - 1, int(r["b"]) - 1) for r in rec}
    true = [(a, b) for a in range(rs.nreads) for b in range(a + 1, rs.nreads)
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

def _gpu(rs, P, filt=None):
    m = mhap.Mhap(P, device=0)
    rec = m.run(rs, filter_kmers=filt)
    st = m.stats()
    m.close()
    return rec, st


def _same(got, want):
    assert got.shape == want.shape, (got.shape, want.shape)
    for f in FIELDS:
        assert np.array_equal(got[f].astype(np.int64), want[f].astype(np.int64)), f
    assert np.max(np.abs(got["erate"] - want["erate"]), initial=0.0) <= 1e-6


CASES = {
    "normal": (dict(), mhap.MhapParameters()),
    "high_ragged_ns": (dict(n=80, L=3000, err=0.05, seed=5, len_jitter=0.5, n_rate=0.002),
                       mhap.MhapParameters.sensitivity("high", min_olap=300)),
    "low_k14": (dict(n=70, L=5000, err=0.03, seed=6),
                mhap.MhapParameters.sensitivity("low", min_olap=500)),
    # BASELINE configs[3]'s read length: 15 kb reads at 25x, 5 % error, the 'normal' preset
    "configs3_15kb": (dict(n=300, L=15000, cov=25, err=0.05, seed=9), mhap.MhapParameters()),
    "utg_small_k": (dict(n=60, L=2500, err=0.02, seed=7),
                    mhap.MhapParameters(k=12, num_hashes=128, num_min_matches=5,
                                        ordered_kmer_size=18, ordered_sketch_size=700,
                                        min_olap_length=200, threshold=0.8)),
}


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(CASES))
def test_gpu_matches_oracle(built, name):
    kw, P = CASES[name]
    rs = _reads(**kw)
    got, st = _gpu(rs, P)
    want = M.run(rs, P.as_oracle())
    assert len(want) > 20
    _same(got, want)
    assert st["overlaps"] == len(want)


@pytest.mark.gpu
def test_gpu_filter_kmers(built, small):
    """-f: frequent k-mers never enter a sketch."""
    P = mhap.MhapParameters()
    r0 = small.read(0).decode()
    filt = [r0[i:i + 16] for i in range(0, 3000, 7)]
    got, _ = _gpu(small, P, filt)
    want = M.run(small, P.as_oracle(), skip_kmers=filt)
    _same(got, want)


@pytest.mark.gpu
def test_gpu_shards_and_text(built, small, small_oracle, tmp_path):
    """Query-range shards (the multi-GPU split) union to the whole job, and the text the
    library writes is byte-identical to the oracle records' lines (and, where built, goes
    through the reference mhapConvert)."""
    P = mhap.MhapParameters()
    m = mhap.Mhap(P, device=0)
    m.load_reads(small)
    m.sketch()
    m.build_index()
    parts = []
    for lo, hi in ((1, 30), (31, 60), (61, small.nreads)):
        m.compare(lo, hi)
        parts.append(m.fetch())
    m.compare()
    path = str(tmp_path / "all.mhap")
    m.write_text(path, 1, small.nreads, 1)
    m.close()
    whole = np.concatenate(parts)
    _same(whole, small_oracle)
    want = "".join(mhap.format_line(r, 1, small.nreads, 1) + "\n" for r in small_oracle)
    assert open(path).read() == want
    oracle.require_reference(mhap_convert=True)
    assert len(oracle.mhap_convert(small, path)) == len(small_oracle)


@pytest.mark.gpu
def test_gpu_sketch_rows_match_oracle(built, small):
    """Stage outputs directly: the MinHash rows and ordered-sketch rows in HBM."""
    import ctypes
    P = mhap.MhapParameters()
    m = mhap.Mhap(P, device=0)
    m.load_reads(small)
    m.sketch()
    pmh, pord, pcnt = m.sketch_buffers()
    n, H, S = small.nreads, P.num_hashes, P.ordered_sketch_size
    mh = np.zeros((n, H), dtype=np.int32)
    od = np.zeros((n, S), dtype=np.uint64)
    oc = np.zeros(n, dtype=np.uint32)
    hip = ctypes.CDLL("libamdhip64.so")        # hipMemcpy D2H (synchronous) of the rows
    hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    assert hip.hipMemcpy(mh.ctypes.data, pmh, mh.nbytes, 2) == 0
    assert hip.hipMemcpy(od.ctypes.data, pord, od.nbytes, 2) == 0
    assert hip.hipMemcpy(oc.ctypes.data, pcnt, oc.nbytes, 2) == 0
    m.close()
    assert np.array_equal(mh, M.sketch(small, P.as_oracle()))
    for i in range(0, n, 7):
        h, pos, s = M.ordered_sketch(small, i, P.as_oracle())
        assert oc[i] == h.shape[0]
        key = (h.astype(np.uint64) << np.uint64(32)) | (pos.astype(np.uint64) << np.uint64(1)) \
            | s.astype(np.uint64)
        assert np.array_equal(od[i, :oc[i]], key), i


@pytest.mark.gpu
@pytest.mark.parametrize("variant", ["canu", "no_tf", "tf_only", "repeat_read", "k20", "noise1",
                                     "noise2"])
def test_gpu_weighted_sketch_rows_match_oracle(built, variant):
    """The weighted MinHash rows in HBM (distinct k-mers by a radix sort, tf as run lengths,
    the -f multipliers) equal the restatement's, bit for bit."""
    import ctypes
    kw = dict(n=40, L=3000, cov=12, seed=19)
    if variant == "repeat_read":
        kw.update(n_repeats=6, repeat_len=400)        # tf > 1 inside reads
    rs = _reads(**kw)
    P = mhap.MhapParameters(num_hashes=128, ordered_sketch_size=600, ordered_kmer_size=14,
                            min_olap_length=300).canu_weighting()
    freq = _freq_for(rs)
    if variant == "no_tf":
        P.no_tf = True
    if variant == "tf_only":
        P.repeat_weight = 1.0
    if variant == "k20":                 # 64-bit (read, code) keys: one sort per batch
        P.k = 20
        freq = ([x + "ACGT" for x in freq[0]], freq[1])
    if variant in ("noise1", "noise2"):  # --supress-noise with an mhapFilterUnique -f list
        P.supress_noise = int(variant[-1])
        freq = _noise_freq(rs)
    m = mhap.Mhap(P, device=0)
    m.load_reads(rs)
    m.set_kmer_frequencies(*freq)
    m.sketch()
    pmh, _, _ = m.sketch_buffers()
    mh = np.zeros((rs.nreads, P.num_hashes), dtype=np.int32)
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    assert hip.hipMemcpy(mh.ctypes.data, pmh, mh.nbytes, 2) == 0
    m.close()
    want = M.sketch_weighted(rs, P.as_oracle(), freq)
    assert np.array_equal(mh, want)


@pytest.mark.gpu
def test_gpu_weighted_job_matches_oracle(built):
    """canu's weighting end to end: records of the weighted all-vs-all equal the
    restatement's (integers bit-exact, erate within 1e-6)."""
    rs = _reads(n=70, L=4000, cov=14, seed=23)
    P = mhap.MhapParameters(num_hashes=256, ordered_sketch_size=1000,
                            min_olap_length=400).canu_weighting()
    freq = _freq_for(rs, every=5)
    m = mhap.Mhap(P, device=0)
    got = m.run(rs, frequencies=freq)
    m.close()
    want = M.run(rs, P.as_oracle(), freq=freq)
    assert len(want) > 20
    _same(got, want)
