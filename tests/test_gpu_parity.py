"""GPU parity: the HIP path through the C-ABI against the oracle (bit-exact records).

The oracle is pinned to the reference overlapInCore (tests/test_oracle_*.py); here every
case compares ovOverlap records (a_iid, b_iid and both bitfield words, i.e. hangs,
orientation, span, evalue) for equality after sorting by ovOverlap::operator<.
"""
import numpy as np
import pytest

from canu_amd.synth import synth_reads
from canu_amd.overlap_in_core import OicParameters, OverlapInCore

import oracle

pytestmark = pytest.mark.gpu


def _params(**kw):
    P = OicParameters(Kmer_Len=kw.pop("k", 22), maxErate=float(np.float32(kw.pop("erate", 0.06))),
                      Min_Olap_Len=kw.pop("minlen", 100))
    for k, v in kw.items():
        setattr(P, k, v)
    return P.finalize()


def _check(rs, P, skip=None, hash_range=None, ref_range=None):
    oic = OverlapInCore(P, device=0)
    oic.load_reads(rs)
    if skip:
        oic.set_skip_kmers(skip)
    hb, he = hash_range or (1, 0xFFFFFFFF)
    rb, re_ = ref_range or (1, 0xFFFFFFFF)
    oic.build_hash_index(hb, he)
    n = oic.find_overlaps(rb, re_)
    got = oic.fetch(n)
    st = oic.stats()
    oic.close()
    want, wst = oracle.run_oracle(rs, P.as_dict(), hash_range=hash_range, ref_range=ref_range,
                                  skip_kmers=skip, with_stats=True)
    assert got.shape == want.shape, (got.shape, want.shape)
    assert np.array_equal(got, want)
    for f in ("kmer_hits_with_olap", "kmer_hits_without_olap", "total_overlaps",
              "contained_overlaps", "dovetail_overlaps", "seed_hits", "multi_overlaps",
              "kmer_hits_skipped"):
        assert st[f] == wst[f], (f, st[f], wst[f])
    return got


def test_basic_default(built):
    rs = synth_reads(150, 2000, 30_000, 0.02, seed=1)
    got = _check(rs, _params())
    assert got.shape[0] > 100


def test_extension_launches_only_classes_with_pairs(built):
    """Later extension classes whose input list is empty are not launched (find_impl reads
    the previous class's defer count): 2 kb reads fit the one staged tier, so the job makes
    one launch plus one per later class (wide, generic) that actually received pairs."""
    rs = synth_reads(150, 2000, 30_000, 0.02, seed=1)
    oic = OverlapInCore(_params(), device=0)
    oic.load_reads(rs)
    oic.build_hash_index(1, 0xFFFFFFFF)
    oic.find_overlaps(1, 0xFFFFFFFF)
    st = oic.stats()
    oic.close()
    assert st["pairs"] > 0
    want = 1 + (st["long_pairs"] > 0) + (st["generic_pairs"] > 0)
    assert st["extend_launches"] == want, (st["extend_launches"], st["staged_pairs"],
                                           st["long_pairs"], st["generic_pairs"])


def test_high_erate(built):
    rs = synth_reads(100, 3000, 30_000, 0.05, seed=2)
    _check(rs, _params(erate=0.144))


def test_partial(built):
    rs = synth_reads(120, 2000, 30_000, 0.02, seed=3)
    _check(rs, _params(Doing_Partial_Overlaps=True))


def test_multiple_per_pair(built):
    rs = synth_reads(100, 2000, 20_000, 0.02, seed=4, n_repeats=4, repeat_len=400)
    _check(rs, _params(Unique_Olap_Per_Pair=False))


def test_ns_repeats_ragged(built):
    rs = synth_reads(150, 2000, 30_000, 0.02, seed=5, n_rate=0.002, n_repeats=6,
                     repeat_len=300, len_jitter=0.6)
    _check(rs, _params())


def test_long_kmer_runs(built):
    # a repeat in 80 copies at ~10x coverage: its k-mers occur up to ~260 times, so their
    # occurrence runs in the index span several 64-record batches (k_table's far path)
    rs = synth_reads(150, 2000, 30_000, 0.02, seed=12, n_repeats=80, repeat_len=300)
    _check(rs, _params(Unique_Olap_Per_Pair=False))


def test_skip_kmers(built):
    rs = synth_reads(120, 2000, 30_000, 0.02, seed=6, n_repeats=5, repeat_len=200)
    skip = [rs.read(0)[i:i + 22].decode() for i in range(0, 1900, 10)]
    skip = [s for s in skip if set(s) <= set("ACGT")]
    _check(rs, _params(), skip=skip)


def test_minkmers(built):
    rs = synth_reads(120, 2000, 30_000, 0.03, seed=7)
    P = _params(minlen=500)
    P.Filter_By_Kmer_Count = int(np.floor(np.exp(-1.0 * 22 * P.maxErate) * (500 - 22 + 1)))
    _check(rs, P)


def test_hash_ref_ranges(built):
    rs = synth_reads(150, 2000, 30_000, 0.02, seed=8)
    _check(rs, _params(), hash_range=(40, 120), ref_range=(10, 90))


def test_small_k(built):
    rs = synth_reads(80, 1500, 20_000, 0.02, seed=9)
    _check(rs, _params(k=16))


def test_pacbio_ecoli_scale(built):
    # BASELINE configs[0]: 1k PacBio-like 3 kb reads at E. coli scale (4.6 Mbp), here the
    # full read count over a scaled genome so the oracle finishes in seconds
    rs = synth_reads(1000, 3000, 300_000, 0.02, seed=10)
    _check(rs, _params(minlen=500))


@pytest.mark.parametrize("case", ["plain", "partial", "multi_ns"])
def test_window_filter(built, case):
    """-w: quality-difference windows along each overlap's alignment (Process_String_
    Overlaps.C:562-621), on reads with low-quality error bursts so that many overlaps are
    rejected; both orientations, 'n' bases (forward wildcards, reverse-complement NULs)."""
    kw = dict(n_reads=90, read_len=2500, genome_len=20_000, error_rate=0.015, seed=51,
              with_quals=True, bursts=1)
    P = dict(k=20, Use_Window_Filter=True)
    if case == "partial":
        P["Doing_Partial_Overlaps"] = True
    if case == "multi_ns":
        kw.update(n_rate=0.003, len_jitter=0.4, bursts=2, seed=52)
        P["Unique_Olap_Per_Pair"] = False
    rs = synth_reads(**kw)
    got = _check(rs, _params(**P))
    nowin = oracle.run_oracle(rs, _params(**{k: v for k, v in P.items()
                                              if k != "Use_Window_Filter"}).as_dict())
    assert 0 < got.shape[0] < nowin.shape[0]      # the filter did reject overlaps


@pytest.mark.parametrize("L", [24_000, 45_000])
def test_long_reads(built, L):
    """Reads past 16,384 bases (32-bit code log) and long enough that the staged kernel
    takes fewer waves per block and more than 64 KB of LDS; ragged lengths."""
    rs = synth_reads(16, L, int(16 * L / 6), 0.015, seed=61, len_jitter=0.3)
    got = _check(rs, _params(minlen=500))
    assert got.shape[0] > 10


@pytest.mark.parametrize("force_regrow", [False, True])
def test_repeat_many_targets(built, force_regrow, monkeypatch):
    """A 300-bp repeat in 150 copies over a 70 kb genome: queries seed against ~160 target
    reads on average and several hundred at most, so most (query, orientation) units take
    several passes of the chain's 128-target table (the second, done-set launch).  With
    force_regrow the pair buffer starts at 4 pairs per unit and the batch is chained again
    with the capacity the counters report -- the result must not change."""
    if force_regrow:
        monkeypatch.setenv("OVL_TEST_PAIRS_PER_UNIT", "4")
    rs = synth_reads(700, 1000, 70_000, 0.02, seed=41, n_repeats=150, repeat_len=300)
    P = _params(minlen=200)
    oic = OverlapInCore(P, device=0)
    oic.load_reads(rs)
    oic.build_hash_index()
    got = oic.fetch(oic.find_overlaps())
    st = oic.stats()
    oic.close()
    want, wst = oracle.run_oracle(rs, P.as_dict(), with_stats=True)
    assert st["multi_pass_units"] > 100
    assert (st["chain_retries"] > 0) == force_regrow
    assert got.shape == want.shape and np.array_equal(got, want)
    for f in ("seed_hits", "pairs", "kmer_hits_with_olap", "kmer_hits_without_olap",
              "total_overlaps"):
        assert st[f] == wst[f], (f, st[f], wst[f])


def _concat(a, b):
    from canu_amd.synth import ReadSet
    off_b = b.offsets.astype(np.uint64) + np.uint64(a.bases.shape[0])
    return ReadSet(bases=np.concatenate([a.bases, b.bases]),
                   offsets=np.concatenate([a.offsets.astype(np.uint64), off_b]),
                   lengths=np.concatenate([a.lengths, b.lengths]).astype(np.uint32))


def test_long_read_among_short(built):
    """One 60 kb read in a set of 3 kb reads at maxErate 0.144.  Before, its error limit
    sized every extension wave (and past ~8,000 errors of LDS failed the job).  Now the
    full-occupancy staged launch keeps its waves and read-length class; the long read's
    pairs carry 'n' bases, so they take the generic kernel, whose row buffers at that error
    limit live in global memory (GR).  Every record matches the oracle."""
    from canu_amd.synth import random_genome
    g = random_genome(np.random.default_rng(82), 60_000)
    short = synth_reads(100, 3000, 60_000, 0.04, seed=81, genome=g)
    long_ = synth_reads(1, 60_000, 60_000, 0.04, seed=83, genome=g, n_rate=0.0005)
    P = _params(erate=0.144, minlen=500)

    def run(rs):
        oic = OverlapInCore(P, device=0)
        oic.load_reads(rs)
        oic.build_hash_index()
        got = oic.fetch(oic.find_overlaps())
        st = oic.stats()
        oic.close()
        return got, st

    _, st_short = run(short)
    both = _concat(short, long_)
    got, st = run(both)
    # the staged class holds overlap SPANS (not whole reads) since round 6: with the long
    # read present its span cap grows to the class's LDS limit, at unchanged occupancy
    assert st["ext_waves"] == st_short["ext_waves"]
    assert st_short["stage_len"] == 3000 and st["stage_len"] >= st_short["stage_len"]
    assert st["generic_pairs"] > 0
    want = oracle.run_oracle(both, P.as_dict())
    assert got.shape == want.shape and np.array_equal(got, want)
    assert np.any((got["a"] == 101) | (got["b"] == 101))


def test_query_over_4096_targets(built):
    """One 300-bp repeat written into every one of 5,200 reads: each of the first queries
    seeds against > 4,096 target reads (round 1's DONE_CAP aborted such a job with
    OVL_ERR_OOM).  The chain's multi-pass launch sizes its done set from the probe's
    counts; records and counters equal the oracle's on a query sub-range."""
    rs = synth_reads(5200, 2000, 500_000, 0.02, seed=91)
    rep = np.frombuffer(b"ACGT", dtype=np.uint8)[np.random.default_rng(92).integers(0, 4, 300)]
    for i in range(rs.nreads):
        o = int(rs.offsets[i]) + 100
        rs.bases[o:o + 300] = rep
    P = _params(minlen=500)
    oic = OverlapInCore(P, device=0)
    oic.load_reads(rs)
    oic.build_hash_index()
    hits = oic.seed_hits(1, 1)
    targets = np.unique(hits["b"][(hits["a_pos_dir"] >> 31) == 0])
    assert targets.shape[0] > 4096
    got = oic.fetch(oic.find_overlaps(1, 8))
    st = oic.stats()
    oic.close()
    want, wst = oracle.run_oracle(rs, P.as_dict(), ref_range=(1, 8), with_stats=True)
    assert st["multi_pass_units"] >= 8
    assert got.shape == want.shape and np.array_equal(got, want)
    for f in ("seed_hits", "pairs", "kmer_hits_with_olap", "kmer_hits_without_olap",
              "total_overlaps"):
        assert st[f] == wst[f], (f, st[f], wst[f])
