"""Edge cases of the overlapInCore path on the GPU, each against the oracle (records and the
reference's counters): a single read, reads shorter than the k-mer or than --minlength,
an all-N read, duplicated reads (containments, long exact matches), a read exactly k long,
and an empty query range.  The reference takes all of these without complaint
(overlapInCore-Process_Overlaps.C:108-116 skips short reads; Find_Overlaps.C:297-303 stops
at the first NUL of a reverse-complemented N run)."""
import numpy as np
import pytest

from canu_amd.overlap_in_core import OicParameters, OverlapInCore
from canu_amd.synth import ReadSet, synth_reads

import oracle

pytestmark = pytest.mark.gpu
STATS = ("kmer_hits_with_olap", "kmer_hits_without_olap", "kmer_hits_skipped",
         "multi_overlaps", "total_overlaps", "contained_overlaps", "dovetail_overlaps")


def _params(minlen=200):
    return OicParameters(Kmer_Len=22, maxErate=float(np.float32(0.06)),
                         Min_Olap_Len=minlen).finalize()


def _readset(seqs):
    lens = np.array([len(x) for x in seqs], dtype=np.uint32)
    offs = np.zeros(len(seqs), dtype=np.uint64)
    if len(seqs) > 1:
        offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    bases = np.frombuffer(b"".join(seqs), dtype=np.uint8).copy()
    return ReadSet(bases=bases, offsets=offs, lengths=lens, first_iid=1)


def _check(rs, P, ref=None):
    oic = OverlapInCore(P, device=0)
    oic.load_reads(rs)
    oic.build_hash_index()
    rb, re_ = ref or (1, 0xFFFFFFFF)
    n = oic.find_overlaps(rb, re_)
    got = oic.fetch(n)
    st = oic.stats()
    oic.close()
    want, wst = oracle.run_oracle(rs, P.as_dict(), ref_range=ref, with_stats=True)
    assert got.shape == want.shape and np.array_equal(got, want)
    for f in STATS:
        assert st[f] == wst[f], (f, st[f], wst[f])
    return got


def _base_reads(n=40, seed=61):
    rs = synth_reads(n, 2000, 25_000, 0.02, seed=seed)
    return [rs.read(i) for i in range(rs.nreads)]


def test_single_read(built):
    assert _check(_readset(_base_reads(1)), _params()).shape[0] == 0


def test_all_reads_below_minlength(built):
    rs = synth_reads(30, 400, 3000, 0.02, seed=62)
    assert _check(rs, _params(minlen=500)).shape[0] == 0


def test_short_all_n_and_k_long_reads_among_normal(built):
    seqs = _base_reads()
    rng = np.random.default_rng(63)
    odd = [b"ACGTACGTAC",                                  # shorter than k
           b"N" * 3000,                                     # all N
           rng.choice(np.frombuffer(b"ACGT", dtype=np.uint8), 22).tobytes(),   # exactly k
           seqs[5][:21],                                    # k - 1, from a real read
           seqs[7][100:1400] + b"N" * 50 + seqs[7][1450:]]  # an N run inside a real read
    mixed = seqs[:20] + odd + seqs[20:]
    got = _check(_readset(mixed), _params())
    assert got.shape[0] > 20


def test_duplicated_reads(built):
    seqs = _base_reads(30, seed=64)
    dup = seqs + [seqs[3], seqs[3], seqs[10][200:1800]]   # identical copies, a contained piece
    got = _check(_readset(dup), _params())
    ids = {tuple(sorted(x)) for x in zip(got["a"].tolist(), got["b"].tolist())}
    assert (4, 31) in ids and (4, 32) in ids and (31, 32) in ids


def test_empty_query_range(built):
    rs = _readset(_base_reads(20, seed=65))
    oic = OverlapInCore(_params(), device=0)
    oic.load_reads(rs)
    oic.build_hash_index()
    assert oic.find_overlaps(15, 10) == 0
    assert oic.find_overlaps(20, 20) == 0                  # the last read has no later reads
    oic.close()
