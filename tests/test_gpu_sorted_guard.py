"""The sorted query windows of OverlapDriver jobs (k_sq_keys / k_probe_sorted, sq_prepare in
ovl_api.hip) against two failure modes that would lose or invent probe records:

* stale window slots: a reverse unit whose strand holds a NUL (the reverse complement of an
  'n') has fewer windows than the L - k + 1 slots its run reserves; those tail slots must be
  written as "no k-mer", or the sort and the probe read an earlier run's (key, wid) pairs --
  with zeroed memory the pair (key 0, wid 0), and key 0 is mix64 of the all-A k-mer.  Reads
  with 'n' bases plus poly-A stretches, two driver jobs in one context;
* a radix sort that keeps the key order but duplicates a window id (what this ROCm's
  partial-range sort did): the check compares the (key, wid) multiset
  before and after the sort; OVL_TEST_SQ_CORRUPT=1 duplicates an id in the first run's sorted
  output, and the run must be sorted again over all bits with the records unchanged.

Reference semantics: Find_Overlaps.C:284-370 (every window's Hash_Find), which the probe
records must equal; checked against the oracle (pinned to the reference overlapInCore).
"""
import numpy as np
import pytest

from canu_amd.synth import synth_reads

import oracle

STAT_KEYS = [("total", "total_overlaps"), ("kmer_hits_with_olap", "kmer_hits_with_olap"),
             ("kmer_hits_without_olap", "kmer_hits_without_olap"), ("multi", "multi_overlaps"),
             ("contained", "contained_overlaps"), ("dovetail", "dovetail_overlaps")]


def _reads():
    rs = synth_reads(n_reads=240, read_len=3000, genome_len=60_000, error_rate=0.03, seed=31,
                     len_jitter=0.4, n_rate=0.002)
    # poly-A stretches (>= k) in every 7th read: the table then holds the all-A k-mer (key 0)
    b = rs.bases.copy()
    for r in range(0, rs.nreads, 7):
        o, L = int(rs.offsets[r]), int(rs.lengths[r])
        if L > 400:
            b[o + 200:o + 240] = ord("A")
    rs.bases = b
    return rs


def _params():
    return oracle.default_params(kmer_len=22, max_erate=0.06, min_olap_len=500)


def _opts(P, rr):
    from canu_amd.overlap_in_core import OicParameters
    O = OicParameters(Kmer_Len=22, maxErate=P["max_erate"], Min_Olap_Len=500,
                      Max_Hash_Strings=45, Num_PThreads=4).finalize()
    O.bgnRefID, O.endRefID = rr
    return O


def _oracle(rs, P, rr):
    want, wst, batches = oracle.run_oracle_driver(rs, P, ref_range=rr, threads=4,
                                                  hashstrings=45, with_stats=True)
    return want, wst, batches


def test_reads_have_nul_tails_and_poly_a():
    """CPU: the read set really exercises the stale-slot case (reads with 'n', so reverse
    units with a NUL, and all-A k-mers)."""
    rs = _reads()
    has_n = [b"N" in rs.read(r) for r in range(rs.nreads)]
    assert sum(has_n) > 50
    assert sum(b"A" * 22 in rs.read(r) for r in range(rs.nreads)) >= 30


@pytest.mark.gpu
def test_gpu_sorted_windows_two_jobs_nul_tails(built, monkeypatch):
    """Two driver jobs in one context through the sorted windows (OVL_SQ=1): the second job
    searches a different -r range over the grown-only buffers the first one left."""
    from canu_amd.overlap_in_core import OverlapInCore
    monkeypatch.setenv("OVL_SQ", "1")
    rs = _reads()
    P = _params()
    oic = OverlapInCore(_opts(P, (1, 240)), device=0)
    try:
        oic.load_reads(rs)
        for rr in [(1, 240), (31, 200)]:
            oic.params.bgnRefID, oic.params.endRefID = rr
            got = oic.fetch(oic.overlap_driver())
            st = oic.stats()
            want, wst, batches = _oracle(rs, P, rr)
            assert st["hash_batches"] == len(batches) >= 5
            assert st["probe_sorted_launches"] > 0
            assert got.shape == want.shape and np.array_equal(got, want), rr
            for _, ok in STAT_KEYS:
                assert st[ok] == wst[ok], (rr, ok, st[ok], wst[ok])
    finally:
        oic.close()


@pytest.mark.gpu
def test_gpu_sorted_windows_corrupt_sort_falls_back(built, monkeypatch):
    """A sorted run whose window ids are no longer a permutation (one id duplicated after the
    sort, keys still ordered) fails the check and is sorted again over all bits: the job's
    records and counters stay the oracle's, and the stats count the re-sorted run."""
    from canu_amd.overlap_in_core import OverlapInCore
    monkeypatch.setenv("OVL_SQ", "1")
    monkeypatch.setenv("OVL_TEST_SQ_CORRUPT", "1")
    rs = _reads()
    P = _params()
    rr = (1, 240)
    oic = OverlapInCore(_opts(P, rr), device=0)
    try:
        got = oic.run_driver(rs)
        st = oic.stats()
    finally:
        oic.close()
    want, wst, batches = _oracle(rs, P, rr)
    assert st["sq_resorted"] >= 1
    assert st["probe_sorted_launches"] > 0
    assert got.shape == want.shape and np.array_equal(got, want)
    for _, ok in STAT_KEYS:
        assert st[ok] == wst[ok], (ok, st[ok], wst[ok])


@pytest.mark.gpu
@pytest.mark.parametrize("chunk_w,sb_w,dense", [("200000", None, None), ("200000", "300000", "1"),
                                                 (None, "250000", None)])
def test_gpu_query_chunks_and_super_batches_are_exact(built, monkeypatch, chunk_w, sb_w, dense):
    """The driver's search plan (ovl_overlap_driver): the reference's hash batches found by
    its loading loop, consecutive batches joined into super-batches (OVL_SB_WINDOWS caps
    their k-mers), and the -r range searched in query chunks whose sorted windows fit
    (OVL_SQ_CHUNK_WINDOWS caps them), every (chunk, super-batch) pair whose reads can meet
    searched once.  On the small job the caps force ~7 chunks and / or ~5 super-batches: the
    same records and -s counters as the oracle's batch-by-batch OverlapDriver, with N bases
    and poly-A stretches.  dense: the half-size tables a chunked full-size job builds
    (OVL_DENSE_TABLES forces them here)."""
    from canu_amd.overlap_in_core import OverlapInCore
    monkeypatch.setenv("OVL_SQ", "1" if chunk_w else "0")
    if dense:
        monkeypatch.setenv("OVL_DENSE_TABLES", dense)
    if chunk_w:
        monkeypatch.setenv("OVL_SQ_CHUNK_WINDOWS", chunk_w)
    if sb_w:
        monkeypatch.setenv("OVL_SB_WINDOWS", sb_w)
    rs = _reads()
    P = _params()
    rr = (1, 240)
    oic = OverlapInCore(_opts(P, rr), device=0)
    try:
        got = oic.run_driver(rs)
        st = oic.stats()
    finally:
        oic.close()
    want, wst, batches = _oracle(rs, P, rr)
    if chunk_w:
        assert st["query_chunks"] >= 5
    if sb_w:
        assert 3 <= st["super_batches"] < len(batches)
    assert st["hash_batches"] == len(batches)
    assert got.shape == want.shape and np.array_equal(got, want)
    for _, ok in STAT_KEYS:
        assert st[ok] == wst[ok], (ok, st[ok], wst[ok])


@pytest.mark.gpu
def test_gpu_batch_by_batch_driver_is_exact(built, monkeypatch):
    """OVL_SUPERBATCH=0: the reference's loop order (build a batch, search it), which -l jobs
    always take -- the same records and counters."""
    from canu_amd.overlap_in_core import OverlapInCore
    monkeypatch.setenv("OVL_SUPERBATCH", "0")
    rs = _reads()
    P = _params()
    rr = (1, 240)
    oic = OverlapInCore(_opts(P, rr), device=0)
    try:
        got = oic.run_driver(rs)
        st = oic.stats()
    finally:
        oic.close()
    want, wst, batches = _oracle(rs, P, rr)
    assert st["super_batches"] == 0 and st["hash_batches"] == len(batches)
    assert got.shape == want.shape and np.array_equal(got, want)
    for _, ok in STAT_KEYS:
        assert st[ok] == wst[ok], (ok, st[ok], wst[ok])
