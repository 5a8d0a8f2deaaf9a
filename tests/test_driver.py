"""OverlapDriver semantics: hash batches and the ref-read block schedule.

canu's jobs run overlapInCore with hash-batch limits (--hashstrings / --hashdatalen /
--hashbits + --hashload; defaults overlapInCore.H:447-450), so one -h range can become
several hash tables (overlapInCore.C:217-287).  Batching changes results in two places:
a final one-read batch is never searched (`while (bgnHashID < endHashID)`, :222) and the
table-load limit moves batch ends (Build_Hash_Index.C:538-541); the ref reads a job
searches depend on -t through Process_Overlaps' blocks (a block that starts at endRefID
is skipped, Process_Overlaps.C:86).

CPU tests pin the oracle's restatement of the driver (oracle.run_oracle_driver) to the
reference overlapInCore (oracle/_ref/oic_ref, built from its sources) -- records AND the
-s counters.  GPU tests run the library's ovl_overlap_driver against both.
"""
import numpy as np
import pytest

from canu_amd.synth import synth_reads

import oracle

STAT_KEYS = [("total", "total_overlaps"), ("kmer_hits_with_olap", "kmer_hits_with_olap"),
             ("kmer_hits_without_olap", "kmer_hits_without_olap"), ("multi", "multi_overlaps"),
             ("contained", "contained_overlaps"), ("dovetail", "dovetail_overlaps")]

# (read set, batch options, threads, -r range)
CASES = {
    # 301 reads, 100 strings per batch: 1-100, 101-200, 201-300, then read 301 alone is
    # never hashed (the reference's `<` at overlapInCore.C:222)
    "strings_one_read_tail": (dict(n_reads=301, read_len=2500, genome_len=80_000, error_rate=0.02,
                                   seed=21, len_jitter=0.4),
                              dict(hashstrings=100), 1, None),
    # bases per batch (--hashdatalen) cut batches by length; 16 threads over -r 17-250:
    # blocks of perThread = 1 reads, the one starting at 250 is skipped
    "datalen_threads": (dict(n_reads=260, read_len=2500, genome_len=70_000, error_rate=0.02,
                             seed=22, len_jitter=0.5),
                        dict(hashstrings=150, hashdatalen=150_000), 16, (17, 250)),
    # a 2^12-bucket table at load 0.5 holds ~43k k-mers: ~17 reads per batch
    "table_load": (dict(n_reads=200, read_len=2500, genome_len=60_000, error_rate=0.02, seed=23),
                   dict(hashbits=12, hashload=0.5), 4, (3, 180)),
}


def _params():
    return oracle.default_params(kmer_len=22, max_erate=0.06, min_olap_len=500)


def _driver_kw(batch):
    return dict(hashstrings=batch.get("hashstrings", 10000),
                hashdatalen=batch.get("hashdatalen", 100_000_000),
                hashbits=batch.get("hashbits", 22), hashload=batch.get("hashload", 0.6))


def _reference(rs, P, batch, threads, rr):
    extra = ["-r", f"{rr[0]}-{rr[1]}"] if rr else []
    return oracle.run_reference(rs, P, threads=threads, hash_bits=batch.get("hashbits", 22),
                                batching={k: v for k, v in batch.items() if k != "hashbits"},
                                extra=extra, with_stats=True)


@pytest.mark.skipif(not oracle.reference_available(), reason="oracle/_ref/oic_ref not built")
@pytest.mark.parametrize("case", sorted(CASES))
def test_oracle_driver_vs_reference(case):
    kw, batch, threads, rr = CASES[case]
    rs = synth_reads(**kw)
    P = _params()
    want, wst, batches = oracle.run_oracle_driver(
        rs, P, ref_range=rr or (1, oracle.UINT32_MAX), threads=threads, with_stats=True,
        **_driver_kw(batch))
    assert len(batches) >= 3
    ref, rst = _reference(rs, P, batch, threads, rr)
    assert want.shape == ref.shape and np.array_equal(want, ref)
    for rk, ok in STAT_KEYS:
        assert wst[ok] == rst[rk], (rk, wst[ok], rst[rk])
    if case == "strings_one_read_tail":
        # the last read is in no batch: nothing overlaps it as the hashed read
        single = oracle.run_oracle(rs, P)
        assert single.shape[0] > ref.shape[0]
        assert not np.any((ref["a"] == 301) | (ref["b"] == 301))


def test_oracle_batch_end_rules():
    """Build_Hash_Index's stop rules on a read set small enough to count by hand."""
    rs = synth_reads(n_reads=40, read_len=1000, genome_len=20_000, error_rate=0.0, seed=24)
    P = _params()
    # strings: 10 IDs per batch
    assert oracle.hash_batch_end(rs, P, 1, 40, 10, 10**8, 22, 0.6) == 10
    # bases: each read adds len + 1 = 1001; the read that reaches 3,500 ends the batch
    assert oracle.hash_batch_end(rs, P, 1, 40, 1000, 3500, 22, 0.6) == 4
    # table load: a 2^7-bucket table at load 1.0 holds 2688 entries; error-free reads of a
    # 20 kb genome bring ~979 new k-mers each until the genome is covered
    end = oracle.hash_batch_end(rs, P, 1, 40, 1000, 10**8, 7, 1.0)
    hist = oracle.first_read_kmers(rs, 1, 40, 22, lambda r: True)
    assert np.cumsum(hist)[end - 1] >= 2688 > np.cumsum(hist)[end - 2]


@pytest.mark.gpu
@pytest.mark.parametrize("case", sorted(CASES))
def test_gpu_driver_vs_oracle_and_reference(built, case):
    from canu_amd.overlap_in_core import OicParameters, OverlapInCore
    kw, batch, threads, rr = CASES[case]
    rs = synth_reads(**kw)
    P = _params()
    want, wst, batches = oracle.run_oracle_driver(
        rs, P, ref_range=rr or (1, oracle.UINT32_MAX), threads=threads, with_stats=True,
        **_driver_kw(batch))
    d = _driver_kw(batch)
    O = OicParameters(Kmer_Len=22, maxErate=P["max_erate"], Min_Olap_Len=500,
                      Max_Hash_Strings=d["hashstrings"], Max_Hash_Data_Len=d["hashdatalen"],
                      Hash_Mask_Bits=d["hashbits"], Max_Hash_Load=d["hashload"],
                      Num_PThreads=threads).finalize()
    if rr:
        O.bgnRefID, O.endRefID = rr
    oic = OverlapInCore(O, device=0)
    got = oic.run_driver(rs)
    st = oic.stats()
    oic.close()
    assert st["hash_batches"] == len(batches)
    assert got.shape == want.shape and np.array_equal(got, want)
    for _, ok in STAT_KEYS:
        assert st[ok] == wst[ok], (ok, st[ok], wst[ok])
    oracle.require_reference()
    ref, rst = _reference(rs, P, batch, threads, rr)
    assert np.array_equal(got, ref)
    assert st["total_overlaps"] == rst["total"]


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["table_load", "datalen_threads"])
def test_gpu_driver_sorted_windows_vs_oracle(built, monkeypatch, case):
    """The driver cases with the job's sorted query windows from the second batch on
    (OVL_SQ=2; off by default): the table-load case is the one whose 882,524-window run a
    partial-range radix sort returned with duplicated window ids."""
    from canu_amd.overlap_in_core import OicParameters, OverlapInCore
    monkeypatch.setenv("OVL_SQ", "2")
    kw, batch, threads, rr = CASES[case]
    rs = synth_reads(**kw)
    P = _params()
    want, wst, batches = oracle.run_oracle_driver(
        rs, P, ref_range=rr or (1, oracle.UINT32_MAX), threads=threads, with_stats=True,
        **_driver_kw(batch))
    d = _driver_kw(batch)
    O = OicParameters(Kmer_Len=22, maxErate=P["max_erate"], Min_Olap_Len=500,
                      Max_Hash_Strings=d["hashstrings"], Max_Hash_Data_Len=d["hashdatalen"],
                      Hash_Mask_Bits=d["hashbits"], Max_Hash_Load=d["hashload"],
                      Num_PThreads=threads).finalize()
    if rr:
        O.bgnRefID, O.endRefID = rr
    oic = OverlapInCore(O, device=0)
    got = oic.run_driver(rs)
    st = oic.stats()
    oic.close()
    assert st["hash_batches"] == len(batches) >= 3
    assert got.shape == want.shape and np.array_equal(got, want)
    for _, ok in STAT_KEYS:
        assert st[ok] == wst[ok], (ok, st[ok], wst[ok])


@pytest.mark.gpu
def test_gpu_driver_10kb_production_batches(built):
    """Reads at the benchmark's 10 kb length under byte-limited batches (canu's
    partitionLength hands each job --hashdatalen; here ~1 Mbp per batch): 4 batches, the
    last a single read that is never hashed.  Bit-exact against the reference itself."""
    from canu_amd.overlap_in_core import OicParameters, OverlapInCore
    rs = synth_reads(n_reads=301, read_len=10_000, genome_len=400_000, error_rate=0.015, seed=25)
    P = _params()
    O = OicParameters(Kmer_Len=22, maxErate=P["max_erate"], Min_Olap_Len=500,
                      Max_Hash_Data_Len=1_000_000, Num_PThreads=8).finalize()
    oic = OverlapInCore(O, device=0)
    got = oic.run_driver(rs)
    st = oic.stats()
    oic.close()
    assert st["hash_batches"] == 3
    want, wst, batches = oracle.run_oracle_driver(rs, P, threads=8, hashdatalen=1_000_000,
                                                  with_stats=True)
    assert batches[-1][1] == 300
    assert np.array_equal(got, want)
    oracle.require_reference()
    ref, rst = oracle.run_reference(rs, P, threads=8, hash_bits=22,
                                    batching={"hashdatalen": 1_000_000}, with_stats=True)
    assert np.array_equal(got, ref)
    for rk, ok in STAT_KEYS:
        assert st[ok] == rst[rk], (rk, st[ok], rst[rk])


@pytest.mark.gpu
def test_gpu_driver_load_cut_within_window_cap(built, monkeypatch):
    """A batch the table load cuts, built from a prefix of the -h range: when the range
    holds more windows than one index may take (OVL_TEST_INDEX_WINDOW_CAP stands in for the
    HBM / 2^32 cap), the first build covers the longest prefix within the cap and the load
    has to stop the batch inside it -- the same batches and records as without the cap.
    A cap the load cannot be reached within fails loudly instead of changing the batches."""
    from canu_amd.overlap_in_core import OicParameters, OverlapInCore, OvlError
    kw, batch, threads, rr = CASES["table_load"]
    rs = synth_reads(**kw)
    P = _params()
    want, wst, batches = oracle.run_oracle_driver(
        rs, P, ref_range=rr, threads=threads, with_stats=True, **_driver_kw(batch))
    d = _driver_kw(batch)

    def run():
        O = OicParameters(Kmer_Len=22, maxErate=P["max_erate"], Min_Olap_Len=500,
                          Hash_Mask_Bits=d["hashbits"], Max_Hash_Load=d["hashload"],
                          Num_PThreads=threads).finalize()
        O.bgnRefID, O.endRefID = rr
        oic = OverlapInCore(O, device=0)
        try:
            got = oic.run_driver(rs)
            return got, oic.stats()
        finally:
            oic.close()

    monkeypatch.setenv("OVL_TEST_INDEX_WINDOW_CAP", "80000")
    got, st = run()
    assert st["hash_batches"] == len(batches)
    assert np.array_equal(got, want)
    for _, ok in STAT_KEYS:
        assert st[ok] == wst[ok], (ok, st[ok], wst[ok])
    monkeypatch.setenv("OVL_TEST_INDEX_WINDOW_CAP", "20000")
    with pytest.raises(OvlError, match="load limit"):
        run()


@pytest.mark.gpu
def test_gpu_driver_batch_past_index_cap_fails_with_its_reason(built, monkeypatch):
    """Super-batch mode (the default): a hash batch the table load cannot cut but no index on
    this GPU could hold (OVL_TEST_INDEX_WINDOW_CAP stands in for the HBM cap) is refused in
    the driver's first phase with the batch-by-batch path's message, not a bare out-of-memory
    later."""
    from canu_amd.overlap_in_core import OicParameters, OverlapInCore, OvlError
    rs = synth_reads(n_reads=60, read_len=3000, genome_len=30_000, error_rate=0.02, seed=27)
    O = OicParameters(Kmer_Len=22, maxErate=0.06, Min_Olap_Len=500, Hash_Mask_Bits=22,
                      Max_Hash_Load=0.75, Max_Hash_Strings=30, Num_PThreads=4).finalize()
    monkeypatch.setenv("OVL_TEST_INDEX_WINDOW_CAP", "20000")
    oic = OverlapInCore(O, device=0)
    try:
        with pytest.raises(OvlError, match="lower --hashstrings"):
            oic.run_driver(rs)
    finally:
        oic.close()


def _lib_case():
    """Reads spread over three gkpStore libraries, -H 1-2 (hash libraries 1 and 2 only) and
    -R 2-3 (search from libraries 2 and 3 only), small hash batches (Build_Hash_Index.C:
    500-503 / :554-556, Process_Overlaps.C:108-109): a skipped read still counts towards
    --hashstrings, so the filters move batch ends."""
    rs = synth_reads(n_reads=150, read_len=2500, genome_len=45_000, error_rate=0.02, seed=26,
                     len_jitter=0.3)
    libs = (np.random.default_rng(26).integers(1, 4, size=rs.nreads)).astype(np.uint32)
    return rs, libs, dict(hashstrings=40), 4, ["-H", "1-2", "-R", "2-3"]


@pytest.mark.skipif(not oracle.reference_available(), reason="oracle/_ref/oic_ref not built")
def test_reference_library_filters_take_effect():
    """CPU: the reference run with -H / -R differs from the unfiltered one, and no record
    pairs two reads the filters exclude from both roles."""
    rs, libs, batch, threads, extra = _lib_case()
    P = _params()
    ref = oracle.run_reference(rs, P, threads=threads, hash_bits=22, batching=batch,
                               libs=libs, extra=extra)
    plain = oracle.run_reference(rs, P, threads=threads, hash_bits=22, batching=batch)
    assert 0 < ref.shape[0] < plain.shape[0]
    la, lb = libs[ref["a"] - 1], libs[ref["b"] - 1]
    # one read of each pair was hashed (library 1-2), the other searched (library 2-3)
    ok = ((la <= 2) & (lb >= 2)) | ((lb <= 2) & (la >= 2))
    assert ok.all()


@pytest.mark.gpu
def test_gpu_driver_library_filters(built):
    """ovl_set_read_libraries + -H / -R through ovl_overlap_driver: records and every -s
    counter equal the reference's, run on a gkpStore with the same libraries."""
    from canu_amd.overlap_in_core import OicParameters, OverlapInCore
    rs, libs, batch, threads, extra = _lib_case()
    P = _params()
    O = OicParameters(Kmer_Len=22, maxErate=P["max_erate"], Min_Olap_Len=500,
                      Max_Hash_Strings=batch["hashstrings"], Num_PThreads=threads,
                      minLibToHash=1, maxLibToHash=2, minLibToRef=2, maxLibToRef=3).finalize()
    oic = OverlapInCore(O, device=0)
    try:
        oic.load_reads(rs)
        oic.set_read_libraries(libs)
        got = oic.fetch(oic.overlap_driver())
        st = oic.stats()
    finally:
        oic.close()
    oracle.require_reference()
    ref, rst = oracle.run_reference(rs, P, threads=threads, hash_bits=22, batching=batch,
                                    libs=libs, extra=extra, with_stats=True)
    assert got.shape == ref.shape and np.array_equal(got, ref)
    for rk, ok in STAT_KEYS:
        assert st[ok] == rst[rk], (rk, st[ok], rst[rk])


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["0", "1"])
def test_gpu_bloom_filter_is_exact(built, monkeypatch, mode):
    """The probe's Bloom filter (OverlapDriver batches probed mostly by reads outside the
    hash range; ensure_bloom / use_bloom in ovl_api.hip) has no false negatives, so records
    and every -s counter are those of the table alone: the production-batch job of
    10 kb reads in 70-read hash batches with the filter forced off (OVL_BLOOM=0) and on
    for every search (OVL_BLOOM=1, also the searches it would skip) against the oracle."""
    from canu_amd.overlap_in_core import OicParameters, OverlapInCore
    monkeypatch.setenv("OVL_BLOOM", mode)
    rs = synth_reads(n_reads=301, read_len=10_000, genome_len=400_000, error_rate=0.015, seed=26)
    P = _params()
    O = OicParameters(Kmer_Len=22, maxErate=P["max_erate"], Min_Olap_Len=500,
                      Max_Hash_Strings=70, Num_PThreads=8).finalize()
    oic = OverlapInCore(O, device=0)
    got = oic.run_driver(rs)
    st = oic.stats()
    oic.close()
    want, wst, batches = oracle.run_oracle_driver(rs, P, threads=8, hashstrings=70,
                                                  with_stats=True)
    assert st["hash_batches"] == len(batches) >= 4
    assert got.shape == want.shape and np.array_equal(got, want)
    for _, ok in STAT_KEYS:
        assert st[ok] == wst[ok], (ok, st[ok], wst[ok])


def _end_skip_kmers(rs, k=22, step=23, span=110):
    """Skip k-mers taken near both ends of every third read: Mark_Skip_Kmers then marks
    those reads' ends screened (Build_Hash_Index.C:147-156), which the hopeless check of
    Process_Matches reads for the TARGET of a single-match pair
    (Process_String_Overlaps.C:445, :455)."""
    out = set()
    for r in range(0, rs.nreads, 3):
        seq = rs.read(r).decode().upper()
        for i in list(range(0, span, step)) + list(range(len(seq) - span, len(seq) - k, step)):
            s = seq[i:i + k]
            if len(s) == k and set(s) <= set("ACGT"):
                out.add(s)
    return sorted(out)


@pytest.mark.gpu
def test_gpu_driver_screened_ends_across_batches(built):
    """Pairs found in one hash batch are extended after later batches have been built (the
    extension accumulator).  The target's screened-end bits must be those of the batch
    that found the pair, as in the reference, where every batch is extended before the
    next is built: a multi-batch job with end skip k-mers, maxErate 0.06 (hopeless check
    on) and noisy reads (many single-match pairs), bit-exact against the reference
    overlapInCore and its -s counters."""
    from canu_amd.overlap_in_core import OicParameters, OverlapInCore
    oracle.require_reference()
    rs = synth_reads(n_reads=240, read_len=3000, genome_len=60_000, error_rate=0.035, seed=27,
                     len_jitter=0.3)
    skip = _end_skip_kmers(rs)
    P = _params()
    O = OicParameters(Kmer_Len=22, maxErate=P["max_erate"], Min_Olap_Len=500,
                      Max_Hash_Strings=50, Num_PThreads=4).finalize()
    oic = OverlapInCore(O, device=0)
    got = oic.run_driver(rs, skip_kmers=skip)
    st = oic.stats()
    oic.close()
    assert st["hash_batches"] >= 4
    ref, rst = oracle.run_reference(rs, P, threads=4, hash_bits=22,
                                    batching={"hashstrings": 50}, skip_kmers=skip,
                                    with_stats=True)
    assert got.shape == ref.shape and np.array_equal(got, ref)
    for rk, ok in STAT_KEYS:
        assert st[ok] == rst[rk], (rk, st[ok], rst[rk])


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["0", "1"])
def test_gpu_sorted_query_windows_are_exact(built, monkeypatch, mode):
    """OverlapDriver batches searched through the job's query windows sorted once by k-mer
    (k_probe_sorted; OVL_SQ=1 from the first batch) and by one random table lookup per
    window (k_probe; OVL_SQ=0): the same records and -s counters, the reference's -- with
    N bases (windows without a k-mer, NUL-ended reverse strands), ragged lengths and end
    skip k-mers (screened ends set from the sorted windows)."""
    from canu_amd.overlap_in_core import OicParameters, OverlapInCore
    oracle.require_reference()
    monkeypatch.setenv("OVL_SQ", mode)
    rs = synth_reads(n_reads=240, read_len=3000, genome_len=60_000, error_rate=0.03, seed=28,
                     len_jitter=0.4, n_rate=0.001)
    skip = _end_skip_kmers(rs)
    P = _params()
    O = OicParameters(Kmer_Len=22, maxErate=P["max_erate"], Min_Olap_Len=500,
                      Max_Hash_Strings=45, Num_PThreads=4).finalize()
    oic = OverlapInCore(O, device=0)
    got = oic.run_driver(rs, skip_kmers=skip)
    st = oic.stats()
    oic.close()
    assert st["hash_batches"] >= 5
    ref, rst = oracle.run_reference(rs, P, threads=4, hash_bits=22,
                                    batching={"hashstrings": 45}, skip_kmers=skip,
                                    with_stats=True)
    assert got.shape == ref.shape and np.array_equal(got, ref)
    for rk, ok in STAT_KEYS:
        assert st[ok] == rst[rk], (rk, st[ok], rst[rk])


def _ref_last(rs, rr, threads):
    nr = rs.first_iid + rs.nreads - 1
    gbr, ger = (max(rr[0], 1), min(rr[1], nr)) if rr else (1, nr)
    per = 1 + (ger - gbr) // max(threads, 1) // 8
    return gbr, (ger - 1 if (ger - gbr) % per == 0 else ger)


@pytest.mark.parametrize("case", sorted(CASES) + ["screened_ends"])
@pytest.mark.parametrize("group", [2, 0])
def test_oracle_super_batches_equal_batches(case, group):
    """The driver's super-batches (ovl_overlap_driver): searching the UNION of consecutive
    hash batches gives the records and every counter that searching them one by one gives --
    a query meets, in any batch, exactly the hashed reads with larger IDs (Find_Overlaps.C:328)
    and a pair's seeds, chain and screened ends depend on the pair alone.  Checked on the
    oracle (pinned to the reference): batches joined two by two (group=2) and all into one
    (group=0), against the batch-by-batch OverlapDriver restatement."""
    if case == "screened_ends":
        rs = synth_reads(n_reads=240, read_len=3000, genome_len=60_000, error_rate=0.035,
                         seed=27, len_jitter=0.3)
        batch, threads, rr, skip = dict(hashstrings=50), 4, None, _end_skip_kmers(rs)
    else:
        kw, batch, threads, rr = CASES[case]
        rs = synth_reads(**kw)
        skip = None
    P = _params()
    want, wst, batches = oracle.run_oracle_driver(
        rs, P, ref_range=rr or (1, oracle.UINT32_MAX), threads=threads, with_stats=True,
        skip_kmers=skip, **_driver_kw(batch))
    assert len(batches) >= 3
    gbr, ref_last = _ref_last(rs, rr, threads)
    groups = [batches] if group == 0 else [batches[i:i + group] for i in range(0, len(batches), group)]
    recs, tot = [], None
    for g in groups:
        rec, st = oracle.run_oracle(rs, P, hash_range=(g[0][0], g[-1][1]), ref_range=(gbr, ref_last),
                                    skip_kmers=skip, with_stats=True)
        recs.append(rec)
        tot = st if tot is None else {f: tot[f] + st[f] for f in st}
    got = oracle.sort_records(np.concatenate(recs))
    assert got.shape == want.shape and np.array_equal(got, want)
    for _, f in STAT_KEYS:
        assert tot[f] == wst[f], (f, tot[f], wst[f])


@pytest.mark.gpu
def test_gpu_cut_index_equals_rebuild(built, monkeypatch):
    """A hash batch the table load cuts inside its first build: the prefix's index cut down
    to the batch by k_cut_index (the default) searches exactly like an index built again over
    the batch's own reads (OVL_CUT_FILTER=0) -- same batch ends, records and every counter,
    for two consecutive batches, with end skip k-mers (screened-end bits set by the prefix
    build on reads past the cut, Build_Hash_Index.C:147-170)."""
    from canu_amd.overlap_in_core import OicParameters, OverlapInCore
    kw, batch, _, _ = CASES["table_load"]
    rs = synth_reads(**kw)
    skip = _end_skip_kmers(rs)
    P = _params()
    out = {}
    for mode in ("1", "0"):
        monkeypatch.setenv("OVL_CUT_FILTER", mode)
        O = OicParameters(Kmer_Len=22, maxErate=P["max_erate"], Min_Olap_Len=500,
                          Hash_Mask_Bits=batch["hashbits"],
                          Max_Hash_Load=batch["hashload"]).finalize()
        oic = OverlapInCore(O, device=0)
        try:
            oic.load_reads(rs)
            oic.set_skip_kmers(skip)
            res = []
            bgn = 1
            for _ in range(2):
                last = oic.build_hash_batch(bgn, rs.nreads)
                got = oic.fetch(oic.find_overlaps(1, rs.nreads))
                st = oic.stats()
                res.append((last, got, {k: st[k] for _, k in STAT_KEYS}))
                bgn = last + 1
        finally:
            oic.close()
        out[mode] = res
    for (l1, g1, s1), (l0, g0, s0) in zip(out["1"], out["0"]):
        assert 1 < l1 < rs.nreads and l1 == l0
        assert g1.shape[0] > 0 and g1.shape == g0.shape and np.array_equal(g1, g0)
        assert s1 == s0
