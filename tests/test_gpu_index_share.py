"""Sharing a built k-mer index between contexts (ovl_export_index / ovl_import_index, ABI 7):
the north star's "one index, shared over xGMI" path.  One context builds the index
(Build_Hash_Index, overlapInCore-Build_Hash_Index.C:443 -- table, occurrence lists, and the
screened-end flags Mark_Skip_Kmers sets on hashed reads); a second context holding the same
reads imports it by device copy and searches it (Find_Overlaps.C:284): its records and -s
counters must equal the builder's own search, and the oracle's.
"""
import numpy as np
import pytest

from canu_amd.synth import synth_reads

import oracle

STAT_KEYS = ["total_overlaps", "kmer_hits_with_olap", "kmer_hits_without_olap",
             "multi_overlaps", "contained_overlaps", "dovetail_overlaps", "kmer_hits_skipped",
             "seed_hits", "pairs"]


def _end_skip_kmers(rs, k=22, step=23, span=110):
    out = set()
    for r in range(0, rs.nreads, 3):
        seq = rs.read(r).decode().upper()
        for i in list(range(0, span, step)) + list(range(len(seq) - span, len(seq) - k, step)):
            s = seq[i:i + k]
            if len(s) == k and set(s) <= set("ACGT"):
                out.add(s)
    return sorted(out)


@pytest.mark.gpu
@pytest.mark.parametrize("batch", [False, True])
def test_gpu_imported_index_searches_like_the_built_one(built, batch):
    """batch=False: ovl_build_hash_index over every read (one table, no filter);
    batch=True: an OverlapDriver batch (ovl_build_hash_batch, reads 1-90, with its Bloom
    filter) searched by every read, most of which lie outside it.  Skip k-mers near read ends
    make the imported screened-end flags matter (the hopeless check reads them)."""
    from canu_amd.overlap_in_core import OicParameters, OverlapInCore
    rs = synth_reads(n_reads=240, read_len=3000, genome_len=60_000, error_rate=0.035, seed=41,
                     len_jitter=0.3, n_rate=0.001)
    skip = _end_skip_kmers(rs)
    P = oracle.default_params(kmer_len=22, max_erate=0.06, min_olap_len=500)
    O = OicParameters(Kmer_Len=22, maxErate=P["max_erate"], Min_Olap_Len=500,
                      Max_Hash_Strings=90).finalize()
    a = OverlapInCore(O, device=0)
    b = OverlapInCore(O, device=0)
    try:
        a.load_reads(rs)
        a.set_skip_kmers(skip)
        if batch:
            last = a.build_hash_batch(1, rs.nreads)
            assert last == 90
        else:
            a.build_hash_index(1, rs.nreads)
        desc = a.export_index()
        assert desc.records > 0 and desc.table_bytes == 16 << desc.tab_bits
        assert (desc.bloom_bytes > 0) == batch
        b.load_reads(rs)
        b.import_index(desc)
        got_b = b.fetch(b.find_overlaps(1, rs.nreads))
        st_b = b.stats()
        got_a = a.fetch(a.find_overlaps(1, rs.nreads))
        st_a = a.stats()
    finally:
        a.close()
        b.close()
    assert got_a.shape[0] > (10 if batch else 100)
    assert got_b.shape == got_a.shape and np.array_equal(got_b, got_a)
    for key in STAT_KEYS:
        assert st_b[key] == st_a[key], (key, st_b[key], st_a[key])
    if not batch:
        want = oracle.run_oracle(rs, P, skip_kmers=skip)
        assert np.array_equal(got_b, want)


@pytest.mark.gpu
def test_gpu_import_rejects_another_read_store(built):
    """An index built over other reads (or another k) is refused, not searched."""
    from canu_amd.overlap_in_core import OicParameters, OverlapInCore, OvlError
    rs = synth_reads(n_reads=60, read_len=2000, genome_len=20_000, error_rate=0.02, seed=42)
    O = OicParameters(Kmer_Len=22, maxErate=0.06, Min_Olap_Len=500).finalize()
    a = OverlapInCore(O, device=0)
    b = OverlapInCore(O, device=0)
    try:
        a.load_reads(rs)
        a.build_hash_index(1, rs.nreads)
        desc = a.export_index()
        rs2 = synth_reads(n_reads=59, read_len=2000, genome_len=20_000, error_rate=0.02, seed=42)
        b.load_reads(rs2)
        with pytest.raises(OvlError, match="index of reads"):
            b.import_index(desc)
    finally:
        a.close()
        b.close()


@pytest.mark.gpu
def test_gpu_share_index_through_torch_buffers(built):
    """dist.share_index, the path bench.py --gpus N takes over RCCL: the exported buffers are
    copied into torch tensors (what a broadcast would fill on every rank) and imported from
    there; without a process group it runs on one GPU.  Same records and counters."""
    import torch
    from canu_amd.dist import share_index
    from canu_amd.overlap_in_core import OicParameters, OverlapInCore
    rs = synth_reads(n_reads=200, read_len=3000, genome_len=50_000, error_rate=0.03, seed=43)
    O = OicParameters(Kmer_Len=22, maxErate=0.06, Min_Olap_Len=500).finalize()
    a = OverlapInCore(O, device=0)
    b = OverlapInCore(O, device=0)
    try:
        a.load_reads(rs)
        a.build_hash_index(41, rs.nreads)
        b.load_reads(rs)
        moved = share_index(a, [b], None, torch.device("cuda", 0))
        assert moved > 0
        got_b = b.fetch(b.find_overlaps(41, 120))
        st_b = b.stats()
        got_a = a.fetch(a.find_overlaps(41, 120))
        st_a = a.stats()
    finally:
        a.close()
        b.close()
    assert got_a.shape[0] > 100
    assert np.array_equal(got_b, got_a)
    for key in STAT_KEYS:
        assert st_b[key] == st_a[key], key


@pytest.mark.gpu
def test_gpu_import_rejects_descriptor_past_build_limits(built):
    """A descriptor the build could not have produced (a corrupted broadcast, another build)
    is refused before any kernel reads it: a filter of more than 2^6 words per fine bucket,
    2^32 or more occurrence records (the table's run offsets are 32-bit), or a slice whose
    wave would not fit 64 KB of LDS."""
    import ctypes
    from canu_amd.overlap_in_core import OicParameters, OverlapInCore, OvlError
    rs = synth_reads(n_reads=120, read_len=3000, genome_len=40_000, error_rate=0.02, seed=44)
    O = OicParameters(Kmer_Len=22, maxErate=0.06, Min_Olap_Len=500,
                      Max_Hash_Strings=60).finalize()
    a = OverlapInCore(O, device=0)
    b = OverlapInCore(O, device=0)
    try:
        a.load_reads(rs)
        b.load_reads(rs)
        assert a.build_hash_batch(1, rs.nreads) == 60
        good = a.export_index()
        assert good.bloom_bytes > 0

        def bad(**kw):
            d = type(good)()
            ctypes.memmove(ctypes.addressof(d), ctypes.addressof(good), ctypes.sizeof(good))
            for f, v in kw.items():
                setattr(d, f, v)
            return d

        nfine = good.table_bytes // 16 >> good.slice_bits
        cases = [
            bad(bloom_w=7, bloom_bytes=8 * (nfine << 7)),
            bad(records=1 << 32, occ_bytes=8 << 32),
            bad(slice_bits=13, bloom_bytes=8 * ((good.table_bytes // 16 >> 13) << good.bloom_w)),
        ]
        for d in cases:
            with pytest.raises(OvlError, match="inconsistent index descriptor|past the build's"):
                b.import_index(d)
        b.import_index(good)                 # the real one still imports and searches
        got_b = b.fetch(b.find_overlaps(1, rs.nreads))
        got_a = a.fetch(a.find_overlaps(1, rs.nreads))
    finally:
        a.close()
        b.close()
    assert np.array_equal(got_b, got_a)
