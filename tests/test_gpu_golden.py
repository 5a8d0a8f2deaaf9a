"""GPU path against the REFERENCE's own output (tests/golden, made by tools/make_golden.py
from overlapInCore compiled from its sources), plus size-independent properties at the
benchmark's read length."""
import numpy as np
import pytest

import oracle
from canu_amd.overlap_in_core import OicParameters, OverlapInCore
from canu_amd.synth import synth_reads
from test_oracle import INDEX, load_golden

pytestmark = pytest.mark.gpu


def _P(p):
    P = OicParameters(Kmer_Len=p["kmer_len"], maxErate=p["max_erate"],
                      Min_Olap_Len=p["min_olap_len"],
                      Doing_Partial_Overlaps=bool(p["partial"]),
                      Unique_Olap_Per_Pair=bool(p["unique_olap_per_pair"]),
                      Use_Window_Filter=bool(p["use_window_filter"]),
                      Use_Hopeless_Check=bool(p["use_hopeless_check"]),
                      Frag_Olap_Limit=int(p["frag_olap_limit"]),
                      Filter_By_Kmer_Count=int(p["filter_by_kmer_count"]))
    return P


@pytest.mark.parametrize("name", sorted(INDEX))
def test_golden_gpu(built, name):
    rs, p, skip, want = load_golden(name)
    oic = OverlapInCore(_P(p), device=0)
    got = oic.run(rs, skip_kmers=skip or None)
    oic.close()
    assert got.shape == want.shape
    assert np.array_equal(got, want)


def _run(rs, P, ref=None, hash_lo=1, with_stats=False):
    oic = OverlapInCore(P, device=0)
    oic.load_reads(rs)
    oic.build_hash_index(hash_lo, rs.nreads)
    n = oic.find_overlaps(*(ref or (1, rs.nreads)))
    rec = oic.fetch(n)
    st = oic.stats()
    oic.close()
    return (rec, st) if with_stats else rec


@pytest.fixture(scope="module")
def ont():
    # the benchmark's read length / error / coverage, 2k reads (the 50k job is 25x this)
    return synth_reads(2000, 10_000, 800_000, 0.015, seed=21)


def test_ont_query_subset_vs_oracle(built, ont):
    """Bit-exact at 10 kb reads: a query sub-range against the oracle over the full index."""
    P = OicParameters(Kmer_Len=22, maxErate=float(np.float32(0.06)), Min_Olap_Len=500)
    got = _run(ont, P, ref=(900, 960))
    want = oracle.run_oracle(ont, P.as_dict(), ref_range=(900, 960))
    assert len(want) > 500
    assert np.array_equal(got, want)


def test_ont_shards_union_and_determinism(built, ont):
    P = OicParameters(Kmer_Len=22, maxErate=float(np.float32(0.06)), Min_Olap_Len=500)
    whole = _run(ont, P)
    again = _run(ont, P)
    assert np.array_equal(whole, again)
    from canu_amd.dist import query_shards
    parts = [_run(ont, P, ref=r) for r in query_shards(ont.nreads, 4)]
    assert np.array_equal(oracle.sort_records(np.concatenate(parts)), whole)
    # a rank indexes only reads lo..n (its queries' targets all have larger IDs): the same
    # records and counters as against the whole index (the multi-GPU bench does this)
    for lo, hi in query_shards(ont.nreads, 4)[1:]:
        full, sf = _run(ont, P, ref=(lo, hi), with_stats=True)
        part, sp = _run(ont, P, ref=(lo, hi), hash_lo=lo, with_stats=True)
        assert np.array_equal(part, full)
        for f in ("kmer_hits_with_olap", "kmer_hits_without_olap", "kmer_hits_skipped",
                  "multi_overlaps", "total_overlaps", "contained_overlaps", "dovetail_overlaps",
                  "pairs"):
            assert sp[f] == sf[f], (f, sp[f], sf[f])
        assert sp["seed_hits"] <= sf["seed_hits"]
    # record invariants: hangs within the reads, span positive, evalue in range
    L = ont.lengths.astype(np.int64)
    a, b = whole["a"].astype(np.int64) - 1, whole["b"].astype(np.int64) - 1
    w0, w1 = whole["w0"], whole["w1"]
    ahg5, ahg3 = (w0 & 0x1FFFFF).astype(np.int64), ((w0 >> 21) & 0x1FFFFF).astype(np.int64)
    bhg5, bhg3 = (w1 & 0x1FFFFF).astype(np.int64), ((w1 >> 21) & 0x1FFFFF).astype(np.int64)
    span = (w1 >> 42) & 0x1FFFFF
    assert np.all(span > 0) and np.all(((w0 >> 42) & 0xFFF) <= 4095)
    assert np.all(ahg5 + ahg3 < L[a]) and np.all(bhg5 + bhg3 < L[b])
    assert np.all(a != b)


def test_gpu_output_files(built, tmp_path):
    """overlapInCore's -o/-s outputs from the GPU job: the .ovb decodes (reference reader
    where built, else the test decoder) to the reference's records, the .counts file is
    byte-identical to the one the reference wrote, the stats text has the reference's lines."""
    import os
    from test_ovb import GOLDEN
    rs, p, skip, want = load_golden("basic")
    oic = OverlapInCore(_P(p), device=0)
    oic.run(rs)
    path = str(tmp_path / "001.ovb.WORKING")
    oic.write_ovb(path)
    oic.write_stats(str(tmp_path / "001.stats"))
    st = oic.stats()
    oic.close()
    oracle.require_reference()
    got = oracle.read_ovb_reference(path)
    assert np.array_equal(got, want)
    assert open(str(tmp_path / "001.counts"), "rb").read() == \
        open(os.path.join(GOLDEN, "basic_ref.counts"), "rb").read()
    txt = open(str(tmp_path / "001.stats")).read().splitlines()
    assert txt[3] == f" Total overlaps produced = {st['total_overlaps']}"
    assert len(txt) == 8
