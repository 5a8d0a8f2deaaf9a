"""-l (Frag_Olap_Limit): per query strand, at most that many overlaps off each end.

Process_String_Olaps (overlapInCore-Process_String_Overlaps.C:687-790) walks a query's
targets in String_Olap_Space order; past the limit it sorts them by average diagonal and
walks the non-negative ones up while A_Olaps_For_Frag < limit, then the negative ones down
while B_Olaps_For_Frag < limit, and Process_Matches (:481-487) stops extending matches off
an end that has its limit.  Results depend on the order, so the GPU runs each query strand's
pairs one after another in that order (k_extend's ORD variant, ovl_api.hip k_olim_*).

CPU tests pin the oracle (oracle/oic_oracle.c) to the reference overlapInCore built from
its sources (records and the -s counters); GPU tests hold the library to the oracle.
"""
import numpy as np
import pytest

import oracle
from canu_amd.synth import synth_reads

STAT_KEYS = [("total", "total_overlaps"), ("kmer_hits_with_olap", "kmer_hits_with_olap"),
             ("kmer_hits_without_olap", "kmer_hits_without_olap"), ("multi", "multi_overlaps"),
             ("contained", "contained_overlaps"), ("dovetail", "dovetail_overlaps")]

# (read-set seed, limit, options): repeats give queries many targets (ties of the average
# diagonal among them); limits from 1 up, unique and non-unique, partial (-G, canu's mode)
CASES = {
    "l1": (203, 1, {}),
    "l3": (201, 3, {}),
    "l5_multi": (202, 5, {"unique_olap_per_pair": 0}),
    "l2_multi": (205, 2, {"unique_olap_per_pair": 0}),
    "l2_partial": (214, 2, {"partial": 1}),
    "l5_partial_multi": (213, 5, {"partial": 1, "unique_olap_per_pair": 0}),
    "l4_partial_0144": (215, 4, {"partial": 1, "max_erate": 0.144}),
}


def _case(name):
    seed, lim, extra = CASES[name]
    extra = dict(extra)
    erate = extra.pop("max_erate", 0.06)
    rs = synth_reads(90, 2200, 12_000, 0.025, seed=seed, len_jitter=0.4, n_repeats=3,
                     repeat_len=250)
    p = oracle.default_params(kmer_len=22, max_erate=erate, min_olap_len=200,
                              frag_olap_limit=lim, **extra)
    return rs, p


needs_ref = pytest.mark.skipif(not oracle.reference_available(),
                               reason="oracle/_ref/oic_ref not built (no /root/reference here)")


@needs_ref
@pytest.mark.parametrize("name", sorted(CASES))
def test_oracle_vs_reference(name):
    rs, p = _case(name)
    # one thread: the reference's global Total_Overlaps count is not thread-safe (with
    # several threads it drifts by a few from run to run; its records do not)
    want, rst = oracle.run_reference(rs, p, threads=1, with_stats=True)
    got, gst = oracle.run_oracle(rs, p, with_stats=True)
    assert np.array_equal(got, want)
    for rk, ok in STAT_KEYS:
        assert gst[ok] == rst[rk], (rk, gst[ok], rst[rk])
    full = oracle.run_oracle(rs, dict(p, frag_olap_limit=(1 << 64) - 1))
    assert len(got) < len(full)            # the limit binds


@needs_ref
def test_oracle_vs_reference_hash_batches():
    """-l under hash batches (StrNum counts from each batch's first read) and a -r range."""
    rs, p = _case("l3")
    want, wst, batches = oracle.run_oracle_driver(rs, p, ref_range=(5, 80), threads=1,
                                                  with_stats=True, hashstrings=30,
                                                  hashdatalen=100_000_000, hashbits=22,
                                                  hashload=0.6)
    assert len(batches) >= 3
    ref, rst = oracle.run_reference(rs, p, threads=1, batching=dict(hashstrings=30),
                                    extra=["-r", "5-80"], with_stats=True)
    assert np.array_equal(want, ref)
    for rk, ok in STAT_KEYS:
        assert wst[ok] == rst[rk], (rk, wst[ok], rst[rk])


def _gpu_params(p):
    from canu_amd.overlap_in_core import OicParameters
    return OicParameters(Kmer_Len=p["kmer_len"], maxErate=p["max_erate"],
                         Min_Olap_Len=p["min_olap_len"],
                         Doing_Partial_Overlaps=bool(p["partial"]),
                         Unique_Olap_Per_Pair=bool(p["unique_olap_per_pair"]),
                         Frag_Olap_Limit=int(p["frag_olap_limit"])).finalize()


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(CASES))
def test_gpu_vs_oracle(built, name):
    from canu_amd.overlap_in_core import OverlapInCore
    rs, p = _case(name)
    P = _gpu_params(p)
    want, wst = oracle.run_oracle(rs, P.as_dict(), with_stats=True)
    oic = OverlapInCore(P, device=0)
    oic.load_reads(rs)
    oic.build_hash_index()
    got = oic.fetch(oic.find_overlaps(1, rs.nreads))
    st = oic.stats()
    oic.close()
    assert got.shape == want.shape and np.array_equal(got, want)
    for _, ok in STAT_KEYS + [(None, "kmer_hits_skipped")]:
        assert st[ok] == wst[ok], (ok, st[ok], wst[ok])


@pytest.mark.gpu
def test_gpu_hash_subrange(built):
    """An index over reads 21..90 only: the hash slots count StrNum from read 21."""
    from canu_amd.overlap_in_core import OverlapInCore
    rs, p = _case("l2_partial")
    P = _gpu_params(p)
    want = oracle.run_oracle(rs, P.as_dict(), hash_range=(21, 90), ref_range=(1, 70))
    oic = OverlapInCore(P, device=0)
    oic.load_reads(rs)
    oic.build_hash_index(21, 90)
    got = oic.fetch(oic.find_overlaps(1, 70))
    oic.close()
    assert len(want) > 50
    assert np.array_equal(got, want)


@pytest.mark.gpu
def test_gpu_driver_hash_batches(built):
    from canu_amd.overlap_in_core import OverlapInCore
    rs, p = _case("l3")
    want, wst, batches = oracle.run_oracle_driver(rs, p, ref_range=(5, 80), threads=2,
                                                  with_stats=True, hashstrings=30,
                                                  hashdatalen=100_000_000, hashbits=22,
                                                  hashload=0.6)
    O = _gpu_params(p)
    O.Max_Hash_Strings = 30
    O.Num_PThreads = 2
    O.bgnRefID, O.endRefID = 5, 80
    oic = OverlapInCore(O, device=0)
    got = oic.run_driver(rs)
    st = oic.stats()
    oic.close()
    assert st["hash_batches"] == len(batches)
    assert got.shape == want.shape and np.array_equal(got, want)
    for _, ok in STAT_KEYS:
        assert st[ok] == wst[ok], (ok, st[ok], wst[ok])


@pytest.mark.gpu
def test_gpu_10kb_partial(built):
    """The benchmark's read length and error under canu's -G with -l 4 (~25 targets per
    query at 25x coverage)."""
    from canu_amd.overlap_in_core import OverlapInCore
    rs = synth_reads(120, 10_000, 48_000, 0.015, seed=216)
    p = oracle.default_params(kmer_len=22, max_erate=0.06, min_olap_len=500, partial=1,
                              frag_olap_limit=4)
    P = _gpu_params(p)
    want, wst = oracle.run_oracle(rs, P.as_dict(), with_stats=True)
    oic = OverlapInCore(P, device=0)
    oic.load_reads(rs)
    oic.build_hash_index()
    got = oic.fetch(oic.find_overlaps(1, rs.nreads))
    st = oic.stats()
    oic.close()
    assert len(want) > 500
    assert got.shape == want.shape and np.array_equal(got, want)
    for _, ok in STAT_KEYS:
        assert st[ok] == wst[ok], (ok, st[ok], wst[ok])
