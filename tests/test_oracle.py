"""The oracle (oracle/oic_oracle.c, a C restatement of overlapInCore) pinned to the
reference.

  * test_golden_*: the records in tests/golden/ were produced by the REFERENCE
    overlapInCore compiled from its own sources (tools/make_golden.py, oracle/_ref); the
    oracle must reproduce them bit for bit.  Runs anywhere (no reference needed).
  * test_vs_reference_*: fresh random cases against oracle/_ref/oic_ref when it is built
    (this container); skipped elsewhere.
"""
import json
import os

import numpy as np
import pytest

import oracle
from canu_amd.synth import ReadSet, synth_reads

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
INDEX = json.load(open(os.path.join(GOLDEN, "index.json")))


def load_golden(name):
    z = np.load(os.path.join(GOLDEN, f"{name}.npz"))        # allow_pickle=False (default)
    lengths = z["lengths"].astype(np.uint32)
    offsets = np.zeros(lengths.shape[0], dtype=np.uint64)
    offsets[1:] = np.cumsum(lengths[:-1], dtype=np.uint64)
    quals = z["quals"] if "quals" in z.files and z["quals"].size else None
    rs = ReadSet(bases=z["bases"], offsets=offsets, lengths=lengths, quals=quals,
                 first_iid=int(z["first_iid"]))
    rec = np.zeros(z["a"].shape[0], dtype=oracle.RECORD_DTYPE)
    for f in ("a", "b", "w0", "w1"):
        rec[f] = z[f]
    skip = [s.decode() for s in z["skip"]]
    p = dict(INDEX[name]["params"])
    p["frag_olap_limit"] = int(p["frag_olap_limit"])
    return rs, p, skip, oracle.sort_records(rec)


@pytest.mark.parametrize("name", sorted(INDEX))
def test_golden_oracle(name):
    rs, p, skip, want = load_golden(name)
    got = oracle.run_oracle(rs, p, skip_kmers=skip or None)
    assert got.shape == want.shape
    assert np.array_equal(got, want)
    assert len(want) > 50


needs_ref = pytest.mark.skipif(not oracle.reference_available(),
                               reason="oracle/_ref/oic_ref not built (no /root/reference here)")


@needs_ref
@pytest.mark.parametrize("seed,erate,k,minlen,extra", [
    (101, 0.06, 22, 300, {}),
    (102, 0.10, 18, 200, {}),
    (103, 0.06, 22, 200, {"partial": 1}),
    (104, 0.06, 20, 200, {"unique_olap_per_pair": 0}),
])
def test_vs_reference_random(seed, erate, k, minlen, extra):
    rs = synth_reads(70, 2200, 14_000, 0.025, seed=seed, len_jitter=0.4, n_repeats=3,
                     repeat_len=250)
    p = oracle.default_params(kmer_len=k, max_erate=erate, min_olap_len=minlen, **extra)
    want = oracle.run_reference(rs, p, threads=4)
    got = oracle.run_oracle(rs, p)
    assert np.array_equal(got, want)


@needs_ref
def test_vs_reference_ranges():
    """-h / -r sub-ranges (the reference's own job partitioning)."""
    rs = synth_reads(80, 2000, 12_000, 0.02, seed=105)
    p = oracle.default_params(kmer_len=22, max_erate=0.06, min_olap_len=200)
    want = oracle.run_reference(rs, p, threads=2, extra=["-h", "21-70", "-r", "5-60"])
    got = oracle.run_oracle(rs, p, hash_range=(21, 70), ref_range=(5, 60))
    assert np.array_equal(got, want)
    assert len(want) > 0


def test_sharded_queries_union():
    """Query shards (-r ranges) are independent: their union is the whole job."""
    from canu_amd.dist import query_shards
    rs = synth_reads(60, 2000, 12_000, 0.02, seed=106)
    p = oracle.default_params(kmer_len=22, max_erate=0.06, min_olap_len=200)
    whole = oracle.run_oracle(rs, p)
    parts = [oracle.run_oracle(rs, p, ref_range=r) for r in query_shards(rs.nreads, 3)
             if r[0] <= r[1]]
    union = oracle.sort_records(np.concatenate(parts))
    assert np.array_equal(union, whole)


def test_match_limit_table():
    """Edit_Match_Limit (prefixEditDistance-matchLimit.C): monotone, and MAX_ERRORS as the
    reference sizes it, 1 + ceil(erate * AS_MAX_READLEN)."""
    import math
    me, lim = oracle.match_limit(float(np.float32(0.06)), 2000)
    assert me == 1 + math.ceil(float(np.float32(0.06)) * ((1 << 21) - 1))
    assert lim[0] == 0 and np.all(np.diff(lim) >= 0)
