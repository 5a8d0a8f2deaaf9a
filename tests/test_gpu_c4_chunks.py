"""The driver's chunked sorted-window search at full scale against the REFERENCE.

tests/golden/c4chunk2000k.json (tools/make_c4_chunk_digest.py) holds the reference
overlapInCore's output (oracle/_ref/oic_ref) for one configs[4]-shaped job over the first
2,000,000 reads of bench.py's 4M x 12 kb configs4-rank read set: a thin hash slice
`-h 1996001-2000000` (one hash batch) searched by every read, `-r 1-2000000`, with canu's
--hashbits 23 --hashload 0.75 (overlapInCore.C:191-300, Find_Overlaps.C:284-370).

On the GPU the same job runs through OverlapInCore.overlap_driver with the sorted query
windows on (OVL_SQ=1: a one-batch job would otherwise probe at random) and NO size caps: the
2M queries are ~48 G windows, several times what one chunk of sorted windows may take of
the device's free HBM, so the driver's own planning (plan_query_chunks) cuts the query
range into >= 4 chunks, each sorted in runs of <= 2^29 windows with the multiset guard, and
the records and -s counters must equal the reference's.  The digest is data: the reference
build is not needed on the GPU box.
"""
import json
import os

import numpy as np
import pytest

from canu_amd import digest

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "c4chunk2000k.json")
STAT_KEYS = [("total", "total_overlaps"), ("kmer_hits_with_olap", "kmer_hits_with_olap"),
             ("kmer_hits_without_olap", "kmer_hits_without_olap"), ("multi", "multi_overlaps"),
             ("contained", "contained_overlaps"), ("dovetail", "dovetail_overlaps")]


_PRE = {}


def _golden():
    with open(GOLDEN) as f:
        return json.load(f)


def _reads():
    from canu_amd.synth import synth_reads_parallel
    w = _golden()["workload"]
    n = w["reads"]
    return synth_reads_parallel(n, w["read_len"], int(n * w["read_len"] / w["coverage"]),
                                w["read_error"], seed=w["seed"], len_jitter=0.2,
                                read_range=(0, w["loaded_reads"]), workers=16)


def pregenerate():
    """conftest's session-start hook: the 2M reads in a forked pool (~40 s) before any test
    initialises the GPU."""
    if "rs" not in _PRE:
        print(f"\n[{os.path.basename(__file__)}] generating the 2M x 12 kb reads", flush=True)
        _PRE["rs"] = _reads()


def test_chunk_digest_is_a_thin_slice_of_the_configs4_reads():
    """CPU: the fixture is bench.py's configs4-rank read set (4M x 12 kb, seed 5), one job
    `-h` a thin slice at the top of the loaded reads, `-r 1-<that top>`."""
    g = _golden()
    w, gj = g["workload"], g["jobs"][0]
    assert w["workload"] == "configs4-rank" and w["reads"] == 4_000_000
    assert w["read_len"] == 12_000 and w["seed"] == 5 and w["coverage"] == 15.0
    hi = w["loaded_reads"]
    assert gj["h"][1] == hi and gj["r"] == [1, hi] and 0 < hi - gj["h"][0] + 1 <= 10_000
    assert gj["records"] == gj["stats"]["total"] > 10_000


@pytest.mark.gpu
def test_gpu_chunked_sorted_search_matches_reference(monkeypatch):
    from canu_amd.overlap_in_core import OicParameters, OverlapInCore
    g = _golden()
    w, gj = g["workload"], g["jobs"][0]
    n = w["reads"]
    rs = _PRE.pop("rs", None) or _reads()
    assert rs.total_bases() == w["loaded_bases"]
    (h_lo, h_hi), (r_lo, r_hi) = gj["h"], gj["r"]
    hashed = int(rs.lengths[h_lo - 1:h_hi].sum(dtype=np.uint64)) + (h_hi - h_lo + 1)
    P = OicParameters(Kmer_Len=w["k"], maxErate=float(np.float32(w["maxerate"])),
                      Min_Olap_Len=w["minlength"], bgnHashID=h_lo, endHashID=h_hi,
                      bgnRefID=r_lo, endRefID=r_hi, Hash_Mask_Bits=23, Max_Hash_Load=0.75,
                      Max_Hash_Strings=10_000_000, Max_Hash_Data_Len=hashed + 1024,
                      Num_PThreads=16).finalize()
    for cap in ("OVL_SQ_CHUNK_WINDOWS", "OVL_SB_WINDOWS", "OVL_SB_PCT", "OVL_HIT_BUDGET_M"):
        monkeypatch.delenv(cap, raising=False)
    monkeypatch.setenv("OVL_SQ", "1")
    oic = OverlapInCore(P, device=0)
    try:
        oic.load_reads(rs)
        del rs
        nrec = oic.overlap_driver(store_num_reads=n)
        st = oic.stats()
        rec = oic.fetch(nrec)
    finally:
        oic.close()
    # the driver cut the 2M-read query range into several chunks on its own
    assert st["query_chunks"] >= 4, st["query_chunks"]
    assert st["hash_batches"] == 1 and st["sq_declined"] == 0
    assert rec.shape[0] == gj["records"]
    assert digest.sha256_sorted(rec) == gj["sha256_sorted"]
    assert f"{digest.multiset_hash(rec):016x}" == gj["multiset_hash"]
    for rk, mk in STAT_KEYS:
        assert int(st[mk]) == int(gj["stats"][rk]), rk
