"""configs[4]'s rank jobs at 20k reads x 12 kb against the REFERENCE's committed digests.

tests/golden/c4rank20k.json holds, for every job of bench.py's `--workload configs4-rank`
8-way plan over 20k reads (canu_amd.dist.hash_block_jobs: `-h lo-hi -r 1-hi`,
--hashbits 23 --hashload 0.75, OverlapDriver's hash batches inside, overlapInCore.C:191-300),
the record count, SHA-256 of the sorted records, multiset hash and -s counters of the
reference overlapInCore (oracle/_ref/oic_ref) run with the same arguments
(tools/make_c4_digest.py).  The digest is data, so this runs without the reference build.

Every job runs here through the drop-in OverlapInCore.overlap_driver (one hash batch each at
this size, probed at random), and the last job -- searched by every read -- once more through
the job's sorted query windows (OVL_SQ=1, k_probe_sorted).
"""
import json
import os

import numpy as np
import pytest

from canu_amd import digest

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "c4rank20k.json")
STAT_KEYS = [("total", "total_overlaps"), ("kmer_hits_with_olap", "kmer_hits_with_olap"),
             ("kmer_hits_without_olap", "kmer_hits_without_olap"), ("multi", "multi_overlaps"),
             ("contained", "contained_overlaps"), ("dovetail", "dovetail_overlaps")]


def _golden():
    with open(GOLDEN) as f:
        return json.load(f)


def test_digest_matches_bench_plan():
    """CPU: the fixture's jobs are bench.py's configs4-rank plan for its read count."""
    from canu_amd.dist import hash_block_jobs
    g = _golden()
    w = g["workload"]
    assert w["workload"] == "configs4-rank" and w["read_len"] == 12_000 and w["seed"] == 5
    jobs = hash_block_jobs(w["reads"], 8, w["read_len"], 36.0, 3.0 * 0.75 * (1 << 23) * 21)
    assert [j["index"] for j in g["jobs"]] == list(range(8))
    for j, gj in zip(jobs, g["jobs"]):
        assert tuple(gj["h"]) == j["h"] and tuple(gj["r"]) == j["r"]
        assert gj["records"] == gj["stats"]["total"] > 1000


def _run_job(rs, gj, w):
    from canu_amd.overlap_in_core import OicParameters, OverlapInCore
    (h_lo, h_hi), (r_lo, r_hi) = gj["h"], gj["r"]
    hashed = int(rs.lengths[h_lo - 1:h_hi].sum(dtype=np.uint64)) + (h_hi - h_lo + 1)
    P = OicParameters(Kmer_Len=w["k"], maxErate=float(np.float32(w["maxerate"])),
                      Min_Olap_Len=w["minlength"], bgnHashID=h_lo, endHashID=h_hi,
                      bgnRefID=r_lo, endRefID=r_hi, Hash_Mask_Bits=23, Max_Hash_Load=0.75,
                      Max_Hash_Strings=10_000_000, Max_Hash_Data_Len=hashed + 1024,
                      Num_PThreads=16).finalize()
    oic = OverlapInCore(P, device=0)
    try:
        oic.load_reads(rs)
        n = oic.overlap_driver(store_num_reads=rs.nreads)
        return oic.fetch(n), oic.stats()
    finally:
        oic.close()


def _check(rec, st, gj):
    assert rec.shape[0] == gj["records"], (gj["index"], rec.shape[0], gj["records"])
    assert digest.sha256_sorted(rec) == gj["sha256_sorted"], gj["index"]
    assert f"{digest.multiset_hash(rec):016x}" == gj["multiset_hash"], gj["index"]
    for rk, mk in STAT_KEYS:
        assert int(st[mk]) == int(gj["stats"][rk]), (gj["index"], rk)


@pytest.mark.gpu
def test_gpu_c4_plan_jobs_match_reference_digest(monkeypatch):
    from canu_amd.synth import synth_reads_parallel
    g = _golden()
    w = g["workload"]
    n = w["reads"]
    rs = synth_reads_parallel(n, w["read_len"], int(n * w["read_len"] / w["coverage"]),
                              w["read_error"], seed=w["seed"], len_jitter=0.2,
                              read_range=(0, n), workers=8)
    assert rs.total_bases() == w["total_bases"]
    for gj in g["jobs"]:
        rec, st = _run_job(rs, gj, w)
        _check(rec, st, gj)
    # the plan's jobs are one hash batch each at this size (the default probes at random
    # then); the last job (searched by every read) once more through the sorted query windows
    monkeypatch.setenv("OVL_SQ", "1")
    rec, st = _run_job(rs, g["jobs"][-1], w)
    _check(rec, st, g["jobs"][-1])
