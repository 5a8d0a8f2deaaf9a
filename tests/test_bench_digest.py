"""The benchmark job pinned at full size: tests/golden/bench50k.json holds the digest of
the records the REFERENCE overlapInCore (oracle/_ref/oic_ref, built from its sources)
writes for bench.py's exact read set -- 50k x 10 kb synthetic ONT reads, one hash batch,
-h 1-n -r 1-n (tools/make_bench_digest.py; overlapInCore.C:191-300).

CPU: the digest functions (canu_amd/digest.py) -- order independence, additivity over
disjoint shards (what bench.py relies on at N > 1).  GPU: the HIP path's records for the
same reads hash to the reference's digest, and its -s counters equal the reference's."""
import json
import os

import numpy as np
import pytest

from canu_amd import digest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden", "bench50k.json")


def _random_records(n, seed):
    rng = np.random.default_rng(seed)
    r = np.zeros(n, dtype=digest.RECORD_DTYPE)
    r["a"] = rng.integers(1, 50_000, n)
    r["b"] = rng.integers(1, 50_000, n)
    r["w0"] = rng.integers(0, 1 << 63, n, dtype=np.uint64)
    r["w1"] = rng.integers(0, 1 << 63, n, dtype=np.uint64)
    return r


def test_digest_is_order_independent_and_additive():
    r = _random_records(5000, 1)
    perm = r[np.random.default_rng(2).permutation(r.shape[0])]
    assert digest.sha256_sorted(r) == digest.sha256_sorted(perm)
    assert digest.multiset_hash(r) == digest.multiset_hash(perm)
    parts = [r[:1234], r[1234:3000], r[3000:]]
    assert digest.combine(digest.multiset_hash(p) for p in parts) == digest.multiset_hash(r)
    s = r.copy()
    s["w1"][17] ^= np.uint64(1)                      # one bit of one record
    assert digest.multiset_hash(s) != digest.multiset_hash(r)
    assert digest.sha256_sorted(s) != digest.sha256_sorted(r)
    assert digest.multiset_hash(r[:0]) == 0


def test_golden_digest_fixture():
    g = json.load(open(GOLDEN))
    assert g["records"] == g["stats"]["total"] == 1187486
    assert len(g["sha256_sorted"]) == 64 and len(g["multiset_hash"]) == 16
    w = g["workload"]
    assert (w["reads"], w["read_len"], w["coverage"], w["seed"], w["k"]) == (50000, 10000, 25.0,
                                                                             1, 22)


def test_configs4_side_line_digest_fixture():
    """tests/golden/c4rank500k.json: the reference overlapInCore's own run (47 min on 8
    threads, tools/make_c4_digest.py --reads 500000 --jobs 0) of the configs4-rank side
    line's job -- rank 0 of the 8-way plan at 1/8 scale, 14 hash batches -- which bench.py's
    side line checks its records against.  Its workload and job are the ones bench.py runs."""
    import bench
    g = json.load(open(os.path.join(ROOT, "tests", "golden", "c4rank500k.json")))
    a = bench.parse_args(["--workload", "configs4-rank"])
    job = bench.Configs4Rank(a, 0, 1, None)
    key = job.workload_key()
    for k in ("reads", "read_len", "coverage", "read_error", "seed", "k", "minlength"):
        assert float(g["workload"][k]) == float(key[k]), k
    from canu_amd.dist import hash_block_jobs
    load = job.HASHLOAD * (1 << job.HASHBITS) * 21             # Configs4Rank.generate's plan
    plan = hash_block_jobs(a.reads, 8, a.read_len, 36.0, 3.0 * load)[a.rank_job]
    (j,) = g["jobs"]
    assert tuple(j["h"]) == tuple(plan["h"]) and tuple(j["r"]) == tuple(plan["r"])
    assert j["records"] == j["stats"]["total"] == 719115
    assert len(j["sha256_sorted"]) == 64 and len(j["multiset_hash"]) == 16


@pytest.mark.gpu
def test_gpu_bench_job_matches_reference_digest(built):
    """The full 50k x 10 kb job (bench.py's step) against the reference's own output."""
    from bench import parse_args, Configs2
    from canu_amd.overlap_in_core import OicParameters, OverlapInCore
    import torch
    g = json.load(open(GOLDEN))
    job = Configs2(parse_args([]), 0, 1, torch.device("cuda", 0))
    assert job.workload_key()["reads"] == g["workload"]["reads"]
    job.generate()
    job.setup(OicParameters, OverlapInCore)
    try:
        n = job.step()
        st = job.oic.stats()
        rec = job.oic.fetch(n)
    finally:
        job.oic.close()
    assert rec.shape[0] == g["records"]
    assert digest.sha256_sorted(rec) == g["sha256_sorted"]
    assert f"{digest.multiset_hash(rec):016x}" == g["multiset_hash"]
    for mine, ref in (("kmer_hits_without_olap", "kmer_hits_without_olap"),
                      ("kmer_hits_with_olap", "kmer_hits_with_olap"),
                      ("multi_overlaps", "multi"), ("total_overlaps", "total"),
                      ("contained_overlaps", "contained"), ("dovetail_overlaps", "dovetail")):
        assert st[mine] == g["stats"][ref], mine
