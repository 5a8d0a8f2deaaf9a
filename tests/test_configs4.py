"""BASELINE configs[4]'s shape on one GPU: hash-block rank jobs of the 8-GPU plan.

configs[4] (4M x 12 kb ONT reads on 8 x MI355X) runs one overlapInCore job per GPU over a
contiguous hash block searched by every earlier read -- `-h lo-hi -r 1-hi`, canu's own
partitioning (overlapInCorePartition.C:73-78) with the blocks cut by
canu_amd.dist.hash_block_jobs -- each job running OverlapDriver's hash batches
(overlapInCore.C:191-300) with canu's production table (--hashbits 23 --hashload 0.75).

Here, at a size the reference finishes in seconds (600 reads x 12 kb +-20 % at 15x):
  * every rank job's records and -s counters equal the reference overlapInCore's
    (oracle/_ref/oic_ref, built from its sources) run with the same arguments;
  * the union of the rank jobs' records is the whole `-h 1-n -r 1-n` job's (every a < b
    pair is found once, by the job whose block holds b).
"""
import numpy as np
import pytest

from canu_amd.synth import synth_reads_parallel

import oracle

N, READ_LEN, COV, SEED = 600, 12_000, 15.0, 5
HASHBITS, HASHLOAD, HASHSTRINGS = 23, 0.75, 97
STAT_KEYS = [("total", "total_overlaps"), ("kmer_hits_with_olap", "kmer_hits_with_olap"),
             ("kmer_hits_without_olap", "kmer_hits_without_olap"), ("multi", "multi_overlaps"),
             ("contained", "contained_overlaps"), ("dovetail", "dovetail_overlaps")]


def _reads():
    return synth_reads_parallel(N, READ_LEN, int(N * READ_LEN / COV), 0.015, seed=SEED,
                                len_jitter=0.2, workers=4)


def _jobs(world):
    from canu_amd.dist import hash_block_jobs
    load = HASHLOAD * (1 << HASHBITS) * 21
    return hash_block_jobs(N, world, READ_LEN, 36.0, 3.0 * load)


def test_plan_covers_pairs_once():
    """CPU: the blocks tile 1..n, each job searches every read up to its block's end, and
    no -h range ends in a one-read batch (the reference never hashes one, :222)."""
    for world in (2, 4, 8):
        js = _jobs(world)
        assert js[0]["h"][0] == 1 and js[-1]["h"][1] == N
        for a, b in zip(js, js[1:]):
            assert b["h"][0] == a["h"][1] + 1
        for j in js:
            lo, hi = j["h"]
            assert j["r"] == (1, hi)
            if world == 2:
                assert (hi - lo + 1) % HASHSTRINGS != 1
    assert N % HASHSTRINGS != 1


def _params(h, r, hashed_bases):
    from canu_amd.overlap_in_core import OicParameters
    return OicParameters(Kmer_Len=22, maxErate=float(np.float32(0.06)), Min_Olap_Len=500,
                         bgnHashID=h[0], endHashID=h[1], bgnRefID=r[0], endRefID=r[1],
                         Hash_Mask_Bits=HASHBITS, Max_Hash_Load=HASHLOAD,
                         Max_Hash_Strings=HASHSTRINGS, Max_Hash_Data_Len=hashed_bases + 1024,
                         Num_PThreads=16).finalize()


def _gpu_job(rs, h, r):
    from canu_amd.overlap_in_core import OverlapInCore
    hashed = int(rs.lengths[h[0] - 1:h[1]].sum()) + (h[1] - h[0] + 1)
    oic = OverlapInCore(_params(h, r, hashed), device=0)
    try:
        oic.load_reads(rs)
        n = oic.overlap_driver(store_num_reads=rs.nreads)
        return oic.fetch(n), oic.stats()
    finally:
        oic.close()


def _ref_job(rs, h, r):
    hashed = int(rs.lengths[h[0] - 1:h[1]].sum()) + (h[1] - h[0] + 1)
    P = oracle.default_params(kmer_len=22, max_erate=0.06, min_olap_len=500)
    return oracle.run_reference(
        rs, P, threads=16, hash_bits=HASHBITS,
        batching={"hashstrings": HASHSTRINGS, "hashdatalen": hashed + 1024,
                  "hashload": HASHLOAD},
        extra=["-h", f"{h[0]}-{h[1]}", "-r", f"{r[0]}-{r[1]}"], with_stats=True)


@pytest.mark.gpu
def test_rank_jobs_union_and_reference():
    rs = _reads()
    whole, whole_st = _gpu_job(rs, (1, N), (1, N))
    assert whole.shape[0] > 1000
    assert whole_st["hash_batches"] >= 6
    parts = []
    for j in _jobs(2):
        rec, st = _gpu_job(rs, j["h"], j["r"])
        assert st["hash_batches"] >= 2
        oracle.require_reference()
        ref, ref_st = _ref_job(rs, j["h"], j["r"])
        assert rec.shape == ref.shape and np.array_equal(rec, ref), j
        for rk, mk in STAT_KEYS:
            assert ref_st[rk] == st[mk], (j, rk)
        parts.append(rec)
    union = oracle.sort_records(np.concatenate(parts))
    assert union.shape == whole.shape and np.array_equal(union, whole)
