"""Host-side logic: the overlapInCore command line, the -k skip file, query sharding and
the synthetic read generator."""
import numpy as np
import pytest

from canu_amd.dist import query_shards, shard_cost
from canu_amd.overlap_in_core import (UINT64_MAX, OicParameters, parse_overlapInCore_args,
                                      read_skip_fasta)
from canu_amd.synth import synth_reads


def test_parse_defaults_and_options():
    P, extra = parse_overlapInCore_args(
        ["-G", "-h", "1-500", "-r", "20-300", "-k", "22", "--maxerate", "0.1", "-m",
         "--minlength", "500", "-w", "-z", "-l", "7", "-t", "8", "-o", "out.ovb",
         "--hashbits", "24", "seq.gkpStore"])
    assert P.Doing_Partial_Overlaps and not P.Unique_Olap_Per_Pair
    assert (P.bgnHashID, P.endHashID, P.bgnRefID, P.endRefID) == (1, 500, 20, 300)
    assert P.Kmer_Len == 22 and P.Min_Olap_Len == 500 and P.Frag_Olap_Limit == 7
    # strtof: the float value of 0.1, not the double
    assert P.maxErate == float(np.float32(0.1))
    # maxErate > 0.06 turns off the window filter and the hopeless check (main() fix-up)
    assert not P.Use_Window_Filter and not P.Use_Hopeless_Check
    assert extra == {"skip_file": None, "store": "seq.gkpStore", "output": "out.ovb",
                     "threads": 8, "stats": None}
    # hash-batch options reach the driver (oicParameters, overlapInCore.H:505-509)
    assert P.Hash_Mask_Bits == 24 and P.Num_PThreads == 8
    assert (P.Max_Hash_Strings, P.Max_Hash_Data_Len, P.Max_Hash_Load) == (10000, 100000000, 0.6)
    P, extra = parse_overlapInCore_args(["-k", "22", "--hashstrings", "300", "--hashdatalen",
                                         "123456", "--hashload", "0.75", "-H", "2-3", "-R", "4",
                                         "-s", "job.stats", "st"])
    assert (P.Max_Hash_Strings, P.Max_Hash_Data_Len, P.Max_Hash_Load) == (300, 123456, 0.75)
    assert (P.minLibToHash, P.maxLibToHash, P.minLibToRef, P.maxLibToRef) == (2, 3, 4, 4)
    assert extra["stats"] == "job.stats"


def test_parse_k_file_and_minkmers_order():
    P, extra = parse_overlapInCore_args(["-k", "mers.fasta", "-k", "18", "--minlength", "100",
                                         "--maxerate", "0.05", "--minkmers", "-l", "0"])
    assert extra["skip_file"] == "mers.fasta" and P.Kmer_Len == 18
    # --minkmers is evaluated where it appears, with the values parsed so far
    want = int(np.floor(np.exp(-18 * float(np.float32(0.05))) * (100 - 18 + 1)))
    assert P.Filter_By_Kmer_Count == want
    assert P.Frag_Olap_Limit == UINT64_MAX          # -l < 1 means no limit
    assert P.Use_Hopeless_Check                      # 0.05 <= 0.06: untouched


def test_read_skip_fasta(tmp_path):
    f = tmp_path / "m.fasta"
    f.write_text(">1\nACGTACGTAC\n>2\nTTTTTTTTTT\n")
    assert read_skip_fasta(str(f), 10) == ["ACGTACGTAC", "TTTTTTTTTT"]
    with pytest.raises(ValueError):
        read_skip_fasta(str(f), 11)


@pytest.mark.parametrize("n,world", [(1, 1), (10, 3), (1000, 8), (50000, 8), (3, 8)])
def test_query_shards_cover_and_balance(n, world):
    sh = query_shards(n, world)
    assert len(sh) == world
    ids = [i for lo, hi in sh for i in range(lo, hi + 1)]
    assert ids == list(range(1, n + 1))
    if n >= 1000:
        # equal modelled time (index lo..n, probe and chain per query, pairs)
        cost = [shard_cost(n, lo, hi) for lo, hi in sh]
        assert max(cost) / (sum(cost) / world) < 1.01



def test_synth_slices_match_whole():
    whole = synth_reads(40, 1500, 10_000, 0.02, seed=9, len_jitter=0.3, n_rate=0.001)
    a = synth_reads(40, 1500, 10_000, 0.02, seed=9, len_jitter=0.3, n_rate=0.001,
                    read_range=(0, 17))
    b = synth_reads(40, 1500, 10_000, 0.02, seed=9, len_jitter=0.3, n_rate=0.001,
                    read_range=(17, 40))
    assert b.first_iid == 18
    assert np.array_equal(np.concatenate([a.bases, b.bases]), whole.bases)
    assert np.array_equal(np.concatenate([a.lengths, b.lengths]), whole.lengths)


def test_hash_block_jobs_cover_and_balance():
    """configs[4]'s per-rank overlapInCore jobs: contiguous hash blocks covering every read,
    each searched by every earlier read (so each a < b pair is found once), equal modelled
    time per rank, the first block the widest (triangular pair count)."""
    from canu_amd.dist import hash_block_jobs
    js = hash_block_jobs(4_000_000, 8, 12_000, 36.0, 1.6e9)
    assert js[0]["h"][0] == 1 and js[-1]["h"][1] == 4_000_000
    for a, b in zip(js, js[1:]):
        assert b["h"][0] == a["h"][1] + 1
    for j in js:
        assert j["r"] == (1, j["h"][1])
    est = [j["est_s"] for j in js]
    assert max(est) / min(est) < 1.02
    widths = [j["h"][1] - j["h"][0] for j in js]
    assert widths == sorted(widths, reverse=True)


# full-size configs[4] rank jobs measured on one MI355X with round 6's harness (the staged bases
# freed before the job): hash block -> (seconds, hash batches, super-batches, query chunks)
# (profiles/r06a{7,0}_c4full.json)
C4_FULL_RUNS = {(3780001, 4000000): (24.97, 20, 3, 17), (1, 1448687): (28.04, 131, 17, 6)}


def test_driver6_replays_the_driver_plans():
    """dist.driver_plan (the driver's packing rules replayed per job) against full-size rank
    jobs measured on the GPU: the same super-batches and query chunks, the hash batches within
    one, the time within 6 %."""
    from canu_amd import dist
    for (lo, hi), (secs, nb, nsb, nch) in C4_FULL_RUNS.items():
        p = dist.driver_plan(4_000_000, 12_000, lo, hi)
        assert abs(p["hash_batches"] - nb) <= 1, (lo, hi, p)
        assert (p["super_batches"], p["query_chunks"]) == (nsb, nch), (lo, hi, p)
        assert abs(p["est_s"] - secs) / secs < 0.06, (lo, hi, p["est_s"], secs)


# round 6: every job of the derived plan (dist.c4_plan) measured at full size, one MI355X
# each (profiles/r06j_c4r{0,3,7}_c4full.json, r06k_c4r{1,2,4,5,6}_c4full.json): block ->
# (seconds, hash batches, super-batches, query chunks)
C4_PLAN_RUNS = {(1, 1429263): (26.67, 129, 17, 6), (1429264, 2049284): (26.90, 56, 7, 8),
                (2049285, 2497633): (26.00, 41, 6, 10), (2497634, 2881292): (26.01, 35, 5, 12),
                (2881293, 3199278): (25.30, 29, 4, 14), (3199279, 3499780): (26.30, 28, 4, 15),
                (3499781, 3762174): (25.75, 24, 4, 16), (3762175, 4000000): (24.77, 22, 3, 17)}


def test_driver6_model_against_the_measured_plan():
    """The eight measured jobs are the plan's, and the model replays each one's structure: the
    same super-batches, query chunks within one (the chunk cap is planned from the free HBM the
    first super-batch leaves, which the model estimates), time within 8 % (all faster)."""
    from canu_amd import dist
    js = dist.c4_plan(4_000_000, 8, 12_000)
    assert sorted(C4_PLAN_RUNS) == [j["h"] for j in js]
    for (lo, hi), (secs, nb, nsb, nch) in C4_PLAN_RUNS.items():
        p = dist.driver_plan(4_000_000, 12_000, lo, hi)
        assert abs(p["hash_batches"] - nb) <= 1 and p["super_batches"] == nsb, (lo, hi, p)
        assert abs(p["query_chunks"] - nch) <= 1, (lo, hi, p)
        assert 0 <= (p["est_s"] - secs) / secs < 0.08, (lo, hi, p["est_s"], secs)


def test_c4_full_plan_covers_the_reads(monkeypatch):
    """configs[4]'s plan at 4M reads (dist.c4_plan, cut on DRIVER6): eight contiguous
    `-h lo-hi -r 1-hi` blocks over 1..4M with equal modelled time, and bench.py's
    configs4-rank workload runs exactly those jobs (checked without reads or a GPU)."""
    from canu_amd import dist
    js = dist.c4_plan(4_000_000, 8, 12_000)
    assert len(js) == 8 and js[0]["h"][0] == 1 and js[-1]["h"][1] == 4_000_000
    for a, b in zip(js, js[1:]):
        assert b["h"][0] == a["h"][1] + 1
    for j in js:
        assert j["r"] == (1, j["h"][1])
    est = [j["est_s"] for j in js]
    # DRIVER6 replays the driver's discrete packing: one more hash batch (or super-batch) in
    # a block costs ~2-3 s at once, so the blocks balance to within a step, not a percent
    assert max(est) / min(est) < 1.10
    import bench
    monkeypatch.delenv("CANU_C4_PLAN", raising=False)
    monkeypatch.delenv("CANU_C4_HBLOCK", raising=False)
    for r in range(8):
        w = bench.Configs4Rank(bench.parse_args(["--workload", "configs4-rank", "--reads",
                                                 "4000000", "--rank-job", str(r)]), 0, 1, None)
        assert w.plan() == "r06"
        jobs, job = w.plan_jobs()            # what generate() runs, without reads or a GPU
        assert [(j["h"], j["r"]) for j in jobs] == [(j["h"], j["r"]) for j in js]
        assert (job["h"], job["r"]) == (js[r]["h"], js[r]["r"])
    # at N ranks rank r runs job r of an N-job plan
    w = bench.Configs4Rank(bench.parse_args(["--workload", "configs4-rank", "--reads",
                                             "4000000"]), 7, 8, None)
    assert w.plan_jobs()[1]["h"] == js[7]["h"]
