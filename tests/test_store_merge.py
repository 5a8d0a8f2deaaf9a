"""configs[4]'s host merge: per-rank overlapInCore outputs -> one ovStore.

On the 8-GPU node every rank runs one canu-shaped job `-h lo-hi -r 1-hi` (its block of
the hash reads searched by every earlier read; overlapInCorePartition.C:73-78 is canu's own
partitioning, canu_amd.dist.hash_block_jobs cuts the blocks) and writes its own .ovb and
.counts.  The host then builds the overlap store from all of them, as canu's ovStoreBuild
does from its overlap jobs (ovStoreBuild.C:348).  The store builder here is the
REFERENCE's (oracle/store_harness.cpp over ovStoreFilter / ovStoreWriter, compiled from
/root/reference/src/stores; its reader dumps the store), so these tests show:

  * CPU: the reference overlapInCore run as rank jobs gives, through the reference store
    build, the same store as the reference's whole-job run -- the partitioning is exact;
  * GPU: the drop-in executable (canu_amd/bin/overlapInCore) run as the rank jobs, on a
    gkpStore the reference wrote, gives that same store, overlap for overlap.
"""
import os
import subprocess
import tempfile

import numpy as np
import pytest

from canu_amd.synth import synth_reads

import oracle

N, READ_LEN, GENOME, ERR, SEED = 240, 6000, 160_000, 0.015, 41
HASHBITS, HASHLOAD = 23, 0.75


def _reads():
    return synth_reads(N, READ_LEN, GENOME, ERR, seed=SEED, len_jitter=0.3)


def _jobs(world):
    from canu_amd.dist import hash_block_jobs
    return hash_block_jobs(N, world, READ_LEN, 2 * READ_LEN * N / GENOME,
                           HASHLOAD * (1 << HASHBITS) * 21)


def _hashlen(rs, h):
    # about three hash batches per job (canu's partitioning hands each job --hashdatalen)
    return int(rs.lengths[h[0] - 1:h[1]].sum()) // 3 + READ_LEN


def _ref_job(rs, P, h, r, wd):
    os.makedirs(wd, exist_ok=True)
    oracle.run_reference(rs, P, threads=8, hash_bits=HASHBITS,
                         batching={"hashstrings": h[1] - h[0] + 1,
                                   "hashdatalen": _hashlen(rs, h), "hashload": HASHLOAD},
                         extra=["-h", f"{h[0]}-{h[1]}", "-r", f"{r[0]}-{r[1]}"], workdir=wd)
    return os.path.join(wd, "w", "ref.ovb"), os.path.join(wd, "w", "ref.gkpStore")


def _params():
    return oracle.default_params(kmer_len=22, max_erate=0.06, min_olap_len=500)


def _whole_store(rs, P, wd):
    ovb, gkp = _ref_job(rs, P, (1, N), (1, N), os.path.join(wd, "whole"))
    store = os.path.join(wd, "whole.ovlStore")
    n = oracle.build_store(gkp, store, [ovb])
    return gkp, oracle.dump_store(gkp, store), n


@pytest.mark.skipif(not (oracle.reference_available() and oracle.store_available()),
                    reason="reference checkers not built")
def test_reference_rank_jobs_merge_to_the_whole_store():
    rs = _reads()
    P = _params()
    with tempfile.TemporaryDirectory() as wd:
        gkp, whole, n_whole = _whole_store(rs, P, wd)
        assert n_whole == whole.shape[0] > 500
        # every overlap is stored from both reads' sides
        assert np.array_equal(np.sort(whole["a"]), np.sort(whole["b"]))
        jobs = _jobs(3)
        ovbs = [_ref_job(rs, P, j["h"], j["r"], os.path.join(wd, f"r{i}"))[0]
                for i, j in enumerate(jobs)]
        store = os.path.join(wd, "ranks.ovlStore")
        assert oracle.build_store(gkp, store, ovbs) == n_whole
        merged = oracle.dump_store(gkp, store)
        assert merged.shape == whole.shape and np.array_equal(merged, whole)


@pytest.mark.gpu
def test_gpu_rank_jobs_merge_to_the_reference_store(built):
    """The drop-in executable as 3 rank jobs of the plan (-h/-r, canu's hash settings,
    three hash batches each) on the reference-written gkpStore; their .ovb files through
    the reference store build equal the store of the reference's whole-job run."""
    from canu_amd import build as B
    oracle.require_reference()
    cli = B.build_cli(verbose=False)
    rs = _reads()
    P = _params()
    with tempfile.TemporaryDirectory() as wd:
        gkp, whole, n_whole = _whole_store(rs, P, wd)
        ovbs = []
        for i, j in enumerate(_jobs(3)):
            (hb, he), (rb, re_) = j["h"], j["r"]
            jobdir = os.path.join(wd, f"{i + 1:03d}")
            os.makedirs(jobdir)
            ovb = os.path.join(jobdir, f"{i + 1:06d}.ovb")
            argv = [cli, "-t", "8", "-k", "22", "--hashbits", str(HASHBITS), "--hashload",
                    str(HASHLOAD), "--maxerate", "0.06", "--minlength", "500",
                    "-h", f"{hb}-{he}", "-r", f"{rb}-{re_}",
                    "--hashstrings", str(he - hb + 1), "--hashdatalen",
                    str(_hashlen(rs, (hb, he))), "-o", ovb, gkp]
            cp = subprocess.run(argv, capture_output=True, text=True, timeout=300)
            assert cp.returncode == 0, cp.stderr[-3000:]
            assert os.path.exists(ovb[:-4] + ".counts")
            ovbs.append(ovb)
        store = os.path.join(wd, "gpu_ranks.ovlStore")
        assert oracle.build_store(gkp, store, ovbs) == n_whole
        merged = oracle.dump_store(gkp, store)
        assert merged.shape == whole.shape and np.array_equal(merged, whole)
