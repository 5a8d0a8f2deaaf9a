"""canu_amd/bin/overlapInCore: the pipeline drop-in (row 7).

canu's overlap.sh runs (src/pipelines/canu/OverlapInCore.pm:207-226)

    $bin/overlapInCore -t N -k K -k ../0-mercounts/<asm>.ms<K>.frequentMers.fasta
        --hashbits B --hashload F --maxerate E --minlength L [--minkmers] $opt
        -o ./$job.ovb.WORKING -s ./$job.stats ../<asm>.gkpStore

with $opt = "-h a-b -r c-d --hashstrings N --hashdatalen M" (overlapInCorePartition.C:78).
The executable reads the gkpStore itself (canu_amd/csrc/gkp_store.h, no reference code);
here the store is written by the reference's gkStore code (oic_ref --gkp-only).
"""
import os
import subprocess
import tempfile

import numpy as np
import pytest

from canu_amd.synth import synth_reads
from canu_amd import build as B

import oracle

needs_ref = pytest.mark.skipif(not oracle.reference_available(),
                               reason="oracle/_ref/oic_ref not built")


@pytest.fixture(scope="module")
def cli(built):
    return B.build_cli(verbose=False)


def _dump(cli, store, args=()):
    with tempfile.TemporaryDirectory() as wd:
        out = os.path.join(wd, "dump.bin")
        cp = subprocess.run([cli, "-k", "22", *args, "--dump-store", out, store],
                            capture_output=True, text=True)
        assert cp.returncode == 0, cp.stderr
        raw = open(out, "rb").read()
    first, n = np.frombuffer(raw[:8], dtype=np.uint32)
    meta = np.frombuffer(raw[8:8 + 8 * n], dtype=np.uint32).reshape(n, 2)
    body = np.frombuffer(raw[8 + 8 * n:], dtype=np.uint8)
    tot = int(meta[:, 1].sum())
    return int(first), meta[:, 0], meta[:, 1], body[:tot], body[tot:2 * tot]


@needs_ref
@pytest.mark.parametrize("quals", [False, True])
def test_store_reader_matches_reads(cli, quals):
    """Every read's length, library, bases (2SEQ for ACGT reads, USEQ for reads with N) and
    QVs (UQLT, or the library default QVAL) as the reference wrote them."""
    rs = synth_reads(60, 1500, 20_000, 0.02, seed=31, n_rate=0.002, len_jitter=0.5,
                     with_quals=quals)
    with tempfile.TemporaryDirectory() as wd:
        store = oracle.build_gkpstore(rs, wd)
        first, libs, lens, bases, qv = _dump(cli, store)
        assert first == 1 and lens.shape[0] == rs.nreads
        assert np.array_equal(lens, rs.lengths)
        assert np.all(libs == 1)                       # the harness's single library
        want = np.frombuffer(bytes(rs.bases), dtype=np.uint8)
        assert np.array_equal(bases | 0x20, want | 0x20)
        if quals:
            assert np.array_equal(qv, np.asarray(rs.quals, dtype=np.uint8))
        else:
            assert np.all(qv == 20)                    # gkLibrary default QV
        # -h / -r select the loaded span
        first, libs, lens, bases, qv = _dump(cli, store, ["-h", "10-20", "-r", "5-12"])
        assert first == 5 and lens.shape[0] == 16
        assert np.array_equal(lens, rs.lengths[4:20])


def test_cli_usage_errors(cli):
    for args in ([], ["-k", "22", "store"], ["-o", "x.ovb", "store"],
                 ["-k", "22", "-o", "x.ovb", "--hashstrings", "0", "store"],
                 ["-k", "22", "-o", "x.ovb", "a", "b"]):
        cp = subprocess.run([cli, *args], capture_output=True, text=True)
        assert cp.returncode == 1, (args, cp.stderr)
    cp = subprocess.run([cli, "-k", "22", "-o", "x.ovb", "/nonexistent.gkpStore"],
                        capture_output=True, text=True)
    assert cp.returncode == 1 and "failed to open" in cp.stderr


def _frequent_mers(rs, k=22, n=40):
    seq = rs.read(0).decode().upper()
    out = []
    for i in range(0, len(seq) - k, 37):
        s = seq[i:i + k]
        if set(s) <= set("ACGT"):
            out.append(s)
        if len(out) == n:
            break
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("job", ["utg", "partial_threads", "partial_limit"])
def test_gpu_cli_canu_job(cli, job):
    """overlap.sh's command line on a reference-written gkpStore: the .ovb read back by the
    reference's ovFile reader equals the reference overlapInCore's records, the .counts
    file is byte-identical, the -s statistics line-identical."""
    oracle.require_reference()
    rs = synth_reads(240, 6000, 150_000, 0.015, seed=33, n_repeats=4, repeat_len=300,
                     len_jitter=0.3)
    hb, he, rb, re_ = (1, 240, 1, 240) if job == "utg" else (31, 230, 11, 200)
    hashlen = int(sum(int(rs.lengths[i - 1]) + 1 for i in range(hb, he + 1)))
    hashlen //= 3                                       # three hash batches per job
    threads = 4 if job == "utg" else 16
    lim = ["-l", "4"] if job == "partial_limit" else []      # -l: Frag_Olap_Limit
    P = oracle.default_params(kmer_len=22, max_erate=0.06, min_olap_len=500,
                              partial=int(job != "utg"), **({"frag_olap_limit": 4} if lim else {}))
    with tempfile.TemporaryDirectory() as wd:
        fm = os.path.join(wd, "asm.ms22.frequentMers.fasta")
        mers = _frequent_mers(rs)
        with open(fm, "w") as f:
            for i, m in enumerate(mers):
                f.write(f">{i}\n{m}\n")
        # the reference job (its own gkpStore + OverlapDriver + ovFile)
        refwd = os.path.join(wd, "ref")
        os.makedirs(refwd)
        opt = ["-h", f"{hb}-{he}", "-r", f"{rb}-{re_}"]
        ref, rst = oracle.run_reference(
            rs, P, threads=threads, hash_bits=23, skip_kmers=mers, minkmers=True,
            batching={"hashstrings": he - hb + 1, "hashdatalen": hashlen, "hashload": 0.75},
            extra=opt + ["-s", os.path.join(wd, "ref.stats")], workdir=refwd, with_stats=True)
        store = os.path.join(refwd, "w", "ref.gkpStore")
        jobdir = os.path.join(wd, "001")
        os.makedirs(jobdir)
        argv = [cli] + (["-G"] if job != "utg" else []) + [
            "-t", str(threads), "-k", "22", "-k", fm, "--hashbits", "23", "--hashload", "0.75",
            "--maxerate", "0.06", "--minlength", "500", "--minkmers",
            *opt, *lim, "--hashstrings", str(he - hb + 1), "--hashdatalen", str(hashlen),
            "-o", os.path.join(jobdir, "000001.ovb.WORKING"),
            "-s", os.path.join(jobdir, "000001.stats"), store]
        cp = subprocess.run(argv, capture_output=True, text=True, timeout=300)
        assert cp.returncode == 0, cp.stderr[-3000:]
        assert "3 hash batches" in cp.stderr
        got = oracle.sort_records(oracle.read_ovb_reference(os.path.join(jobdir, "000001.ovb.WORKING")))
        assert got.shape[0] > 100
        assert got.shape == ref.shape and np.array_equal(got, ref)
        assert open(os.path.join(jobdir, "000001.counts"), "rb").read() == \
            open(os.path.join(refwd, "w", "ref.counts"), "rb").read()
        mine = open(os.path.join(jobdir, "000001.stats")).read().splitlines()
        theirs = open(os.path.join(wd, "ref.stats")).read().splitlines()
        if job == "utg":
            assert mine == theirs
        else:
            # -G: Output_Partial_Overlap counts with `Total_Overlaps++` on the GLOBAL
            # (overlapInCore-Output.C:253) from every thread without a lock, so with -t > 1
            # the reference's total can lose increments.  Every other line is exact; ours is
            # the number of records written.
            assert [l for l in mine if "Total overlaps" not in l] == \
                [l for l in theirs if "Total overlaps" not in l]
            tot = lambda lines: int([l for l in lines if "Total overlaps" in l][0].split("=")[1])
            assert tot(mine) == got.shape[0] and tot(theirs) <= tot(mine)
