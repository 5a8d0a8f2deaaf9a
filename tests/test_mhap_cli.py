"""canu_amd/bin/mhap: the MHAP command line canu's precompute.sh and mhap.sh run
(src/pipelines/canu/OverlapMhap.pm:374-498), over libcanu_mhap.so.

A job = one hash block (-s block.dat) against itself (unless --no-self) and against the
query blocks linked into queries/<job>/ (-q), numbered the jar's way: hash reads 1..N, query
reads N+1.. in file order (OverlapMhap.pm:227-232).  The executable's lines are checked
against the restatement of the jar's bytecode (oracle/mhap_jar.py, see tests/test_mhap.py)
with the jar's block semantics (the self search, then the -q search), and, where built, the
reference's mhapConvert reads them with canu's own conversion arguments."""
import dataclasses
import os
import subprocess

import numpy as np
import pytest

import mhap_jar as M
import oracle
from canu_amd import build as B
from canu_amd import mhap
from canu_amd.synth import ReadSet, synth_reads

FIELDS = ("a", "b", "raw", "a_bgn", "a_end", "a_len", "o", "b_bgn", "b_end", "b_len")
N, L, BLOCK = 60, 3000, 20
OPTS = ["-k", "16", "--num-hashes", "128", "--num-min-matches", "3", "--threshold", "0.78",
        "--ordered-sketch-size", "1536", "--ordered-kmer-size", "12", "--min-olap-length",
        "500", "--num-threads", "8"]
CANU_EXTRA = ["--repeat-weight", "0.9", "--repeat-idf-scale", "10",
              "--filter-threshold", "0.000005"]


@pytest.fixture(scope="module")
def cli():
    return B.build_mhap_cli(verbose=False)


def _run(cli, args, cwd=None):
    return subprocess.run([cli, *args], capture_output=True, text=True, cwd=cwd, timeout=300)


def test_cli_usage_errors(cli):
    for args in ([], ["-p", "x.fasta"], ["-p", "x.fasta", "-s", "y.dat", "-q", "."],
                 ["--bogus"], ["-k"], ["--no-tf", "-s", "missing.dat"],
                 ["--supress-noise", "5", "-s", "y.dat"],
                 ["--supress-noise", "-1", "-p", "x.fasta", "-q", "."]):
        cp = _run(cli, args)
        assert cp.returncode == 1, (args, cp.stderr)


def _reads():
    return synth_reads(n_reads=N, read_len=L, genome_len=int(N * L / 15), error_rate=0.04,
                       seed=3)


def _block(rs, lo, hi, first=1):
    """Reads lo..hi-1 (0-based) of rs as a read set numbered from `first`."""
    o0 = int(rs.offsets[lo])
    end = int(rs.offsets[hi - 1]) + int(rs.lengths[hi - 1])
    offs = rs.offsets[lo:hi] - np.uint64(o0)
    return ReadSet(bases=rs.bases[o0:end].copy(), offsets=offs.copy(),
                   lengths=rs.lengths[lo:hi].copy(), first_iid=first)


def _concat(blocks):
    bases = np.concatenate([b.bases for b in blocks])
    lens = np.concatenate([b.lengths for b in blocks])
    offs = np.zeros(lens.shape[0], dtype=np.uint64)
    offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    return ReadSet(bases=bases, offsets=offs, lengths=lens, first_iid=1)


def _parse(text):
    rows = []
    for line in text.splitlines():
        w = line.split()
        rows.append((int(w[0]), int(w[1]), float(w[2]), float(w[3]), int(w[5]), int(w[6]),
                     int(w[7]), int(w[8]), int(w[9]), int(w[10]), int(w[11]), 0))
    return np.array(rows, dtype=M.MHAP_DTYPE)


def _same(got, want):
    assert got.shape == want.shape, (got.shape, want.shape)
    for f in FIELDS:
        assert np.array_equal(got[f], want[f]), f
    # the line holds erate rounded half-up to 6 places (String.format)
    assert [mhap.java_fixed6(x) for x in want["erate"]] == [f"{x:.6f}" for x in got["erate"]]


@pytest.mark.gpu
def test_gpu_cli_precompute_and_jobs(cli, tmp_path):
    """canu's precompute.sh and mhap.sh command lines, with canu's weighting and a -f file
    holding k-mers on both sides of --filter-threshold."""
    import gzip
    extra = CANU_EXTRA
    rs = _reads()
    blocks = [_block(rs, i, i + BLOCK) for i in range(0, N, BLOCK)]
    bdir = tmp_path / "blocks"
    bdir.mkdir()
    # the -f file canu writes (Meryl.pm:699-716): a count line, kmer<TAB>fraction, both
    # strands; some of read 1's 16-mers at graded fractions
    r0 = rs.read(0).decode()
    comp = str.maketrans("ACGT", "TGCA")
    km, fr = [], []
    for j, i0 in enumerate(range(0, 2800, 9)):
        m = r0[i0:i0 + 16]
        km += [m, m.translate(comp)[::-1]]
        fr += [5e-6 * 1.4 ** (j % 15) * (0.05 if j % 3 == 0 else 1.0)] * 2
    fpath = tmp_path / "asm.ms16.frequentMers.ignore.gz"
    with gzip.open(fpath, "wt") as f:
        f.write(f"{len(km)}\n")
        for m, x in zip(km, fr):
            f.write(f"{m}\t{x:e}\n")
    fr_read = [float(f"{x:e}") for x in fr]          # the fractions as the file holds them
    for i, b in enumerate(blocks, start=1):
        fa = bdir / f"{i:06d}.input.fasta"
        with open(fa, "w") as f:
            for r in range(b.nreads):
                f.write(f">{BLOCK * (i - 1) + r + 1}\n{b.read(r).decode()}\n")
        cp = _run(cli, [*OPTS, *extra, "-f", str(fpath), "-p", f"./{fa.name}", "-q", "."],
                  cwd=bdir)
        assert cp.returncode == 0, cp.stderr
        os.replace(bdir / f"{i:06d}.input.dat", bdir / f"{i:06d}.dat")
    # the sketches are canu's weighted ones (tf-idf with the -f table)
    P = mhap.MhapParameters(num_hashes=128).canu_weighting(0.000005).as_oracle()
    freq = (km, np.array(fr_read))

    # job 1: block 1 against itself and blocks 2-3 (OverlapMhap.pm's "(and self)" case)
    q1 = tmp_path / "queries" / "000001"
    q1.mkdir(parents=True)
    for i in (2, 3):
        os.symlink(f"../../blocks/{i:06d}.dat", q1 / f"{i:06d}.dat")
    cp = _run(cli, [*OPTS, "-s", "./blocks/000001.dat", "-q", "queries/000001"], cwd=tmp_path)
    assert cp.returncode == 0, cp.stderr
    got = _parse(cp.stdout)
    self_want = M.run(blocks[0], P, freq=freq)
    cross_want = M.run(_concat(blocks), P, q_range=(BLOCK, N), t_range=(0, BLOCK), freq=freq,
                       to_self=False)
    assert len(self_want) > 5 and len(cross_want) > 5
    _same(got[:len(self_want)], self_want)
    _same(got[len(self_want):], cross_want)
    oracle.require_reference(mhap_convert=True)
    out = tmp_path / "000001.mhap"
    out.write_text(cp.stdout)
    # canu's conversion arguments for an "(and self)" job: -h <block bgn> 0 -q <block bgn>
    assert len(oracle.mhap_convert(rs, str(out), 1, 0, 1)) == len(got)

    # job 2: block 2 against block 3 only (--no-self); IDs are 1..20 (hash), 21..40 (query)
    cp = _run(cli, [*OPTS, "-s", "./blocks/000002.dat", "--no-self", "-q",
                    "./blocks/000003.dat"], cwd=tmp_path)
    assert cp.returncode == 0, cp.stderr
    got2 = _parse(cp.stdout)
    want2 = M.run(_concat(blocks[1:]), P, q_range=(BLOCK, 2 * BLOCK), t_range=(0, BLOCK),
                  freq=freq, to_self=False)
    _same(got2, want2)

    # a sketch file made with other options is refused
    cp = _run(cli, ["-k", "14", *OPTS[2:], "-s", "./blocks/000001.dat"], cwd=tmp_path)
    assert cp.returncode == 1 and "other -k" in cp.stderr
