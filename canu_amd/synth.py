"""Synthetic read sets for the overlapInCore path (no network, no datasets here).

A random genome is sampled into reads with substitution / insertion / deletion errors,
random strand, optional 'N' bases and optional planted repeats.  The generator is
deterministic in its seed.  Reads are returned the way gkStore hands them to
overlapInCore (Process_Overlaps.C:118-126): one byte per base, upper case, concatenated,
with 64-bit offsets and 32-bit lengths; read i gets gkStore ID first_iid + i.
"""
from __future__ import annotations

import dataclasses
import struct

import numpy as np

_ACGT = np.frombuffer(b"ACGT", dtype=np.uint8)
_COMP = np.zeros(256, dtype=np.uint8)
for _a, _b in zip(b"ACGTN", b"TGCAN"):
    _COMP[_a] = _b


@dataclasses.dataclass
class ReadSet:
    bases: np.ndarray        # uint8, concatenated
    offsets: np.ndarray      # uint64, start of each read in bases
    lengths: np.ndarray      # uint32
    quals: np.ndarray | None = None   # uint8 0..60, same layout as bases
    first_iid: int = 1
    starts: np.ndarray | None = None  # synthetic truth: genome start of each read
    strands: np.ndarray | None = None # synthetic truth: 1 = reverse-complemented

    @property
    def nreads(self) -> int:
        return int(self.lengths.shape[0])

    def read(self, i: int) -> bytes:
        o = int(self.offsets[i])
        return self.bases[o:o + int(self.lengths[i])].tobytes()

    def total_bases(self) -> int:
        return int(self.lengths.sum(dtype=np.uint64))


# Named profiles of BASELINE.json's configs.  "ont" is the headline workload.
PROFILES = {
    # configs[0]: 1k PacBio-like 3 kb reads at E. coli scale (4.6 Mbp genome).
    "pacbio-ecoli": dict(n_reads=1000, read_len=3000, genome_len=4_600_000, error_rate=0.02),
    # configs[1]/[2]: 50k ONT-like 10 kb reads; 20 Mbp genome -> 25x coverage.
    "ont-50k": dict(n_reads=50_000, read_len=10_000, genome_len=20_000_000, error_rate=0.015),
}


def random_genome(rng: np.random.Generator, length: int, n_repeats: int = 0,
                  repeat_len: int = 0) -> np.ndarray:
    g = _ACGT[rng.integers(0, 4, size=length, dtype=np.int64)]
    if n_repeats and repeat_len:
        unit = _ACGT[rng.integers(0, 4, size=repeat_len, dtype=np.int64)]
        for _ in range(n_repeats):
            p = int(rng.integers(0, max(1, length - repeat_len)))
            g[p:p + repeat_len] = unit
    return g


def _mutate(rng: np.random.Generator, seg: np.ndarray, out_len: int, error_rate: float,
            sub_frac: float, ins_frac: float) -> np.ndarray:
    n = seg.shape[0]
    r = rng.random(n)
    p_sub = error_rate * sub_frac
    p_ins = error_rate * ins_frac
    is_sub = r < p_sub
    is_ins = (r >= p_sub) & (r < p_sub + p_ins)
    is_del = (r >= p_sub + p_ins) & (r < error_rate)
    out = seg.copy()
    if is_sub.any():
        shift = rng.integers(1, 4, size=int(is_sub.sum()))
        idx = np.searchsorted(_ACGT, out[is_sub])
        out[is_sub] = _ACGT[(idx + shift) % 4]
    counts = np.ones(n, dtype=np.int64)
    counts[is_del] = 0
    counts[is_ins] = 2
    rep = np.repeat(out, counts)
    # the first copy of each inserted position becomes a random base
    ins_pos = np.cumsum(counts)[is_ins] - 2
    if ins_pos.size:
        rep[ins_pos] = _ACGT[rng.integers(0, 4, size=ins_pos.size)]
    return rep[:out_len]


def synth_reads(n_reads: int, read_len: int, genome_len: int, error_rate: float,
                seed: int = 1, sub_frac: float = 0.4, ins_frac: float = 0.3,
                len_jitter: float = 0.0, n_rate: float = 0.0, n_repeats: int = 0,
                repeat_len: int = 0, with_quals: bool = False, bursts: int = 0,
                genome: np.ndarray | None = None, read_range: tuple[int, int] | None = None
                ) -> ReadSet:
    """Sample `n_reads` reads of about `read_len` bases from a random genome.

    Read i is drawn from its own stream (seed, i), so any sub-range [lo, hi) of the reads
    can be generated on its own (read_range): ranks build their slice and all-gather."""
    if genome is None:
        genome = random_genome(np.random.default_rng(seed), genome_len, n_repeats, repeat_len)
    genome_len = genome.shape[0]
    lo, hi = read_range if read_range else (0, n_reads)
    lengths = np.empty(hi - lo, dtype=np.uint32)
    starts = np.empty(hi - lo, dtype=np.int64)
    strands = np.zeros(hi - lo, dtype=np.uint8)
    chunks = []
    for i in range(lo, hi):
        rng = np.random.default_rng([seed, i])
        L = read_len
        if len_jitter > 0:
            L = max(64, int(read_len * (1.0 + len_jitter * (2.0 * rng.random() - 1.0))))
        L = min(L, genome_len)
        span = min(genome_len, int(L * (1.0 + 2.0 * error_rate)) + 32)
        start = int(rng.integers(0, genome_len - span + 1))
        seg = genome[start:start + span]
        rd = _mutate(rng, seg, L, error_rate, sub_frac, ins_frac)
        starts[i - lo] = start
        if bursts:
            # low-quality stretches: 60 bases with 30 % substitutions (window-filter cases)
            brng = np.random.default_rng([seed, i, 11])
            rd = rd.copy()
            for _ in range(bursts):
                b0 = int(brng.integers(0, max(1, rd.shape[0] - 60)))
                sel = b0 + np.nonzero(brng.random(60) < 0.3)[0]
                sel = sel[sel < rd.shape[0]]
                idx = np.searchsorted(_ACGT, rd[sel])
                rd[sel] = _ACGT[(idx + brng.integers(1, 4, size=sel.size)) % 4]
        if rng.random() < 0.5:
            rd = _COMP[rd[::-1]]
            strands[i - lo] = 1
        if n_rate > 0:
            m = rng.random(rd.shape[0]) < n_rate
            rd = rd.copy()
            rd[m] = ord("N")
        chunks.append(rd)
        lengths[i - lo] = rd.shape[0]
    bases = np.concatenate(chunks) if chunks else np.zeros(0, np.uint8)
    offsets = np.zeros(hi - lo, dtype=np.uint64)
    if hi - lo > 1:
        offsets[1:] = np.cumsum(lengths[:-1], dtype=np.uint64)
    quals = None
    if with_quals:
        quals = np.random.default_rng([seed, n_reads, 7]).integers(
            2, 41, size=bases.shape[0]).astype(np.uint8)
    return ReadSet(bases=bases, offsets=offsets, lengths=lengths, quals=quals,
                   first_iid=1 + lo, starts=starts, strands=strands)


_PAR = {}


def _par_slice(lo_hi):
    g = _PAR
    return synth_reads(g["n"], g["len"], g["glen"], g["err"], seed=g["seed"],
                       len_jitter=g["jit"], genome=g["genome"], read_range=lo_hi)


def concat_read_sets(parts: list[ReadSet], first_iid: int) -> ReadSet:
    lengths = np.concatenate([p.lengths for p in parts])
    offsets = np.zeros(lengths.shape[0], dtype=np.uint64)
    if lengths.shape[0] > 1:
        offsets[1:] = np.cumsum(lengths[:-1], dtype=np.uint64)
    return ReadSet(bases=np.concatenate([p.bases for p in parts]), offsets=offsets,
                   lengths=lengths, quals=None, first_iid=first_iid,
                   starts=np.concatenate([p.starts for p in parts]),
                   strands=np.concatenate([p.strands for p in parts]))


def synth_reads_parallel(n_reads: int, read_len: int, genome_len: int, error_rate: float,
                         seed: int = 1, len_jitter: float = 0.0,
                         read_range: tuple[int, int] | None = None,
                         workers: int = 8) -> ReadSet:
    """synth_reads over [lo, hi) in `workers` forked processes (read i depends only on
    (seed, i), so the slices concatenate to exactly what one synth_reads call returns)."""
    import multiprocessing as mp
    import sys
    lo, hi = read_range if read_range else (0, n_reads)
    genome = random_genome(np.random.default_rng(seed), genome_len)
    # no worker pool is forked from a process that has initialised the GPU (its children
    # would inherit the device state); such a caller generates serially
    torch = sys.modules.get("torch")
    oic = sys.modules.get("canu_amd.overlap_in_core")
    if (torch is not None and torch.cuda.is_initialized()) or \
            (oic is not None and getattr(oic, "_lib", None) is not None):
        workers = 1
    if workers <= 1 or hi - lo < 1024:
        return synth_reads(n_reads, read_len, genome_len, error_rate, seed=seed,
                           len_jitter=len_jitter, genome=genome, read_range=(lo, hi))
    _PAR.update(n=n_reads, len=read_len, glen=genome_len, err=error_rate, seed=seed,
                jit=len_jitter, genome=genome)
    pieces = max(workers * 4, 1)
    cuts = [(lo + (hi - lo) * i // pieces, lo + (hi - lo) * (i + 1) // pieces)
            for i in range(pieces)]
    # close + join (not the context manager's terminate): the workers exit on their own, so
    # no SIGTERM reaches them (a profiler's inherited signal handler logs one as an abort)
    pool = mp.get_context("fork").Pool(workers)
    try:
        parts = pool.map(_par_slice, cuts)
        pool.close()
    except BaseException:
        pool.terminate()
        raise
    finally:
        pool.join()
    _PAR.clear()
    return concat_read_sets(parts, first_iid=1 + lo)


def profile(name: str, seed: int = 1, **over) -> ReadSet:
    kw = dict(PROFILES[name])
    kw.update(over)
    return synth_reads(seed=seed, **kw)


def scaled_profile(name: str, n_reads: int, seed: int = 1) -> ReadSet:
    """The same read length / error / coverage as `name`, with fewer reads (the genome
    shrinks with the read count, so per-read work stays the same)."""
    kw = dict(PROFILES[name])
    scale = n_reads / kw["n_reads"]
    kw["genome_len"] = max(kw["read_len"] * 4, int(kw["genome_len"] * scale))
    kw["n_reads"] = n_reads
    return synth_reads(seed=seed, **kw)


def write_reads_file(path: str, rs: ReadSet) -> None:
    """The reads file oracle/ref_harness.cpp reads ("OICR" v1)."""
    with open(path, "wb") as f:
        f.write(b"OICR")
        f.write(struct.pack("<III", 1, rs.nreads, 1 if rs.quals is not None else 0))
        f.write(rs.lengths.astype("<u4").tobytes())
        f.write(rs.bases.tobytes())
        if rs.quals is not None:
            f.write(rs.quals.tobytes())
