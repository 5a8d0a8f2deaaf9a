"""CPU model of k_cut_index (canu_amd/csrc/ovl_index.hip): a load-cut driver batch takes its
index from the index of the longer prefix built to find the cut, instead of building it again
over the cut range (Build_Hash_Index.C:495-541 decides the cut).

The index keeps each k-mer's occurrences as one run in chain order -- position descending,
(iid << 32 | offset), the order Hash_Insert chains them (Build_Hash_Index.C:296-341) -- so a
k-mer's occurrences in reads past the cut lead its run.  The kernel moves each table entry
past them (binary search); a k-mer left with none keeps its slot with an empty run, which the
probe reads as {off 0, cnt 0}, the record of a miss.  This checks, on random reads with
repeats, that every lookup of the cut index equals the same lookup of an index built over
the cut range alone (the GPU side is checked against the reference in the driver tests'
table-load case and the configs[4] digests, -m gpu).
"""
import random

import pytest


def build(reads, lo, hi, k):
    """k-mer -> its occurrences in reads lo..hi, position descending (one sorted run)."""
    idx = {}
    for iid in range(lo, hi + 1):
        s = reads[iid]
        for p in range(len(s) - k + 1):
            idx.setdefault(s[p:p + k], []).append((iid << 32) | p)
    occ, table = [], {}
    for kmer, run in idx.items():
        run.sort(reverse=True)
        table[kmer] = (len(occ), len(run))
        occ.extend(run)
    return table, occ


def cut(table, occ, last):
    """k_cut_index: skip each run's leading occurrences in reads > last."""
    out = {}
    for kmer, (off, n) in table.items():
        lo, hi = 0, n
        while lo < hi:
            mid = (lo + hi) // 2
            if (occ[off + mid] >> 32) > last:
                lo = mid + 1
            else:
                hi = mid
        out[kmer] = (off + lo if lo < n else 0, n - lo)
    return out


def lookup(table, occ, kmer):
    """What a probe record and the chain read: the occurrence list ({0, 0} on a miss)."""
    off, n = table.get(kmer, (0, 0))
    return [occ[off + i] for i in range(n)]


@pytest.mark.parametrize("seed", [1, 2, 3, 4, 5])
def test_cut_index_equals_rebuild(seed):
    rng = random.Random(seed)
    k = 5
    genome = "".join(rng.choice("ACGT") for _ in range(400))
    reads = {}
    for iid in range(1, 61):                     # overlapping pieces of one genome: shared k-mers
        b = rng.randrange(0, 300)
        reads[iid] = genome[b:b + rng.randrange(30, 100)]
    lo, hi = 11, 60
    t_pre, occ_pre = build(reads, lo, hi, k)
    for last in (lo, 25, 40, hi - 1, hi):
        t_cut = cut(t_pre, occ_pre, last)
        t_ref, occ_ref = build(reads, lo, last, k)
        kmers = set(t_pre) | set(t_ref) | {"".join(rng.choice("ACGT") for _ in range(k))
                                           for _ in range(50)}
        for kmer in kmers:
            assert lookup(t_cut, occ_pre, kmer) == lookup(t_ref, occ_ref, kmer), (last, kmer)
