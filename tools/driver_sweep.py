#!/usr/bin/env python3
"""Randomised parity sweep of the OverlapDriver path (ovl_overlap_driver) against the oracle's
restatement of OverlapDriver (oracle.run_oracle_driver, pinned to the reference overlapInCore
by tests/test_driver.py): each case draws a read set (count, length, error, ragged lengths,
'n' bases, skip k-mers near read ends), canu's batch options (--hashstrings, --hashbits /
--hashload, -t, a -h / -r sub-range) and the driver's own plan knobs -- sorted windows on or
off (OVL_SQ), query-chunk and super-batch caps (OVL_SQ_CHUNK_WINDOWS, OVL_SB_WINDOWS), dense
tables (OVL_DENSE_TABLES), batch by batch (OVL_SUPERBATCH=0) -- and compares the records and
the -s counters bit for bit.  Run on a GPU box:

    python tools/driver_sweep.py [--cases 24] [--seed 11]
"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

from canu_amd.overlap_in_core import OicParameters, OverlapInCore  # noqa: E402
from canu_amd.synth import synth_reads  # noqa: E402
import oracle  # noqa: E402

STATS = [("total", "total_overlaps"), ("kmer_hits_with_olap", "kmer_hits_with_olap"),
         ("kmer_hits_without_olap", "kmer_hits_without_olap"), ("multi", "multi_overlaps"),
         ("contained", "contained_overlaps"), ("dovetail", "dovetail_overlaps")]
KNOBS = ("OVL_SQ", "OVL_SQ_CHUNK_WINDOWS", "OVL_SB_WINDOWS", "OVL_DENSE_TABLES", "OVL_SUPERBATCH")


def end_skip_kmers(rs, k, every):
    out = set()
    for r in range(0, rs.nreads, every):
        seq = rs.read(r).decode().upper()
        for i in (0, 23, 46, len(seq) - k - 40, len(seq) - k - 1):
            s = seq[max(i, 0):max(i, 0) + k]
            if len(s) == k and set(s) <= set("ACGT"):
                out.add(s)
    return sorted(out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cases", type=int, default=24)
    ap.add_argument("--seed", type=int, default=11)
    a = ap.parse_args()
    rng = np.random.default_rng(a.seed)
    ok_all = True
    for c in range(a.cases):
        n = int(rng.integers(120, 360))
        L = int(rng.integers(1500, 6000))
        err = float(rng.choice([0.01, 0.02, 0.035]))
        rs = synth_reads(n_reads=n, read_len=L, genome_len=int(n * L / rng.uniform(10, 25)),
                         error_rate=err, seed=int(rng.integers(1, 1 << 30)),
                         len_jitter=float(rng.choice([0.0, 0.3])),
                         n_rate=float(rng.choice([0.0, 0.0, 0.001])))
        k = int(rng.choice([22, 22, 16]))
        maxerate = 0.06 if k == 22 else 0.12
        P = oracle.default_params(kmer_len=k, max_erate=maxerate, min_olap_len=500)
        hs = int(rng.choice([30, 60, 100, 10000]))
        hbits, hload = (int(rng.choice([12, 13, 22])), float(rng.choice([0.5, 0.75])))
        threads = int(rng.choice([1, 4, 16]))
        hr = (1, n) if rng.random() < 0.7 else (int(rng.integers(1, n // 3)), n)
        rr = (1, n) if rng.random() < 0.6 else (int(rng.integers(1, n // 4)), int(rng.integers(n // 2, n)))
        skip = end_skip_kmers(rs, k, int(rng.choice([3, 7]))) if rng.random() < 0.4 else None
        knobs = {}
        mode = rng.integers(0, 5)
        if mode == 0:
            knobs["OVL_SUPERBATCH"] = "0"
        knobs["OVL_SQ"] = str(int(rng.choice([0, 1, 3])))
        if rng.random() < 0.5:
            knobs["OVL_SQ_CHUNK_WINDOWS"] = str(int(rng.integers(50_000, 400_000)))
        if rng.random() < 0.5:
            knobs["OVL_SB_WINDOWS"] = str(int(rng.integers(80_000, 500_000)))
        if rng.random() < 0.3:
            knobs["OVL_DENSE_TABLES"] = "1"
        for kn in KNOBS:
            os.environ.pop(kn, None)
        os.environ.update(knobs)
        O = OicParameters(Kmer_Len=k, maxErate=P["max_erate"], Min_Olap_Len=500,
                          Max_Hash_Strings=hs, Hash_Mask_Bits=hbits, Max_Hash_Load=hload,
                          Num_PThreads=threads).finalize()
        O.bgnHashID, O.endHashID = hr
        O.bgnRefID, O.endRefID = rr
        t0 = time.time()
        oic = OverlapInCore(O, device=0)
        try:
            got = oic.run_driver(rs, skip_kmers=skip)
            st = oic.stats()
        finally:
            oic.close()
        t1 = time.time()
        want, wst, batches = oracle.run_oracle_driver(
            rs, P, hash_range=hr, ref_range=rr, threads=threads, hashstrings=hs,
            hashbits=hbits, hashload=hload, skip_kmers=skip, with_stats=True)
        same = got.shape == want.shape and np.array_equal(got, want) and \
            all(st[g] == wst[g] for _, g in STATS) and st["hash_batches"] == len(batches)
        ok_all &= same
        print(f"case {c}: {n} reads x {L} bp err {err} k {k} -h {hr[0]}-{hr[1]} -r {rr[0]}-{rr[1]} "
              f"hs {hs} hb {hbits}/{hload} t {threads} skip {len(skip) if skip else 0} "
              f"{knobs} -> batches {len(batches)} sb {st['super_batches']} chunks "
              f"{st['query_chunks']} records {got.shape[0]} vs {want.shape[0]}: "
              f"{'ok' if same else 'MISMATCH'} ({t1 - t0:.1f} s gpu)", flush=True)
    print("ALL OK" if ok_all else "MISMATCHES")
    sys.exit(0 if ok_all else 1)


if __name__ == "__main__":
    main()
