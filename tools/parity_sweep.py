#!/usr/bin/env python3
"""Randomised GPU-vs-oracle parity sweep (beyond tests/test_gpu_parity.py's fixed cases).

Each case draws a read set (count, length, error rate, seed, ragged lengths, 'n' bases)
and an option mix (k,
maxErate, minimum overlap, -G partial, -m multiple-per-pair) and compares the HIP path's
ovOverlap records and counters with the oracle bit for bit.  Run on a GPU box:

    python tools/parity_sweep.py [--cases 20] [--seed 7]
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

COUNTERS = ("kmer_hits_with_olap", "kmer_hits_without_olap", "total_overlaps",
            "contained_overlaps", "dovetail_overlaps", "seed_hits", "multi_overlaps",
            "kmer_hits_skipped")


def one_case(rng, i):
    n = int(rng.integers(80, 320))
    L = int(rng.choice([1500, 3000, 6000, 10000, 14000]))
    err = float(rng.choice([0.01, 0.02, 0.04, 0.07]))
    cov = float(rng.uniform(8, 25))
    glen = max(4 * L, int(n * L / cov))
    k = int(rng.choice([16, 22]))
    erate = float(np.float32(rng.choice([0.06, 0.1, 0.144])))
    if L >= 10000:                 # keep each oracle run well under a minute
        n = min(n, 140)
        if err >= 0.04:
            erate = float(np.float32(0.06))
    P = OicParameters(Kmer_Len=k, maxErate=erate, Min_Olap_Len=int(rng.choice([100, 500])))
    if rng.random() < 0.25:
        P.Doing_Partial_Overlaps = True
    if rng.random() < 0.25:
        P.Unique_Olap_Per_Pair = False
    P = P.finalize()
    # ragged lengths (the extension's length classes) and 'n' bases (the generic kernel)
    jitter = float(rng.choice([0.0, 0.0, 0.3]))
    n_rate = float(rng.choice([0.0, 0.0, 0.001]))
    rs = synth_reads(n, L, glen, err, seed=int(rng.integers(1, 1 << 30)), len_jitter=jitter,
                     n_rate=n_rate)
    t0 = time.time()
    oic = OverlapInCore(P, device=0)
    oic.load_reads(rs)
    oic.build_hash_index(1, 0xFFFFFFFF)
    got = oic.fetch(oic.find_overlaps(1, 0xFFFFFFFF))
    st = oic.stats()
    oic.close()
    t1 = time.time()
    print(f"  case {i}: gpu done ({got.shape[0]} records), running the oracle", flush=True)
    want, wst = oracle.run_oracle(rs, P.as_dict(), with_stats=True)
    t2 = time.time()
    ok = got.shape == want.shape and np.array_equal(got, want) and \
        all(st[f] == wst[f] for f in COUNTERS)
    desc = (f"case {i}: {n} reads x {L} bp err {err} cov {cov:.0f} k {k} erate {erate:.3f} "
            f"partial {int(P.Doing_Partial_Overlaps)} unique {int(P.Unique_Olap_Per_Pair)}: "
            f"{got.shape[0]} vs {want.shape[0]} records, gpu {t1 - t0:.1f}s oracle {t2 - t1:.1f}s")
    return ok, desc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cases", type=int, default=20)
    ap.add_argument("--seed", type=int, default=7)
    a = ap.parse_args()
    rng = np.random.default_rng(a.seed)
    bad = 0
    for i in range(a.cases):
        ok, desc = one_case(rng, i)
        print(("OK   " if ok else "FAIL ") + desc, flush=True)
        bad += 0 if ok else 1
    print(f"{a.cases - bad}/{a.cases} cases bit-exact", flush=True)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
