#!/usr/bin/env python3
"""Pin the benchmark job at full size: run the REFERENCE overlapInCore (oracle/_ref/oic_ref,
compiled from /root/reference's own sources by oracle/Makefile) on bench.py's exact read set
and commit the digest of its records as tests/golden/bench50k.json.

The read set is bench.py's: synth_reads(50k reads, 10 kb, 25x of a 20 Mbp random genome,
1.5 % error, seed 1).  The reference runs it as ONE hash batch (--hashstrings > n,
--hashdatalen > bases + n) searched by every read (-r 1-n), so every a < b pair is searched
once -- the job bench.py times (overlapInCore.C:191-300 OverlapDriver, one iteration).

The fixture is data: record count, SHA-256 of the sorted 24-B records, the additive
multiset hash (canu_amd/digest.py), and the reference's -s counters.  bench.py and
tests/test_gpu_bench_digest.py compare the HIP path's records with it.

    python tools/make_bench_digest.py [--reads 50000] [--threads 8]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import oracle  # noqa: E402
from canu_amd import digest  # noqa: E402
from canu_amd.synth import random_genome, synth_reads  # noqa: E402


def bench_reads(n: int, read_len: int, coverage: float, error: float, seed: int):
    """Exactly bench.py's read set (same genome, same per-read streams)."""
    genome_len = int(n * read_len / coverage)
    genome = random_genome(np.random.default_rng(seed), genome_len)
    return synth_reads(n_reads=n, read_len=read_len, genome_len=genome_len, error_rate=error,
                       seed=seed, genome=genome, read_range=(0, n))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--reads", type=int, default=50_000)
    ap.add_argument("--read-len", type=int, default=10_000)
    ap.add_argument("--coverage", type=float, default=25.0)
    ap.add_argument("--read-error", type=float, default=0.015)
    ap.add_argument("--k", type=int, default=22)
    ap.add_argument("--maxerate", type=float, default=0.06)
    ap.add_argument("--minlength", type=int, default=500)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--hashbits", type=int, default=25)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    out = args.out or os.path.join(ROOT, "tests", "golden",
                                   f"bench{args.reads // 1000}k.json")

    t0 = time.time()
    rs = bench_reads(args.reads, args.read_len, args.coverage, args.read_error, args.seed)
    t_gen = time.time() - t0
    p = oracle.default_params(kmer_len=args.k, max_erate=args.maxerate,
                              min_olap_len=args.minlength)
    t1 = time.time()
    rec, stats = oracle.run_reference(rs, p, threads=args.threads, hash_bits=args.hashbits,
                                      with_stats=True)
    t_ref = time.time() - t1
    fx = {
        "workload": {"reads": args.reads, "read_len": args.read_len, "coverage": args.coverage,
                     "read_error": args.read_error, "seed": args.seed, "k": args.k,
                     "maxerate": p["max_erate"], "minlength": args.minlength,
                     "total_bases": rs.total_bases()},
        "reference": {"binary": "oracle/_ref/oic_ref (reference overlapInCore built from its "
                                "sources; one hash batch, -h 1-n -r 1-n)",
                      "threads": args.threads, "hashbits": args.hashbits,
                      "wall_s": round(t_ref, 1), "gen_s": round(t_gen, 1)},
        "records": int(rec.shape[0]),
        "sha256_sorted": digest.sha256_sorted(rec),
        "multiset_hash": f"{digest.multiset_hash(rec):016x}",
        "stats": stats,
    }
    with open(out, "w") as f:
        json.dump(fx, f, indent=1)
        f.write("\n")
    print(json.dumps(fx))


if __name__ == "__main__":
    main()
