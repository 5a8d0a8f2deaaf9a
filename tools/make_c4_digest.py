#!/usr/bin/env python3
"""Pin configs[4]'s rank jobs at a size past the unit tests: run the REFERENCE overlapInCore
(oracle/_ref/oic_ref, compiled from /root/reference's own sources by oracle/Makefile) on
every job of bench.py's `--workload configs4-rank` plan and commit the digests of their
records as tests/golden/c4rank<reads/1000>k.json.

The read set is bench.py's configs4-rank one (synth_reads_parallel: ONT-like reads, 12 kb
+-20 %, 15x, 1.5 % error, seed 5) at `--reads`; the plan is canu_amd.dist.hash_block_jobs'
8-way cut, each job `-h lo-hi -r 1-hi` with --hashbits 23 --hashload 0.75 and the hash
batches OverlapDriver cuts (overlapInCore.C:191-300), exactly as bench.py's job sets them.

The fixture is data: per job the record count, SHA-256 of the sorted 24-B records, the
additive multiset hash (canu_amd/digest.py) and the reference's -s counters.  bench.py
(configs4-rank at this size) and tests/test_gpu_c4_digest.py compare the HIP path with it.

    python tools/make_c4_digest.py [--reads 20000] [--threads 8] [--jobs 0,7]
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
from canu_amd.dist import hash_block_jobs  # noqa: E402
from canu_amd.synth import synth_reads_parallel  # noqa: E402

HASHBITS, HASHLOAD, HASHSTRINGS, PLAN_RANKS = 23, 0.75, 10_000_000, 8


def c4_reads(n: int, read_len: int, coverage: float, error: float, seed: int):
    """bench.py Configs4Rank's read set at one rank (world 1)."""
    return synth_reads_parallel(n, read_len, int(n * read_len / coverage), error, seed=seed,
                                len_jitter=0.2, read_range=(0, n), workers=8)


def c4_jobs(n: int, read_len: int) -> list[dict]:
    load = HASHLOAD * (1 << HASHBITS) * 21
    return hash_block_jobs(n, PLAN_RANKS, read_len, 36.0, 3.0 * load)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--reads", type=int, default=20_000)
    ap.add_argument("--read-len", type=int, default=12_000)
    ap.add_argument("--coverage", type=float, default=15.0)
    ap.add_argument("--read-error", type=float, default=0.015)
    ap.add_argument("--k", type=int, default=22)
    ap.add_argument("--maxerate", type=float, default=0.06)
    ap.add_argument("--minlength", type=int, default=500)
    ap.add_argument("--seed", type=int, default=5)
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--jobs", default=None, help="comma list of plan jobs (default: all)")
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    out = args.out or os.path.join(ROOT, "tests", "golden", f"c4rank{args.reads // 1000}k.json")

    t0 = time.time()
    rs = c4_reads(args.reads, args.read_len, args.coverage, args.read_error, args.seed)
    t_gen = time.time() - t0
    jobs = c4_jobs(args.reads, args.read_len)
    pick = range(len(jobs)) if args.jobs is None else [int(x) for x in args.jobs.split(",")]
    p = oracle.default_params(kmer_len=args.k, max_erate=args.maxerate,
                              min_olap_len=args.minlength)
    res = []
    for ji in pick:
        (h_lo, h_hi), (r_lo, r_hi) = jobs[ji]["h"], jobs[ji]["r"]
        hashed = int(rs.lengths[h_lo - 1:h_hi].sum(dtype=np.uint64)) + (h_hi - h_lo + 1)
        t1 = time.time()
        rec, stats = oracle.run_reference(
            rs, p, threads=args.threads, hash_bits=HASHBITS,
            batching={"hashstrings": HASHSTRINGS, "hashdatalen": hashed + 1024,
                      "hashload": HASHLOAD},
            extra=["-h", f"{h_lo}-{h_hi}", "-r", f"{r_lo}-{r_hi}"], with_stats=True)
        wall = time.time() - t1
        res.append({"index": ji, "h": [h_lo, h_hi], "r": [r_lo, r_hi],
                    "records": int(rec.shape[0]), "sha256_sorted": digest.sha256_sorted(rec),
                    "multiset_hash": f"{digest.multiset_hash(rec):016x}", "stats": stats,
                    "wall_s": round(wall, 1)})
        print(json.dumps(res[-1]), flush=True)
    fx = {
        "workload": {"workload": "configs4-rank", "reads": args.reads,
                     "read_len": args.read_len, "coverage": args.coverage,
                     "read_error": args.read_error, "seed": args.seed, "k": args.k,
                     "maxerate": p["max_erate"], "minlength": args.minlength,
                     "total_bases": rs.total_bases()},
        "reference": {"binary": "oracle/_ref/oic_ref (reference overlapInCore built from its "
                                "sources), one run per plan job: -h lo-hi -r 1-hi",
                      "threads": args.threads, "hashbits": HASHBITS, "hashload": HASHLOAD,
                      "hashstrings": HASHSTRINGS, "hashdatalen": "job's hashed bases + 1024",
                      "plan_ranks": PLAN_RANKS, "gen_s": round(t_gen, 1)},
        "jobs": res,
    }
    with open(out, "w") as f:
        json.dump(fx, f, indent=1)
        f.write("\n")


if __name__ == "__main__":
    main()
