#!/usr/bin/env python3
"""Pin the driver's chunked sorted-window search at full scale: a thin hash slice of the
configs[4] read set searched by a large query range, run by the REFERENCE overlapInCore
(oracle/_ref/oic_ref, compiled from /root/reference's sources by oracle/Makefile), digest
committed as tests/golden/c4chunk<reads/1000>k.json.

The read set is bench.py's configs4-rank one at 4M reads (synth_reads_parallel: 12 kb +-20 %,
15x, 1.5 % error, seed 5); the job is `-h HI-SLICE+1-HI -r 1-HI` with canu's --hashbits 23
--hashload 0.75: one hash batch, every read 1..HI a query (Find_Overlaps.C:328 pairs each
query with the slice's reads of larger ID).  On the GPU the same job runs with the sorted
query windows on (OVL_SQ=1; the chunk sizes are the driver's own, planned from free HBM):
2M queries are ~48 G windows, more than one chunk's worth of HBM several times over, so
the driver cuts the query range into several chunks on its own (no OVL_SQ_CHUNK_WINDOWS /
OVL_SB_WINDOWS caps) -- tests/test_gpu_c4_chunks.py and bench.py's c4chunk side line.

The reads file is written piecewise (2M x 12 kb is 24 GB; the host holds one piece at a
time), then handed to the reference by path.

    python tools/make_c4_chunk_digest.py [--hi 2000000] [--slice 4000] [--threads 8]
"""
from __future__ import annotations

import argparse
import json
import os
import struct
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import oracle  # noqa: E402
from canu_amd import digest  # noqa: E402
from canu_amd.synth import synth_reads_parallel  # noqa: E402

HASHBITS, HASHLOAD, HASHSTRINGS = 23, 0.75, 10_000_000


def write_reads_piecewise(path: str, n: int, hi: int, read_len: int, coverage: float,
                          error: float, seed: int, piece: int = 250_000) -> tuple[int, int]:
    """Reads 1..hi of the n-read set into an "OICR" v1 file (synth.write_reads_file's
    format), generated piece by piece; returns (total bases, bases of the last `slice`)."""
    genome_len = int(n * read_len / coverage)
    lens = np.zeros(hi, dtype="<u4")
    with open(path, "wb") as f:
        f.write(b"OICR")
        f.write(struct.pack("<III", 1, hi, 0))
        f.seek(4 * hi, os.SEEK_CUR)                  # the lengths, written at the end
        for lo in range(0, hi, piece):
            h = min(hi, lo + piece)
            rs = synth_reads_parallel(n, read_len, genome_len, error, seed=seed,
                                      len_jitter=0.2, read_range=(lo, h), workers=8)
            lens[lo:h] = rs.lengths
            f.write(memoryview(np.ascontiguousarray(rs.bases)))
            del rs
            print(f"  reads {lo + 1}-{h} written", flush=True)
        f.seek(16)
        f.write(lens.tobytes())
    return int(lens.sum(dtype=np.uint64)), lens


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--reads", type=int, default=4_000_000)
    ap.add_argument("--hi", type=int, default=2_000_000)
    ap.add_argument("--slice", type=int, default=4000)
    ap.add_argument("--read-len", type=int, default=12_000)
    ap.add_argument("--coverage", type=float, default=15.0)
    ap.add_argument("--read-error", type=float, default=0.015)
    ap.add_argument("--k", type=int, default=22)
    ap.add_argument("--maxerate", type=float, default=0.06)
    ap.add_argument("--minlength", type=int, default=500)
    ap.add_argument("--seed", type=int, default=5)
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--workdir", default=None)
    ap.add_argument("--reuse", action="store_true", help="reuse <workdir>/reads.bin")
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    out = args.out or os.path.join(ROOT, "tests", "golden", f"c4chunk{args.hi // 1000}k.json")
    wd = args.workdir or tempfile.mkdtemp(prefix="c4chunk_", dir=os.environ.get("TMPDIR", "/tmp"))
    os.makedirs(wd, exist_ok=True)
    reads = os.path.join(wd, "reads.bin")
    t0 = time.time()
    if args.reuse and os.path.exists(reads):          # a reads file an earlier run wrote
        with open(reads, "rb") as f:
            assert f.read(4) == b"OICR" and struct.unpack("<III", f.read(12))[1] == args.hi
            lens = np.frombuffer(f.read(4 * args.hi), dtype="<u4")
        total = int(lens.sum(dtype=np.uint64))
    else:
        total, lens = write_reads_piecewise(reads, args.reads, args.hi, args.read_len,
                                            args.coverage, args.read_error, args.seed)
    t_gen = time.time() - t0
    h_lo, h_hi = args.hi - args.slice + 1, args.hi
    hashed = int(lens[h_lo - 1:h_hi].sum(dtype=np.uint64)) + (h_hi - h_lo + 1)
    p = oracle.default_params(kmer_len=args.k, max_erate=args.maxerate,
                              min_olap_len=args.minlength)
    t1 = time.time()
    rec, stats = oracle.run_reference(
        None, p, threads=args.threads, hash_bits=HASHBITS,
        batching={"hashstrings": HASHSTRINGS, "hashdatalen": hashed + 1024, "hashload": HASHLOAD},
        extra=["-h", f"{h_lo}-{h_hi}", "-r", f"1-{h_hi}"], with_stats=True, workdir=wd,
        reads_path=reads)
    wall = time.time() - t1
    job = {"h": [h_lo, h_hi], "r": [1, h_hi], "records": int(rec.shape[0]),
           "sha256_sorted": digest.sha256_sorted(rec),
           "multiset_hash": f"{digest.multiset_hash(rec):016x}", "stats": stats,
           "wall_s": round(wall, 1)}
    print(json.dumps(job), flush=True)
    fx = {
        "workload": {"workload": "configs4-rank", "reads": args.reads, "read_len": args.read_len,
                     "coverage": args.coverage, "read_error": args.read_error,
                     "seed": args.seed, "k": args.k, "maxerate": p["max_erate"],
                     "minlength": args.minlength, "loaded_reads": args.hi,
                     "loaded_bases": total},
        "reference": {"binary": "oracle/_ref/oic_ref (reference overlapInCore built from its "
                                "sources): -h slice -r 1-hi, one hash batch",
                      "threads": args.threads, "hashbits": HASHBITS, "hashload": HASHLOAD,
                      "hashstrings": HASHSTRINGS, "hashdatalen": "the slice's bases + 1024",
                      "gen_s": round(t_gen, 1)},
        "jobs": [job],
    }
    with open(out, "w") as f:
        json.dump(fx, f, indent=1)
        f.write("\n")
    if args.workdir is None:
        import shutil
        shutil.rmtree(wd, ignore_errors=True)


if __name__ == "__main__":
    main()
