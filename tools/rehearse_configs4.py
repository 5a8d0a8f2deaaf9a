#!/usr/bin/env python3
"""A scaled rehearsal of BASELINE configs[4] (4M x 12 kb ONT reads, 8 x MI355X) on one GPU.

One rank of configs[4] holds the whole read store and runs OverlapDriver over its share of
the hash blocks: every hash batch of its -h range is built and searched by the -r reads.
This script runs that loop -- ovl_overlap_driver, the reference's batch semantics
(overlapInCore.C:217-287) with canu-style --hashbits / --hashload / --hashstrings /
--hashdatalen limits -- on a 1/8-size read set (default 500k x 12 kb at 15x), and reports
per-phase times, the hash batches taken, and the device memory the library holds (free HBM
before the load minus free HBM after the job: the library's buffers only grow, so this is
its high-water mark).  The reference asserts when the whole -h range holds more bases than
--hashdatalen (Build_Hash_Index.C:521-523), so batches are cut by the hash load
(--hashbits / --hashload) and --hashstrings.  DESIGN.md's configs[4] memory plan extrapolates from these numbers.

    python tools/rehearse_configs4.py [--reads 500000] [--read-len 12000] [--coverage 15]
                                      [--hashbits 26] [--hashdatalen 8000000000]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


_G = {}


def _part(lo_hi):
    from canu_amd.synth import synth_reads
    g = _G
    return synth_reads(g["n"], g["len"], g["glen"], g["err"], seed=g["seed"], len_jitter=0.2,
                       genome=g["genome"], read_range=lo_hi)


def _generate(n, read_len, genome_len, err, seed, workers=12):
    """synth_reads' read i depends only on (seed, i): slices are generated in parallel
    (fork-shared genome) and concatenated -- the same reads as one synth_reads call."""
    import multiprocessing as mp
    from canu_amd.synth import ReadSet, random_genome
    _G.update(n=n, len=read_len, glen=genome_len, err=err, seed=seed,
              genome=random_genome(np.random.default_rng(seed), genome_len))
    cuts = [(n * i // 64, n * (i + 1) // 64) for i in range(64)]
    with mp.get_context("fork").Pool(workers) as pool:
        parts = pool.map(_part, cuts)
    lengths = np.concatenate([p.lengths for p in parts])
    offsets = np.zeros(n, dtype=np.uint64)
    offsets[1:] = np.cumsum(lengths[:-1], dtype=np.uint64)
    return ReadSet(bases=np.concatenate([p.bases for p in parts]), offsets=offsets,
                   lengths=lengths, quals=None, first_iid=1,
                   starts=np.concatenate([p.starts for p in parts]),
                   strands=np.concatenate([p.strands for p in parts]))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--reads", type=int, default=500_000)
    ap.add_argument("--read-len", type=int, default=12_000)
    ap.add_argument("--coverage", type=float, default=15.0)
    ap.add_argument("--read-error", type=float, default=0.015)
    ap.add_argument("--hashbits", type=int, default=26)
    ap.add_argument("--hashload", type=float, default=0.75)
    ap.add_argument("--hashstrings", type=int, default=1_000_000)
    ap.add_argument("--hashdatalen", type=int, default=8_000_000_000)
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--seed", type=int, default=5)
    args = ap.parse_args()

    import torch
    from canu_amd.overlap_in_core import OicParameters, OverlapInCore

    n = args.reads
    genome_len = int(n * args.read_len / args.coverage)
    t0 = time.time()
    rs = _generate(n, args.read_len, genome_len, args.read_error, args.seed)
    gen_s = time.time() - t0
    print(f"generated {n} reads, {rs.total_bases() / 1e9:.2f} Gbp in {gen_s:.0f} s", flush=True)

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    torch.cuda.synchronize()
    free0, total = torch.cuda.mem_get_info()
    bases = torch.from_numpy(rs.bases).to(dev)
    d_offsets = torch.from_numpy(rs.offsets.view(np.int64)).to(dev)
    torch.cuda.synchronize()
    free_staged, _ = torch.cuda.mem_get_info()

    P = OicParameters(Kmer_Len=22, maxErate=float(np.float32(0.06)), Min_Olap_Len=500,
                      Hash_Mask_Bits=args.hashbits, Max_Hash_Load=args.hashload,
                      Max_Hash_Strings=args.hashstrings, Max_Hash_Data_Len=args.hashdatalen,
                      Num_PThreads=args.threads).finalize()
    oic = OverlapInCore(P, device=0)
    oic.load_reads_device(1, bases.data_ptr(), d_offsets.data_ptr(), rs.lengths)
    torch.cuda.synchronize()
    free_loaded, _ = torch.cuda.mem_get_info()
    t1 = time.perf_counter()
    nrec = oic.overlap_driver(store_num_reads=n)
    torch.cuda.synchronize()
    job_s = time.perf_counter() - t1
    free_end, _ = torch.cuda.mem_get_info()
    st = oic.stats()
    oic.close()

    gib = float(1 << 30)
    out = {
        "workload": f"configs[4] rehearsal: {n} x {args.read_len} bp at {args.coverage}x "
                    f"(1/{4_000_000 // n} of configs[4]'s reads), one GPU, OverlapDriver "
                    "hash batches",
        "gbp": round(rs.total_bases() / 1e9, 3),
        "limits": {"hashbits": args.hashbits, "hashload": args.hashload,
                   "hashstrings": args.hashstrings, "hashdatalen": args.hashdatalen},
        "hash_batches": st["hash_batches"],
        "overlaps": nrec,
        "job_s": round(job_s, 2),
        "overlaps_per_s": round(nrec / job_s, 1),
        "ms": {"index": round(st["ms_index"], 1), "seed": round(st["ms_seed"], 1),
               "extend": round(st["ms_extend"], 1)},
        "seed_hits": st["seed_hits"], "pairs": st["pairs"],
        "staged_pairs": st["staged_pairs"], "long_pairs": st["long_pairs"],
        "generic_pairs": st["generic_pairs"],
        "extra": {k: st[k] for k in ("chain_retries", "multi_pass_units", "ms_probe_kernel",
                                     "ext_waves", "generic_waves", "stage_len",
                                     "long_stage_len", "extend_launches") if k in st},
        "hbm_gib": {"total": round(total / gib, 1),
                    "raw_bases_staged": round((free0 - free_staged) / gib, 2),
                    "library_store": round((free_staged - free_loaded) / gib, 2),
                    "library_job_high_water": round((free_loaded - free_end) / gib, 2)},
        "generate_s": round(gen_s, 1),
    }
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
