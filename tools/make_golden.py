#!/usr/bin/env python3
"""Generate tests/golden/*.npz: small read sets and the ovOverlap records the REFERENCE
overlapInCore (oracle/_ref/oic_ref, compiled from /root/reference's own sources by
oracle/Makefile) produces for them.

The fixtures are data only: the inputs (bases, lengths, options) and the reference's
output records and counters.  tests/test_golden.py checks the C restatement (oracle/) and,
on the GPU box, the HIP path against them -- /root/reference is not needed there.

    python tools/make_golden.py            # needs oracle/_ref/oic_ref (built by `make -C oracle`)
    python tools/make_golden.py --only window   # (re)generate some cases only
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import oracle  # noqa: E402
from canu_amd.synth import synth_reads  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden")

# name -> (read-set kwargs, oracle params, reference extras)
CASES = {
    "basic": (dict(n_reads=60, read_len=2500, genome_len=20000, error_rate=0.02, seed=11),
              dict(kmer_len=22, max_erate=0.06, min_olap_len=200), {}),
    "ont_like": (dict(n_reads=40, read_len=6000, genome_len=30000, error_rate=0.015, seed=12,
                      len_jitter=0.3),
                 dict(kmer_len=22, max_erate=0.06, min_olap_len=500), {}),
    "high_erate": (dict(n_reads=50, read_len=2000, genome_len=15000, error_rate=0.05, seed=13),
                   dict(kmer_len=16, max_erate=0.144, min_olap_len=100), {}),
    "partial": (dict(n_reads=50, read_len=2000, genome_len=15000, error_rate=0.02, seed=14),
                dict(kmer_len=22, max_erate=0.06, min_olap_len=100, partial=1), {}),
    "multi": (dict(n_reads=50, read_len=2000, genome_len=12000, error_rate=0.02, seed=15,
                   n_repeats=6, repeat_len=400),
              dict(kmer_len=20, max_erate=0.06, min_olap_len=100, unique_olap_per_pair=0), {}),
    "ns_ragged": (dict(n_reads=60, read_len=1800, genome_len=12000, error_rate=0.02, seed=16,
                       len_jitter=0.6, n_rate=0.003, n_repeats=4, repeat_len=300),
                  dict(kmer_len=22, max_erate=0.06, min_olap_len=100), {}),
    "minkmers": (dict(n_reads=50, read_len=2000, genome_len=15000, error_rate=0.03, seed=17),
                 dict(kmer_len=22, max_erate=0.06, min_olap_len=100), {"minkmers": True}),
    "no_hopeless": (dict(n_reads=40, read_len=2000, genome_len=12000, error_rate=0.02, seed=18),
                    dict(kmer_len=22, max_erate=0.06, min_olap_len=100, use_hopeless_check=0),
                    {}),
    # -w: qualities + low-quality error bursts, so the window filter rejects overlaps
    "window": (dict(n_reads=60, read_len=2500, genome_len=15000, error_rate=0.015, seed=41,
                    with_quals=True, bursts=1),
               dict(kmer_len=20, max_erate=0.06, min_olap_len=100, use_window_filter=1), {}),
}


def main() -> None:
    only = sys.argv[sys.argv.index("--only") + 1].split(",") if "--only" in sys.argv else None
    if not oracle.reference_available():
        sys.exit("oracle/_ref/oic_ref is missing: run `make -C oracle` with /root/reference present")
    os.makedirs(OUT, exist_ok=True)
    index = {}
    if only:
        with open(os.path.join(OUT, "index.json")) as f:
            index = json.load(f)
    for name, (rkw, pkw, extra) in CASES.items():
        if only and name not in only:
            continue
        rs = synth_reads(**rkw)
        p = oracle.default_params(**pkw)
        skip = None
        if name == "ns_ragged":
            # a few k-mers of read 0 on the skip list (the -k file)
            r0 = rs.read(0).decode()
            k = p["kmer_len"]
            skip = [r0[i:i + k] for i in (100, 400, 900) if "N" not in r0[i:i + k]]
        minkmers = bool(extra.get("minkmers"))
        rec = oracle.run_reference(rs, p, threads=4, skip_kmers=skip, minkmers=minkmers)
        if minkmers:
            # main(): --minkmers sets Filter_By_Kmer_Count = int(floor(exp(-k e) (minlen-k+1)))
            import math
            fb = int(math.floor(math.exp(-1.0 * p["kmer_len"] * p["max_erate"]) *
                                (p["min_olap_len"] - p["kmer_len"] + 1)))
            p["filter_by_kmer_count"] = fb
        np.savez_compressed(
            os.path.join(OUT, f"{name}.npz"),
            bases=rs.bases, lengths=rs.lengths, first_iid=np.uint32(rs.first_iid),
            skip=np.array([s.encode() for s in (skip or [])], dtype="S64"),
            quals=(rs.quals if rs.quals is not None else np.zeros(0, np.uint8)),
            a=rec["a"], b=rec["b"], w0=rec["w0"], w1=rec["w1"])
        index[name] = {"params": {k: (v if k != "frag_olap_limit" else str(v))
                                  for k, v in p.items()},
                       "reads": rs.nreads, "bases": int(rs.total_bases()),
                       "records": int(len(rec)), "generator": rkw}
        print(f"{name}: {rs.nreads} reads, {len(rec)} reference records", flush=True)
    with open(os.path.join(OUT, "index.json"), "w") as f:
        json.dump(index, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
