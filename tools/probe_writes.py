#!/usr/bin/env python3
"""Where k_probe's WRITE_SIZE comes from: the bench's read set, one index, then the seed-hit
path (k_probe + k_hitlist count pass, no extension) twice in a row.  Run under
`rocprofv3 --pmc WRITE_SIZE`: the first k_probe follows the index build (k_table's dirty
table lines), the second follows k_hitlist (which writes one word per unit).  Prints the
probe records' bytes (8 B per query window) for comparison.

    rocprofv3 --pmc WRITE_SIZE -d out -o run -- python3 tools/probe_writes.py [--reads 50000]
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--reads", type=int, default=50_000)
    ap.add_argument("--read-len", type=int, default=10_000)
    args = ap.parse_args()
    import torch
    from canu_amd.synth import random_genome, synth_reads
    from canu_amd.overlap_in_core import OicParameters, OverlapInCore
    n = args.reads
    gl = int(n * args.read_len / 25.0)
    g = random_genome(np.random.default_rng(1), gl)
    rs = synth_reads(n, args.read_len, gl, 0.015, seed=1, genome=g)
    P = OicParameters(Kmer_Len=22, maxErate=float(np.float32(0.06)), Min_Olap_Len=500).finalize()
    oic = OverlapInCore(P, device=0)
    oic.load_reads(rs)
    oic.build_hash_index(1, n)
    for _ in range(2):
        oic.seed_hits(1, n, fetch=False)
    torch.cuda.synchronize()
    windows = int(2 * np.maximum(rs.lengths.astype(np.int64) - 22 + 1, 1).sum())
    print(f"query windows {windows}, probe records {8 * windows} B", flush=True)
    oic.close()


if __name__ == "__main__":
    main()
