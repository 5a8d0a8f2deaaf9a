#!/usr/bin/env python3
"""Write bench.py's configs4-rank read set (one rank, default sizes or --reads N) to the cache
directory CANU_C4_READS_CACHE names, so that runs under rocprofv3 (tools/prof_traffic.sh)
load it instead of generating it with a worker pool.  usage: CANU_C4_READS_CACHE=dir
python tools/c4_cache.py [bench.py configs4-rank options]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

import bench  # noqa: E402
from canu_amd.synth import synth_reads_parallel  # noqa: E402


def main():
    a = bench.parse_args(["--workload", "configs4-rank"] + sys.argv[1:])
    cache = os.environ["CANU_C4_READS_CACHE"]
    n = a.reads
    key = f"c4_{n}_{a.read_len}_{a.coverage}_{a.read_error}_{a.seed}"
    if os.path.exists(os.path.join(cache, key + "_lengths.npy")):
        print("cached", key)
        return
    part = synth_reads_parallel(n, a.read_len, int(n * a.read_len / a.coverage), a.read_error,
                                seed=a.seed, len_jitter=0.2, read_range=(0, n), workers=16)
    os.makedirs(cache, exist_ok=True)
    np.save(os.path.join(cache, key + "_bases.npy"), part.bases)
    np.save(os.path.join(cache, key + "_lengths.npy"), part.lengths)
    print("wrote", key, part.total_bases(), "bases")


if __name__ == "__main__":
    main()
