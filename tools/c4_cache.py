#!/usr/bin/env python3
"""Write bench.py's configs4-rank read set (one GPU: the reads of the --rank-job's job) to the
cache directory CANU_C4_READS_CACHE names, so that runs under rocprofv3 load it instead of
generating it with a worker pool (a pool forked by a process the profiler has attached to the
GPU).  usage: CANU_C4_READS_CACHE=dir python tools/c4_cache.py [bench.py configs4-rank options]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def main():
    assert os.environ.get("CANU_C4_READS_CACHE"), "set CANU_C4_READS_CACHE"
    a = bench.parse_args(["--workload", "configs4-rank"] + sys.argv[1:])
    job = bench.Configs4Rank(a, 0, 1, None)
    job.generate()                       # writes the cache (or finds it there)
    print("cached", job._part.lengths.shape[0], "reads,", int(job._part.lengths.sum()), "bases")


if __name__ == "__main__":
    main()
