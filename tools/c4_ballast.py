#!/usr/bin/env python3
"""The driver's natural query chunking at a size the reference pins: the configs[4] 1/8-scale
rank-0 job (`-h 1-158209 -r 1-158209` of the 500k x 12 kb set, 14 hash batches; the
reference's own run is tests/golden/c4rank500k.json) run with most of the HBM held by a
ballast tensor, so the driver plans super-batches and query chunks from free HBM the way it
does at full size -- no OVL_SQ_CHUNK_WINDOWS / OVL_SB_WINDOWS caps.  For each target free
HBM: the driver's batch structure and whether records and counters equal the reference's.

    python tools/c4_ballast.py 110 90 75      (GB free when the job starts)
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    targets = [float(x) for x in sys.argv[1:]] or [90.0]
    from canu_amd.synth import synth_reads_parallel
    with open(os.path.join(ROOT, "tests", "golden", "c4rank500k.json")) as f:
        g = json.load(f)
    w, gj = g["workload"], g["jobs"][0]
    n, hi = w["reads"], gj["h"][1]
    t0 = time.time()
    rs = synth_reads_parallel(n, w["read_len"], int(n * w["read_len"] / w["coverage"]),
                              w["read_error"], seed=w["seed"], len_jitter=0.2,
                              read_range=(0, hi), workers=16)
    print(f"generated {hi} reads in {time.time() - t0:.1f} s", flush=True)
    import torch
    from canu_amd import digest
    from canu_amd.overlap_in_core import OicParameters, OverlapInCore
    hashed = int(rs.lengths.sum(dtype=np.uint64)) + hi
    P = OicParameters(Kmer_Len=w["k"], maxErate=float(np.float32(w["maxerate"])),
                      Min_Olap_Len=w["minlength"], bgnHashID=1, endHashID=hi, bgnRefID=1,
                      endRefID=hi, Hash_Mask_Bits=23, Max_Hash_Load=0.75,
                      Max_Hash_Strings=10_000_000, Max_Hash_Data_Len=hashed + 1024,
                      Num_PThreads=16).finalize()
    for tgt in targets:
        torch.cuda.empty_cache()
        oic = OverlapInCore(P, device=0)
        try:
            oic.load_reads(rs)
            free, _ = torch.cuda.mem_get_info(0)
            ballast = None
            if free > tgt * 1e9:
                ballast = torch.empty(int(free - tgt * 1e9), dtype=torch.uint8, device="cuda:0")
            t1 = time.time()
            try:
                nrec = oic.overlap_driver(store_num_reads=n)
            except Exception as e:                      # reported, the next target runs
                print(json.dumps({"free_gb_at_start": tgt, "error": str(e)[:300]}), flush=True)
                continue
            dt = time.time() - t1
            st = oic.stats()
            rec = oic.fetch(nrec)
            del ballast
            names = {"total": "total_overlaps", "kmer_hits_with_olap": "kmer_hits_with_olap",
                     "kmer_hits_without_olap": "kmer_hits_without_olap",
                     "multi": "multi_overlaps", "contained": "contained_overlaps",
                     "dovetail": "dovetail_overlaps"}
            ok = (rec.shape[0] == gj["records"] and
                  digest.sha256_sorted(rec) == gj["sha256_sorted"] and
                  f"{digest.multiset_hash(rec):016x}" == gj["multiset_hash"] and
                  all(int(st[m]) == int(gj["stats"][r]) for r, m in names.items()))
            print(json.dumps({"free_gb_at_start": tgt, "job_s": round(dt, 2),
                              "records": int(rec.shape[0]), "parity_ok": bool(ok),
                              **{k: int(st[k]) for k in ("hash_batches", "super_batches",
                                                         "query_chunks", "sq_declined",
                                                         "find_releases", "sq_resorted")}}),
                  flush=True)
        finally:
            oic.close()


if __name__ == "__main__":
    main()
