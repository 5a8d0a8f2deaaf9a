#!/usr/bin/env python3
"""profiles/traffic_mhap.json from tools/mhap_pmc.sh's rocprofv3 passes on bench_mhap.py's
configs[3] job (one step): per MHAP kernel, per launch, the VALU / SALU wave-instructions
(issue pass) and the HBM bytes (FETCH_SIZE pass x the coalesced-read correction 2, the
guide's half undercount, + the WRITE_SIZE pass; both in KiB), keyed by the workload and a hash
of the MHAP sources, so that bench_mhap.py uses them only for the same job and code.
usage: python tools/pmc_mhap.py TAG [out.json]     (reads gpurun_out/TAG_{issue,fetch,write})"""
import csv
import glob
import hashlib
import json
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNELS = ("k_mh_minhash", "k_mh_bitslice", "k_mh_keys", "k_mh_ordered", "k_mh_candidates",
           "k_mh_compare")


def mhap_source_hash() -> str:
    h = hashlib.sha256()
    for rel in ("canu_amd/csrc/mhap.hip", "include/canu_mhap.h"):
        with open(os.path.join(ROOT, rel), "rb") as f:
            h.update(rel.encode() + b"\0" + f.read())
    return h.hexdigest()[:16]


def default_workload() -> dict:
    """bench_mhap.py's defaults (its workload_key)."""
    sys.path.insert(0, ROOT)
    import bench_mhap
    return bench_mhap.workload_key(bench_mhap.parse_args([]))


def sums(d):
    tot = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(path)):
            for k in KERNELS:
                if k in row["Kernel_Name"]:
                    tot[k][row["Counter_Name"]] += float(row["Counter_Value"])
                    disp[k].add(row["Dispatch_Id"])
    return tot, disp


def main():
    tag = sys.argv[1]
    out = sys.argv[2] if len(sys.argv) > 2 else os.path.join(ROOT, "profiles", "traffic_mhap.json")
    base = os.path.join(ROOT, "gpurun_out", tag)
    iss, di = sums(base + "_issue")
    fet, _ = sums(base + "_fetch")
    wri, _ = sums(base + "_write")
    res = {"_method": {"tag": tag, "src_sha": mhap_source_hash(), "workload": default_workload(),
                       "hbm_bytes": "(2 * FETCH_SIZE + WRITE_SIZE) KiB per launch",
                       "issue": "SQ_INSTS_VALU / SQ_INSTS_SALU wave-instructions per launch"}}
    for k in KERNELS:
        n = len(di.get(k, ()))
        if not n:
            continue
        res[k] = {"launches_per_step": n,
                  "valu_insts": iss[k].get("SQ_INSTS_VALU", 0.0) / n,
                  "salu_insts": iss[k].get("SQ_INSTS_SALU", 0.0) / n,
                  "wait_inst_any_frac": iss[k].get("SQ_WAIT_INST_ANY", 0.0) /
                  max(iss[k].get("SQ_WAVE_CYCLES", 0.0), 1.0),
                  "hbm_bytes_per_launch": (2.0 * fet[k].get("FETCH_SIZE", 0.0) +
                                           wri[k].get("WRITE_SIZE", 0.0)) * 1024.0 / n}
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res)[:800])


if __name__ == "__main__":
    main()
