#!/usr/bin/env python3
"""Turn the calib_traffic PMC passes into profiles/calib_traffic.json: for each access
pattern, the bytes FETCH_SIZE / WRITE_SIZE report per byte actually moved (read_factor /
write_factor) -- tools/pmc_traffic.py divides each kernel's counters by the factor of its
dominant pattern instead of assuming the streaming-read x2 everywhere.

    python tools/calib_traffic.py <dir with calib.log, calib_fetch/, calib_write/>
"""
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def counter(d, name):
    """Per kernel, the largest dispatch value of `name` (the measured launch; the warm-up
    launch of each kernel moves 1/64 of the bytes)."""
    out = {}
    for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(path)):
            if row["Counter_Name"] != name:
                continue
            k = row["Kernel_Name"].split("(")[0].strip()
            out[k] = max(out.get(k, 0.0), float(row["Counter_Value"]))
    return out


def main():
    d = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "gpurun_out")
    known = {}
    for line in open(os.path.join(d, "calib.log")):
        if line.startswith("CALIB "):
            f = line.split()
            known[f[1]] = {"read_bytes": int(f[3]), "write_bytes": int(f[5])}
    fetch = counter(os.path.join(d, "calib_fetch"), "FETCH_SIZE")
    write = counter(os.path.join(d, "calib_write"), "WRITE_SIZE")
    res = {}
    for k, kb in known.items():
        r = {"known_read_bytes": kb["read_bytes"], "known_write_bytes": kb["write_bytes"],
             "fetch_size_bytes": fetch.get(k, 0.0) * 1024, "write_size_bytes": write.get(k, 0.0) * 1024}
        if kb["read_bytes"]:
            r["read_factor"] = round(r["fetch_size_bytes"] / kb["read_bytes"], 4)
        if kb["write_bytes"]:
            r["write_factor"] = round(r["write_size_bytes"] / kb["write_bytes"], 4)
        res[k] = r
    out = os.path.join(ROOT, "profiles", "calib_traffic.json")
    with open(out, "w") as f:
        json.dump(res, f, indent=1, sort_keys=True)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
