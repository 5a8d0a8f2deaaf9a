#!/usr/bin/env python3
"""Sum rocprofv3 counter_collection.csv values per counter for kernels whose name contains
a substring (default k_extend):  python tools/pmc_sum.py <rocprofv3 -d dir> [substring]"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main():
    d = sys.argv[1]
    sub = sys.argv[2] if len(sys.argv) > 2 else "k_extend"
    tot, disp = defaultdict(float), set()
    for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(path)):
            if sub in row["Kernel_Name"]:
                tot[row["Counter_Name"]] += float(row["Counter_Value"])
                disp.add(row["Dispatch_Id"])
    print(os.path.basename(d.rstrip("/")), f"dispatches={len(disp)}",
          " ".join(f"{k}={v:.4g}" for k, v in sorted(tot.items())))


if __name__ == "__main__":
    main()
