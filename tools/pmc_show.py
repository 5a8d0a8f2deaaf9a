import csv, glob, sys
from collections import defaultdict
tag = sys.argv[1]
tot = defaultdict(float)
for f in glob.glob(f"gpurun_out/{tag}_*/**/*counter_collection.csv", recursive=True):
    for row in csv.DictReader(open(f)):
        if "k_extend" in row["Kernel_Name"]:
            tot[row["Counter_Name"]] += float(row["Counter_Value"])
for k in sorted(tot):
    print(f"{k:28s} {tot[k]:.4g}")
