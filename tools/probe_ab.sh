# WRITE_SIZE and duration of k_probe per library variant (canu_amd/lib/ab_*.so) on the
# seed-hit path (tools/probe_writes.py), one rocprofv3 PMC pass each.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
cd /tmp
for f in $R/canu_amd/lib/ab_*.so; do
  n=$(basename $f .so)
  CANU_OVL_LIB=$f timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/${n}_pw -o run -- python3 $R/tools/probe_writes.py > $R/gpurun_out/${n}_pw.log 2>&1 || exit 1
  python3 - $R/gpurun_out/${n}_pw $n <<'PY'
import csv, glob, sys
rows = []
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if r["Kernel_Name"].split("(")[0].endswith("k_probe"):
            rows.append((float(r["Counter_Value"]) * 1024 / 1e9,
                         (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6))
print(sys.argv[2], "k_probe WRITE_SIZE GB / ms:", [(round(a, 2), round(b, 2)) for a, b in rows])
PY
done
