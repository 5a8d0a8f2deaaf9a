# configs4-rank with the sorted query windows' arrays kept across jobs (the warmup job pays
# their allocation): OVL_SQ = 1 (from the first batch), 2 (from the second), 0 (never)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd $R
export CANU_C4_READS_CACHE=/tmp/canu_c4_cache
timeout -k 10 300 python tools/c4_cache.py > gpurun_out/r04x_cache.log 2>&1 || { tail -5 gpurun_out/r04x_cache.log; exit 1; }
for m in 1 0 2 1; do
OVL_SQ=$m OVL_TIMING=1 timeout -k 10 300 python bench.py --workload configs4-rank --steps 1 --warmup 1 --no-cpu-baseline --no-side > gpurun_out/r04x_c4_sq$m.log 2>&1 || { echo "c4 sq$m failed"; tail -20 gpurun_out/r04x_c4_sq$m.log; exit 1; }
grep -a "sorted query\|alloc" gpurun_out/r04x_c4_sq$m.log | tail -4
python3 - $m <<'PY'
import json, sys
for l in open(f"gpurun_out/r04x_c4_sq{sys.argv[1]}.log"):
    if l.startswith("{"):
        d = json.loads(l)
        pr = d.get("probe_roofline") or {}
        print("OVL_SQ", sys.argv[1], d["value"], d["ms_per_step"], d["breakdown_ms"], "probe launches", pr.get("launches"), "avg ms", pr.get("avg_launch_ms"), "parity", d.get("parity"))
PY
done
rm -rf /tmp/canu_c4_cache
