# table slice sizing A/B (OVL_SLICE_Q: slots per slice = Q/4 x the largest fine bucket's
# distinct k-mers): the headline job's index + seed (tools/index_ab.py, 50k reads) and the
# configs4-rank job (the sorted-window probe streams the whole table per launch)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd $R
( for i in $(seq 1 40); do date > gpurun_out/r04_call34.heartbeat; sleep 50; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
for v in SL8 SL6 SL4 SL8; do
  echo -n "$v (50000 reads): "
  env CANU_OVL_LIB=$R/canu_amd/lib/ab_$v.so timeout -k 10 240 python tools/index_ab.py --reads 50000 --reps 1 --finds 3 2>&1 | grep -v amdgpu.ids | grep -v OVL_DEBUG | tail -1 || exit 1
done
export CANU_C4_READS_CACHE=/tmp/canu_c4_cache
timeout -k 10 300 python tools/c4_cache.py > gpurun_out/r04zn_cache.log 2>&1 || { tail -5 gpurun_out/r04zn_cache.log; exit 1; }
for v in SL8 SL6 SL4; do
CANU_OVL_LIB=$R/canu_amd/lib/ab_$v.so timeout -k 10 300 python bench.py --workload configs4-rank --steps 1 --warmup 1 --no-cpu-baseline --no-side > gpurun_out/r04zn_c4_$v.log 2>&1 || { echo "c4 $v failed"; tail -20 gpurun_out/r04zn_c4_$v.log; exit 1; }
python3 - $v <<'PY'
import json, sys
for l in open(f"gpurun_out/r04zn_c4_{sys.argv[1]}.log"):
    if l.startswith("{"):
        d = json.loads(l)
        pr = d.get("probe_roofline") or {}
        print(sys.argv[1], d["value"], d["ms_per_step"], d["breakdown_ms"], "records", d.get("overlaps_per_step"), "probe", pr.get("kernel"), pr.get("launches"), "avg ms", pr.get("avg_launch_ms"))
PY
done
rm -rf /tmp/canu_c4_cache
