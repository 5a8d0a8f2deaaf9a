# configs4-rank: a load-cut batch's index cut from its prefix's (OVL_CUT_FILTER=1, default) vs
# built again (0), with the default sorted-window rule; then the GPU suite on these sources
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd $R
( for i in $(seq 1 40); do date > gpurun_out/r04_call25.heartbeat; sleep 50; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
export CANU_C4_READS_CACHE=/tmp/canu_c4_cache
timeout -k 10 300 python tools/c4_cache.py > gpurun_out/r04za_cache.log 2>&1 || { tail -5 gpurun_out/r04za_cache.log; exit 1; }
for v in 1 0 1; do
OVL_CUT_FILTER=$v OVL_TIMING=1 timeout -k 10 300 python bench.py --workload configs4-rank --steps 1 --warmup 1 --no-cpu-baseline --no-side > gpurun_out/r04za_c4_cut$v.log 2>&1 || { echo "c4 cut$v failed"; tail -20 gpurun_out/r04za_c4_cut$v.log; exit 1; }
python3 - $v <<'PY'
import json, sys
for l in open(f"gpurun_out/r04za_c4_cut{sys.argv[1]}.log"):
    if l.startswith("{"):
        d = json.loads(l)
        pr = d.get("probe_roofline") or {}
        print("CUT", sys.argv[1], d["value"], d["ms_per_step"], d["breakdown_ms"], "records", d.get("overlaps_per_step"), "probe launches", pr.get("launches"), "avg ms", pr.get("avg_launch_ms"))
PY
done
rm -rf /tmp/canu_c4_cache
unset CANU_C4_READS_CACHE
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r04za_gpu_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r04za_gpu_tests.log
grep -E "FAILED|ERROR" gpurun_out/r04za_gpu_tests.log | head -20
exit $rc
