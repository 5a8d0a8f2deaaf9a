# configs4-rank with the sorted query windows (top-24-bit sort for long runs) and without;
# the driver / configs4-digest GPU tests (both sort paths)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd $R
for m in 2 0; do
OVL_SQ=$m OVL_TIMING=1 timeout -k 10 400 python bench.py --workload configs4-rank --steps 1 --warmup 1 --no-cpu-baseline --no-side > gpurun_out/r04o_c4_sq$m.log 2>&1; echo "c4 sq$m rc $?"
grep -a "sorted query" gpurun_out/r04o_c4_sq$m.log | head -2
python3 - $m <<'PY'
import json, sys
for l in open(f"gpurun_out/r04o_c4_sq{sys.argv[1]}.log"):
    if l.startswith("{"):
        d = json.loads(l)
        pr = d.get("probe_roofline") or {}
        print("OVL_SQ", sys.argv[1], d["value"], d["ms_per_step"], d["breakdown_ms"], "probe launches", pr.get("launches"), "avg ms", pr.get("avg_launch_ms"))
PY
done
timeout -k 10 600 python -u -m pytest tests/test_driver.py tests/test_gpu_c4_digest.py -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r04o_tests.log 2>&1
grep -E "PASSED|FAILED|passed|failed" gpurun_out/r04o_tests.log | tail -20
