# configs4-rank with the sorted query windows (2^29-window runs) and without, then the GPU
# suite and the default bench line
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd $R
for m in 2 0; do
OVL_SQ=$m OVL_TIMING=1 timeout -k 10 400 python bench.py --workload configs4-rank --steps 1 --warmup 1 --no-cpu-baseline --no-side > gpurun_out/r04m_c4_sq$m.log 2>&1; echo "c4 sq$m rc $?"
grep -a "sorted query" gpurun_out/r04m_c4_sq$m.log | head -1
python3 - $m <<'PY'
import json, sys
for l in open(f"gpurun_out/r04m_c4_sq{sys.argv[1]}.log"):
    if l.startswith("{"):
        d = json.loads(l)
        pr = d.get("probe_roofline") or {}
        print("OVL_SQ", sys.argv[1], d["value"], d["ms_per_step"], d["breakdown_ms"], "probe launches", pr.get("launches"), "avg ms", pr.get("avg_launch_ms"))
PY
done
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r04m_gpu_tests.log 2>&1; rc=$?
grep -E "FAILED|passed|failed" gpurun_out/r04m_gpu_tests.log | tail -12
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 700 python bench.py > gpurun_out/r04m_bench.log 2>&1 || { tail -30 gpurun_out/r04m_bench.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r04m_bench.log | cut -c1-400
