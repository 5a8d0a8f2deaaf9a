# configs4-rank: sorted query windows with the batch's Bloom filter in front of the table
# (OVL_SQ_BLOOM=1) and without, both from the first batch; the auto default (OVL_SQ=3); then the
# GPU suite on these sources
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd $R
( for i in $(seq 1 40); do date > gpurun_out/r04_call23.heartbeat; sleep 50; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
export CANU_C4_READS_CACHE=/tmp/canu_c4_cache
timeout -k 10 300 python tools/c4_cache.py > gpurun_out/r04y_cache.log 2>&1 || { tail -5 gpurun_out/r04y_cache.log; exit 1; }
for v in "1 1" "1 0" "3 1"; do
set -- $v
OVL_SQ=$1 OVL_SQ_BLOOM=$2 OVL_TIMING=1 timeout -k 10 300 python bench.py --workload configs4-rank --steps 1 --warmup 1 --no-cpu-baseline --no-side > gpurun_out/r04y_c4_sq$1b$2.log 2>&1 || { echo "c4 sq$1 b$2 failed"; tail -20 gpurun_out/r04y_c4_sq$1b$2.log; exit 1; }
python3 - $1 $2 <<'PY'
import json, sys
for l in open(f"gpurun_out/r04y_c4_sq{sys.argv[1]}b{sys.argv[2]}.log"):
    if l.startswith("{"):
        d = json.loads(l)
        pr = d.get("probe_roofline") or {}
        print("OVL_SQ", sys.argv[1], "BLOOM", sys.argv[2], d["value"], d["ms_per_step"], d["breakdown_ms"], "probe launches", pr.get("launches"), "avg ms", pr.get("avg_launch_ms"))
PY
done
rm -rf /tmp/canu_c4_cache
unset CANU_C4_READS_CACHE
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r04y_gpu_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r04y_gpu_tests.log
grep -E "FAILED|ERROR" gpurun_out/r04y_gpu_tests.log | head -20
exit $rc
