# final sources: smoke(), the default bench line (traffic keyed to these sources for both
# workloads); then an A/B of k_probe_sorted variants on the configs4-rank job (libraries built
# from a scratch copy of the sources: Q0 = as committed, QP = next step's windows loaded
# ahead, QS = filter word and table entry loaded together, W8 = 8 windows per thread)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd $R
( for i in $(seq 1 40); do date > gpurun_out/r04_call27.heartbeat; sleep 50; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r04zd_smoke.log 2>&1 || { tail -20 gpurun_out/r04zd_smoke.log; exit 1; }
tail -2 gpurun_out/r04zd_smoke.log
timeout -k 10 700 python bench.py > gpurun_out/r04zd_bench.log 2>&1 || { tail -30 gpurun_out/r04zd_bench.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r04zd_bench.log | cut -c1-300
export CANU_C4_READS_CACHE=/tmp/canu_c4_cache
timeout -k 10 300 python tools/c4_cache.py > gpurun_out/r04ze_cache.log 2>&1 || { tail -5 gpurun_out/r04ze_cache.log; exit 1; }
for v in Q0 QP QS QPS QP8 QPS8 Q0; do
CANU_OVL_LIB=$R/canu_amd/lib/ab_$v.so timeout -k 10 300 python bench.py --workload configs4-rank --steps 1 --warmup 1 --no-cpu-baseline --no-side > gpurun_out/r04ze_c4_$v.log 2>&1 || { echo "c4 $v failed"; tail -20 gpurun_out/r04ze_c4_$v.log; exit 1; }
python3 - $v <<'PY'
import json, sys
for l in open(f"gpurun_out/r04ze_c4_{sys.argv[1]}.log"):
    if l.startswith("{"):
        d = json.loads(l)
        pr = d.get("probe_roofline") or {}
        print(sys.argv[1], d["value"], d["ms_per_step"], d["breakdown_ms"], "records", d.get("overlaps_per_step"), "probe launches", pr.get("launches"), "avg ms", pr.get("avg_launch_ms"))
PY
done
rm -rf /tmp/canu_c4_cache
