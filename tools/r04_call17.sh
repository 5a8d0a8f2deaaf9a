# chain occupancy A/B on the 50k-read job (CH6 = current 6 waves/SIMD with 47 spilled VGPRs,
# CH5 = 5 waves with 13, CH4 = 4 waves with none), then configs4-rank with the sorted query
# windows (OVL_SQ=1, top-24-bit sort) and without
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd $R
run() {
  echo -n "$1 ($3 reads): "
  env CANU_OVL_LIB=$R/canu_amd/lib/ab_$2.so timeout -k 10 240 python tools/index_ab.py --reads $3 --reps 1 --finds 3 2>&1 | grep -v amdgpu.ids | grep -v OVL_DEBUG | tail -1 || exit 1
}
for v in CH6 CH5 CH4 CH6 CH5 CH4; do run $v $v 50000 || exit 1; done
for m in 1 0; do
OVL_SQ=$m OVL_TIMING=1 timeout -k 10 300 python bench.py --workload configs4-rank --steps 1 --warmup 1 --no-cpu-baseline --no-side > gpurun_out/r04s_c4_sq$m.log 2>&1; echo "c4 sq$m rc $?"
grep -a "sorted query" gpurun_out/r04s_c4_sq$m.log | head -2
python3 - $m <<'PY'
import json, sys
for l in open(f"gpurun_out/r04s_c4_sq{sys.argv[1]}.log"):
    if l.startswith("{"):
        d = json.loads(l)
        pr = d.get("probe_roofline") or {}
        print("OVL_SQ", sys.argv[1], d["value"], d["ms_per_step"], d["breakdown_ms"], "probe launches", pr.get("launches"), "avg ms", pr.get("avg_launch_ms"))
PY
done
