# chain A/B on the 50k-read job (X0 = current: old row loop, run replay with lane-exchange
# run bits; N0 = without run replay; SB0 = + batched staging loads; RP0 = phase profile), then
# the configs4-rank job with the sorted query windows (ILP probe) and without (OVL_SQ=0)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd $R
run() {
  echo -n "$1 ($3 reads): "
  env CANU_OVL_LIB=$R/canu_amd/lib/ab_$2.so timeout -k 10 240 python tools/index_ab.py --reads $3 --reps 1 --finds 3 2>&1 | grep -v amdgpu.ids | grep -v OVL_DEBUG | tail -2 || exit 1
}
for v in X0 N0 SB0 X0 N0 SB0 RP0; do run $v $v 50000 || exit 1; done
for m in 2 0; do
OVL_SQ=$m timeout -k 10 400 python bench.py --workload configs4-rank --steps 1 --warmup 1 --no-cpu-baseline --no-side > gpurun_out/r04l_c4_sq$m.log 2>&1; echo "c4 sq$m rc $?"
python3 - $m <<'PY'
import json, sys
for l in open(f"gpurun_out/r04l_c4_sq{sys.argv[1]}.log"):
    if l.startswith("{"):
        d = json.loads(l)
        pr = d.get("probe_roofline") or {}
        print("OVL_SQ", sys.argv[1], d["value"], d["ms_per_step"], d["breakdown_ms"], "probe launches", pr.get("launches"), "avg ms", pr.get("avg_launch_ms"))
PY
done
