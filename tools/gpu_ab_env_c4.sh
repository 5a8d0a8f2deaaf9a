# configs4-rank (one timed step) under two settings of one environment knob, twice each in
# alternating order: bash tools/gpu_ab_env_c4.sh VAR VALUE_A VALUE_B
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
for pass in 1 2; do
  for v in $2 $3; do
    env $1=$v timeout -k 10 400 python $R/bench.py --workload configs4-rank --steps 1 --warmup 1 --no-cpu-baseline --no-parity > $R/gpurun_out/abenv_c4_$v.log 2>&1 || { tail -20 $R/gpurun_out/abenv_c4_$v.log; exit 1; }
    echo "$pass $1=$v $(grep -o '"ms_per_step": [0-9.]*\|"overlaps_per_step": [0-9]*\|"breakdown_ms": {[^}]*}' $R/gpurun_out/abenv_c4_$v.log | tr '\n' ' ')"
  done
done
