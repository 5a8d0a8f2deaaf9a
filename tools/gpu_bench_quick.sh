# 50k-read bench (2 steps) with per-stage breakdown and kernel stats
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bq.log 2>&1 || exit 1
grep -o '"value": [0-9.]*\|"breakdown_ms": {[^}]*}\|"launches": [0-9]*' gpurun_out/bq.log
