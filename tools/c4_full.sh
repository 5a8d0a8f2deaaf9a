# configs[4] at its real size on one GPU: one rank job of the 8-GPU plan for 4M x 12 kb ONT
# reads (dist.c4_plan: the blocks cut on DRIVER6, the driver's own packing replayed per job;
# CANU_C4_PLAN=r02 gives the rehearsal-cost plan, rank 0 -h 1-1145091), canu's --hashbits 23 --hashload 0.75, the job's reads generated before GPU
# init.  One timed job (no warm-up: its first-use allocations are inside it, OVL_TIMING shows
# them), per-search timing lines, the HBM high-water from rocm-smi beside it, and the rank's
# .ovb + .counts written after the timed region (bench.py --ovb-out, timed).
# usage: bash tools/c4_full.sh TAG [rank_job] [extra bench.py args]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-c4full}
JOB=${2:-0}
shift 2 2>/dev/null
mkdir -p $R/gpurun_out
( while sleep 5; do rocm-smi --showmeminfo vram --json 2>/dev/null | tr -d '\n' >> $R/gpurun_out/${TAG}_vram.jsonl; echo >> $R/gpurun_out/${TAG}_vram.jsonl; done ) &
SMI=$!
OVL_TIMING=1 timeout -k 10 1000 python -u $R/bench.py --workload configs4-rank --reads 4000000 \
  --rank-job $JOB --steps 1 --warmup 0 --no-parity --ovb-out /tmp/c4ovb_$JOB "$@" > $R/gpurun_out/${TAG}.json \
  2> $R/gpurun_out/${TAG}.log
rc=$?
kill $SMI
tail -c 3000 $R/gpurun_out/${TAG}.json
exit $rc
