# rocprofv3 evidence on the final sources: kernel trace + FETCH_SIZE / WRITE_SIZE / issue PMC
# passes of one bench step, for the headline workload (r04p) and the configs4-rank job (r04q)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd $R
# progress marks for the long PMC passes (each pass has its own time limit)
( for i in $(seq 1 40); do date > gpurun_out/r04_call16.heartbeat; sleep 50; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
bash tools/prof_traffic.sh r04p || { echo "configs2 passes failed"; exit 1; }
echo "configs2 passes done"
bash tools/prof_traffic.sh r04q --workload configs4-rank --steps 1 --warmup 0 --no-cpu-baseline --no-side || { echo "configs4 passes failed"; exit 1; }
echo "configs4 passes done"
ls gpurun_out | grep -E "r04[pq]_" | head -20
