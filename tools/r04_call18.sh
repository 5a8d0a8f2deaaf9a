# rocprofv3 evidence on the final sources: kernel trace + FETCH_SIZE / WRITE_SIZE / issue PMC
# passes of one bench step for the headline workload (TAG1) and the configs4-rank job (TAG2,
# its read set generated once outside the profiler: tools/c4_cache.py)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG1=${1:-r04t}; TAG2=${2:-r04u}
mkdir -p $R/gpurun_out
cd $R
( for i in $(seq 1 40); do date > gpurun_out/r04_call18.heartbeat; sleep 50; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
export CANU_C4_READS_CACHE=/tmp/canu_c4_cache
timeout -k 10 300 python tools/c4_cache.py > gpurun_out/${TAG2}_cache.log 2>&1 || { tail -5 gpurun_out/${TAG2}_cache.log; exit 1; }
cat gpurun_out/${TAG2}_cache.log
if [ "$TAG1" != "-" ]; then
bash tools/prof_traffic.sh $TAG1 || { echo "configs2 passes failed"; exit 1; }
echo "configs2 passes done"
fi
bash tools/prof_traffic.sh $TAG2 --workload configs4-rank --steps 1 --warmup 0 --no-cpu-baseline --no-side || { echo "configs4 passes failed"; tail -5 gpurun_out/${TAG2}_*.log; exit 1; }
echo "configs4 passes done"
rm -rf /tmp/canu_c4_cache
