# rocprofv3 --kernel-trace --stats of one full-size configs[4] rank job (4M x 12 kb plan,
# --rank-job J): the job's reads cached first (tools/c4_cache.py: no worker pool is forked
# under the profiler), then one timed job under the profiler.
# usage: bash tools/c4_rank_prof.sh TAG J
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-c4rprof}; J=${2:-1}
mkdir -p $R/gpurun_out
export CANU_C4_READS_CACHE=/tmp/canu_c4_cache TMPDIR=/tmp
mkdir -p $CANU_C4_READS_CACHE
cd $R
timeout -k 10 300 python tools/c4_cache.py --reads 4000000 --rank-job $J > gpurun_out/${TAG}_cache.log 2>&1 || { tail -5 gpurun_out/${TAG}_cache.log; exit 1; }
cd /tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${TAG}_kt -o run -- python3 $R/bench.py --workload configs4-rank --reads 4000000 --rank-job $J --steps 1 --warmup 0 --no-cpu-baseline --no-parity > $R/gpurun_out/${TAG}_kt.json 2> $R/gpurun_out/${TAG}_kt.log || { tail -20 $R/gpurun_out/${TAG}_kt.log; exit 1; }
f=$(find $R/gpurun_out/${TAG}_kt -name "*kernel_stats.csv" | head -1)
cp $f $R/gpurun_out/${TAG}_kernel_stats.csv
head -24 $f | cut -d, -f1-4 | cut -c1-150
