# Index-build profile: kernel trace and HBM traffic (separate PMC passes) of tools/index_ab.py
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-idx}
mkdir -p $R/gpurun_out
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${TAG}_kt -o run -- python3 $R/tools/index_ab.py --reps 3 > $R/gpurun_out/${TAG}_kt.log 2>&1 || exit 1
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $c --output-format csv -d $R/gpurun_out/${TAG}_$c -o run -- python3 $R/tools/index_ab.py --reps 1 > $R/gpurun_out/${TAG}_$c.log 2>&1 || exit 1
done
find $R/gpurun_out/${TAG}_kt -name "*kernel_stats.csv" | head -1 | xargs head -12 | cut -c1-160
