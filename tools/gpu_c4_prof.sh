# configs4-rank kernel stats (rocprofv3 --kernel-trace --stats, one timed step) and the
# probe filter's exactness test.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-c4prof}
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 300 python -u -m pytest tests/test_driver.py -m gpu -x -q --timeout 240 --timeout-method thread -k bloom > gpurun_out/${TAG}_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -n 1 gpurun_out/${TAG}_tests.log
export TMPDIR=/tmp
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${TAG}_kt -o run -- python3 $R/bench.py --workload configs4-rank --steps 1 --warmup 0 --no-cpu-baseline --no-parity > $R/gpurun_out/${TAG}_kt.log 2>&1 || { tail -20 $R/gpurun_out/${TAG}_kt.log; exit 1; }
find $R/gpurun_out/${TAG}_kt -name "*kernel_stats.csv" | head -1 | xargs head -14 | cut -d, -f1-4 | cut -c1-150
