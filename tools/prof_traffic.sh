# rocprofv3 evidence for the bench's default workload (one step):
#   <tag>_kt    --kernel-trace --stats  (per-kernel durations)
#   <tag>_fetch --pmc FETCH_SIZE        (separate passes, no tracing domains with --pmc)
#   <tag>_write --pmc WRITE_SIZE
#   <tag>_issue --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES GRBM_GUI_ACTIVE
# then tools/pmc_traffic.py writes profiles/traffic.json + profiles/<tag>_*.csv summaries.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r01}; shift
ARGS=${@:---steps 1 --warmup 0 --no-cpu-baseline --no-shard-timing --no-seed-only --no-side}
export TMPDIR=/tmp
mkdir -p $R/gpurun_out
cd /tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${TAG}_kt -o run -- python3 $R/bench.py $ARGS > $R/gpurun_out/${TAG}_kt.log 2>&1 && \
timeout -k 10 500 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/${TAG}_fetch -o run -- python3 $R/bench.py $ARGS > $R/gpurun_out/${TAG}_fetch.log 2>&1 && \
timeout -k 10 500 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/${TAG}_write -o run -- python3 $R/bench.py $ARGS > $R/gpurun_out/${TAG}_write.log 2>&1 && \
timeout -k 10 500 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/${TAG}_issue -o run -- python3 $R/bench.py $ARGS > $R/gpurun_out/${TAG}_issue.log 2>&1
