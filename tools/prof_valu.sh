set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-valu}
ARGS="--reads 10000 --steps 1 --warmup 0 --no-cpu-baseline"
export TMPDIR=/tmp
mkdir -p $R/gpurun_out
cd /tmp
timeout -k 10 300 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_BUSY_CU_CYCLES SQ_CYCLES SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU2 SQ_INSTS_VALU SQ_INSTS_VALU_INT64 SQ_WAVE_CYCLES --output-format csv -d $R/gpurun_out/${TAG}_1 -o run -- python3 $R/bench.py $ARGS > $R/gpurun_out/${TAG}_1.log 2>&1
