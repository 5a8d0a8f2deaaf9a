# PMC passes over the 10k-read bench (one step).  Usage: bash tools/prof_pmc.sh <tag> [bench args]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-pmc}; shift
ARGS=${@:---reads 10000 --steps 1 --warmup 0 --no-cpu-baseline}
export TMPDIR=/tmp
mkdir -p $R/gpurun_out
cd /tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU -d $R/gpurun_out/${TAG}_1 -o run -- python3 $R/bench.py $ARGS > $R/gpurun_out/${TAG}_1.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_BRANCH -d $R/gpurun_out/${TAG}_2 -o run -- python3 $R/bench.py $ARGS > $R/gpurun_out/${TAG}_2.log 2>&1
