set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-pmc}
ARGS="--reads 10000 --steps 1 --warmup 0 --no-cpu-baseline"
export TMPDIR=/tmp
mkdir -p $R/gpurun_out
cd /tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU --output-format csv -d $R/gpurun_out/${TAG}_1 -o run -- python3 $R/bench.py $ARGS > $R/gpurun_out/${TAG}_1.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_SCA SQ_IFETCH SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_BRANCH --output-format csv -d $R/gpurun_out/${TAG}_2 -o run -- python3 $R/bench.py $ARGS > $R/gpurun_out/${TAG}_2.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc SQ_INST_CYCLES_SALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC SQ_INSTS_SMEM SQ_ACTIVE_INST_EXP SQ_INST_LEVEL_LDS SQ_ACTIVE_INST_FLAT SQ_INSTS_FLAT --output-format csv -d $R/gpurun_out/${TAG}_3 -o run -- python3 $R/bench.py $ARGS > $R/gpurun_out/${TAG}_3.log 2>&1
