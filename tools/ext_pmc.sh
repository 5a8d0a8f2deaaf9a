# k_extend stall profile on the 10k-read job: two PMC passes (8 SQ counters each, no tracing
# domains), each under its own time limit, summed over k_extend dispatches.
# usage: bash tools/ext_pmc.sh TAG   (CANU_OVL_LIB may name a variant library)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-ext}
export TMPDIR=/tmp
mkdir -p $R/gpurun_out
cd /tmp
timeout -k 10 -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS --output-format csv -d $R/gpurun_out/${TAG}_stall -o run -- python3 $R/tools/index_ab.py --reads 10000 --reps 1 --finds 1 > $R/gpurun_out/${TAG}_stall.log 2>&1 || { tail -5 $R/gpurun_out/${TAG}_stall.log; exit 1; }
python3 $R/tools/pmc_sum.py $R/gpurun_out/${TAG}_stall k_extend
timeout -k 10 -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAVES --output-format csv -d $R/gpurun_out/${TAG}_mix -o run -- python3 $R/tools/index_ab.py --reads 10000 --reps 1 --finds 1 > $R/gpurun_out/${TAG}_mix.log 2>&1 || { tail -5 $R/gpurun_out/${TAG}_mix.log; exit 1; }
python3 $R/tools/pmc_sum.py $R/gpurun_out/${TAG}_mix k_extend
