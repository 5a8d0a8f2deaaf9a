# k_extend instruction-fetch and stall profile on the 10k-read job (tools/index_ab.py): PMC
# passes of <= 8 SQ-block counters each, no tracing domains, each under its own time limit,
# summed over k_extend dispatches by tools/pmc_sum.py.
#   pass 1 (fetch):  instruction fetches and the SQC instruction cache
#   pass 2 (stall):  wait / active cycles beside the instruction mix
#   pass 3 (vmem):   vector-memory write issue and its FIFO stalls, LDS / VALU / SALU busy
#   pass 4 (tc):     texture-address busy and stalls, L2 -> fabric write requests
#   pass 5 (lat):    LDS / vector-memory / scalar-memory instructions and their outstanding
#                    levels (level / count = average latency in the counters' cycle unit)
# usage: bash tools/ext_icache.sh TAG [reads]   (CANU_OVL_LIB may name a variant library)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-ext}
READS=${2:-10000}
export TMPDIR=/tmp
mkdir -p $R/gpurun_out
cd /tmp
JOB="python3 $R/tools/index_ab.py --reads $READS --reps 1 --finds 1"
pass() {   # name counters...
  local name=$1; shift
  timeout -k 10 -s KILL 150 rocprofv3 --pmc "$@" --output-format csv -d $R/gpurun_out/${TAG}_$name \
    -o run -- $JOB > $R/gpurun_out/${TAG}_$name.log 2>&1 || { tail -5 $R/gpurun_out/${TAG}_$name.log; return 1; }
  python3 $R/tools/pmc_sum.py $R/gpurun_out/${TAG}_$name k_extend | tee -a $R/gpurun_out/${TAG}_pmc.txt
}
pass fetch SQ_IFETCH SQ_IFETCH_LEVEL SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES \
  SQC_ICACHE_MISSES_DUPLICATE SQ_WAVE_CYCLES SQ_BUSY_CYCLES && \
pass stall SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM SQ_INSTS_BRANCH \
  SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES && \
pass vmem SQ_INSTS_VMEM_WR SQ_INST_CYCLES_VMEM_WR SQ_VMEM_WR_TA_DATA_FIFO_FULL \
  SQ_VMEM_TA_ADDR_FIFO_FULL SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS && \
pass tc TA_BUSY_avr TA_DATA_STALLED_BY_TC_CYCLES_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum \
  GRBM_GUI_ACTIVE && \
pass lat SQ_INSTS_LDS SQ_INST_LEVEL_LDS SQ_INSTS_VMEM_RD SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_WR \
  SQ_INSTS_FLAT SQ_INSTS_SMEM SQ_INST_LEVEL_SMEM
