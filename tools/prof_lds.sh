# One rocprofv3 pass of the extension's LDS and issue counters on the 10k-read job (one
# step): LDS array cycles, bank-conflict / unaligned extra cycles, LDS issue stalls.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-lds}
export TMPDIR=/tmp
mkdir -p $R/gpurun_out
cd /tmp
timeout -k 10 -s KILL 240 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/${TAG}_pmc -o run -- python3 $R/bench.py --reads 10000 --steps 1 --warmup 0 --no-cpu-baseline --no-shard-timing --no-seed-only > $R/gpurun_out/${TAG}_pmc.log 2>&1 || exit 1
python3 $R/tools/pmc_sum.py $R/gpurun_out/${TAG}_pmc k_extend
