# MHAP configs[3] counter evidence (bench_mhap.py, one step, serial read generation): PMC
# passes summed over the sketch kernels (k_mh_minhash: the weighted MinHash draws;
# k_mh_ordered: the ordered sketch), each pass a run of its own under its own time limit:
#   issue:  VALU / SALU instructions, active / wait cycles, wave cycles
#   bytes:  FETCH_SIZE, then WRITE_SIZE (HBM traffic, the guide's passes)
# and a kernel trace; then tools/pmc_mhap.py sums them per launch into
# gpurun_out/TAG_traffic_mhap.json (copy it to profiles/traffic_mhap.json for bench_mhap.py).
# usage: bash tools/mhap_pmc.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-mh}
export TMPDIR=/tmp
mkdir -p $R/gpurun_out
cd /tmp
JOB="python3 $R/bench_mhap.py --steps 1 --warmup 0 --no-cpu-baseline"
pass() {   # name counters...
  local name=$1; shift
  timeout -k 10 -s KILL 300 rocprofv3 --pmc "$@" --output-format csv -d $R/gpurun_out/${TAG}_$name \
    -o run -- $JOB > $R/gpurun_out/${TAG}_$name.log 2>&1 || { tail -5 $R/gpurun_out/${TAG}_$name.log; return 1; }
  for k in k_mh_minhash k_mh_bitslice k_mh_keys k_mh_ordered k_mh_compare; do
    python3 $R/tools/pmc_sum.py $R/gpurun_out/${TAG}_$name $k | sed "s/^/$k /" | tee -a $R/gpurun_out/${TAG}_pmc.txt
  done
}
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${TAG}_kt -o run \
  -- $JOB > $R/gpurun_out/${TAG}_kt.log 2>&1 && \
pass issue SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY \
  SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES && \
pass fetch FETCH_SIZE && \
pass write WRITE_SIZE && \
python3 $R/tools/pmc_mhap.py $TAG $R/gpurun_out/${TAG}_traffic_mhap.json
