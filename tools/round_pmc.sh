# The PMC evidence of both bench.py workloads on the current sources, each pass a run of its
# own under its own time limit (tools/prof_traffic.sh): configs2 (the headline) as TAG2, then
# the configs4-rank side line as TAG4 with its read set cached first (tools/c4_cache.py: no
# worker pool under the profiler).  Afterwards, on the host:
#   python tools/pmc_traffic.py TAG2
#   python tools/pmc_traffic.py TAG4 --workload configs4-rank
# usage: bash tools/round_pmc.sh TAG2 TAG4
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
T2=${1:-pmc2}
T4=${2:-pmc4}
cd $R
bash tools/prof_traffic.sh $T2 || exit 1
export CANU_C4_READS_CACHE=/tmp/canu_c4_cache
mkdir -p $CANU_C4_READS_CACHE
timeout -k 10 400 python tools/c4_cache.py > gpurun_out/${T4}_cache.log 2>&1 || { tail -5 gpurun_out/${T4}_cache.log; exit 1; }
bash tools/prof_traffic.sh $T4 --workload configs4-rank --steps 1 --warmup 0 --no-cpu-baseline --no-parity
