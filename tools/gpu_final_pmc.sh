# The PMC passes that key profiles/traffic*.json to the current sources, in one GPU call:
# the overlapInCore headline and configs4-rank side line (tools/round_pmc.sh), then the MHAP
# configs[3] line (tools/mhap_pmc.sh).  Afterwards, on the host:
#   python tools/pmc_traffic.py TAG2 ; python tools/pmc_traffic.py TAG4 --workload configs4-rank
#   cp gpurun_out/TAGM_traffic_mhap.json profiles/traffic_mhap.json
# usage: bash tools/gpu_final_pmc.sh TAG2 TAG4 TAGM
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash tools/round_pmc.sh ${1:-pmc2} ${2:-pmc4} || exit 1
bash tools/mhap_pmc.sh ${3:-pmcm}
