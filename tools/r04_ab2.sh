# Shared-strand A/B after the slot-claim fix, 10k-read job (records' CRC must agree):
#   B_sh0 in-place row loop, per-pair strands; B_sh1 + shared query strand (64 VGPRs, 32
#   waves/CU); Bs6_sh1 shared strand at 80 VGPRs (24 waves/CU: the protocol's cost alone)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
run() {
  echo -n "$1: "
  env CANU_OVL_LIB=$R/canu_amd/lib/ab_$2.so OVL_SHARED=$3 timeout -k 10 180 python $R/tools/index_ab.py --reads 10000 --reps 1 --finds 3 2>&1 | grep -v amdgpu.ids | tail -1 || exit 1
}
run B_sh0 B 0 || exit 1
run B_sh1 B 1 || exit 1
run Bs6_sh1 Bs6 1 || exit 1
run B_sh1 B 1 || exit 1
