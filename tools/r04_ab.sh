# Round-4 extension A/B on the 10k-read job (10 kb reads), two alternating passes:
#   A_sh0   original row loop (ab_A.so), per-pair strands            = the round-3 kernel
#   B_sh0   in-place row loop (ab_B.so), per-pair strands
#   B_sh1   in-place row loop, block-shared query strand (32 waves/CU)
#   A_sh1   original row loop, block-shared query strand
#   A_occ4  the round-3 kernel with LDS padded to 2 blocks per CU (occupancy sensitivity)
# each line: the library's extend ms (median of 3 finds) and the records' CRC (must agree).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
run() {   # name lib shared [extra env]
  echo -n "$1: "
  env CANU_OVL_LIB=$R/canu_amd/lib/ab_$2.so OVL_SHARED=$3 $4 timeout -k 10 180 python $R/tools/index_ab.py ${EAB_ARGS:---reads 10000 --reps 1 --finds 3} 2>&1 | grep -v amdgpu.ids | tail -1 || exit 1
}
for pass in 1 2; do
  run A_sh0 A 0 || exit 1
  run B_sh0 B 0 || exit 1
  run B_sh1 B 1 || exit 1
  run A_sh1 A 1 || exit 1
done
run A_occ4 A 0 OVL_EXT_BLOCKS_PER_CU=2 || exit 1
