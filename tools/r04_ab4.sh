# Extension A/B on the 10k-read job (records' CRC must agree): D = current (24 waves/CU),
# G6 = Edit_Match_Limit from global + removal thresholds in global scratch at 6 waves/SIMD,
# G8 = the same at 8 waves/SIMD (32 waves/CU: a wave's LDS is its two strands only).
# Then the chain A/B on the 50k-read job: B = staged indices, C = payload lists, C5 = C at
# 5 waves/SIMD (no spills).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
run() {
  echo -n "$1 ($3 reads): "
  env CANU_OVL_LIB=$R/canu_amd/lib/ab_$2.so timeout -k 10 240 python $R/tools/index_ab.py --reads $3 --reps 1 --finds 3 2>&1 | grep -v amdgpu.ids | tail -1 || exit 1
}
CANU_OVL_LIB=$R/canu_amd/lib/ab_D.so timeout -k 10 200 python -u $R/tools/dbg_driver.py table_load 0,1c 2>&1 | grep -v amdgpu.ids | head -60
for v in D G6 G8 D G8; do run $v $v 10000 || exit 1; done
for v in B C C5 B C; do run $v $v 50000 || exit 1; done
