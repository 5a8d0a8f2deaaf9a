# k_chain A/B on the bench's 50k-read job (records' CRC must agree): B = the chain with
# staged indices, C = per-target payload lists with the next payload prefetched
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
run() {
  echo -n "$1: "
  env CANU_OVL_LIB=$R/canu_amd/lib/ab_$2.so timeout -k 10 240 python $R/tools/index_ab.py --reads 50000 --reps 1 --finds 3 2>&1 | grep -v amdgpu.ids | tail -1 || exit 1
}
for v in ${@:-B C B C}; do run $v $v || exit 1; done
