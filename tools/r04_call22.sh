# extension A/B: SK1 = the reverse extension skipped when the forward one stopped short of the
# ends (its result is unread unless partial overlaps are on), SK0 = always run; 10k and 50k
# reads, alternating; each line: extend ms (median of the finds) and the records' CRC
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd $R
run() {
  echo -n "$1 ($2 reads): "
  env CANU_OVL_LIB=$R/canu_amd/lib/ab_$1.so timeout -k 10 240 python tools/index_ab.py --reads $2 --reps 1 --finds 3 2>&1 | grep -v amdgpu.ids | grep -v OVL_DEBUG | tail -1 || exit 1
}
for v in SK0 SK1 SK0 SK1; do run $v 10000 || exit 1; done
for v in SK1 SK0 SK1; do run $v 50000 || exit 1; done
