# OVL_SLICE_Q 8 (default) vs 4 on the headline job, alternating, three passes each
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd $R
for v in SL8 SL4 SL8 SL4 SL8 SL4; do
  echo -n "$v (50000 reads): "
  env CANU_OVL_LIB=$R/canu_amd/lib/ab_$v.so timeout -k 10 240 python tools/index_ab.py --reads 50000 --reps 1 --finds 3 2>&1 | grep -v amdgpu.ids | grep -v OVL_DEBUG | tail -1 || exit 1
done
