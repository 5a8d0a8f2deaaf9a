# Extension A/B on the GPU box: every canu_amd/lib/ab_*.so twice, alternating, on the
# 10k-read job (EAB_ARGS overrides); each line carries the records' CRC.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
for pass in 1 2; do
  for f in $R/canu_amd/lib/ab_*.so; do
    CANU_OVL_LIB=$f timeout -k 10 180 python $R/tools/index_ab.py ${EAB_ARGS:---reads 10000 --reps 1 --finds 3} 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
