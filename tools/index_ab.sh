# Index-build A/B on the GPU box: every canu_amd/lib/ab_*.so twice, alternating.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
for pass in 1 2; do
  for f in $R/canu_amd/lib/ab_*.so; do
    CANU_OVL_LIB=$f timeout -k 10 180 python $R/tools/index_ab.py ${IAB_ARGS:-} 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
