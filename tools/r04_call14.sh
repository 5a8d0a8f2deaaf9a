# hipcub partial-range radix sorts checked (tools/sortcheck.hip), then the chain scatter A/B
# on the 50k-read job (B1 = ballot ranks, B0 = LDS lane masks)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 300 ./tools/sortcheck > gpurun_out/r04n_sortcheck.log 2>&1; echo "sortcheck rc $?"; cat gpurun_out/r04n_sortcheck.log
run() {
  echo -n "$1 ($3 reads): "
  env CANU_OVL_LIB=$R/canu_amd/lib/ab_$2.so timeout -k 10 240 python tools/index_ab.py --reads $3 --reps 1 --finds 3 2>&1 | grep -v amdgpu.ids | grep -v OVL_DEBUG | tail -2 || exit 1
}
for v in B1 B0 B1 B0; do run $v $v 50000 || exit 1; done
