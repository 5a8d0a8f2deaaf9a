# extension A/B without the shared-strand instance (R3 = round 3, E0 = old row loop,
# E1 = in-place row loop, both with the chain's run replay; N = E1 without it; RP = chain
# phase profile), then the configs4-rank job with the sorted query windows (S, OVL_TIMING)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd $R
run() {
  echo -n "$1 ($3 reads): "
  env CANU_OVL_LIB=$R/canu_amd/lib/ab_$2.so timeout -k 10 240 python tools/index_ab.py --reads $3 --reps 1 --finds 3 2>&1 | grep -v amdgpu.ids | grep -v OVL_DEBUG | tail -2 || exit 1
}
for v in R3 E0 E1 N R3 E0 E1 RP; do run $v $v 50000 || exit 1; done
CANU_OVL_LIB=$R/canu_amd/lib/ab_S.so OVL_TIMING=1 timeout -k 10 400 python bench.py --workload configs4-rank --steps 1 --warmup 1 --no-cpu-baseline --no-side > gpurun_out/r04k_c4.log 2>&1; echo "c4 rc $?"
grep -a "sorted query\|^{" gpurun_out/r04k_c4.log | cut -c1-700 | head -4
