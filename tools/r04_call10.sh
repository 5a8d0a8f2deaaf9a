# the GPU suite (no -x), the default bench line (with its configs4-rank / MHAP side lines),
# then the chain A/B: D = current, Q = unrolled short-list qualifying, + phase profiles
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r04j_gpu_tests.log 2>&1; rc=$?
grep -E "FAILED|passed|failed" gpurun_out/r04j_gpu_tests.log | tail -12
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 700 python bench.py > gpurun_out/r04j_bench.log 2>&1 || { tail -30 gpurun_out/r04j_bench.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r04j_bench.log | cut -c1-600
run() {
  echo -n "$1 ($3 reads): "
  env CANU_OVL_LIB=$R/canu_amd/lib/ab_$2.so timeout -k 10 240 python tools/index_ab.py --reads $3 --reps 1 --finds 3 2>&1 | grep -v amdgpu.ids | grep -v OVL_DEBUG | tail -2 || exit 1
}
for v in D Q D Q CP QP; do run $v $v 50000 || exit 1; done
