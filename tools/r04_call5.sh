# (1) the sorted-window probe checked against the random-lookup probe on the failing driver
#     case (OVL_SQ_CHECK), (2) extension A/B on 10k and 50k reads: R3 = round 3's library,
#     D = current, G6 / G8 = Edit_Match_Limit + removal thresholds out of LDS at 6 / 8 waves
#     per SIMD; chain A/B: C5 = current chain at 5 waves/SIMD (no spills); (3) driver tests
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd $R
CANU_OVL_LIB=$R/canu_amd/lib/ab_D.so timeout -k 10 200 python -u tools/dbg_driver.py table_load 0,1c > gpurun_out/r04e_dbg.log 2>&1; echo "dbg rc $?"
grep -v amdgpu.ids gpurun_out/r04e_dbg.log | head -40
run() {
  echo -n "$1 ($3 reads): "
  env CANU_OVL_LIB=$R/canu_amd/lib/ab_$2.so timeout -k 10 240 python tools/index_ab.py --reads $3 --reps 1 --finds 3 2>&1 | grep -v amdgpu.ids | tail -1 || exit 1
}
for v in R3 D G8 G6 D G8 R3; do run $v $v 10000 || exit 1; done
for v in R3 D G8 C5 D G8; do run $v $v 50000 || exit 1; done
timeout -k 10 600 python -u -m pytest tests/test_driver.py tests/test_gpu_c4_digest.py tests/test_olap_limit.py -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r04e_tests.log 2>&1
grep -E "PASSED|FAILED|passed|failed" gpurun_out/r04e_tests.log | tail -30
