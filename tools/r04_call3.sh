# driver debugging (tools/dbg_driver.py), then the whole GPU suite without -x, then the bench
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 300 python -u tools/dbg_driver.py table_load > gpurun_out/r04c_dbg.log 2>&1; rc=$?
cat gpurun_out/r04c_dbg.log | grep -v amdgpu.ids
[ $rc -eq 0 ] || exit $rc
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r04c_gpu_tests.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/r04c_gpu_tests.log | tail -100
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python bench.py > gpurun_out/r04c_bench.log 2>&1 || { tail -30 gpurun_out/r04c_bench.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r04c_bench.log | cut -c1-1500
