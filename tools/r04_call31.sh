# final sources: the GPU suite, smoke(), then the default bench line (traffic keyed to these
# sources for both workloads)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r04zk_gpu_tests.log 2>&1; rc=$?
grep -E "FAILED|passed|failed" gpurun_out/r04zk_gpu_tests.log | tail -12
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r04zk_smoke.log 2>&1; echo "smoke rc $?"; tail -2 gpurun_out/r04zk_smoke.log
timeout -k 10 700 python bench.py > gpurun_out/r04zk_bench.log 2>&1 || { tail -30 gpurun_out/r04zk_bench.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r04zk_bench.log | cut -c1-300
