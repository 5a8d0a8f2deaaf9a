# GPU tests selected by -k, then the default bench line and the MHAP bench line.
# usage: bash tools/gpu_tests_bench.sh TAG "pytest -k expression" [mhap]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-chk}
K=${2:-""}
mkdir -p $R/gpurun_out
cd $R
if [ -n "$K" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$K" > gpurun_out/${TAG}_gpu_tests.log 2>&1 || { tail -40 gpurun_out/${TAG}_gpu_tests.log; exit 1; }
  tail -n 3 gpurun_out/${TAG}_gpu_tests.log
fi
timeout -k 10 600 python bench.py > gpurun_out/${TAG}_bench.log 2>&1 || { tail -30 gpurun_out/${TAG}_bench.log; exit 1; }
grep -v amdgpu.ids gpurun_out/${TAG}_bench.log | cut -c1-1500
if [ "$3" = "mhap" ]; then
  timeout -k 10 600 python bench_mhap.py > gpurun_out/${TAG}_mhap.log 2>&1 || { tail -30 gpurun_out/${TAG}_mhap.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/${TAG}_mhap.log | cut -c1-2500
fi
