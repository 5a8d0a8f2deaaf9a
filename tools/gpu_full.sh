# The whole GPU suite, then the default bench line and a configs4-rank line.
# usage: bash tools/gpu_full.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-full}
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.log 2>&1 || { tail -40 gpurun_out/${TAG}_gpu_tests.log; exit 1; }
tail -n 3 gpurun_out/${TAG}_gpu_tests.log
timeout -k 10 600 python bench.py > gpurun_out/${TAG}_bench.log 2>&1 || { tail -30 gpurun_out/${TAG}_bench.log; exit 1; }
grep -v amdgpu.ids gpurun_out/${TAG}_bench.log | cut -c1-1200
timeout -k 10 400 python bench.py --workload configs4-rank --steps 1 --warmup 1 > gpurun_out/${TAG}_c4.log 2>&1 || { tail -30 gpurun_out/${TAG}_c4.log; exit 1; }
grep -v amdgpu.ids gpurun_out/${TAG}_c4.log | cut -c1-1500
if [ "$2" = "mhap" ]; then
  timeout -k 10 600 python bench_mhap.py > gpurun_out/${TAG}_mhap.log 2>&1 || { tail -30 gpurun_out/${TAG}_mhap.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/${TAG}_mhap.log | cut -c1-2500
fi
