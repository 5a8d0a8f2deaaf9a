# GPU suite + bench line for the current tree (TAG names the outputs under gpurun_out/).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-chk}
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_gpu_tests.log; exit 1; }
tail -n 2 gpurun_out/${TAG}_gpu_tests.log
timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > gpurun_out/${TAG}_bench.log 2>&1 || { tail -30 gpurun_out/${TAG}_bench.log; exit 1; }
grep -v amdgpu.ids gpurun_out/${TAG}_bench.log | cut -c1-700
