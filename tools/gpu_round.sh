# GPU evidence for the current tree: GPU tests, rocprofv3 kernel stats of the bench, bench line.
# usage: bash tools/gpu_round.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r01}
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.log 2>&1; rc=$?
tail -n 5 gpurun_out/${TAG}_gpu_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py > gpurun_out/${TAG}_bench.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/${TAG}_bench.log | cut -c1-3000
export TMPDIR=/tmp
cd /tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${TAG}_kt -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $R/gpurun_out/${TAG}_kt.log 2>&1 || exit $?
