# Round-1 GPU evidence: full GPU tests, rocprofv3 kernel stats of the bench, full bench line.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -n 5 gpurun_out/gpu_tests.log
[ $rc -ne 0 ] && exit $rc
export TMPDIR=/tmp
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r01_kt -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $R/gpurun_out/r01_kt.log 2>&1 || exit $?
cd $R
timeout -k 10 900 python bench.py > gpurun_out/bench_full.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/bench_full.log | cut -c1-3000
