# Round evidence: full GPU test suite, rocprofv3 passes (kernel stats, FETCH/WRITE, issue) and the bench line.
# full evidence pass for the current tree (round 1, tag r01d)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r01d_gpu_tests.log 2>&1; rc=$?
tail -n 3 gpurun_out/r01d_gpu_tests.log
[ $rc -ne 0 ] && exit $rc
bash tools/prof_traffic.sh ${TAG:-r01d} || exit 1
timeout -k 10 600 python bench.py > gpurun_out/r01d_bench.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r01d_bench.log | cut -c1-400
