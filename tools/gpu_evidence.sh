# Round evidence: full GPU test suite, rocprofv3 passes (kernel stats, FETCH/WRITE, issue) and the bench line.
# full evidence pass for the current tree (tag from $TAG, default r01e)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG:-r01e}_gpu_tests.log 2>&1; rc=$?
tail -n 3 gpurun_out/${TAG:-r01e}_gpu_tests.log
[ $rc -ne 0 ] && exit $rc
bash tools/prof_traffic.sh ${TAG:-r01e} || exit 1
timeout -k 10 600 python bench.py > gpurun_out/${TAG:-r01e}_bench.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/${TAG:-r01e}_bench.log | cut -c1-400
