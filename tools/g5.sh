set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -q -m gpu -x > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -n 3 gpurun_out/gpu_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/b50k.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/b50k.log | cut -c1-2500
bash tools/prof_traffic.sh r01
