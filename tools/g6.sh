set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -q -m gpu -x > gpurun_out/parity.log 2>&1; rc=$?
tail -n 2 gpurun_out/parity.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/b50k.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/b50k.log | cut -c1-1500
