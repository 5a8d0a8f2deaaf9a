set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_gpu_parity.py -q -m gpu -x > gpurun_out/parity.log 2>&1; rc=$?
tail -n 30 gpurun_out/parity.log
[ $rc -ne 0 ] && exit $rc
OVL_DEBUG=1 timeout -k 10 300 python bench.py --reads 10000 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/b10k.log 2>&1 && \
timeout -k 10 400 python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/b50k.log 2>&1
rc=$?
cat gpurun_out/b10k.log gpurun_out/b50k.log | grep -v amdgpu.ids | cut -c1-1200
exit $rc
