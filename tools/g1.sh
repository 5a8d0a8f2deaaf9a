set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_gpu_parity.py -q -m gpu -x > gpurun_out/parity.log 2>&1 && \
timeout -k 10 300 python bench.py --reads 10000 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/b10k.log 2>&1 && \
timeout -k 10 400 python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/b50k.log 2>&1
rc=$?
tail -n 3 gpurun_out/parity.log; cat gpurun_out/b10k.log gpurun_out/b50k.log | cut -c1-1500
exit $rc
