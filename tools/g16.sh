set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_mhap.py -m gpu -x -q --timeout 120 --timeout-method thread -k "oracle or rows" > gpurun_out/mhap_gpu.log 2>&1; rc=$?
tail -n 2 gpurun_out/mhap_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench_mhap.py --reads 50000 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/mhA.log 2>&1 || exit 1
MHAP_SKETCH_B64=1 timeout -k 10 300 python bench_mhap.py --reads 50000 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/mhB.log 2>&1 || exit 1
grep -o '"breakdown_ms": {[^}]*}' gpurun_out/mhA.log gpurun_out/mhB.log
