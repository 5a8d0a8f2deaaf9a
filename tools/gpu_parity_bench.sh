# GPU parity + golden tests, then the quick 50k bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_golden.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/par.log 2>&1; rc=$?
tail -n 2 gpurun_out/par.log
[ $rc -ne 0 ] && exit $rc
bash tools/gpu_bench_quick.sh
