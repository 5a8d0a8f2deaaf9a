# GPU parity + golden tests, then 10k- and 50k-read bench timings.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_golden.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/par.log 2>&1; rc=$?
tail -n 3 gpurun_out/par.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --reads 10000 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/b10k.log 2>&1 || exit 1
grep -o '"extend": [0-9.]*' gpurun_out/b10k.log
timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/b50k.log 2>&1 || exit 1
grep -o '"value": [0-9.]*\|"breakdown_ms": {[^}]*}' gpurun_out/b50k.log
