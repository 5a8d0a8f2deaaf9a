set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -q -m gpu -x > gpurun_out/parity.log 2>&1; rc=$?
tail -n 3 gpurun_out/parity.log
exit $rc
