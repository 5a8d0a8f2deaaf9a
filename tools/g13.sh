set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_mhap.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/mhap_gpu.log 2>&1; rc=$?
tail -n 25 gpurun_out/mhap_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -m pytest tests/test_gpu_golden.py -m gpu -x -q --timeout 120 --timeout-method thread -k output_files > gpurun_out/ovb_gpu.log 2>&1; rc=$?
tail -n 5 gpurun_out/ovb_gpu.log
exit $rc
