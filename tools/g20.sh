set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_golden.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/par.log 2>&1; rc=$?
tail -n 3 gpurun_out/par.log
[ $rc -ne 0 ] && exit $rc
export TMPDIR=/tmp; R=$PWD; cd /tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/g20_kt -o run -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline > $R/gpurun_out/g20_kt.log 2>&1 || exit 1
cut -c1-110 $R/gpurun_out/g20_kt/run_kernel_stats.csv | head -12
