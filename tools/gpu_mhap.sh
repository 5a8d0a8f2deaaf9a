# MHAP GPU tests, bench_mhap.py at configs[3] and its rocprofv3 kernel stats.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_mhap.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/mhap_gpu.log 2>&1; rc=$?
tail -n 3 gpurun_out/mhap_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench_mhap.py --steps 2 --warmup 1 > gpurun_out/mh200k.log 2>&1 || { tail -20 gpurun_out/mh200k.log; exit 1; }
grep -v amdgpu.ids gpurun_out/mh200k.log | cut -c1-3000
export TMPDIR=/tmp
R=$PWD
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r01_mhap_kt -o run -- python3 $R/bench_mhap.py --steps 1 --warmup 0 --no-cpu-baseline > $R/gpurun_out/r01_mhap_kt.log 2>&1
