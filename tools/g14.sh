set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench_mhap.py --reads 20000 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/mh20k.log 2>&1 || { tail -20 gpurun_out/mh20k.log; exit 1; }
grep -v amdgpu.ids gpurun_out/mh20k.log | cut -c1-2500
timeout -k 10 600 python bench_mhap.py --steps 2 --warmup 1 > gpurun_out/mh200k.log 2>&1 || { tail -20 gpurun_out/mh200k.log; exit 1; }
grep -v amdgpu.ids gpurun_out/mh200k.log | cut -c1-3000
