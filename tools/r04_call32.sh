# the N > 1 path on one GPU: 2 ranks of bench.py (self-launched, gloo, both on device 0), the
# headline workload at 8k reads and a configs4-rank plan at 20k reads (each rank its job,
# checked against the committed reference digests)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd $R
CANU_DEVICE=0 CANU_DIST_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --reads 8000 --steps 2 --no-cpu-baseline --no-side > gpurun_out/r04zl_gpus2.log 2>&1 || { tail -30 gpurun_out/r04zl_gpus2.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r04zl_gpus2.log | grep '^{' | cut -c1-700
CANU_DEVICE=0 CANU_DIST_BACKEND=gloo timeout -k 10 400 python bench.py --gpus 2 --workload configs4-rank --reads 20000 --steps 1 --warmup 0 --no-cpu-baseline --no-side > gpurun_out/r04zl_c4_gpus2.log 2>&1 || { tail -30 gpurun_out/r04zl_c4_gpus2.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r04zl_c4_gpus2.log | grep '^{' | cut -c1-900
timeout -k 10 400 python bench.py --workload configs4-rank --reads 20000 --rank-job 7 --steps 1 --warmup 1 --no-cpu-baseline --no-side > gpurun_out/r04zl_c4_job7.log 2>&1 || { tail -30 gpurun_out/r04zl_c4_job7.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r04zl_c4_job7.log | grep '^{' | cut -c1-900
