# Round-3 GPU checks: new GPU tests, the bench line (parity, roofline fields, CPU share),
# the --gpus 2 self-launch (gloo rehearsal on one device) and the configs4-rank workload.
# usage: bash tools/gpu_r03.sh TAG [pytest -k expression]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r03}
K=${2:-"configs4 or library or launch"}
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$K" > gpurun_out/${TAG}_gpu_tests.log 2>&1 || { tail -40 gpurun_out/${TAG}_gpu_tests.log; exit 1; }
tail -n 3 gpurun_out/${TAG}_gpu_tests.log
timeout -k 10 600 python bench.py > gpurun_out/${TAG}_bench.log 2>&1 || { tail -30 gpurun_out/${TAG}_bench.log; exit 1; }
grep -v amdgpu.ids gpurun_out/${TAG}_bench.log | cut -c1-4000
CANU_DEVICE=0 CANU_DIST_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --reads 8000 --steps 2 --no-cpu-baseline > gpurun_out/${TAG}_gpus2.log 2>&1 || { tail -30 gpurun_out/${TAG}_gpus2.log; exit 1; }
grep -v amdgpu.ids gpurun_out/${TAG}_gpus2.log | cut -c1-1500
timeout -k 10 400 python bench.py --workload configs4-rank --steps 1 --warmup 1 > gpurun_out/${TAG}_c4.log 2>&1 || { tail -30 gpurun_out/${TAG}_c4.log; exit 1; }
grep -v amdgpu.ids gpurun_out/${TAG}_c4.log | cut -c1-2000
