# the 2-rank configs4-rank rehearsal again, first without a warmup job (as r04zl) and then with
# one: how much of the step is the ranks' first allocations
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd $R
for w in 0 1; do
CANU_DEVICE=0 CANU_DIST_BACKEND=gloo OVL_TIMING=1 timeout -k 10 400 python bench.py --gpus 2 --workload configs4-rank --reads 20000 --steps 1 --warmup $w --no-cpu-baseline --no-side > gpurun_out/r04zm_c4_gpus2_w$w.log 2>&1 || { tail -30 gpurun_out/r04zm_c4_gpus2_w$w.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r04zm_c4_gpus2_w$w.log | grep '^{' | cut -c1-400
grep -a "OVL_TIMING batch" gpurun_out/r04zm_c4_gpus2_w$w.log | tail -4 | cut -c1-250
done
