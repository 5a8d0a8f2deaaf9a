set -o pipefail
mkdir -p gpurun_out
for nb in 2 3; do
OVL_EXT_BLOCKS_PER_CU=$nb timeout -k 10 300 python bench.py --reads 10000 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/occ$nb.log 2>&1 || exit $?
grep -o '"ms_per_step": [0-9.]*\|"extend": [0-9.]*' gpurun_out/occ$nb.log
done
bash tools/prof_traffic.sh r01c
