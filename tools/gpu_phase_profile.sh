# Profiling build (s_memtime stamps per extension phase, OVL_DEBUG=1) on 10k reads, then prof_pmc.sh passes.
set -o pipefail
mkdir -p gpurun_out
CANU_OVL_LIB=$PWD/canu_amd/lib/libcanu_ovl_prof.so OVL_DEBUG=1 timeout -k 10 300 python bench.py --reads 10000 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/prof.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/prof.log | tail -5 | cut -c1-1500
bash tools/prof_pmc.sh pmcA
