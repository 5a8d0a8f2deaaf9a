# A/B timing of library variants (canu_amd/lib/ab_*.so, built beforehand) on the
# 10k-read workload (AB_READS, AB_STEPS override): per-variant breakdown, twice each in
# alternating order; with
# AB_PMC=1 also one rocprofv3 issue-counter pass per variant (k_extend instruction mix).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
for pass in 1 2; do
  for f in $R/canu_amd/lib/ab_*.so; do
    n=$(basename $f .so)
    CANU_OVL_LIB=$f timeout -k 10 240 python $R/bench.py --reads ${AB_READS:-10000} --steps ${AB_STEPS:-3} --warmup 1 --no-cpu-baseline ${AB_ARGS:-} > $R/gpurun_out/ab_run_$n.log 2>&1 || exit 1
    echo "$pass $n $(grep -o "\"multiset_hash\": \"[0-9a-f]*\"" $R/gpurun_out/ab_run_$n.log) $(grep -o "\"ms_per_step\": [0-9.]*" $R/gpurun_out/ab_run_$n.log) $(grep -o "\"breakdown_ms\": {[^}]*}" $R/gpurun_out/ab_run_$n.log)"
  done
done
[ "${AB_PMC:-0}" = 1 ] || exit 0
export TMPDIR=/tmp
cd /tmp
for f in $R/canu_amd/lib/ab_*.so; do
  n=$(basename $f .so)
  CANU_OVL_LIB=$f timeout -k 10 -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/${n}_pmc -o run -- python3 $R/bench.py --reads 10000 --steps 1 --warmup 0 --no-cpu-baseline > $R/gpurun_out/${n}_pmc.log 2>&1 || exit 1
  python3 $R/tools/pmc_sum.py $R/gpurun_out/${n}_pmc k_extend
done
