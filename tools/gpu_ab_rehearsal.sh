# A/B of library variants (canu_amd/lib/ab_*.so) on the configs[4] rehearsal workload
# (AB_READS reads x 12 kb, 15x, jittered lengths): extension / seed / index ms per variant,
# twice each in alternating order.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
for pass in 1 2; do
  for f in $R/canu_amd/lib/ab_*.so; do
    n=$(basename $f .so)
    CANU_OVL_LIB=$f timeout -k 10 240 python $R/tools/rehearse_configs4.py --reads ${AB_READS:-200000} --hashbits ${AB_HASHBITS:-25} > $R/gpurun_out/${n}_c4.log 2>&1 || exit 1
    echo "$pass $n $(grep -o '"job_s": [0-9.]*' $R/gpurun_out/${n}_c4.log) $(grep -o '"ms": {[^}]*}' $R/gpurun_out/${n}_c4.log)"
  done
done
