# k_fine phase costs: rocprofv3 kernel stats of tools/index_ab.py (timing only) for every
# canu_amd/lib/ab_*.so (phase-cut builds: -DOVL_FINE_PHASE=1 / 2 stop after the fine
# histogram / the fine split and leave empty buckets for k_table).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
export TMPDIR=/tmp
cd /tmp
for f in $R/canu_amd/lib/ab_*.so; do
  n=$(basename $f .so)
  CANU_OVL_LIB=$f timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${n}_kt -o run -- python3 $R/tools/index_ab.py --reps 3 --finds 0 > $R/gpurun_out/${n}_kt.log 2>&1 || exit 1
  echo "== $n $(grep 'index ms' $R/gpurun_out/${n}_kt.log)"
  find $R/gpurun_out/${n}_kt -name "*kernel_stats.csv" | head -1 | xargs grep -E "k_fine|k_coarse|k_table" | cut -d, -f1-4
done
