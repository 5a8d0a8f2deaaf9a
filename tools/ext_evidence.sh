# Extension evidence on the 10k-read job, each step under its own time limit:
#   1. A/B of every canu_amd/lib/ab_*.so (tools/ext_ab.sh: twice each, alternating, records'
#      CRC per line)                                              -> gpurun_out/TAG_ab.txt
#   2. the phase profile (libcanu_ovl_prof.so, s_memtime stamps per extension phase; build
#      it with `python -m canu_amd.build --profile`)              -> gpurun_out/TAG_phase.log
#   3. instruction-fetch and stall PMC passes (tools/ext_icache.sh) -> gpurun_out/TAG_pmc.txt
# usage: bash tools/ext_evidence.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-ext}
mkdir -p $R/gpurun_out
bash $R/tools/ext_ab.sh > $R/gpurun_out/${TAG}_ab.txt 2>&1 || { tail -5 $R/gpurun_out/${TAG}_ab.txt; exit 1; }
cat $R/gpurun_out/${TAG}_ab.txt
if [ -f $R/canu_amd/lib/libcanu_ovl_prof.so ]; then
  CANU_OVL_LIB=$R/canu_amd/lib/libcanu_ovl_prof.so OVL_DEBUG=1 timeout -k 10 180 \
    python $R/tools/index_ab.py --reads 10000 --reps 1 --finds 1 > $R/gpurun_out/${TAG}_phase.log 2>&1 \
    || { tail -5 $R/gpurun_out/${TAG}_phase.log; exit 1; }
  grep OVL_DEBUG $R/gpurun_out/${TAG}_phase.log | tail -3
fi
bash $R/tools/ext_icache.sh $TAG
