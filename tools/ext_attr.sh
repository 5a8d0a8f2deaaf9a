# k_extend HBM traffic by source: FETCH_SIZE / WRITE_SIZE passes (one counter group per run)
# of the 50k x 10 kb job for the shipped library and three measurement-only builds
# (canu_amd/lib/attr_*.so; their records are wrong by construction):
#   attr_log   every row of the traceback log stored to row 0's stripe (log writes stay in L2)
#   attr_tb    every traceback load reads row 0 (the walk's log reads stay in L2)
#   attr_both  both
# base - attr_log = the log's write traffic, base - attr_tb = the traceback's reads; what
# attr_both keeps is the rest (strand staging, match nodes, deltas, scratch spills).
# usage: bash tools/ext_attr.sh TAG      -> gpurun_out/TAG_attr.txt
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-attr}
export TMPDIR=/tmp
mkdir -p $R/gpurun_out
cd /tmp
for lib in libcanu_ovl attr_log attr_tb attr_both; do
  for ctr in FETCH_SIZE WRITE_SIZE; do
    d=$R/gpurun_out/${TAG}_${lib}_${ctr}
    CANU_OVL_LIB=$R/canu_amd/lib/$lib.so timeout -k 10 240 rocprofv3 --pmc $ctr --output-format csv -d $d -o run -- \
      python3 $R/tools/index_ab.py --reads 50000 --reps 1 --finds 1 > $d.log 2>&1 || { tail -5 $d.log; exit 1; }
    grep -h "index ms" $d.log
    python3 $R/tools/pmc_sum.py $d k_extend | tee -a $R/gpurun_out/${TAG}_attr.txt
  done
done
