# Occupancy sensitivity of k_extend: the same library at its natural occupancy (3 blocks of
# 8 waves per CU at 10 kb) and with LDS padded to 2 blocks per CU (OVL_EXT_BLOCKS_PER_CU),
# twice each, alternating, on the 10k-read job; then the counter list of this device.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
for pass in 1 2; do
  for nb in 0 2; do
    if [ $nb = 0 ]; then unset OVL_EXT_BLOCKS_PER_CU; else export OVL_EXT_BLOCKS_PER_CU=$nb; fi
    echo "pass $pass blocks_per_cu=$nb"
    timeout -k 10 180 python $R/tools/index_ab.py --reads 10000 --reps 1 --finds 3 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
unset OVL_EXT_BLOCKS_PER_CU
export TMPDIR=/tmp
cd /tmp
timeout -k 10 -s KILL 60 rocprofv3 -L > $R/gpurun_out/counters_list.txt 2>&1 || true
grep -c "SQ_" $R/gpurun_out/counters_list.txt || true
