# the sorted-window keys checked (OVL_SQ_CHECK) on the failing driver case, and the chain's
# phase profile (OVL_CHAIN_PROF build) on the 50k-read job
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 200 python -u tools/dbg_driver.py table_load 1c > gpurun_out/r04f_dbg.log 2>&1; echo "dbg rc $?"
grep -v amdgpu.ids gpurun_out/r04f_dbg.log | head -24
CANU_OVL_LIB=$R/canu_amd/lib/ab_CP.so timeout -k 10 240 python tools/index_ab.py --reads 50000 --reps 1 --finds 1 > gpurun_out/r04f_chainprof.log 2>&1; echo "prof rc $?"
grep -v amdgpu.ids gpurun_out/r04f_chainprof.log | tail -5
