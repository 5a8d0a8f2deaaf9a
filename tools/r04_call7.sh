# the sorted-window probe: host emulation and a relaunch beside the random-lookup probe
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 200 python -u tools/dbg_driver.py table_load 1c > gpurun_out/r04i_dbg.log 2>&1; echo "dbg rc $?"
grep -v amdgpu.ids gpurun_out/r04i_dbg.log | grep -v "OVL_SQ_CHECK window" | head -30
