# FETCH_SIZE / WRITE_SIZE calibration on known byte counts (tools/calib_traffic.hip), then
# profiles/calib_traffic.json (tools/calib_traffic.py).  One counter per pass, no tracing.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
mkdir -p $R/gpurun_out
cd /tmp
timeout -k 10 120 $R/tools/bin/calib_traffic > $R/gpurun_out/calib.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/calib_fetch -o run -- $R/tools/bin/calib_traffic > $R/gpurun_out/calib_fetch.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/calib_write -o run -- $R/tools/bin/calib_traffic > $R/gpurun_out/calib_write.log 2>&1 && \
python3 $R/tools/calib_traffic.py $R/gpurun_out
