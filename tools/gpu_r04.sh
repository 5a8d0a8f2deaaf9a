# Round 4 evidence call: the whole GPU suite, the default bench line, then an optional
# extra script (e.g. tools/occ_ab.sh).  usage: bash tools/gpu_r04.sh TAG [extra.sh]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r04}
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.log 2>&1 || { tail -40 gpurun_out/${TAG}_gpu_tests.log; exit 1; }
tail -n 3 gpurun_out/${TAG}_gpu_tests.log
timeout -k 10 600 python bench.py > gpurun_out/${TAG}_bench.log 2>&1 || { tail -30 gpurun_out/${TAG}_bench.log; exit 1; }
grep -v amdgpu.ids gpurun_out/${TAG}_bench.log | cut -c1-1200
if [ -n "$2" ]; then bash $2 || exit 1; fi
