# A/B (tools/r04_ab2.sh), then the GPU suite and the default bench line (tools/gpu_r04.sh)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
bash $R/tools/r04_ab2.sh > $R/gpurun_out/r04_ab2.log 2>&1; cat $R/gpurun_out/r04_ab2.log
bash $R/tools/gpu_r04.sh r04b
