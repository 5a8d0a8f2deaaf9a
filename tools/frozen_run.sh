# Run a command inside .gpu_frozen/ (tools/freeze.sh) on the GPU box, with its gpurun_out/
# pointing at the top-level one that gpurun merges back.   usage: bash tools/frozen_run.sh CMD...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out"
cd "$R/.gpu_frozen" || exit 1
rm -rf gpurun_out
ln -s "$R/gpurun_out" gpurun_out
export GRAFT_REPO_ROOT="$R/.gpu_frozen"
"$@"
