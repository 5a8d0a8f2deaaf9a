# configs[4] at full size: several rank jobs of the 8-GPU plan one after another on one GPU
# (tools/c4_full.sh per job, each under its own time limit); stops at the first failure.
# usage: bash tools/c4_ranks.sh TAG JOB [JOB ...]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
for J in "$@"; do
  echo "=== rank job $J $(date +%T)"
  bash $R/tools/c4_full.sh ${TAG}${J} $J > /dev/null || { echo "rank job $J failed"; exit 1; }
  python3 - $R/gpurun_out/${TAG}${J}.json <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
c = d.get("counters", {})
print(json.dumps({"job": d["config"]["job"], "ms": d["ms_per_step"], "setup_s": d["setup_s"],
                  "records": d["overlaps_per_step"], "breakdown_ms": d["breakdown_ms"],
                  "sb": c.get("super_batches"), "chunks": c.get("query_chunks"),
                  "free_gb": d["setup_hbm"]["device_free_gb"], "ovb": d.get("ovb_output")}))
PY
done
