# Run GPU steps in order, each under its own time limit; stop at the first step that timed
# out or crashed (124 / 137 / 134 / 139), go on after an ordinary failure.
# usage: bash tools/gpu_steps.sh "SECONDS CMD" ["SECONDS CMD" ...]
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
for step in "$@"; do
  secs=${step%% *}; cmd=${step#* }
  echo "=== $(date +%T) $cmd"
  timeout -k 10 $secs bash -c "$cmd"
  rc=$?
  echo "=== rc $rc"
  case $rc in 124|137|134|139) echo "stopping: step timed out or crashed"; exit $rc;; esac
done
