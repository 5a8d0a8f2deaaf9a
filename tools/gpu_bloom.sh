# The probe's Bloom filter: driver / configs[4] GPU tests with the filter forced on for every
# search (OVL_BLOOM=1, exactness), then the configs4-rank bench line with it off and on.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-bloom}
mkdir -p $R/gpurun_out
cd $R
OVL_BLOOM=1 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "driver or configs4 or golden" > gpurun_out/${TAG}_tests_forced.log 2>&1 || { tail -30 gpurun_out/${TAG}_tests_forced.log; exit 1; }
tail -n 1 gpurun_out/${TAG}_tests_forced.log
for b in 0 auto; do
  if [ $b = auto ]; then unset OVL_BLOOM; else export OVL_BLOOM=$b; fi
  timeout -k 10 400 python bench.py --workload configs4-rank --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}_c4_$b.log 2>&1 || { tail -30 gpurun_out/${TAG}_c4_$b.log; exit 1; }
  echo "bloom=$b $(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"overlaps_per_step": [0-9]*\|"breakdown_ms": {[^}]*}' gpurun_out/${TAG}_c4_$b.log | tr '\n' ' ')"
done
