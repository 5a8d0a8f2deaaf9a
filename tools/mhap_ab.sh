# A/B of MHAP library variants (canu_amd/lib/mhab_*.so, built by hand with extra -D flags) on
# bench_mhap.py's configs[3] job: two alternating passes, each variant's sketch / compare time
# and its overlap and candidate counts (equal counts: the same sketches).  Each run under its
# own time limit.   usage: bash tools/mhap_ab.sh > gpurun_out/TAG_mhab.txt
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
for pass in 1 2; do
  for lib in $R/canu_amd/lib/mhab_*.so; do
    CANU_MHAP_LIB=$lib timeout -k 10 240 python $R/bench_mhap.py --steps 2 --warmup 1 \
      --no-cpu-baseline > /tmp/mhab.json 2> /tmp/mhab.err || { tail -5 /tmp/mhab.err; exit 1; }
    python3 -c "
import json,sys
d=json.loads(open('/tmp/mhab.json').read().strip().splitlines()[-1])
b=d['breakdown_ms']
print('$(basename $lib)', 'sketch', b['sketch'], 'compare', b['compare'], 'step', d['ms_per_step'],
      'overlaps', d['overlaps_per_step'], 'candidates', d.get('candidates_per_step'), flush=True)"
  done
done
