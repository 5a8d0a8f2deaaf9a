import sys, os
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R); sys.path.insert(0, os.path.join(R, 'oracle'))
import numpy as np
from canu_amd.synth import synth_reads
from canu_amd.overlap_in_core import OicParameters, OverlapInCore
import oracle
kw = dict(n_rate=0.002, n_repeats=6, repeat_len=300, len_jitter=0.6)
which = sys.argv[1] if len(sys.argv) > 1 else 'all'
variants = {'n': dict(n_rate=0.002), 'rep': dict(n_repeats=6, repeat_len=300), 'jit': dict(len_jitter=0.6), 'all': kw}
for name, v in variants.items():
    rs = synth_reads(150, 2000, 30_000, 0.02, seed=5, **v)
    P = OicParameters(Kmer_Len=22, maxErate=float(np.float32(0.06)), Min_Olap_Len=100).finalize()
    oic = OverlapInCore(P, device=0)
    got = oic.run(rs); st = oic.stats(); oic.close()
    want, wst = oracle.run_oracle(rs, P.as_dict(), with_stats=True)
    print(name, len(got), len(want), np.array_equal(got, want))
    print('  gpu', {k: st[k] for k in ('seed_hits','pairs','kmer_hits_with_olap','kmer_hits_without_olap')})
    print('  ora', {k: wst[k] for k in ('seed_hits','pairs','kmer_hits_with_olap','kmer_hits_without_olap')})
    if not np.array_equal(got, want):
        gs = set(map(tuple, got.tolist())); ws = set(map(tuple, want.tolist()))
        print('  only gpu', sorted(gs - ws)[:5]); print('  only ora', sorted(ws - gs)[:5])
