import sys, os, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'oracle'))
import numpy as np
from canu_amd.synth import synth_reads
from canu_amd.overlap_in_core import OicParameters, OverlapInCore
import oracle
n = int(sys.argv[1]) if len(sys.argv) > 1 else 150
rs = synth_reads(n, 2000, 200*n, 0.02, seed=1)
P = OicParameters(Kmer_Len=22, maxErate=float(np.float32(0.06)), Min_Olap_Len=100).finalize()
oic = OverlapInCore(P, device=0)
oic.load_reads(rs)
oic.build_hash_index()
n_ = oic.find_overlaps()
print("gpu n", n_, oic.stats())
got = oic.fetch(n_)
want, wst = oracle.run_oracle(rs, P.as_dict(), with_stats=True)
print("oracle", len(want), wst)
print("equal", np.array_equal(got, want))
if len(got) and len(want):
    print(got[:3]); print(want[:3])
