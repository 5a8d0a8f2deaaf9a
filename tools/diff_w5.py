import os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
import oracle
from canu_amd.synth import synth_reads
from canu_amd.overlap_in_core import OicParameters, OverlapInCore
rs = synth_reads(150, 2000, 30_000, 0.02, seed=1)
P = OicParameters(Kmer_Len=22, maxErate=float(np.float32(0.06)), Min_Olap_Len=100).finalize()
want = oracle.run_oracle(rs, P.as_dict())
for rep in range(3):
    oic = OverlapInCore(P, device=0)
    got = oic.run(rs)
    oic.close()
    wa = set(map(tuple, want.tolist())); ga = set(map(tuple, got.tolist()))
    print(os.environ.get("CANU_OVL_LIB", "default"), rep, len(got), len(want), "missing", sorted(wa - ga)[:3], "extra", sorted(ga - wa)[:3], flush=True)
