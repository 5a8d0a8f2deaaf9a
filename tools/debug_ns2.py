import sys, os
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R); sys.path.insert(0, os.path.join(R, 'oracle'))
import numpy as np
from canu_amd.synth import synth_reads
from canu_amd.overlap_in_core import OicParameters, OverlapInCore
import oracle
rs = synth_reads(150, 2000, 30_000, 0.02, seed=5, n_rate=0.002)
P = OicParameters(Kmer_Len=22, maxErate=float(np.float32(0.06)), Min_Olap_Len=100).finalize()
oic = OverlapInCore(P, device=0)
oic.load_reads(rs); oic.build_hash_index()
k = 22
comp = {'A':'T','C':'G','G':'C','T':'A'}
reads = [rs.read(i).decode().lower() for i in range(rs.nreads)]
idx = {}
for i, s in enumerate(reads):
    for o in range(len(s) - k + 1):
        w = s[o:o+k]
        if set(w) <= set('acgt'):
            idx.setdefault(w, []).append((i + 1, o))
def rc(s):
    m = {'a':'t','c':'g','g':'c','t':'a'}
    return ''.join(m.get(c, '\0') for c in reversed(s))
bad = 0
for a in range(1, rs.nreads + 1):
    s = reads[a - 1]
    cnt = 0
    for d, q in ((0, s), (1, rc(s))):
        for o in range(len(q) - k + 1):
            if o > 0 and q[o + k - 1] == '\0': break
            w = q[o:o+k]
            for (b, p) in idx.get(w, []):
                if b > a: cnt += 1
    oic.find_overlaps(a, a)
    g = oic.stats()['seed_hits']
    if g != cnt:
        bad += 1
        if bad < 6:
            print('read', a, 'gpu', g, 'py', cnt, 'has n', 'n' in s, 'len', len(s), 'n at', [i for i, c in enumerate(s) if c == 'n'])
print('bad', bad)
