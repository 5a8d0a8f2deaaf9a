"""CPU restatement of the MHAP MinHash sketch / filter stage (TEST INFRASTRUCTURE ONLY).

Only tests/, __graft_entry__.smoke() and bench_mhap.py's cpu_baseline leg use this module.

PARITY UNPINNED against MHAP itself.  The reference ships MHAP only as a prebuilt Java
archive (src/mhap/mhap-2.1.2.tar -> mhap-2.1.2.jar, third-party: MHAP 2.1.2, Berlin et al.,
Nat. Biotechnol. 33:623, 2015), which is never run or loaded here, and no Java toolchain is
present.  This module restates the published algorithm with the options canu passes
(src/pipelines/canu/OverlapMhap.pm:109-150, :381-392 / :481-493):
  --num-hashes H, --num-min-matches, --threshold, --ordered-sketch-size S,
  --ordered-kmer-size k', -k (MhapMerSize, Defaults.pm:704), --min-olap-length,
  -f <frequent k-mers> (filtered).
It is pinned instead to (a) the reference's CONSUMER of MHAP output, mhapConvert.C, built
from the reference sources (oracle/Makefile -> oracle/_ref/mhapConvert): every line we write
must pass its format asserts and convert to the ovOverlap records we expect
(tests/test_mhap.py), and (b) the GPU path, bit-exact on integers, erate within 1e-6.

The algorithm, as specified here (and implemented identically in canu_amd/csrc/mhap.hip):

Stage 1 -- MinHash sketch (MinHashSketch in MHAP):
  k-mers of A/C/G/T (any other byte breaks k-mers), 2 bits per base, first base most
  significant; canonical code c = min(fwd, revcomp); k-mers on the filter list dropped.
  x = splitmix64(c); for j in 0..H-1: x ^= x << 21; x ^= x >> 35 (logical); x ^= x << 4;
  sketch[j] = min over the read's k-mers of int32(low 32 bits of x).  A read with no
  k-mer has sketch[j] = INT32_MAX and never matches.
Stage 2 -- candidate search (the MinHash index): for query q and every other read t > q
  (each pair once), count(q, t) = #{j : sketch_q[j] == sketch_t[j] != INT32_MAX};
  candidates have count >= num-min-matches.
Stage 3 -- second-stage filter (OrderKmerHashes / the ordered sketch):
  per read, the S smallest distinct values h = high 32 bits of splitmix64(canonical k'-mer)
  with the k'-mer's forward position p and strand bit s (1 if revcomp < fwd); on equal h
  the smallest p is kept.  Only entries of the smallest 4096-bin (h >> 20) histogram bins
  that reach S entries are considered, at most 4096 of them (whole bins dropped from the
  top beyond that) -- this bounds the work per read; it changes the sketch only for reads
  with thousands of copies of one k'-mer.  For a candidate (A = q, B = t):
    shared = equal h in both sketches; orientation o = 0 if #(sA == sB) >= #(sA != sB)
    else 1 (B reverse-complemented); consistent = shared entries with (sA == sB) == (o == 0);
    pB' = pB (o = 0) or len(B) - k' - pB (o = 1); d = pA - pB';
    dm = lower median of d over the consistent entries (sorted, index (n - 1) // 2);
    A range [a_bgn, a_end) = [max(0, dm), min(len A, len B + dm)); must be >= min-olap-len;
    B' range = A range - dm;
    cA / cB = sketch entries whose k'-mer lies inside the A / B' range;
    m = consistent entries inside both ranges; J = m / (cA + cB - m);
    D = -ln(2J / (1 + J)) / k' (the Mash distance of Jaccard J); accept if 1 - D >= threshold;
    erate = min(D, 1).
Output (MHAP's text line, read by mhapConvert.C:114-150):
    a  b  erate  count  0  a_bgn  a_end  len_a  o  b_bgn  b_end  len_b
  with B's coordinates on the strand o (o = 1: on the reverse complement).
"""
from __future__ import annotations

import numpy as np

INT32_MAX = np.int32(0x7FFFFFFF)
NBIN = 4096          # ordered-sketch histogram bins (h >> 20)
OCAP = 4096          # most entries collected per read for the ordered sketch
U64 = np.uint64
M64 = (1 << 64) - 1

MHAP_DTYPE = np.dtype([("a", "<u4"), ("b", "<u4"), ("erate", "<f8"), ("count", "<u4"),
                       ("a_bgn", "<i4"), ("a_end", "<i4"), ("a_len", "<i4"), ("o", "<u4"),
                       ("b_bgn", "<i4"), ("b_end", "<i4"), ("b_len", "<i4")])

_CODE = np.full(256, 255, dtype=np.uint8)
for _c, _v in zip(b"ACGTacgt", (0, 1, 2, 3, 0, 1, 2, 3)):
    _CODE[_c] = _v


def default_params(**kw) -> dict:
    """canu's 'normal' sensitivity for correction (OverlapMhap.pm:116-121, Defaults.pm)."""
    p = dict(k=16, num_hashes=512, min_matches=3, threshold=0.78, ordered_sketch=1536,
             ordered_k=12, min_olap=500, repeat_weight=-1.0, repeat_idf_scale=10.0,
             filter_threshold=1e-5, no_tf=False, supress_noise=0)
    p.update(kw)
    return p


def splitmix64(c: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = c.astype(U64) + U64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> U64(30))) * U64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> U64(27))) * U64(0x94D049BB133111EB)
        return z ^ (z >> U64(31))


def kmers(seq_codes: np.ndarray, k: int):
    """(positions, canonical codes, strand bits) of the valid k-mers of one read."""
    n = seq_codes.shape[0]
    if n < k:
        e = np.zeros(0, dtype=np.int64)
        return e, np.zeros(0, dtype=U64), np.zeros(0, dtype=np.uint8)
    bad = seq_codes == 255
    b = np.where(bad, 0, seq_codes).astype(U64)
    fwd = np.zeros(n - k + 1, dtype=U64)
    rc = np.zeros(n - k + 1, dtype=U64)
    for t in range(k):
        fwd = (fwd << U64(2)) | b[t:n - k + 1 + t]
        rc = rc | ((U64(3) - b[t:n - k + 1 + t]) << U64(2 * t))
    cb = np.concatenate([[0], np.cumsum(bad)])
    ok = (cb[k:] - cb[:-k]) == 0
    pos = np.nonzero(ok)[0]
    f, r = fwd[ok], rc[ok]
    can = np.minimum(f, r)
    strand = (r < f).astype(np.uint8)
    return pos.astype(np.int64), can, strand


def read_codes(rs, i: int) -> np.ndarray:
    o, L = int(rs.offsets[i]), int(rs.lengths[i])
    return _CODE[np.frombuffer(rs.bases[o:o + L].tobytes(), dtype=np.uint8)]


def sketch(rs, p: dict, skip: np.ndarray | None = None) -> np.ndarray:
    """Stage 1: int32 [nreads, H]."""
    H, k = p["num_hashes"], p["k"]
    out = np.full((rs.nreads, H), INT32_MAX, dtype=np.int32)
    for i in range(rs.nreads):
        _, c, _ = kmers(read_codes(rs, i), k)
        if skip is not None and skip.size and c.size:
            c = c[~np.isin(c, skip)]
        if c.size == 0:
            continue
        x = splitmix64(c)
        with np.errstate(over="ignore"):
            for j in range(H):
                x ^= x << U64(21)
                x ^= x >> U64(35)
                x ^= x << U64(4)
                out[i, j] = (x & U64(0xFFFFFFFF)).astype(np.uint32).view(np.int32).min()
    return out


def kmer_multipliers(freq_kmers, fractions, p: dict):
    """The -f table of the weighted sketch (canu_amd mhap_set_kmer_frequencies, restated from
    MHAP 2.x's tf-idf; parity with the jar unpinned): canonical codes of the -f k-mers with
    a fraction >= filter_threshold (largest fraction per code), their multipliers
      m = r + (1 - r) * (1 + (X - 1) * (idf - idf_min) / (idf_max - idf_min)),
      idf = ln(1 / fraction), idf_max = ln(1 / filter_threshold), idf_min over the table,
    r = repeat_weight, X = repeat_idf_scale (m = 1 when r >= 1 or the table is empty), and
    the multiplier of every other k-mer (idf = idf_max).  Logs and arithmetic in Python
    floats (C doubles, libm log), in the library's order of operations.
    supress_noise (--supress-noise, canu_mhap.h): with a -f table, every listed k-mer is
    kept (below the threshold: idf = idf_max) and an unlisted k-mer's multiplier is that of
    the most frequent one (2) or -1, i.e. removed from the sketch (1)."""
    import math
    k, thr = p["k"], p["filter_threshold"]
    r, X = p["repeat_weight"], p["repeat_idf_scale"]
    noise = int(p.get("supress_noise", 0)) != 0 and len(freq_kmers) > 0
    best = {}
    for km, f in zip(freq_kmers, fractions):
        f = float(f)
        c = _CODE[np.frombuffer(km.encode() if isinstance(km, str) else km, dtype=np.uint8)]
        if c.shape[0] != k or (c == 255).any() or (not (f >= thr) and not noise):
            continue
        _, can, _ = kmers(c, k)
        cc = int(can[0])
        best[cc] = max(best.get(cc, f), f)
    codes = sorted(best)
    idf_max = math.log(1.0 / thr)
    idf = [math.log(1.0 / best[c]) if best[c] >= thr else idf_max for c in codes]
    idf_min = min([idf_max] + idf)

    def mult(v):
        if r >= 1.0 or not codes:
            return 1.0
        sc = 1.0 + (X - 1.0) * (v - idf_min) / (idf_max - idf_min) if idf_max > idf_min else X
        return r + (1.0 - r) * sc

    dm = mult(idf_max) if not noise else mult(idf_min) if int(p["supress_noise"]) == 2 else -1.0
    return (np.array(codes, dtype=U64), np.array([mult(v) for v in idf], dtype=np.float64), dm)


def sketch_weighted(rs, p: dict, freq=None) -> np.ndarray:
    """Stage 1 with repeat weighting (p["repeat_weight"] >= 0): every DISTINCT canonical
    k-mer c of a read, with tf = its occurrences (1 with no_tf) and multiplier m (the -f
    table, kmer_multipliers; m = 1 without one), has weight w = max(1, floor(tf * m + 0.5))
    and takes w consecutive steps of its xorshift64 chain (seeded by splitmix64(c)) per
    hash function j; sketch[j] = min over the read's k-mers and their w values of
    int32(low 32 bits).  With w = 1 everywhere this is sketch() exactly."""
    import math
    H, k = p["num_hashes"], p["k"]
    if freq is not None:
        fcodes, fmult, dmult = kmer_multipliers(freq[0], freq[1], p)
    else:
        fcodes, fmult, dmult = np.zeros(0, dtype=U64), np.zeros(0), 1.0
    out = np.full((rs.nreads, H), INT32_MAX, dtype=np.int32)
    for i in range(rs.nreads):
        _, c, _ = kmers(read_codes(rs, i), k)
        if c.size == 0:
            continue
        u, tf = np.unique(c, return_counts=True)
        if p.get("no_tf"):
            tf = np.ones_like(tf)
        m = np.full(u.shape[0], dmult, dtype=np.float64)
        if fcodes.size:
            q = np.searchsorted(fcodes, u)
            hit = (q < fcodes.size) & (fcodes[np.minimum(q, fcodes.size - 1)] == u)
            m[hit] = fmult[q[hit]]
        keep = m >= 0.0                        # --supress-noise 1: unlisted k-mers removed
        u, tf, m = u[keep], tf[keep], m[keep]
        if u.size == 0:
            continue
        w = np.array([max(1, int(math.floor(float(t) * float(mm) + 0.5)))
                      for t, mm in zip(tf.tolist(), m.tolist())], dtype=np.int64)
        x = splitmix64(u)
        wmax = int(w.max())
        with np.errstate(over="ignore"):
            for j in range(H):
                best = np.full(u.shape[0], INT32_MAX, dtype=np.int32)
                for t in range(wmax):
                    act = t < w
                    xa = x[act]
                    xa ^= xa << U64(21)
                    xa ^= xa >> U64(35)
                    xa ^= xa << U64(4)
                    x[act] = xa
                    v = (xa & U64(0xFFFFFFFF)).astype(np.uint32).view(np.int32)
                    best[act] = np.minimum(best[act], v)
                out[i, j] = best.min()
    return out


def ordered_sketch(rs, i: int, p: dict):
    """Stage 3 input for read i: (h uint32 ascending, pos int32, strand uint8)."""
    kk, S = p["ordered_k"], p["ordered_sketch"]
    pos, c, s = kmers(read_codes(rs, i), kk)
    h = (splitmix64(c) >> U64(32)).astype(np.uint32)
    # candidate entries: the 4096-bin histogram of h >> 20 picks the smallest bin B whose
    # cumulative count reaches S (the last bin if none does), then whole bins are dropped
    # from the top while more than OCAP entries would be collected (the GPU's LDS budget)
    bins = (h >> np.uint32(20)).astype(np.int64)
    cnt = np.bincount(bins, minlength=NBIN)
    cs = np.cumsum(cnt)
    reach = np.nonzero(cs >= S)[0]
    B = int(reach[0]) if reach.size else NBIN - 1
    tot = int(cs[B])
    while B >= 0 and tot > OCAP:
        tot -= int(cnt[B])
        B -= 1
    sel = bins <= B
    h, pos, s = h[sel], pos[sel], s[sel]
    order = np.lexsort((pos, h))                 # by h, then smallest position first
    h, pos, s = h[order], pos[order], s[order]
    keep = np.ones(h.shape[0], dtype=bool)
    keep[1:] = h[1:] != h[:-1]
    h, pos, s = h[keep][:S], pos[keep][:S], s[keep][:S]
    return h, pos.astype(np.int32), s


def candidates(sk: np.ndarray, q_range, min_matches: int, t_range=None):
    """Stage 2: [(q, t, count)] with t > q, 0-based read indices, sorted by (q, t).  With
    t_range ([lo, hi), 0-based: the jar's hash block) every t in it but q itself."""
    n = sk.shape[0]
    out = []
    for q in range(q_range[0], q_range[1]):
        lo, hi = (q + 1, n) if t_range is None else t_range
        if lo >= hi:
            continue
        eq = (sk[lo:hi] == sk[q][None, :]) & (sk[q][None, :] != INT32_MAX)
        cnt = eq.sum(axis=1)
        for t in np.nonzero(cnt >= min_matches)[0]:
            if lo + int(t) != q:
                out.append((q, lo + int(t), int(cnt[t])))
    return out


def compare(A, B, la: int, lb: int, p: dict):
    """Stage 3 for one candidate: None or (erate, a_bgn, a_end, o, b_bgn, b_end)."""
    kk = p["ordered_k"]
    ha, pa, sa = A
    hb, pb, sb = B
    common, ia, ib = np.intersect1d(ha, hb, assume_unique=True, return_indices=True)
    if common.size == 0:
        return None
    same = sa[ia] == sb[ib]
    o = 0 if int(same.sum()) >= int((~same).sum()) else 1
    cons = same if o == 0 else ~same
    ia, ib = ia[cons], ib[cons]
    if ia.size == 0:
        return None
    pA = pa[ia].astype(np.int64)
    pB = pb[ib].astype(np.int64) if o == 0 else (lb - kk - pb[ib].astype(np.int64))
    d = np.sort(pA - pB)
    dm = int(d[(d.size - 1) // 2])
    a_bgn, a_end = max(0, dm), min(la, lb + dm)
    if a_end - a_bgn < p["min_olap"]:
        return None
    b_bgn, b_end = a_bgn - dm, a_end - dm
    pa_all = pa.astype(np.int64)
    pb_all = pb.astype(np.int64) if o == 0 else (lb - kk - pb.astype(np.int64))
    cA = int(((pa_all >= a_bgn) & (pa_all <= a_end - kk)).sum())
    cB = int(((pb_all >= b_bgn) & (pb_all <= b_end - kk)).sum())
    inside = (pA >= a_bgn) & (pA <= a_end - kk) & (pB >= b_bgn) & (pB <= b_end - kk)
    m = int(inside.sum())
    if m == 0:
        return None
    J = m / (cA + cB - m)
    D = -np.log(2.0 * J / (1.0 + J)) / kk
    if 1.0 - D < p["threshold"]:
        return None
    return (min(D, 1.0), a_bgn, a_end, o, b_bgn, b_end)


def run(rs, p: dict, q_range=None, skip_kmers=None, t_range=None, freq=None) -> np.ndarray:
    """All-vs-all over rs (queries in q_range, 0-based [lo, hi)): MHAP_DTYPE records with
    1-based read IDs (rs.first_iid based), sorted by (a, b).  t_range (0-based [lo, hi)):
    the targets are the reads in it (every one but the query), not the later reads.
    p["repeat_weight"] >= 0: weighted sketches (sketch_weighted, -f table freq =
    (k-mers, fractions) or none)."""
    skip = None
    if skip_kmers:
        codes = []
        for s in skip_kmers:
            c = _CODE[np.frombuffer(s.encode() if isinstance(s, str) else s, dtype=np.uint8)]
            _, can, _ = kmers(c, p["k"])
            codes.extend(can.tolist())
        skip = np.unique(np.array(codes, dtype=U64))
    q_range = q_range or (0, rs.nreads)
    if p.get("repeat_weight", -1.0) >= 0:
        sk = sketch_weighted(rs, p, freq)
    else:
        sk = sketch(rs, p, skip)
    cands = candidates(sk, q_range, p["min_matches"], t_range)
    cache = {}

    def osk(i):
        if i not in cache:
            cache[i] = ordered_sketch(rs, i, p)
        return cache[i]

    rows = []
    for q, t, cnt in cands:
        la, lb = int(rs.lengths[q]), int(rs.lengths[t])
        r = compare(osk(q), osk(t), la, lb, p)
        if r is None:
            continue
        er, a0, a1, o, b0, b1 = r
        rows.append((rs.first_iid + q, rs.first_iid + t, er, cnt, a0, a1, la, o, b0, b1, lb))
    return np.array(rows, dtype=MHAP_DTYPE)
