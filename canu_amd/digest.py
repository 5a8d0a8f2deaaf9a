"""Size-independent digests of ovOverlap record sets (parity at the benchmark's full size).

Two digests of a record multiset, both independent of the order the records come out in:

* `sha256_sorted` -- SHA-256 of the 24-byte records sorted by ovOverlap::operator<
  (a_iid, b_iid, dat) -- the order ovStore keeps them in (ovOverlap.H:300).
* `multiset_hash` -- the sum mod 2^64 of a 64-bit mix of every record.  Additive, so the
  query shards of a multi-GPU job each hash their own records and the ranks' sums add up
  to the whole job's (no records move between ranks).

Both are computed on the host from the records a job hands back; the reference's values
for the bench workload are committed in tests/golden/bench50k.json (tools/make_bench_digest.py
runs the reference overlapInCore, built from its own sources, on the bench's exact reads).
"""
from __future__ import annotations

import hashlib

import numpy as np

RECORD_DTYPE = np.dtype([("a", "<u4"), ("b", "<u4"), ("w0", "<u8"), ("w1", "<u8")])
_M64 = (1 << 64) - 1


def sort_records(rec: np.ndarray) -> np.ndarray:
    """ovOverlap::operator< order: a_iid, b_iid, then the packed dat words."""
    return rec[np.lexsort((rec["w1"], rec["w0"], rec["b"], rec["a"]))]


def sha256_sorted(rec: np.ndarray) -> str:
    r = np.ascontiguousarray(sort_records(np.asarray(rec, dtype=RECORD_DTYPE)))
    return hashlib.sha256(r.tobytes()).hexdigest()


def _mix64(x: np.ndarray) -> np.ndarray:
    """splitmix64's finaliser, lane-wise on uint64 (wrapping arithmetic)."""
    x = x ^ (x >> np.uint64(30))
    x = x * np.uint64(0xBF58476D1CE4E5B9)
    x = x ^ (x >> np.uint64(27))
    x = x * np.uint64(0x94D049BB133111EB)
    return x ^ (x >> np.uint64(31))


def record_hashes(rec: np.ndarray) -> np.ndarray:
    r = np.asarray(rec, dtype=RECORD_DTYPE)
    ab = r["a"].astype(np.uint64) | (r["b"].astype(np.uint64) << np.uint64(32))
    with np.errstate(over="ignore"):
        h = _mix64(ab ^ np.uint64(0x9E3779B97F4A7C15))
        h = _mix64(h ^ r["w0"])
        return _mix64(h ^ r["w1"])


def multiset_hash(rec: np.ndarray) -> int:
    """Sum mod 2^64 of record_hashes (order-independent, additive over shards)."""
    h = record_hashes(rec)
    if h.size == 0:
        return 0
    # exact modular sum: split into 32-bit halves so nothing overflows silently
    lo = int(np.sum(h & np.uint64(0xFFFFFFFF), dtype=np.uint64))
    hi = int(np.sum(h >> np.uint64(32), dtype=np.uint64))
    return (lo + (hi << 32)) & _M64


def combine(hashes) -> int:
    """The multiset hash of a union of disjoint record sets."""
    s = 0
    for h in hashes:
        s = (s + int(h)) & _M64
    return s
