"""Host side of the MHAP stage: ctypes binding of libcanu_mhap.so (include/canu_mhap.h) and
the MHAP command-line options canu passes (src/pipelines/canu/OverlapMhap.pm:374-498).

There is no CPU fallback: every compute call goes to the gfx950 library, and loading it
fails loudly when it was not built."""
from __future__ import annotations

import ctypes
import dataclasses
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "lib", "libcanu_mhap.so")

# the C struct mhap_record
MHAP_DTYPE = np.dtype([("a", "<u4"), ("b", "<u4"), ("erate", "<f8"), ("raw", "<f8"),
                       ("a_bgn", "<i4"), ("a_end", "<i4"), ("a_len", "<i4"), ("o", "<u4"),
                       ("b_bgn", "<i4"), ("b_end", "<i4"), ("b_len", "<i4"),
                       ("count", "<u4")], align=True)

EXPORTS = ["mhap_params_init", "mhap_ctx_create", "mhap_ctx_destroy", "mhap_last_error",
           "mhap_abi_version", "mhap_load_reads", "mhap_load_reads_device",
           "mhap_set_weighting", "mhap_sketch", "mhap_sketch_buffers", "mhap_copy_sketches",
           "mhap_build_index", "mhap_build_index_range", "mhap_compare_all",
           "mhap_copy_sketches_host", "mhap_weighting_init", "mhap_set_kmer_frequencies",
           "mhap_set_kmer_frequencies_ex",
           "mhap_compare", "mhap_fetch", "mhap_write_text", "mhap_format_line",
           "mhap_get_stats"]

ABI_VERSION = 7          # MHAP_ABI_VERSION of include/canu_mhap.h


class MhapError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"[{code}] {msg}")
        self.code = code


class _Params(ctypes.Structure):
    _fields_ = [("k", ctypes.c_uint32), ("num_hashes", ctypes.c_uint32),
                ("min_matches", ctypes.c_uint32), ("ordered_sketch", ctypes.c_uint32),
                ("ordered_k", ctypes.c_uint32), ("min_olap", ctypes.c_int32),
                ("threshold", ctypes.c_double), ("max_shift", ctypes.c_double),
                ("min_store", ctypes.c_int32), ("no_rc", ctypes.c_int32)]


class _Weighting(ctypes.Structure):
    _fields_ = [("repeat_weight", ctypes.c_double), ("repeat_idf_scale", ctypes.c_double),
                ("filter_threshold", ctypes.c_double), ("no_tf", ctypes.c_int32),
                ("supress_noise", ctypes.c_int32)]


class _Stats(ctypes.Structure):
    _fields_ = [("sketched_reads", ctypes.c_uint64), ("candidates", ctypes.c_uint64),
                ("overlaps", ctypes.c_uint64), ("ms_sketch", ctypes.c_double),
                ("ms_index", ctypes.c_double), ("ms_candidates", ctypes.c_double),
                ("ms_compare", ctypes.c_double), ("sketch_kmers", ctypes.c_uint64),
                ("ms_sketch_kernel", ctypes.c_double), ("sketch_launches", ctypes.c_uint64),
                ("sketch_draws", ctypes.c_uint64)]


_lib = None


def load_library(path: str | None = None):
    global _lib
    if _lib is not None:
        return _lib
    path = path or os.environ.get("CANU_MHAP_LIB") or LIB_PATH
    if not os.path.exists(path):
        raise MhapError(-1, f"{path} missing: run __graft_entry__.build()")
    lib = ctypes.CDLL(path)
    # the structs below mirror include/canu_mhap.h of this ABI: refuse a stale library
    if lib.mhap_abi_version() != ABI_VERSION:
        raise MhapError(-1, f"{path} has ABI {lib.mhap_abi_version()}, this binding expects "
                            f"{ABI_VERSION}: rebuild with __graft_entry__.build()")
    P, V, U32, U64 = ctypes.POINTER, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64
    lib.mhap_params_init.argtypes = [P(_Params)]
    lib.mhap_ctx_create.argtypes = [P(_Params), ctypes.c_int, P(V)]
    lib.mhap_ctx_destroy.argtypes = [V]
    lib.mhap_last_error.restype = ctypes.c_char_p
    lib.mhap_load_reads.argtypes = [V, U32, U32, V, V, V]
    lib.mhap_load_reads_device.argtypes = [V, U32, U32, V, V, V]
    lib.mhap_set_weighting.argtypes = [V, P(_Weighting)]
    lib.mhap_sketch.argtypes = [V, U32, U32]
    lib.mhap_sketch_buffers.argtypes = [V, P(V), P(V), P(V)]
    lib.mhap_copy_sketches.argtypes = [V, U32, U32, V, V, V, ctypes.c_int]
    lib.mhap_build_index.argtypes = [V]
    lib.mhap_build_index_range.argtypes = [V, U32, U32]
    lib.mhap_copy_sketches_host.argtypes = [V, U32, U32, V, V, V, ctypes.c_int]
    lib.mhap_compare_all.argtypes = [V, U32, U32, P(U64)]
    lib.mhap_compare.argtypes = [V, U32, U32, P(U64)]
    lib.mhap_fetch.argtypes = [V, V, U64, P(U64)]
    lib.mhap_write_text.argtypes = [V, ctypes.c_char_p, U32, U32, U32]
    lib.mhap_format_line.argtypes = [V, U32, U32, U32, ctypes.c_char_p, ctypes.c_size_t]
    lib.mhap_get_stats.argtypes = [V, P(_Stats)]
    lib.mhap_weighting_init.argtypes = [P(_Weighting)]
    lib.mhap_set_kmer_frequencies.argtypes = [V, ctypes.c_char_p, V, U64, P(_Weighting)]
    lib.mhap_set_kmer_frequencies_ex.argtypes = [V, ctypes.c_char_p, V, U64, U64, P(_Weighting)]
    _lib = lib
    return lib


@dataclasses.dataclass
class MhapParameters:
    """MHAP options canu sets (OverlapMhap.pm:109-150, :380-392; Defaults.pm:698-706) and
    the jar's own defaults for the rest (MhapMain.<init> option table)."""
    k: int = 16
    num_hashes: int = 512
    num_min_matches: int = 3
    threshold: float = 0.78
    ordered_sketch_size: int = 1536
    ordered_kmer_size: int = 12
    min_olap_length: int = 500
    max_shift: float = 0.2
    min_store_length: int = 0
    no_rc: bool = False
    # repeat weighting (canu_mhap.h mhap_weighting; the jar's defaults 0.9 / 3 / 1e-5, canu
    # passes --repeat-weight 0.9 --repeat-idf-scale 10 --filter-threshold, OverlapMhap.pm:382,
    # :390); without -f frequencies a k-mer weighs its count (repeat_weight >= 0) or 1
    repeat_weight: float = 0.9
    repeat_idf_scale: float = 3.0
    filter_threshold: float = 1e-5
    no_tf: bool = False
    # --supress-noise (canu: 2 with mhapFilterUnique, OverlapMhap.pm:483): with a -f table, 1
    # keeps only k-mers the jar's Guava Bloom filter of the file's keys accepts (keepKmer),
    # 2 builds that filter and never reads it
    supress_noise: int = 0

    @classmethod
    def sensitivity(cls, level: str, tag: str = "cor", nanopore: bool = False,
                    ordered_mer: int | None = None, min_olap: int = 500) -> "MhapParameters":
        """The presets of OverlapMhap.pm:109-150 ('low' / 'normal' / 'high', +0.05
        threshold for nanopore-raw libraries, obt/utg hash count override)."""
        om = ordered_mer if ordered_mer is not None else (12 if tag == "cor" else 18)
        if level == "low":
            p = cls(num_hashes=256, num_min_matches=3, threshold=0.80, ordered_sketch_size=1000,
                    ordered_kmer_size=om + 2)
        elif level == "normal":
            p = cls(num_hashes=512, num_min_matches=3, threshold=0.78, ordered_sketch_size=1536,
                    ordered_kmer_size=om)
        elif level == "high":
            p = cls(num_hashes=768, num_min_matches=2, threshold=0.73, ordered_sketch_size=1536,
                    ordered_kmer_size=om)
        else:
            raise ValueError(f"invalid MhapSensitivity={level}")
        if nanopore:
            p.threshold += 0.05
        if tag in ("obt", "utg"):
            p.num_hashes, p.num_min_matches = 128, 5
        p.min_olap_length = min_olap
        return p

    def to_c(self) -> _Params:
        return _Params(self.k, self.num_hashes, self.num_min_matches, self.ordered_sketch_size,
                       self.ordered_kmer_size, self.min_olap_length, self.threshold,
                       self.max_shift, self.min_store_length, 1 if self.no_rc else 0)

    def weighting_c(self) -> _Weighting:
        return _Weighting(self.repeat_weight, self.repeat_idf_scale, self.filter_threshold,
                          1 if self.no_tf else 0, int(self.supress_noise))

    def canu_weighting(self, filter_threshold: float = 0.000005) -> "MhapParameters":
        """The weighting canu always asks the jar for (OverlapMhap.pm:382, :390;
        mhapFilterThreshold, Defaults.pm:699)."""
        self.repeat_weight, self.repeat_idf_scale = 0.9, 10.0
        self.filter_threshold = filter_threshold
        return self

    def as_oracle(self) -> dict:
        return dict(k=self.k, num_hashes=self.num_hashes, min_matches=self.num_min_matches,
                    threshold=self.threshold, ordered_sketch=self.ordered_sketch_size,
                    ordered_k=self.ordered_kmer_size, min_olap=self.min_olap_length,
                    repeat_weight=self.repeat_weight, repeat_idf_scale=self.repeat_idf_scale,
                    filter_threshold=self.filter_threshold, no_tf=bool(self.no_tf),
                    supress_noise=int(self.supress_noise), max_shift=self.max_shift,
                    min_store=self.min_store_length, no_rc=bool(self.no_rc))


def parse_mhap_args(argv: list[str]) -> tuple[MhapParameters, dict]:
    """The jar's options as canu writes them (OverlapMhap.pm:380-395, :480-495).  Options
    that only steer the jar's own I/O (-p, -q, -s, --num-threads, ...) are returned in the
    second dict; weighting options this build does not implement raise."""
    p = MhapParameters()
    io: dict = {}
    i = 0
    while i < len(argv):
        a = argv[i]
        val = argv[i + 1] if i + 1 < len(argv) else None
        if a == "-k":
            p.k = int(val); i += 1
        elif a == "--num-hashes":
            p.num_hashes = int(val); i += 1
        elif a == "--num-min-matches":
            p.num_min_matches = int(val); i += 1
        elif a == "--threshold":
            p.threshold = float(val); i += 1
        elif a == "--ordered-sketch-size":
            p.ordered_sketch_size = int(val); i += 1
        elif a == "--ordered-kmer-size":
            p.ordered_kmer_size = int(val); i += 1
        elif a == "--min-olap-length":
            p.min_olap_length = int(val); i += 1
        elif a == "--max-shift":
            p.max_shift = float(val); i += 1
        elif a == "--min-store-length":
            p.min_store_length = int(val); i += 1
        elif a == "--no-rc":
            p.no_rc = True
        elif a in ("-f", "-p", "-q", "-s", "--num-threads"):
            io[a] = val; i += 1
        elif a == "--repeat-weight":
            p.repeat_weight = float(val); i += 1
        elif a == "--repeat-idf-scale":
            p.repeat_idf_scale = float(val); i += 1
        elif a == "--filter-threshold":
            p.filter_threshold = float(val); i += 1
        elif a == "--no-tf":
            p.no_tf = True
        elif a in ("--no-self",):
            io[a] = True
        elif a == "--supress-noise":
            p.supress_noise = int(val); i += 1
            if p.supress_noise not in (0, 1, 2):
                raise MhapError(-2, f"--supress-noise {val}: 0, 1 or 2")
        else:
            raise MhapError(-2, f"unknown MHAP option '{a}'")
        i += 1
    return p, io


def read_frequency_file(path: str, k: int, with_count: bool = False):
    """The -f file canu writes (Meryl.pm:699-716): optionally gzipped, a first line with
    the number of k-mer lines, then "kmer<TAB>fraction" lines (both strands).  Returns
    (k-mers, fractions), with_count: and the count line's value (the number of k-mer lines
    when the file has none), which sizes the jar's --supress-noise Bloom filter."""
    import gzip
    op = gzip.open if path.endswith(".gz") else open
    kmers, fr = [], []
    count = None
    with op(path, "rt") as f:
        for j, line in enumerate(f):
            parts = line.split()
            if not parts:
                continue
            if j == 0 and len(parts) == 1 and parts[0].isdigit():
                count = int(parts[0])
                continue                                   # the count line
            if len(parts[0]) != k:
                raise MhapError(-4, f"{path}:{j + 1}: k-mer of length {len(parts[0])}, not {k}")
            kmers.append(parts[0])
            fr.append(float(parts[1]) if len(parts) > 1 else 1.0)
    if with_count:
        return kmers, np.asarray(fr, dtype=np.float64), len(kmers) if count is None else count
    return kmers, np.asarray(fr, dtype=np.float64)


class Mhap:
    """One MHAP job on one gfx950 device: load -> sketch -> index -> compare -> fetch."""

    def __init__(self, params: MhapParameters, device: int = 0):
        self.lib = load_library()
        self.params = params
        cp = params.to_c()
        ctx = ctypes.c_void_p()
        self._check(self.lib.mhap_ctx_create(ctypes.byref(cp), device, ctypes.byref(ctx)))
        self.ctx = ctx
        self.first_iid, self.nreads = 1, 0

    def _check(self, rc: int):
        if rc != 0:
            raise MhapError(rc, self.lib.mhap_last_error().decode())

    def close(self):
        if getattr(self, "ctx", None):
            self.lib.mhap_ctx_destroy(self.ctx)
            self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def load_reads(self, rs) -> None:
        bases = np.ascontiguousarray(rs.bases, dtype=np.uint8)
        offs = np.ascontiguousarray(rs.offsets, dtype=np.uint64)
        lens = np.ascontiguousarray(rs.lengths, dtype=np.uint32)
        self._check(self.lib.mhap_load_reads(self.ctx, rs.first_iid, rs.nreads,
                                             bases.ctypes.data, offs.ctypes.data,
                                             lens.ctypes.data))
        self.first_iid, self.nreads = rs.first_iid, rs.nreads

    def load_reads_device(self, first_iid: int, d_bases: int, d_offsets: int,
                          lengths: np.ndarray) -> None:
        lens = np.ascontiguousarray(lengths, dtype=np.uint32)
        self._check(self.lib.mhap_load_reads_device(self.ctx, first_iid, lens.shape[0],
                                                    d_bases, d_offsets, lens.ctypes.data))
        self.first_iid, self.nreads = first_iid, int(lens.shape[0])

    def set_weighting(self) -> None:
        """This job's weighting options (params.repeat_weight ...) without a -f table."""
        w = self.params.weighting_c()
        self._check(self.lib.mhap_set_weighting(self.ctx, ctypes.byref(w)))

    def set_kmer_frequencies(self, kmers: list[str], fractions, expected: int | None = None
                             ) -> None:
        """-f with fractions (file order), under this job's weighting options; expected = the
        file's count line (sizes --supress-noise's Bloom filter; None: the number of lines)."""
        blob = "".join(kmers).encode()
        fr = np.ascontiguousarray(fractions, dtype=np.float64)
        w = self.params.weighting_c()
        n = len(kmers)
        self._check(self.lib.mhap_set_kmer_frequencies_ex(
            self.ctx, blob, fr.ctypes.data if fr.size else None, n,
            n if expected is None else int(expected), ctypes.byref(w)))

    def sketch(self, bgn: int | None = None, end: int | None = None) -> None:
        bgn = self.first_iid if bgn is None else bgn
        end = self.first_iid + self.nreads - 1 if end is None else end
        self._check(self.lib.mhap_sketch(self.ctx, bgn, end))

    def sketch_buffers(self) -> tuple[int, int, int]:
        a, b, c = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_void_p()
        self._check(self.lib.mhap_sketch_buffers(self.ctx, ctypes.byref(a), ctypes.byref(b),
                                                 ctypes.byref(c)))
        return a.value, b.value, c.value

    def copy_sketches(self, first_iid: int, n: int, d_minhash: int, d_ordered: int,
                      d_ocount: int, to_ctx: bool) -> None:
        """Export (to_ctx=False) / import (True) the sketch rows of n reads from first_iid
        to / from caller device buffers (e.g. torch tensors' data_ptr())."""
        self._check(self.lib.mhap_copy_sketches(self.ctx, first_iid, n, d_minhash, d_ordered,
                                                d_ocount, 1 if to_ctx else 0))

    def build_index(self, bgn: int | None = None, end: int | None = None) -> None:
        """Index every loaded read, or reads bgn..end only (the jar's hash block)."""
        if bgn is None and end is None:
            self._check(self.lib.mhap_build_index(self.ctx))
        else:
            bgn = self.first_iid if bgn is None else bgn
            end = self.first_iid + self.nreads - 1 if end is None else end
            self._check(self.lib.mhap_build_index_range(self.ctx, bgn, end))

    def compare(self, bgn: int | None = None, end: int | None = None,
                all_targets: bool = False) -> int:
        """The jar's self search: queries bgn..end (forward strands) against the indexed
        strands of reads with smaller IDs; or (all_targets, the -q search) against every
        indexed read but themselves."""
        bgn = self.first_iid if bgn is None else bgn
        end = self.first_iid + self.nreads - 1 if end is None else end
        n = ctypes.c_uint64()
        fn = self.lib.mhap_compare_all if all_targets else self.lib.mhap_compare
        self._check(fn(self.ctx, bgn, end, ctypes.byref(n)))
        return n.value

    def fetch(self) -> np.ndarray:
        n = self.stats()["overlaps"]
        rec = np.zeros(max(n, 1), dtype=MHAP_DTYPE)
        got = ctypes.c_uint64()
        self._check(self.lib.mhap_fetch(self.ctx, rec.ctypes.data, n, ctypes.byref(got)))
        return rec[:got.value]

    def write_text(self, path: str, hash_base: int = 1, num_hash: int | None = None,
                   query_base: int = 1) -> None:
        nh = self.nreads if num_hash is None else num_hash
        self._check(self.lib.mhap_write_text(self.ctx, path.encode(), hash_base, nh, query_base))

    def stats(self) -> dict:
        s = _Stats()
        self._check(self.lib.mhap_get_stats(self.ctx, ctypes.byref(s)))
        return {f: getattr(s, f) for f, _ in _Stats._fields_}

    def run(self, rs, frequencies=None) -> np.ndarray:
        """The jar's self job over rs (-s block without --no-self): records sorted by
        (a, b, o), a the query (larger ID).  frequencies = (k-mers, fractions) of a -f
        file."""
        self.load_reads(rs)
        if frequencies is not None:
            km, fr = frequencies[0], frequencies[1]
            self.set_kmer_frequencies(list(km), fr,
                                      frequencies[2] if len(frequencies) > 2 else None)
        else:
            self.set_weighting()
        self.sketch()
        self.build_index()
        self.compare()
        return self.fetch()


def java_fixed6(x: float) -> str:
    """String.format("%.6f", x) as Java does it: the shortest decimal that reads back as x
    (FloatingDecimal), rounded half-up to 6 places (FormattedFloatingDecimal)."""
    from decimal import Decimal, ROUND_HALF_UP
    return str(Decimal(repr(float(x))).quantize(Decimal("0.000001"), rounding=ROUND_HALF_UP))


def format_line(r, hash_base: int = 1, num_hash: int = 0, query_base: int = 1) -> str:
    """One record as MatchResult.toString's line (the layout mhap_write_text writes)."""
    w0 = int(r["a"]) - (query_base - 1) + num_hash
    w1 = int(r["b"]) - (hash_base - 1)
    return (f"{w0} {w1} {java_fixed6(r['erate'])} {java_fixed6(r['raw'])} 0 "
            f"{int(r['a_bgn'])} {int(r['a_end'])} {int(r['a_len'])} {int(r['o'])} "
            f"{int(r['b_bgn'])} {int(r['b_end'])} {int(r['b_len'])}")
