"""Host-side mirror of canu's overlapInCore interface over the MI355X C-ABI.

Names follow the reference: `OicParameters` is oicParameters (overlapInCore.H:418) and
`parse_overlapInCore_args` accepts overlapInCore's own options (overlapInCore.C:316-412).
`OverlapInCore` drives what OverlapDriver() does (overlapInCore.C:190): load the reads,
Build_Hash_Index over the -h range, search the -r range in both orientations, and hand
back ovOverlap records.  Everything runs in libcanu_ovl.so on a gfx950 device; there is
no CPU fallback -- a missing library or device raises.
"""
from __future__ import annotations

import ctypes
import dataclasses
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "lib", "libcanu_ovl.so")

RECORD_DTYPE = np.dtype([("a", "<u4"), ("b", "<u4"), ("w0", "<u8"), ("w1", "<u8")])
# ovl_seed_hit: query, target, query window | orientation << 31, target offset
SEED_HIT_DTYPE = np.dtype([("a", "<u4"), ("b", "<u4"), ("a_pos_dir", "<u4"), ("b_pos", "<u4")])

OVL_STATUS = {0: "OVL_OK", -1: "OVL_ERR_NO_DEVICE", -2: "OVL_ERR_BAD_PARAM",
              -3: "OVL_ERR_UNSUPPORTED", -4: "OVL_ERR_BAD_INPUT", -5: "OVL_ERR_HIP",
              -6: "OVL_ERR_OOM", -7: "OVL_ERR_STATE"}

UINT64_MAX = (1 << 64) - 1


class OvlError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"{OVL_STATUS.get(code, code)}: {msg}")
        self.code = code


class _Params(ctypes.Structure):
    _fields_ = [("kmer_len", ctypes.c_uint32), ("max_erate", ctypes.c_double),
                ("min_olap_len", ctypes.c_int32), ("partial", ctypes.c_int32),
                ("unique_olap_per_pair", ctypes.c_int32), ("use_window_filter", ctypes.c_int32),
                ("use_hopeless_check", ctypes.c_int32), ("frag_olap_limit", ctypes.c_uint64),
                ("filter_by_kmer_count", ctypes.c_uint64)]


class _Record(ctypes.Structure):
    _fields_ = [("a_iid", ctypes.c_uint32), ("b_iid", ctypes.c_uint32),
                ("dat", ctypes.c_uint64 * 2)]


class _Stats(ctypes.Structure):
    _fields_ = [(n, ctypes.c_uint64) for n in (
        "kmer_hits_without_olap", "kmer_hits_with_olap", "kmer_hits_skipped", "multi_overlaps",
        "total_overlaps", "contained_overlaps", "dovetail_overlaps", "seed_hits", "pairs")] + \
        [("ms_index", ctypes.c_double), ("ms_seed", ctypes.c_double),
         ("ms_extend", ctypes.c_double), ("ms_probe_kernel", ctypes.c_double),
         ("probe_bytes", ctypes.c_uint64), ("probe_launches", ctypes.c_uint32),
         ("extend_launches", ctypes.c_uint32), ("bad_short_window", ctypes.c_uint64),
         ("bad_long_window", ctypes.c_uint64), ("hash_batches", ctypes.c_uint64),
         ("ref_reads", ctypes.c_uint64), ("multi_pass_units", ctypes.c_uint64),
         ("chain_retries", ctypes.c_uint64), ("ms_seed_hits", ctypes.c_double),
         ("staged_pairs", ctypes.c_uint64), ("long_pairs", ctypes.c_uint64),
         ("generic_pairs", ctypes.c_uint64), ("ext_waves", ctypes.c_uint32),
         ("generic_waves", ctypes.c_uint32), ("stage_len", ctypes.c_uint32),
         ("long_stage_len", ctypes.c_uint32), ("seed_nodes", ctypes.c_uint64),
         ("probe_sorted_launches", ctypes.c_uint32), ("sq_resorted", ctypes.c_uint32),
         ("query_chunks", ctypes.c_uint32), ("super_batches", ctypes.c_uint32),
         ("sq_declined", ctypes.c_uint32), ("find_releases", ctypes.c_uint32)]


class _IndexDesc(ctypes.Structure):
    """ovl_index_desc (include/canu_ovl.h, ABI 7+): a built index as device buffers."""
    _fields_ = [(n, ctypes.c_uint32) for n in (
        "bgn_iid", "end_iid", "first_iid", "nreads", "kmer_len", "tab_bits", "slice_bits",
        "bloom_w", "hash_lib_lo", "hash_lib_hi")] + \
        [("records", ctypes.c_uint64),
         ("table", ctypes.c_void_p), ("table_bytes", ctypes.c_uint64),
         ("occ", ctypes.c_void_p), ("occ_bytes", ctypes.c_uint64),
         ("bloom", ctypes.c_void_p), ("bloom_bytes", ctypes.c_uint64),
         ("read_flags", ctypes.c_void_p), ("read_flags_bytes", ctypes.c_uint64)]


class _HashLimits(ctypes.Structure):
    _fields_ = [("max_hash_strings", ctypes.c_uint32), ("max_hash_data_len", ctypes.c_uint64),
                ("hash_mask_bits", ctypes.c_uint32), ("max_hash_load", ctypes.c_double),
                ("min_lib_hash", ctypes.c_uint32), ("max_lib_hash", ctypes.c_uint32)]


class _DriverParams(ctypes.Structure):
    _fields_ = [("bgn_hash_iid", ctypes.c_uint32), ("end_hash_iid", ctypes.c_uint32),
                ("bgn_ref_iid", ctypes.c_uint32), ("end_ref_iid", ctypes.c_uint32),
                ("min_lib_ref", ctypes.c_uint32), ("max_lib_ref", ctypes.c_uint32),
                ("num_threads", ctypes.c_uint32), ("store_num_reads", ctypes.c_uint32),
                ("limits", _HashLimits)]


# Every symbol include/canu_ovl.h declares (tests check the library exports them all).
EXPORTS = ["ovl_params_init", "ovl_params_finalize", "ovl_ctx_create", "ovl_ctx_destroy",
           "ovl_last_error", "ovl_abi_version", "ovl_load_reads", "ovl_load_reads_device",
           "ovl_set_skip_kmers", "ovl_build_hash_index", "ovl_find_overlaps",
           "ovl_fetch_overlaps", "ovl_get_stats", "ovl_ctx_stream", "ovl_write_ovb",
           "ovl_ctx_write_ovb", "ovl_ctx_write_stats", "ovl_set_read_libraries",
           "ovl_hash_limits_init", "ovl_build_hash_batch", "ovl_driver_params_init",
           "ovl_overlap_driver", "ovl_seed_hits", "ovl_probe_ceiling", "ovl_probe_replay",
           "ovl_export_index", "ovl_import_index"]

_lib = None


ABI_VERSION = 8          # OVL_ABI_VERSION of include/canu_ovl.h


def load_library(path: str | None = None):
    """Load libcanu_ovl.so.  Raises if it was not built -- there is no fallback.
    CANU_OVL_LIB names another build of the same library (e.g. the profiling build)."""
    global _lib
    if _lib is not None:
        return _lib
    path = path or os.environ.get("CANU_OVL_LIB") or LIB_PATH
    if not os.path.exists(path):
        raise OvlError(-1, f"{path} missing: run __graft_entry__.build()")
    lib = ctypes.CDLL(path)
    # the structs below mirror include/canu_ovl.h of this ABI: a library of another ABI
    # would read or write past them (ovl_stats grew in ABI 3)
    if lib.ovl_abi_version() != ABI_VERSION:
        raise OvlError(-1, f"{path} has ABI {lib.ovl_abi_version()}, this binding expects "
                           f"{ABI_VERSION}: rebuild with __graft_entry__.build()")
    P = ctypes.POINTER
    lib.ovl_params_init.argtypes = [P(_Params)]
    lib.ovl_params_finalize.argtypes = [P(_Params)]
    lib.ovl_ctx_create.argtypes = [P(_Params), ctypes.c_int, P(ctypes.c_void_p)]
    lib.ovl_ctx_destroy.argtypes = [ctypes.c_void_p]
    lib.ovl_last_error.restype = ctypes.c_char_p
    lib.ovl_load_reads.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32,
                                   ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                   ctypes.c_void_p]
    lib.ovl_load_reads_device.argtypes = lib.ovl_load_reads.argtypes
    lib.ovl_set_skip_kmers.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_uint64]
    lib.ovl_build_hash_index.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32]
    lib.ovl_find_overlaps.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32,
                                      P(ctypes.c_uint64)]
    lib.ovl_fetch_overlaps.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                       P(ctypes.c_uint64)]
    lib.ovl_get_stats.argtypes = [ctypes.c_void_p, P(_Stats)]
    lib.ovl_probe_ceiling.argtypes = [ctypes.c_void_p, P(ctypes.c_double), P(ctypes.c_uint64)]
    lib.ovl_probe_replay.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32,
                                     P(ctypes.c_double), P(ctypes.c_uint64)]
    lib.ovl_ctx_stream.argtypes = [ctypes.c_void_p]
    lib.ovl_ctx_stream.restype = ctypes.c_void_p
    lib.ovl_write_ovb.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_char_p, ctypes.c_int]
    lib.ovl_ctx_write_ovb.argtypes = [ctypes.c_void_p, ctypes.c_char_p]
    lib.ovl_ctx_write_stats.argtypes = [ctypes.c_void_p, ctypes.c_char_p]
    lib.ovl_set_read_libraries.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    lib.ovl_hash_limits_init.argtypes = [P(_HashLimits)]
    lib.ovl_build_hash_batch.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32,
                                         P(_HashLimits), P(ctypes.c_uint32)]
    lib.ovl_driver_params_init.argtypes = [P(_DriverParams)]
    lib.ovl_overlap_driver.argtypes = [ctypes.c_void_p, P(_DriverParams), P(ctypes.c_uint64)]
    lib.ovl_seed_hits.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32,
                                  ctypes.c_void_p, ctypes.c_uint64, P(ctypes.c_uint64)]
    lib.ovl_export_index.argtypes = [ctypes.c_void_p, P(_IndexDesc)]
    lib.ovl_import_index.argtypes = [ctypes.c_void_p, P(_IndexDesc)]
    _lib = lib
    return lib


@dataclasses.dataclass
class OicParameters:
    """oicParameters (overlapInCore.H:418-530), the options this path honours."""
    Kmer_Len: int = 0
    maxErate: float = 0.06
    Min_Olap_Len: int = 0
    Doing_Partial_Overlaps: bool = False
    Unique_Olap_Per_Pair: bool = True
    Use_Window_Filter: bool = False
    Use_Hopeless_Check: bool = True
    Frag_Olap_Limit: int = UINT64_MAX
    Filter_By_Kmer_Count: int = 0
    bgnHashID: int = 1
    endHashID: int = 0xFFFFFFFF
    bgnRefID: int = 1
    endRefID: int = 0xFFFFFFFF
    minLibToHash: int = 0
    maxLibToHash: int = 0xFFFFFFFF
    minLibToRef: int = 0
    maxLibToRef: int = 0xFFFFFFFF
    Hash_Mask_Bits: int = 22
    Max_Hash_Load: float = 0.6
    Max_Hash_Strings: int = 10000
    Max_Hash_Data_Len: int = 100000000
    Num_PThreads: int = 1

    def finalize(self) -> "OicParameters":
        """main()'s fix-ups after option parsing (overlapInCore.C:416-421)."""
        if self.maxErate > 0.06:
            self.Use_Window_Filter = False
            self.Use_Hopeless_Check = False
        return self

    def to_c(self) -> _Params:
        return _Params(kmer_len=self.Kmer_Len, max_erate=self.maxErate,
                       min_olap_len=self.Min_Olap_Len, partial=int(self.Doing_Partial_Overlaps),
                       unique_olap_per_pair=int(self.Unique_Olap_Per_Pair),
                       use_window_filter=int(self.Use_Window_Filter),
                       use_hopeless_check=int(self.Use_Hopeless_Check),
                       frag_olap_limit=self.Frag_Olap_Limit,
                       filter_by_kmer_count=self.Filter_By_Kmer_Count)

    def driver_c(self, store_num_reads: int = 0) -> _DriverParams:
        d = _DriverParams()
        load_library().ovl_driver_params_init(ctypes.byref(d))
        d.bgn_hash_iid, d.end_hash_iid = self.bgnHashID, min(self.endHashID, 0xFFFFFFFF)
        d.bgn_ref_iid, d.end_ref_iid = self.bgnRefID, min(self.endRefID, 0xFFFFFFFF)
        d.min_lib_ref, d.max_lib_ref = self.minLibToRef, self.maxLibToRef
        d.num_threads = self.Num_PThreads
        d.store_num_reads = store_num_reads
        L = d.limits
        L.max_hash_strings, L.max_hash_data_len = self.Max_Hash_Strings, self.Max_Hash_Data_Len
        L.hash_mask_bits, L.max_hash_load = self.Hash_Mask_Bits, self.Max_Hash_Load
        L.min_lib_hash, L.max_lib_hash = self.minLibToHash, self.maxLibToHash
        return d

    def as_dict(self) -> dict:
        return dict(kmer_len=self.Kmer_Len, max_erate=self.maxErate,
                    min_olap_len=self.Min_Olap_Len, partial=int(self.Doing_Partial_Overlaps),
                    unique_olap_per_pair=int(self.Unique_Olap_Per_Pair),
                    use_window_filter=int(self.Use_Window_Filter),
                    use_hopeless_check=int(self.Use_Hopeless_Check),
                    frag_olap_limit=self.Frag_Olap_Limit,
                    filter_by_kmer_count=self.Filter_By_Kmer_Count)


def _decode_range(s: str) -> tuple[int, int]:
    """AS_UTL_decodeRange: 'a-b' or 'a'."""
    if "-" in s:
        a, b = s.split("-", 1)
        return int(a), int(b)
    return int(s), int(s)


def parse_overlapInCore_args(argv: list[str]) -> tuple[OicParameters, dict]:
    """Parse overlapInCore's command line (overlapInCore.C:316-412) the way main() does:
    --maxerate through strtof (a float), --minkmers evaluated where it appears."""
    P = OicParameters()
    extra = {"skip_file": None, "store": None, "output": None, "threads": 1, "stats": None}
    i = 0
    while i < len(argv):
        a = argv[i]
        if a == "-G":
            P.Doing_Partial_Overlaps = True
        elif a == "-h":
            i += 1; P.bgnHashID, P.endHashID = _decode_range(argv[i])
        elif a == "-r":
            i += 1; P.bgnRefID, P.endRefID = _decode_range(argv[i])
        elif a == "-H":
            i += 1; P.minLibToHash, P.maxLibToHash = _decode_range(argv[i])
        elif a == "-R":
            i += 1; P.minLibToRef, P.maxLibToRef = _decode_range(argv[i])
        elif a == "--hashbits":
            i += 1; P.Hash_Mask_Bits = int(argv[i])
        elif a == "--hashstrings":
            i += 1; P.Max_Hash_Strings = int(argv[i])
        elif a == "--hashdatalen":
            i += 1; P.Max_Hash_Data_Len = int(argv[i])
        elif a == "--hashload":
            i += 1; P.Max_Hash_Load = float(argv[i])
        elif a == "-s":
            i += 1; extra["stats"] = argv[i]
        elif a == "-k":
            i += 1
            v = argv[i]
            if v.isdigit() and len(v) <= 2:
                P.Kmer_Len = int(v)
            else:
                extra["skip_file"] = v
        elif a == "-l":
            i += 1
            v = int(argv[i])
            P.Frag_Olap_Limit = UINT64_MAX if v < 1 else v
        elif a == "-m":
            P.Unique_Olap_Per_Pair = False
        elif a == "-u":
            P.Unique_Olap_Per_Pair = True
        elif a == "--minlength":
            i += 1; P.Min_Olap_Len = int(argv[i])
        elif a == "--minkmers":
            P.Filter_By_Kmer_Count = int(np.floor(np.exp(-1.0 * P.Kmer_Len * P.maxErate) *
                                                  (P.Min_Olap_Len - P.Kmer_Len + 1)))
        elif a == "--maxerate":
            i += 1; P.maxErate = float(np.float32(float(argv[i])))
        elif a == "-w":
            P.Use_Window_Filter = True
        elif a == "-z":
            P.Use_Hopeless_Check = False
        elif a == "-o":
            i += 1; extra["output"] = argv[i]
        elif a == "-t":
            i += 1; extra["threads"] = P.Num_PThreads = int(argv[i])
        elif a == "--maxreadlen":
            i += 1      # the CPU table's bit packing of (read, offset); no limit here
        else:
            extra["store"] = a
        i += 1
    P.finalize()
    return P, extra


def read_skip_fasta(path: str, k: int) -> list[str]:
    """The -k <frequentMers.fasta> file: '>' line then one k-mer line (Mark_Skip_Kmers)."""
    out = []
    with open(path) as f:
        lines = f.read().split("\n")
    for j in range(0, len(lines) - 1, 2):
        if not lines[j].startswith(">"):
            raise ValueError(f"bad skip-kmer line {j + 1}")
        km = lines[j + 1].strip()
        if len(km) != k:
            raise ValueError(f"bad skip-kmer line {j + 2}")
        out.append(km)
    return out


class OverlapInCore:
    """One overlapInCore job on one gfx950 device (one process per GPU)."""

    def __init__(self, params: OicParameters, device: int = 0):
        self.lib = load_library()
        self.params = params
        cp = params.to_c()
        ctx = ctypes.c_void_p()
        self._check(self.lib.ovl_ctx_create(ctypes.byref(cp), device, ctypes.byref(ctx)))
        self.ctx = ctx
        self.first_iid = 1
        self.nreads = 0

    def _check(self, rc: int):
        if rc != 0:
            raise OvlError(rc, self.lib.ovl_last_error().decode())

    def close(self):
        if getattr(self, "ctx", None):
            self.lib.ovl_ctx_destroy(self.ctx)
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
        quals = None if rs.quals is None else np.ascontiguousarray(rs.quals, dtype=np.uint8)
        self._check(self.lib.ovl_load_reads(self.ctx, rs.first_iid, rs.nreads,
                                            bases.ctypes.data, offs.ctypes.data,
                                            lens.ctypes.data,
                                            None if quals is None else quals.ctypes.data))
        self.first_iid = rs.first_iid
        self.nreads = rs.nreads

    def load_reads_device(self, first_iid: int, d_bases: int, d_offsets: int,
                          lengths: np.ndarray) -> None:
        """Reads already in HBM (device pointers, e.g. from torch tensors)."""
        lens = np.ascontiguousarray(lengths, dtype=np.uint32)
        self._check(self.lib.ovl_load_reads_device(self.ctx, first_iid, lens.shape[0],
                                                   d_bases, d_offsets, lens.ctypes.data, None))
        self.first_iid = first_iid
        self.nreads = int(lens.shape[0])

    def set_skip_kmers(self, kmers: list[str]) -> None:
        blob = "".join(kmers).encode()
        self._check(self.lib.ovl_set_skip_kmers(self.ctx, blob, len(kmers)))

    def build_hash_index(self, bgn: int | None = None, end: int | None = None) -> None:
        bgn = self.params.bgnHashID if bgn is None else bgn
        end = self.params.endHashID if end is None else end
        self._check(self.lib.ovl_build_hash_index(self.ctx, bgn, min(end, 0xFFFFFFFF)))

    def find_overlaps(self, bgn: int | None = None, end: int | None = None) -> int:
        bgn = self.params.bgnRefID if bgn is None else bgn
        end = self.params.endRefID if end is None else end
        n = ctypes.c_uint64()
        self._check(self.lib.ovl_find_overlaps(self.ctx, bgn, min(end, 0xFFFFFFFF),
                                               ctypes.byref(n)))
        return n.value

    def fetch(self, n: int | None = None) -> np.ndarray:
        if n is None:
            n = self.stats()["total_overlaps"]
        rec = np.zeros(max(n, 1), dtype=RECORD_DTYPE)
        got = ctypes.c_uint64()
        self._check(self.lib.ovl_fetch_overlaps(self.ctx, rec.ctypes.data, n,
                                                ctypes.byref(got)))
        return rec[:got.value]

    def stats(self) -> dict:
        s = _Stats()
        self._check(self.lib.ovl_get_stats(self.ctx, ctypes.byref(s)))
        return {f: getattr(s, f) for f, _ in _Stats._fields_}

    def stream(self) -> int:
        return self.lib.ovl_ctx_stream(self.ctx)

    def probe_ceiling(self) -> tuple[float, int]:
        """(G random 16-B loads/s over the current index table's allocation, its bytes):
        the ceiling of one random lookup per query window here (ovl_probe_ceiling)."""
        g, b = ctypes.c_double(), ctypes.c_uint64()
        self._check(self.lib.ovl_probe_ceiling(self.ctx, ctypes.byref(g), ctypes.byref(b)))
        return g.value, b.value

    def probe_replay(self, bgn: int, end: int) -> tuple[float, int]:
        """(G loads/s, windows): the probe's own table lookups for the query windows of reads
        bgn..end (first 2^28) replayed as pure loads (ovl_probe_replay)."""
        g, n = ctypes.c_double(), ctypes.c_uint64()
        self._check(self.lib.ovl_probe_replay(self.ctx, bgn, end, ctypes.byref(g),
                                              ctypes.byref(n)))
        return g.value, n.value

    def write_ovb(self, path: str) -> None:
        """overlapInCore's -o output: the last find's records as an .ovb + .counts."""
        self._check(self.lib.ovl_ctx_write_ovb(self.ctx, path.encode()))

    def write_stats(self, path: str) -> None:
        """overlapInCore's -s statistics file."""
        self._check(self.lib.ovl_ctx_write_stats(self.ctx, path.encode()))

    def set_read_libraries(self, libs) -> None:
        lib = np.ascontiguousarray(libs, dtype=np.uint32)
        assert lib.shape[0] == self.nreads
        self._check(self.lib.ovl_set_read_libraries(self.ctx, lib.ctypes.data))

    def build_hash_batch(self, bgn: int, end: int) -> int:
        """Build_Hash_Index(gkpStore, bgn, end): returns the last ID the batch loaded."""
        d = self.params.driver_c()
        last = ctypes.c_uint32()
        self._check(self.lib.ovl_build_hash_batch(self.ctx, bgn, min(end, 0xFFFFFFFF),
                                                  ctypes.byref(d.limits), ctypes.byref(last)))
        return last.value

    def overlap_driver(self, store_num_reads: int = 0) -> int:
        """OverlapDriver(): every hash batch of the -h range searched by the -r reads."""
        d = self.params.driver_c(store_num_reads)
        n = ctypes.c_uint64()
        self._check(self.lib.ovl_overlap_driver(self.ctx, ctypes.byref(d), ctypes.byref(n)))
        return n.value

    def run_driver(self, rs, skip_kmers=None) -> np.ndarray:
        """The whole overlapInCore job (hash batches, Process_Overlaps' ref schedule)."""
        self.load_reads(rs)
        if skip_kmers:
            self.set_skip_kmers(skip_kmers)
        return self.fetch(self.overlap_driver())

    def seed_hits(self, bgn: int | None = None, end: int | None = None,
                  fetch: bool = True) -> np.ndarray | int:
        """The Add_Ref hit list of the ref reads against the current index (SEED_HIT_DTYPE,
        reference order); fetch=False only counts (the lookup still runs in full)."""
        bgn = self.params.bgnRefID if bgn is None else bgn
        end = min(self.params.endRefID if end is None else end, 0xFFFFFFFF)
        n = ctypes.c_uint64()
        self._check(self.lib.ovl_seed_hits(self.ctx, bgn, end, None, 0, ctypes.byref(n)))
        if not fetch:
            return n.value
        h = np.zeros(max(n.value, 1), dtype=SEED_HIT_DTYPE)
        self._check(self.lib.ovl_seed_hits(self.ctx, bgn, end, h.ctypes.data, n.value,
                                           ctypes.byref(n)))
        return h[:n.value]

    def export_index(self) -> "_IndexDesc":
        """The context's built index as device buffers (valid until its next build)."""
        d = _IndexDesc()
        self._check(self.lib.ovl_export_index(self.ctx, ctypes.byref(d)))
        return d

    def import_index(self, desc: "_IndexDesc") -> None:
        """Copy an exported index (this GPU, a peer, or buffers a collective filled) into
        this context, which then searches it as if it had built it."""
        self._check(self.lib.ovl_import_index(self.ctx, ctypes.byref(desc)))

    def run(self, rs, skip_kmers=None) -> np.ndarray:
        """OverlapDriver() for one hash batch: load, index, search, fetch (sorted)."""
        self.load_reads(rs)
        if skip_kmers:
            self.set_skip_kmers(skip_kmers)
        self.build_hash_index()
        n = self.find_overlaps()
        return self.fetch(n)


def write_ovb(records: np.ndarray, path: str, counts: bool = True) -> None:
    """Write ovOverlap records (RECORD_DTYPE, in the given order) as an ovFileFullWrite
    .ovb (src/stores/ovStoreFile.C:198) plus its .counts file (ovStoreHistogram.C:322)."""
    lib = load_library()
    rec = np.ascontiguousarray(records, dtype=RECORD_DTYPE)
    rc = lib.ovl_write_ovb(rec.ctypes.data if rec.size else None, rec.shape[0],
                           path.encode(), 1 if counts else 0)
    if rc != 0:
        raise OvlError(rc, lib.ovl_last_error().decode())
