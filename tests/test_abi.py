"""The drop-in boundary: libcanu_ovl.so loads, exports exactly what include/canu_ovl.h
declares, and behaves on the host without a GPU (no compute calls here)."""
import ctypes
import os
import re

import numpy as np
import pytest

from canu_amd import overlap_in_core as oic

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "canu_ovl.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(ovl_[a-z_]+)\s*\(", src)))


def test_header_declares_the_python_exports():
    assert declared_functions() == sorted(oic.EXPORTS)


def test_library_exports_every_declared_symbol(built):
    lib = oic.load_library()
    missing = [f for f in declared_functions() if not hasattr(lib, f)]
    assert not missing, missing


def test_abi_version(built):
    assert oic.load_library().ovl_abi_version() == 8


def test_driver_defaults_match_reference(built):
    """ovl_driver_params_init / ovl_hash_limits_init = oicParameters::initialize()
    (overlapInCore.H:429-450): -h / -r 1-UINT32_MAX, 10000 strings, 1e8 bases, 22 bits,
    load 0.6, all libraries, one thread."""
    lib = oic.load_library()
    d = oic._DriverParams()
    lib.ovl_driver_params_init(ctypes.byref(d))
    assert (d.bgn_hash_iid, d.end_hash_iid, d.bgn_ref_iid, d.end_ref_iid) == \
        (1, 0xFFFFFFFF, 1, 0xFFFFFFFF)
    assert (d.min_lib_ref, d.max_lib_ref, d.num_threads, d.store_num_reads) == (0, 0xFFFFFFFF, 1, 0)
    L = d.limits
    assert (L.max_hash_strings, L.max_hash_data_len, L.hash_mask_bits) == (10000, 100000000, 22)
    assert abs(L.max_hash_load - 0.6) < 1e-15
    assert (L.min_lib_hash, L.max_lib_hash) == (0, 0xFFFFFFFF)
    assert ctypes.sizeof(oic._HashLimits) == 40 and ctypes.sizeof(oic._DriverParams) == 72


@pytest.mark.gpu
def test_failed_load_leaves_no_reads(built):
    """A load the GPU path rejects leaves the context without reads: a later build is a
    call-order error, not a kernel over stale buffers."""
    o = oic.OverlapInCore(oic.OicParameters(Kmer_Len=22), device=0)
    lib = o.lib
    bases = np.frombuffer(b"ACGTXACGT" * 100, dtype=np.uint8).copy()
    offs = np.array([0], dtype=np.uint64)
    lens = np.array([bases.shape[0]], dtype=np.uint32)
    rc = lib.ovl_load_reads(o.ctx, 1, 1, bases.ctypes.data, offs.ctypes.data,
                            lens.ctypes.data, None)
    assert rc == -4
    assert lib.ovl_build_hash_index(o.ctx, 1, 1) == -7
    n = ctypes.c_uint64()
    assert lib.ovl_find_overlaps(o.ctx, 1, 1, ctypes.byref(n)) == -7
    o.close()


def test_params_init_matches_reference_defaults(built):
    """ovl_params_init = oicParameters::initialize() (overlapInCore.H:425)."""
    lib = oic.load_library()
    p = oic._Params()
    lib.ovl_params_init(ctypes.byref(p))
    assert p.kmer_len == 0
    assert p.min_olap_len == 0
    assert p.partial == 0 and p.unique_olap_per_pair == 1
    assert p.use_window_filter == 0 and p.use_hopeless_check == 1
    assert p.frag_olap_limit == (1 << 64) - 1 and p.filter_by_kmer_count == 0
    assert abs(p.max_erate - 0.06) < 1e-12


def test_params_finalize_erate_fixups(built):
    """main(): maxErate > 0.06 turns off the window filter and the hopeless check."""
    lib = oic.load_library()
    p = oic._Params()
    lib.ovl_params_init(ctypes.byref(p))
    p.kmer_len = 16
    p.max_erate = 0.144
    p.use_window_filter = 1
    lib.ovl_params_finalize(ctypes.byref(p))
    assert p.use_window_filter == 0 and p.use_hopeless_check == 0


def test_ctx_create_fails_loudly_without_gpu(built):
    """No silent CPU fallback: without a gfx950 device the context cannot be created."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    lib = oic.load_library()
    cp = oic.OicParameters(Kmer_Len=22).to_c()
    ctx = ctypes.c_void_p()
    rc = lib.ovl_ctx_create(ctypes.byref(cp), 0, ctypes.byref(ctx))
    assert rc == -1 and not ctx.value
    assert b"device" in lib.ovl_last_error()
    with pytest.raises(oic.OvlError):
        oic.OverlapInCore(oic.OicParameters(Kmer_Len=22), device=0)


def test_ctx_create_rejects_bad_params(built):
    lib = oic.load_library()
    cp = oic.OicParameters(Kmer_Len=0).to_c()
    ctx = ctypes.c_void_p()
    assert lib.ovl_ctx_create(ctypes.byref(cp), 0, ctypes.byref(ctx)) == -2


def test_missing_library_raises(tmp_path, monkeypatch):
    monkeypatch.setattr(oic, "_lib", None)
    with pytest.raises(oic.OvlError):
        oic.load_library(str(tmp_path / "nope.so"))


def test_record_layout():
    """ovl_record = {uint32 a_iid, uint32 b_iid, uint64 dat[2]} (ovOverlap.H:270)."""
    assert ctypes.sizeof(oic._Record) == 24
    assert oic.RECORD_DTYPE.itemsize == 24
    r = np.zeros(1, dtype=oic.RECORD_DTYPE)
    assert r.dtype.names == ("a", "b", "w0", "w1")


def test_struct_layouts_match_header(tmp_path):
    """The ctypes mirrors of ovl_stats and ovl_index_desc have the header's sizes and field
    offsets (compiled against include/canu_ovl.h with the host C compiler)."""
    import subprocess
    inc = os.path.join(ROOT, "include")
    src = tmp_path / "layout.c"
    src.write_text(
        '#include <stddef.h>\n#include <stdio.h>\n#include "canu_ovl.h"\n'
        'int main(void) { printf("%zu %zu %zu %zu %zu %zu\\n", sizeof(ovl_stats), '
        'offsetof(ovl_stats, sq_resorted), offsetof(ovl_stats, query_chunks), '
        'offsetof(ovl_stats, find_releases), '
        'sizeof(ovl_index_desc), offsetof(ovl_index_desc, read_flags_bytes)); return 0; }\n')
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-std=c99", "-I", inc, str(src), "-o", str(exe)], check=True)
    got = [int(x) for x in subprocess.run([str(exe)], capture_output=True, text=True,
                                          check=True).stdout.split()]
    assert got == [ctypes.sizeof(oic._Stats), oic._Stats.sq_resorted.offset,
                   oic._Stats.query_chunks.offset, oic._Stats.find_releases.offset,
                   ctypes.sizeof(oic._IndexDesc),
                   oic._IndexDesc.read_flags_bytes.offset]
