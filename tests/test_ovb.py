"""overlapInCore's output files written by the library (canu_amd/csrc/ovl_ovb.h):
the .ovb (ovFile full-write format, snappy-framed blocks) and the .counts histogram,
checked against the files the REFERENCE overlapInCore wrote for the "basic" golden set
(tests/golden/basic_ref.*, tools/make_golden_ovb.py) and, where oracle/_ref/oic_ref is
built, read back by the reference's own ovFile reader."""
import os
import struct

import numpy as np
import pytest

import oracle
from canu_amd import overlap_in_core as oic
from test_oracle import load_golden

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def snappy_decode(buf: bytes) -> bytes:
    """Raw snappy stream -> bytes (the published format: varint length, then literal and
    copy elements).  Test-only decoder for reading the reference's .ovb blocks."""
    n, shift, i = 0, 0, 0
    while True:
        b = buf[i]
        i += 1
        n |= (b & 0x7F) << shift
        shift += 7
        if not b & 0x80:
            break
    out = bytearray()
    while i < len(buf):
        tag = buf[i]
        i += 1
        kind = tag & 3
        if kind == 0:
            ln = tag >> 2
            if ln >= 60:
                nb = ln - 59
                ln = int.from_bytes(buf[i:i + nb], "little")
                i += nb
            ln += 1
            out += buf[i:i + ln]
            i += ln
            continue
        if kind == 1:
            ln = ((tag >> 2) & 7) + 4
            off = ((tag >> 5) << 8) | buf[i]
            i += 1
        elif kind == 2:
            ln = (tag >> 2) + 1
            off = int.from_bytes(buf[i:i + 2], "little")
            i += 2
        else:
            ln = (tag >> 2) + 1
            off = int.from_bytes(buf[i:i + 4], "little")
            i += 4
        for _ in range(ln):
            out.append(out[-off])
    assert len(out) == n
    return bytes(out)


def read_ovb_py(path: str) -> np.ndarray:
    """Records of a snappy-framed full .ovb in file order (ovStoreFile.C:266 readBuffer)."""
    data = open(path, "rb").read()
    words = []
    i = 0
    while i < len(data):
        (cl,) = struct.unpack_from("<Q", data, i)
        i += 8
        words.append(np.frombuffer(snappy_decode(data[i:i + cl]), dtype="<u4"))
        i += cl
    w = np.concatenate(words) if words else np.zeros(0, dtype="<u4")
    w = w.reshape(-1, 6).astype(np.uint64)
    rec = np.zeros(w.shape[0], dtype=oracle.RECORD_DTYPE)
    rec["a"] = w[:, 0]
    rec["b"] = w[:, 1]
    rec["w0"] = (w[:, 2] << np.uint64(32)) | w[:, 3]
    rec["w1"] = (w[:, 4] << np.uint64(32)) | w[:, 5]
    return rec


@pytest.fixture(scope="module")
def ref_file_order():
    return read_ovb_py(os.path.join(GOLDEN, "basic_ref.ovb"))


def test_reference_ovb_fixture_holds_the_golden_records(ref_file_order):
    _, _, _, want = load_golden("basic")
    assert np.array_equal(oracle.sort_records(ref_file_order), want)


def test_counts_file_is_byte_identical(built, tmp_path, ref_file_order):
    want = open(os.path.join(GOLDEN, "basic_ref.counts"), "rb").read()
    for order, rec in (("file", ref_file_order), ("sorted", oracle.sort_records(ref_file_order))):
        p = str(tmp_path / f"{order}.ovb")
        oic.write_ovb(rec, p)
        assert open(str(tmp_path / f"{order}.counts"), "rb").read() == want, order


def test_ovb_round_trip(built, tmp_path, ref_file_order):
    p = str(tmp_path / "job.ovb")
    oic.write_ovb(ref_file_order, p)
    assert np.array_equal(read_ovb_py(p), ref_file_order)


def test_counts_name_follows_findBaseFileName(built, tmp_path, ref_file_order):
    """canu writes '-o ./001.ovb.WORKING' and stashes '001.counts' (OverlapInCore.pm)."""
    p = str(tmp_path / "001.ovb.WORKING")
    oic.write_ovb(ref_file_order[:5], p)
    assert os.path.exists(str(tmp_path / "001.counts"))


def test_multi_block_and_empty(built, tmp_path):
    """More than one 43,680-record block, and an empty job."""
    n = 100_000
    rng = np.random.default_rng(5)
    rec = np.zeros(n, dtype=oracle.RECORD_DTYPE)
    rec["a"] = rng.integers(1, 5000, n)
    rec["b"] = rng.integers(1, 5000, n)
    rec["w0"] = rng.integers(0, 1 << 63, n, dtype=np.uint64)
    rec["w1"] = rng.integers(0, 1 << 63, n, dtype=np.uint64)
    p = str(tmp_path / "big.ovb")
    oic.write_ovb(rec, p)
    assert np.array_equal(read_ovb_py(p), rec)
    opr = np.fromfile(str(tmp_path / "big.counts"), dtype="<u4")
    assert opr[0] == max(rec["a"].max(), rec["b"].max()) + 1
    assert opr[1:].sum() == 2 * n
    e = str(tmp_path / "empty.ovb")
    oic.write_ovb(rec[:0], e)
    assert os.path.getsize(e) == 0
    assert np.fromfile(str(tmp_path / "empty.counts"), dtype="<u4").tolist() == [0]


@pytest.mark.skipif(not oracle.reference_available(), reason="oracle/_ref/oic_ref not built")
def test_reference_reader_reads_our_ovb(built, tmp_path, ref_file_order):
    """The reference's ovFile(…, ovFileFull)::readOverlap decodes our file to the same
    records in the same order, across several blocks."""
    rec = np.concatenate([ref_file_order] * 300)          # 132,300 records: 4 blocks
    p = str(tmp_path / "ours.ovb")
    oic.write_ovb(rec, p)
    got = oracle.read_ovb_reference(p)
    assert np.array_equal(got, rec)
    assert np.array_equal(oracle.read_ovb_reference(os.path.join(GOLDEN, "basic_ref.ovb")),
                          ref_file_order)
