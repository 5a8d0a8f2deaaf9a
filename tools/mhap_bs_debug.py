#!/usr/bin/env python3
"""Bit-sliced MinHash draws vs the exact path and the restatement on test_mhap's weighted
'canu' case: prints the (read, strand, function) entries that differ.
    python tools/mhap_bs_debug.py"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import torch  # noqa: E402,F401
import mhap_jar as M  # noqa: E402
from canu_amd import mhap  # noqa: E402
from test_mhap import _reads, _rows, _freq_for  # noqa: E402


def run(rs, P, freq, env):
    for k in ("MHAP_BITSLICE", "MHAP_BS_ZMAX"):
        os.environ.pop(k, None)
    os.environ.update(env)
    m = mhap.Mhap(P, device=0)
    m.load_reads(rs)
    m.set_kmer_frequencies(*freq)
    m.sketch()
    got = _rows(m, rs.nreads, P)
    m.close()
    return got


def main():
    rs = _reads(n=24, L=3000, cov=8, seed=19)
    P = mhap.MhapParameters(num_hashes=48, ordered_sketch_size=600, ordered_kmer_size=14,
                            min_olap_length=300).canu_weighting()
    freq = _freq_for(rs)
    want = M.sketch_rows(rs, P.as_oracle(), freq)
    for name, env in (("exact", {"MHAP_BITSLICE": "0"}), ("bitslice", {}),
                      ("bitslice_z0", {"MHAP_BS_ZMAX": "0"}),
                      ("bitslice_z6", {"MHAP_BS_ZMAX": "6"})):
        mh = run(rs, P, freq, env)[0]
        bad = np.argwhere(mh != want[0])
        print(name, "mismatches:", len(bad), flush=True)
        for r, st, j in bad[:12]:
            print("  read", r, "strand", st, "j", j, "gpu", mh[r, st, j], "want",
                  want[0][r, st, j], "len", rs.lengths[r])


if __name__ == "__main__" and not os.environ.get("DUMP_CHECK"):
    main()


def dump_check():
    """MHAP_BS_DUMP: the exact pass's per-strand minima against the restatement's minima over
    the same k-mers (the first 2048 sorted positions, and every k-mer of another weight)."""
    rs = _reads(n=24, L=3000, cov=8, seed=19)
    P = mhap.MhapParameters(num_hashes=48, ordered_sketch_size=600, ordered_kmer_size=14,
                            min_olap_length=300).canu_weighting()
    freq = _freq_for(rs)
    path = os.path.join(ROOT, "gpurun_out", "bsdump.bin")
    run(rs, P, freq, {"MHAP_BS_DUMP": path})
    raw = open(path, "rb").read()
    nb = np.frombuffer(raw[:4], dtype=np.uint32)[0]
    sids = np.frombuffer(raw[4:4 + 4 * nb], dtype=np.uint32)
    cnt = np.frombuffer(raw[4 + 4 * nb:4 + 8 * nb], dtype=np.uint32)
    rec = np.frombuffer(raw[4 + 8 * nb:], dtype=[("val", "<i8"), ("fp", "<u4"), ("v", "<u4")])
    rec = rec.reshape(nb, -1)
    print("strands", nb, "listed", cnt.tolist())
    print("fp==NONE entries per strand", [(int(sids[b]), int((rec[b]["fp"] == 0xFFFFFFFF).sum())) for b in range(nb)])
    print("val==0 entries per strand", [(int(sids[b]), int((rec[b]["val"] == 0).sum())) for b in range(nb)])


if __name__ == "__main__" and os.environ.get("DUMP_CHECK"):
    dump_check()
