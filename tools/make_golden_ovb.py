#!/usr/bin/env python3
"""Generate tests/golden/basic_ref.ovb and basic_ref.counts: the output files the REFERENCE
overlapInCore (oracle/_ref/oic_ref, one thread) writes with its own ovFile for the "basic"
golden read set -- the byte-level fixtures for the library's .ovb/.counts writer.

    python tools/make_golden_ovb.py          # needs oracle/_ref/oic_ref
"""
from __future__ import annotations

import os
import shutil
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import oracle  # noqa: E402
from test_oracle import load_golden  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden")


def main() -> None:
    if not oracle.reference_available():
        sys.exit("oracle/_ref/oic_ref is missing: run `make -C oracle`")
    rs, p, skip, _ = load_golden("basic")
    wd = tempfile.mkdtemp(prefix="ovbgold_")
    try:
        oracle.run_reference(rs, p, threads=1, workdir=wd)
        shutil.copy(os.path.join(wd, "w", "ref.ovb"), os.path.join(OUT, "basic_ref.ovb"))
        shutil.copy(os.path.join(wd, "w", "ref.counts"), os.path.join(OUT, "basic_ref.counts"))
    finally:
        shutil.rmtree(wd)
    print("wrote", os.path.join(OUT, "basic_ref.ovb"), os.path.join(OUT, "basic_ref.counts"))


if __name__ == "__main__":
    main()
