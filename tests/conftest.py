import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

# torch first: it and libcanu_ovl.so both need libamdhip64.so.7, and the process keeps the
# first one loaded.  bench.py and smoke() load torch's before the library; so do the tests
# (with the library's /opt/rocm runtime loaded first, torch's HIP init fails)
import torch  # noqa: E402,F401


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 device (runs on the GPU box)")


def pytest_collection_finish(session):
    # Large synthetic read sets are generated here, before any test touches the GPU: after
    # that, synth_reads_parallel generates serially (no pool forked from a GPU process), and
    # 2M x 12 kb serially is minutes of silence in the middle of the suite.
    if session.config.option.collectonly:
        return
    for item in session.items:
        pre = getattr(item.module, "pregenerate", None)
        if pre is not None and item.get_closest_marker("gpu") is not None:
            pre()


@pytest.fixture(scope="session")
def built():
    import __graft_entry__
    __graft_entry__.build()
    return True
