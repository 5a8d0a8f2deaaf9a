import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 device (runs on the GPU box)")


@pytest.fixture(scope="session")
def built():
    import __graft_entry__
    __graft_entry__.build()
    return True
