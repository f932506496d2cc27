import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "tensorkrylov.jl_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU and libtkhip.so")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def ctx():
    import tkamd
    c = tkamd.Context(0)
    yield c
    c.close()
