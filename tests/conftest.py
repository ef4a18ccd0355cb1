import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "deflate.hpp_amd")
for p in (PKG, os.path.dirname(os.path.abspath(__file__))):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 GPU (run on the MI355X box)")


@pytest.fixture(scope="session")
def ctx():
    import dmx
    c = dmx.Context()
    yield c
    c.close()


@pytest.fixture(scope="session")
def oracle():
    from oracle_bind import Oracle
    return Oracle()
