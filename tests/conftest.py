import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "large-scale-recommendation_amd"), os.path.join(ROOT, "oracle"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libmfhip on the device)")


@pytest.fixture(scope="session", autouse=True)
def _built():
    """Make sure the native artefacts exist (build() is idempotent and fast when up to date)."""
    import __graft_entry__ as g
    lib = os.path.join(ROOT, "large-scale-recommendation_amd", "lib", "libmfhip.so")
    orc = os.path.join(ROOT, "oracle", "build", "libmforacle.so")
    if not (os.path.exists(lib) and os.path.exists(orc)):
        g.build()
    yield


def golden(name):
    import numpy as np
    return dict(np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False))
