import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU; runs the HIP kernels")


@pytest.fixture(scope="session", autouse=True)
def _built_library():
    """The native library is part of the product: build it (hipcc cross-compiles without a GPU)."""
    from lbt_amd import _build
    _build.build()
    yield
