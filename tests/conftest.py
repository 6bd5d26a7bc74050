import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)
GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libdsx.so)")


@pytest.fixture(scope="session")
def golden():
    def read(name):
        with open(os.path.join(GOLDEN, name), "rb") as f:
            return f.read()
    return read


@pytest.fixture(scope="session")
def dctx():
    """One dsx context for the whole GPU session (one process on the card)."""
    from desync_amd import _lib
    return _lib.default_context(0)
