import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)
GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libdsx.so)")


# The GPU suite runs under -x: the parity files first, the tests that start
# other processes (torch.distributed.run, spawned ranks, a child on the
# diagnostic build) last, so that a problem in a process launch cannot keep
# the parity tests from running (round 5's driver run stopped at test 59 of
# 162, before all of test_gpu_parity.py).
_LAST = ("test_gpu_multiproc.py", "test_gpu_variants.py", "test_gpu_behind.py")


def pytest_collection_modifyitems(session, config, items):
    def rank(item):
        name = os.path.basename(str(item.fspath))
        return _LAST.index(name) + 1 if name in _LAST else 0
    items[:] = sorted(items, key=rank)  # (stable: file and test order kept otherwise)


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
