import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture
def lib_option():
    """set(name, value): a run-time option of the HIP library (include/dmdqn.h
    DMDQN_OPT_*, dmdqn_amd._lib.set_option) for this test, restored after it."""
    from dmdqn_amd import _lib
    saved = []

    def set_(name, value):
        saved.append((name, _lib.set_option(name, value)))

    yield set_
    for name, old in reversed(saved):
        _lib.set_option(name, old)
