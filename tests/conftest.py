import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "genomics-gpu_amd"), os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI)")
    config.addinivalue_line("markers", "slow: longer-running parity sweep")


def pytest_collection_modifyitems(config, items):
    # GPU tests require the device; fail loudly (not skip) when the marker is selected on a box without it
    pass


@pytest.fixture(scope="session")
def engine():
    import gasal_ffi
    eng = gasal_ffi.Engine(0)
    yield eng
    eng.close()
