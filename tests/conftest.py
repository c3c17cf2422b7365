import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU (MI355X) and the HIP kernel extension")
    config.addinivalue_line("markers", "slow: multi-process / longer tests")


@pytest.fixture(scope="session", autouse=True)
def _native_built():
    # build the in-tree native modules once if they are missing (no-op when up to date)
    from simple_distributed_machine_learning_amd import _native

    _native.runtime()
    yield


def free_port():
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p
