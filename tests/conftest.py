import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X GPU (run on the gpurun box)")
    config.addinivalue_line("markers", "slow: long-running CPU test")
    # Build the (fast, g++) host runtime library before collection so the native trust-layer
    # code is what the tests exercise; NumPy-fallback tests force the fallback explicitly.
    try:
        from bcfl.csrc.build import build_host
        build_host()
    except Exception as e:  # pragma: no cover - toolchain missing
        print("host lib build skipped:", e)


@pytest.fixture
def tmp_out(tmp_path):
    return str(tmp_path / "run")
