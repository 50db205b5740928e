import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "isaklm-raytracer_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI)")
    config.addinivalue_line("markers", "slow: multi-second CPU test")


@pytest.fixture(scope="session", autouse=True)
def _built():
    """Make sure the in-tree library and the oracle exist (builds if stale)."""
    import importlib.util

    spec = importlib.util.spec_from_file_location("rt_build", os.path.join(ROOT, "isaklm-raytracer_amd", "build.py"))
    b = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(b)
    b.build()
    import oracle

    oracle.build()
