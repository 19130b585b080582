"""Shared fixtures. Tests marked `gpu` need a gfx950 device (run on the MI355X box); everything
else runs on CPU. The oracle (oracle/) is imported only here in tests, as the checker."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hakai-fem_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

REF_TENSILE = "/root/reference/HAKAI-v0.0.0/input/Tensile5e.inp"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 (MI355X) GPU")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def has_gpu():
    import hakai
    return hakai.device_count() > 0
