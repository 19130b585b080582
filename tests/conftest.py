"""Shared fixtures. Tests marked `gpu` need a gfx950 device (run on the MI355X box); everything
else runs on CPU. The oracle (oracle/) is imported only here in tests, as the checker.

GPU test order: the BASELINE configurations and the reference's own decks run first (C2/C4/C5 in
test_gpu_configs, C3 in test_gpu_fullsize, C1 and the decks in test_gpu_exact / test_gpu_decks /
test_gpu_parity), so a `-x` stop in a later, narrower test cannot hide them."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hakai-fem_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

REF_TENSILE = "/root/reference/HAKAI-v0.0.0/input/Tensile5e.inp"

_FIRST = ("test_gpu_exact.py", "test_gpu_configs.py", "test_gpu_fullsize.py", "test_gpu_decks.py",
          "test_gpu_parity.py")
_LAST = ("test_gpu_own.py", "test_gpu_multirank.py", "test_gpu_rccl.py")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 (MI355X) GPU")
    config.addinivalue_line("markers", "slow: long-running")


def pytest_collection_modifyitems(config, items):
    def rank(item):
        f = os.path.basename(str(item.fspath))
        if f in _FIRST:
            return _FIRST.index(f)
        if f in _LAST:
            return 100 + _LAST.index(f)
        return 50
    items.sort(key=rank)  # stable: file order within a rank, test order within a file


@pytest.fixture(scope="session")
def has_gpu():
    import hakai
    return hakai.device_count() > 0
