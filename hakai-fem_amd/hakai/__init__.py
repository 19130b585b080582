"""hakai -- MI355X-native explicit-dynamics inner loop of HAKAI (yozoyugen/HAKAI-fem v0.0.2).

Python host layer over libhakai_hip.so (include/hakai_hip.h). Import path: add the
``hakai-fem_amd`` directory to ``sys.path`` (the repo's conftest, bench and __graft_entry__ do).
"""
from ._abi import HakaiError, device_count, lib  # noqa: F401
from .model import BCGroup, Material, Model, read_inp  # noqa: F401
from .solver import Solver, State, cal_stress_hexa, cal_triax_stress, comm_unique_id, hakai  # noqa: F401

__all__ = ["HakaiError", "device_count", "lib", "BCGroup", "Material", "Model", "read_inp", "Solver", "State",
           "cal_stress_hexa", "cal_triax_stress", "comm_unique_id", "hakai"]
