import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
for p in (str(ROOT), str(ROOT / "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")
    config.addinivalue_line("markers", "slow: long-running CPU test")
    config.addinivalue_line("markers", "spawns: starts GPU-using child processes; runs before any test initialises "
                                       "HIP in the pytest process")


def pytest_collection_modifyitems(session, config, items):
    # Child processes that use the GPU are started from a parent that has not initialised HIP yet:
    # those tests run first (stable order otherwise).
    items.sort(key=lambda it: 0 if it.get_closest_marker("spawns") else 1)


def assert_hip_untouched():
    """For `spawns` tests: the pytest process must not have initialised HIP before starting children."""
    import torch

    assert not torch.cuda.is_initialized(), "HIP already initialised in the pytest process"
