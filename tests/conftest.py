import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for _p in (ROOT, os.path.join(ROOT, "tests")):
    if _p not in sys.path:
        sys.path.insert(0, _p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI)")
    config.addinivalue_line("markers", "slow: larger CPU cases")
    config.addinivalue_line("markers", "gpu_extended: GPU variants kept out of the default -m gpu run "
                            "(GLOO_AMD_GPU_EXTENDED=1 selects them)")


def pytest_collection_modifyitems(config, items):
    """GPU variants marked gpu_extended repeat what a default case already
    covers at other sizes: deselected unless GLOO_AMD_GPU_EXTENDED=1, so the
    default GPU suite keeps to its time budget."""
    if os.environ.get("GLOO_AMD_GPU_EXTENDED") == "1":
        return
    keep, drop = [], []
    for it in items:
        (drop if it.get_closest_marker("gpu_extended") else keep).append(it)
    if drop:
        config.hook.pytest_deselected(items=drop)
        items[:] = keep


@pytest.fixture(scope="session")
def golden_math():
    import numpy as np
    return np.load(os.path.join(ROOT, "tests", "golden", "math_golden.npz"))


@pytest.fixture(scope="session")
def golden_sched():
    import numpy as np
    return np.load(os.path.join(ROOT, "tests", "golden", "sched_golden.npz"))
