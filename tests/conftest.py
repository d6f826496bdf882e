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


@pytest.fixture(scope="session")
def golden_math():
    import numpy as np
    return np.load(os.path.join(ROOT, "tests", "golden", "math_golden.npz"))


@pytest.fixture(scope="session")
def golden_sched():
    import numpy as np
    return np.load(os.path.join(ROOT, "tests", "golden", "sched_golden.npz"))
