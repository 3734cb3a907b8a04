import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box)")


@pytest.fixture(scope="session")
def golden():
    import numpy as np

    return dict(np.load(os.path.join(ROOT, "tests", "golden", "golden_dynamics.npz")))


@pytest.fixture(scope="session")
def golden_env():
    import numpy as np

    return dict(np.load(os.path.join(ROOT, "tests", "golden", "golden_env.npz")))


@pytest.fixture(scope="session")
def golden_freerun():
    import numpy as np

    return dict(np.load(os.path.join(ROOT, "tests", "golden", "golden_freerun.npz")))
