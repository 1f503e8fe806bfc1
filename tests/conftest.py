import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) and runs libsyzsig.so kernels")
    config.addinivalue_line("markers", "slow: a larger case (tens of millions of entries)")


@pytest.fixture(scope="session")
def ctx():
    from syzkaller_amd.cover import Context, default_context

    c = default_context()
    assert isinstance(c, Context)
    yield c


@pytest.fixture(scope="session")
def kats():
    import json

    with open(os.path.join(GOLDEN, "cover_kats.json")) as f:
        return json.load(f)["tests"]


@pytest.fixture(scope="session")
def exec_golden():
    import numpy as np

    with np.load(os.path.join(GOLDEN, "exec_signal_golden.npz"), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}
