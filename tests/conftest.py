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


HIP_ERROR_INVALID_DEVICE = 101  # hipErrorInvalidDevice


@pytest.fixture(autouse=True)
def _stale_hip_error(request):
    """Before each GPU test: drop the "invalid device ordinal" error that tests
    spawning worker processes leave pending on this process's main thread
    (torch's allocator would report it at the next test's first allocation).
    Any other pending error is left in place, to fail where it shows."""
    if request.node.get_closest_marker("gpu"):
        import ctypes

        try:
            hip = ctypes.CDLL("libamdhip64.so")
        except OSError:
            hip = None
        if hip is not None and hip.hipPeekAtLastError() == HIP_ERROR_INVALID_DEVICE:
            hip.hipGetLastError()
    yield


@pytest.fixture(scope="session")
def ctx():
    from syzkaller_amd.cover import Context, default_context

    c = default_context()
    assert isinstance(c, Context)
    yield c


@pytest.fixture
def ctx_option():
    """set(context, key, value): a context option (sg_ctx_set_option) for one
    test, restored after it."""
    saved = []

    def set_(c, key, value):
        saved.append((c, key, c.get_option(key)))
        c.set_option(key, value)

    yield set_
    for c, key, v in reversed(saved):
        if c.h:
            c.set_option(key, v)


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
