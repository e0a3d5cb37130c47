import os
import sys
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
TESTS = os.path.dirname(os.path.abspath(__file__))
if TESTS not in sys.path:
    sys.path.insert(0, TESTS)



# JIT code objects live here for the session (and across sessions on the same machine); a fresh
# GPU box starts empty and the `gpu` fixture fills it in parallel before the first GPU test
JIT_CACHE = os.path.join(ROOT, ".jitcache")
os.makedirs(JIT_CACHE, exist_ok=True)
os.environ.setdefault("MIMIC_JIT_CACHE", JIT_CACHE)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP engine)")
    config.addinivalue_line("markers", "slow: long-running")


def _session_kernels(session):
    """Every JIT kernel the selected GPU tests will run: the jit_kernels() of their modules."""
    kernels, seen = [], set()
    for item in session.items:
        if item.get_closest_marker("gpu") is None:
            continue
        mod = getattr(item, "module", None)
        if mod is None or mod.__name__ in seen:
            continue
        seen.add(mod.__name__)
        fn = getattr(mod, "jit_kernels", None)
        if fn is not None:
            kernels.extend(fn())
    return kernels


@pytest.fixture(autouse=True)
def _gpu_settle(request):
    """After every GPU test the device is synchronised: an error its asynchronous work left (a
    faulting kernel, a copy into freed memory) is reported at that test's teardown, not at the next
    test's first HIP call."""
    yield
    if request.node.get_closest_marker("gpu") is None:
        return
    import torch

    if torch.cuda.is_available():
        torch.cuda.synchronize()


@pytest.fixture(scope="session")
def gpu(request):
    """The GPU session: first compiles the session's JIT kernels in parallel worker processes
    (hipRTC only, no device), then checks that a GPU is visible."""
    from mimic_amd import jit as J

    t0 = time.time()
    kernels = _session_kernels(request.session)
    info = J.prewarm(kernels)
    sys.stderr.write(f"\n[jit prewarm] {info['kernels']} kernels in {time.time() - t0:.1f}s\n")
    import torch

    if not torch.cuda.is_available():
        pytest.fail("GPU test run without a visible GPU")
    return 0
