import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
TESTS = os.path.dirname(os.path.abspath(__file__))
if TESTS not in sys.path:
    sys.path.insert(0, TESTS)


# JIT kernels compiled by earlier processes (or prewarmed on a CPU host with
# MIMIC_JIT_PREWARM=1 python -m pytest tests -m gpu -n 8) are reused from here
JIT_CACHE = os.path.join(ROOT, ".jitcache")
os.makedirs(JIT_CACHE, exist_ok=True)
os.environ.setdefault("MIMIC_JIT_CACHE", JIT_CACHE)
PREWARM = bool(os.environ.get("MIMIC_JIT_PREWARM"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP engine)")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def gpu():
    import torch

    if PREWARM:
        return 0
    if not torch.cuda.is_available():
        pytest.fail("GPU test run without a visible GPU")
    return 0
