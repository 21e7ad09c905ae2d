import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU (MI355X) and libfvo.so")


@pytest.fixture(scope="session")
def oracle_mod():
    import oracle  # noqa: E402  (test infrastructure)
    oracle.build()
    return oracle


def gpu_available():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False
