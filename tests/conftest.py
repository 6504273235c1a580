import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")


def gpu_available():
    try:
        import torch  # device probe only
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def om():
    import raytracingoneweekend_amd as m
    return m


@pytest.fixture(scope="session")
def oracle():
    from oracle import oracle as O
    return O
