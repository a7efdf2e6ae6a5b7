import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")
INPUT_DATA = os.path.join(ROOT, "scenes", "input_data")
REF_SCENE = os.path.join(ROOT, "scenes", "reference_scene.txt")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")
    config.addinivalue_line("markers", "slow: long-running check")


@pytest.fixture(scope="session")
def oracle_mod():
    import oracle
    oracle.build()
    return oracle


@pytest.fixture(scope="session")
def pt_mod():
    import pathtracerap_amd as P
    if not os.path.exists(os.path.join(ROOT, "pathtracerap_amd", "libpathtracer_amd.so")):
        P.build()
    return P


@pytest.fixture(scope="session")
def gpu():
    """Skips nothing: a -m gpu run without a device must fail loudly."""
    import torch
    assert torch.cuda.is_available(), "gpu tests need a ROCm device"
    return torch.device("cuda:0")
