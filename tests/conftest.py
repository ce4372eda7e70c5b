import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box only)")


@pytest.fixture(scope="session")
def gpu():
    """Fail (never skip) when a gpu-marked test runs without a usable GPU + libgrs."""
    import torch

    assert torch.cuda.is_available(), "gpu test without a visible GPU"
    import gpuradixsort_amd as grs

    grs.lib()  # raises if libgrs.so is missing: there is no fallback
    return torch.device("cuda", 0)
