import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 GPU (runs on the MI355X box)")


@pytest.fixture
def gpu():
    """GPU tests FAIL (never skip) without a device: the HIP path has no fallback."""
    import torch
    assert torch.cuda.is_available(), "gpu test selected but no GPU is visible"
    from posfeat_amd import _lib
    _lib.require_device()
    return torch.device("cuda", torch.cuda.current_device())


GOLDEN = os.path.join(ROOT, "tests", "golden")
