import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (gfx950) GPU")


def has_gpu() -> bool:
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def golden():
    import json

    def load(name):
        with open(os.path.join(GOLDEN, name)) as f:
            return json.load(f)
    return load


@pytest.fixture(scope="session")
def gpu():
    # GPU tests fail (never skip) without a GPU: a skipped parity test must
    # not read as a pass on the GPU box.
    import torch
    assert torch.cuda.is_available(), "gpu-marked test needs a visible MI355X"
    torch.cuda.init()
    return torch.device("cuda:0")
