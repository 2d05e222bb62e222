import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU (MI355X); parity tests through the C ABI")


@pytest.fixture(scope="session")
def O():
    from oracle import oracle

    oracle.build()
    return oracle


@pytest.fixture(scope="session")
def cuda():
    import torch

    if not torch.cuda.is_available():
        pytest.fail("gpu test needs a GPU (run with -m 'not gpu' on CPU)")
    torch.cuda.set_device(0)
    return torch.device("cuda:0")
