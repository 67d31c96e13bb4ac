import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run on the GPU box)")


@pytest.fixture(scope="session")
def oracle_lib():
    from oracle import binding
    binding.build()
    return binding.load()


@pytest.fixture(scope="session")
def hip_lib():
    from raysnail_amd import _abi
    return _abi.load()


@pytest.fixture(scope="session")
def gpu():
    import torch
    assert torch.cuda.is_available(), "gpu tests need a GPU"
    torch.cuda.set_device(0)
    return torch
