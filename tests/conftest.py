import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (gfx950) GPU")
    config.addinivalue_line("markers", "slow: long-running test")


@pytest.fixture(scope="session")
def gpu():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from nv_genai_amd import ops

    ops.kernels()  # fail loudly if the HIP extension is missing
    return torch.device("cuda:0")


@pytest.fixture
def kernel_form():
    """Select an A/B kernel form for one test (csrc/kernels/kernels.h KernelForm) and restore
    it afterwards: ``kernel_form("decode_dma", 2)``."""
    from nv_genai_amd import ops

    saved = {}

    def set_form(name, value):
        if name not in saved:
            saved[name] = ops.kernel_form(name)
        ops.kernels().set_kernel_form(name, int(value))

    yield set_form
    for k, v in saved.items():
        ops.kernels().set_kernel_form(k, v)
