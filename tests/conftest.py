import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# the fp32 ATen / MIOpen oracle of the GPU parity tests: immediate-mode kernel choice
# instead of a per-shape search (minutes at the shipped batch sizes; numerics unchanged)
os.environ.setdefault("MIOPEN_FIND_MODE", "FAST")
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU and the native extension")
    config.addinivalue_line("markers", "slow: long-running test")


@pytest.fixture(scope="session")
def cuda_dev():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from unet_distributed_amd import native
    native.require()      # the HIP path must load on a GPU box: fail loudly, never skip
    return torch.device("cuda:0")
