import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu on the GPU box)")


@pytest.fixture(scope="session")
def hip_ext():
    """The built _C extension (GPU tests only; the product has no CPU path)."""
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import relightable3dgaussian_amd as r

    return r._C
