import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU; run with -m gpu")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def engine_lib():
    """The engine library, built if needed (build needs only hipcc, no GPU)."""
    from rapido_amd import build
    build.build_engine()
    import rapido_amd
    return rapido_amd.lib()


@pytest.fixture(scope="session")
def gpu(engine_lib):
    import rapido_amd
    if not rapido_amd.is_supported():
        pytest.fail("no gfx950 GPU visible, but a gpu-marked test was selected")
    import torch
    torch.cuda.init()
    return torch.device("cuda:0")
