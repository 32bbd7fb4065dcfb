import contextlib
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


# the kernel families every parity test runs on (rapido_amd/csrc/gcm_engine.hip plan_launch): the window kernels
# with 64-position segments, with 32-position segments (8 lanes, 4 steps), with 32-position segments and 16 lanes
# (2 steps), the split kernels (runs of 16 such segments on separate workgroups), and the batch kernels (K lanes per
# record)
FAMILIES = ["window", "window32", "window16", "split", "batch"]


@contextlib.contextmanager
def kernel_family(name: str, framing: bool):
    """Routes every batch to the kernel family `name` (FAMILIES) for the duration of the block."""
    import rapido_amd as ra
    set_window = ra.set_tls_window_records if framing else ra.set_aead_window_records
    prev = set_window(0 if name == "batch" else 1 << 30)
    prev32 = ra.set_seg32_records(1 << 30 if name == "window32" else 0)
    prev16 = ra.set_win16_records(1 << 30 if name == "window16" else 0)
    prevs = ra.set_split_records(1 << 30 if name == "split" else 0)
    try:
        yield name
    finally:
        set_window(prev)
        ra.set_seg32_records(prev32)
        ra.set_win16_records(prev16)
        ra.set_split_records(prevs)


@pytest.fixture(params=["launch", "resident"])
def rl_mode(request, gpu):
    """Record layers created during the test launch kernels per window, or post jobs to the resident grid
    (include/ptls_mi355x.h section 6): the record-layer suites run both ways."""
    import rapido_amd as ra
    prev = ra.RecordLayer.default_resident
    ra.RecordLayer.default_resident = request.param == "resident"
    try:
        yield request.param
    finally:
        ra.RecordLayer.default_resident = prev
