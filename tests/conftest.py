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


@pytest.fixture(autouse=True)
def _gpu_work_checked(request):
    """After every GPU test: the objects it dropped are finalised now (their free paths synchronise and report), the
    device is synchronised, and any fault of the test's GPU work -- or an error a free path met -- fails THIS test.
    A fault is reported by whatever HIP call comes next; without this check the next test's first call takes the
    blame (round 4: an illegal address surfaced at the first H2D copy of an unrelated test).  A page fault is signalled
    asynchronously, possibly after the kernel has completed (a faulting store does not stop its wave), so the check
    runs twice, RAPIDO_FAULT_SETTLE_MS (default 20) apart: round 5 saw the round-4 report again at the same place
    with the checks 3 ms apart, i.e. the report arrived later than that."""
    yield
    if request.node.get_closest_marker("gpu") is None:
        return
    import gc
    import time

    import rapido_amd as ra
    nerr = len(ra.FINALIZER_ERRORS)
    gc.collect()
    ra.device_check()
    time.sleep(float(os.environ.get("RAPIDO_FAULT_SETTLE_MS", "20")) * 1e-3)
    ra.device_check()
    new = ra.FINALIZER_ERRORS[nerr:]
    if new:
        pytest.fail("finalizer errors: " + "; ".join(new))


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
# (2 steps), the split kernels (runs of 8 such segments on separate workgroups), and the batch kernels (K lanes per
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
