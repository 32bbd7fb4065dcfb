import contextlib
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

# where the engine's fault journal (rapido_amd/csrc/fault_journal.c) appends its report if the GPU signals a memory
# fault: read after every GPU test (below), and merged back from the GPU box with the rest of gpurun_out/
FAULT_LOG = os.environ.setdefault("RAPIDO_FAULT_LOG", os.path.join(ROOT, "gpurun_out", "fault_journal.log"))


def _fault_log_size() -> int:
    try:
        return os.path.getsize(FAULT_LOG)
    except OSError:
        return 0


def _fault_log_since(offset: int) -> str:
    try:
        with open(FAULT_LOG, "rb") as f:
            f.seek(offset)
            return f.read().decode(errors="replace")
    except OSError:
        return ""


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
    gpu = request.node.get_closest_marker("gpu") is not None
    if gpu:
        os.makedirs(os.path.dirname(FAULT_LOG), exist_ok=True)
    log0 = _fault_log_size()
    import rapido_amd as ra
    engines0 = set(id(e) for e in ra.LIVE_ENGINES)
    yield
    if not gpu:
        return
    import gc
    import time

    nerr = ra.FINALIZER_ERROR_COUNT
    # engines the test left open are released here, explicitly and in creation-independent order, before the checks
    # (not at some later garbage collection): each release synchronises and reports, so an error is this test's
    for eng in [e for e in list(ra.LIVE_ENGINES) if id(e) not in engines0]:
        eng.close()
    gc.collect()
    try:
        ra.device_check()
        time.sleep(float(os.environ.get("RAPIDO_FAULT_SETTLE_MS", "20")) * 1e-3)
        ra.device_check()
    except RuntimeError as e:
        # the journal's report, if the handler wrote one, names the faulting address and the launches around it
        raise RuntimeError(f"{e}\n{_fault_log_since(log0)}") from None
    report = _fault_log_since(log0)
    if report:
        pytest.fail("the GPU signalled a memory fault during this test (fault journal):\n" + report)
    k = ra.FINALIZER_ERROR_COUNT - nerr
    if k:
        pytest.fail("finalizer errors: " + "; ".join(ra.FINALIZER_ERRORS[-k:]))


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
