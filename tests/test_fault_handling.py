"""Fault handling of the engine.

* The fault journal (rapido_amd/csrc/fault_journal.c): the report the memory-fault observer writes -- the faulting
  address, its reasons, and the engine's last device events with the range that holds the address marked -- checked on
  the CPU through its on-demand entry point; on the GPU, that the observer is registered with the HSA runtime.
  A deliberate GPU page fault is not part of the suite: the pool's rules forbid running kernels that fault.
* The AEAD slot fails closed: an engine error inside do_decrypt refuses the record as a bad MAC (SIZE_MAX, which
  picotls turns into PTLS_ALERT_BAD_RECORD_MAC, lib/picotls.c:645-654) with its output zeroed, and the process lives;
  do_encrypt, whose ABI has no error return, still aborts.
"""
import os
import subprocess
import sys

import pytest

import rapido_amd as ra

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _with_report_path(path):
    """Points the journal's report at `path` (install sets the path first, even where no GPU lets it register)."""
    ra.lib().ptls_mi355x_fault_journal_install(path.encode())


def test_fault_journal_report_marks_the_range_holding_the_address(engine_lib, tmp_path):
    log = str(tmp_path / "fault.log")
    _with_report_path(log)
    try:
        ra.fault_journal_note(b"hipMalloc key image", 0x7F1000000000, 128 << 10)
        ra.fault_journal_note(b"hipFree scratch", 0x7F1000400000, 1 << 20)
        ra.fault_journal_note(b"hipMalloc work counters", 0x7F1000800000, 1024)
        ra.fault_journal_report(0x7F1000400123, 0x1)
        text = open(log).read()
    finally:
        _with_report_path(os.environ["RAPIDO_FAULT_LOG"])
    assert "GPU memory fault at VA 0x00007f1000400123" in text
    assert "page not present" in text
    lines = [ln for ln in text.splitlines() if "HOLDS THE FAULTING ADDRESS" in ln]
    assert len(lines) == 1 and "hipFree scratch" in lines[0], text
    assert text.rstrip().endswith("=== end of fault journal ===")


def test_fault_report_says_what_the_address_is(engine_lib, tmp_path):
    """The report describes the faulting address as it is at the fault: the runtime's view of it and of the byte
    before its page (hsa_amd_pointer_info; here, without a GPU, its status), and the /proc/self/maps line holding it
    -- an address in no mapping is reported as such, with its neighbours."""
    import numpy as np
    log = str(tmp_path / "fault.log")
    host = np.zeros(1 << 20, np.uint8)
    _with_report_path(log)
    try:
        ra.fault_journal_report(host.ctypes.data + 8192, 0x1)
        ra.fault_journal_report(0x10, 0x1)  # below every mapping
        text = open(log).read()
    finally:
        _with_report_path(os.environ["RAPIDO_FAULT_LOG"])
    first, second = text.split("=== end of fault journal ===")[:2]
    assert "the faulting address now:" in first and "fault VA 0x" in first and "byte before its page" in first
    maps = [ln for ln in first.splitlines() if ln.strip().startswith("maps:")]
    assert len(maps) == 1 and "rw" in maps[0], first  # the array's own (writable) mapping
    assert "is in no mapping" in second, second


def test_fault_journal_keeps_the_last_256_events(engine_lib, tmp_path):
    log = str(tmp_path / "fault.log")
    _with_report_path(log)
    try:
        for i in range(300):
            ra.fault_journal_note(b"event", 0x1000 * (i + 1), 16)
        ra.fault_journal_report(0x1000 * 300 + 4, 0x2)
        text = open(log).read()
    finally:
        _with_report_path(os.environ["RAPIDO_FAULT_LOG"])
    events = [ln for ln in text.splitlines() if ln.startswith("#")]
    assert len(events) == 256
    assert "HOLDS THE FAULTING ADDRESS" in events[-1] and "read-only" in text


def _slot_probe(code: str) -> subprocess.CompletedProcess:
    env = dict(os.environ, RAPIDO_FAULT_JOURNAL="0")
    return subprocess.run([sys.executable, "-c", code], cwd=ROOT, env=env, capture_output=True, text=True, timeout=120)


SLOT_SETUP = """
import rapido_amd as ra
L = ra.lib()
L.ptls_mi355x_test_slot_without_engine(1)
dec = ra.aead_new_direct("aes128gcm", False, bytes(16), bytes(12))
L.ptls_mi355x_test_slot_without_engine(0)
"""


def test_slot_decrypt_fails_closed_on_an_engine_error(engine_lib):
    """A context whose every engine call fails (test hook): do_decrypt returns SIZE_MAX, zeroes the output in place,
    counts the error, and the process goes on -- twice in a row."""
    r = _slot_probe(SLOT_SETUP + """
import ctypes as C
assert L.ptls_mi355x_slot_engine_errors() == 0
for k in range(2):
    buf = C.create_string_buffer(b"\\x5a" * 64, 64)
    n = dec.ctx.do_decrypt(dec.ptr, buf, buf, 64, 7, None, 0)
    assert n == ra.SIZE_MAX, n
    assert buf.raw[:48] == bytes(48), buf.raw  # in place: no byte of the 48-byte output is left
assert L.ptls_mi355x_slot_engine_errors() == 2
assert dec.decrypt(bytes(40), 1) is None
dec.free()
print("ALIVE")
""")
    assert r.returncode == 0, r.stderr
    assert "ALIVE" in r.stdout
    assert r.stderr.count("failed closed") == 3


def test_slot_encrypt_aborts_on_an_engine_error(engine_lib):
    """do_encrypt is void in picotls' ABI (include/picotls.h:351): an engine error there aborts rather than emit a
    record that was never encrypted."""
    r = _slot_probe(SLOT_SETUP + """
dec.encrypt(b"hello", 1)  # both halves are populated (lib/fusion.c:951-957)
print("NOT REACHED")
""")
    assert r.returncode != 0 and "NOT REACHED" not in r.stdout
    assert "seal failed" in r.stderr


@pytest.mark.gpu
def test_fault_journal_is_registered_on_the_gpu(gpu):
    """The memory-fault observer is registered with the HSA runtime (status 0) in the test process."""
    assert ra.FAULT_JOURNAL_STATUS == 0, ra.FAULT_JOURNAL_STATUS
    assert ra.lib().ptls_mi355x_fault_journal_installed() == 1
    assert ra.fault_journal_faults() == 0


@pytest.mark.gpu
def test_slot_decrypt_fails_closed_on_an_injected_gpu_error(gpu):
    """An injected engine error in the real slot's decrypt: SIZE_MAX and a zeroed output; the next call of the same
    context opens the record."""
    L = ra.lib()
    key, iv = bytes(range(16)), bytes(range(12))
    enc = ra.aead_new_direct("aes128gcm", True, key, iv)
    dec = ra.aead_new_direct("aes128gcm", False, key, iv)
    try:
        ct = enc.encrypt(b"record body " * 100, 5, b"\x17\x03\x03\x04\xc0")
        before = L.ptls_mi355x_slot_engine_errors()
        L.ptls_mi355x_test_inject_engine_errors(1)
        assert dec.decrypt(ct, 5, b"\x17\x03\x03\x04\xc0") is None
        assert L.ptls_mi355x_slot_engine_errors() == before + 1
        assert dec.decrypt(ct, 5, b"\x17\x03\x03\x04\xc0") == b"record body " * 100
    finally:
        L.ptls_mi355x_test_inject_engine_errors(0)
        enc.free()
        dec.free()


@pytest.mark.gpu
def test_fault_report_describes_gpu_runtime_memory(gpu, tmp_path):
    """On the GPU the report's address description comes from the HSA runtime (hsa_amd_pointer_info): device memory
    and pinned host memory (hipHostMalloc) are the runtime's allocations with their extents; a range the record layer
    registered (hipHostRegister) is NOT in the runtime's allocation map on this stack -- HIP maps it through the kernel
    driver's shared-virtual-memory ranges, device address = host address -- so the report's record-layer table is what
    names it; a plain heap array is unknown to the runtime and named by its /proc/self/maps line."""
    import numpy as np
    import torch
    log = str(tmp_path / "fault.log")
    d = torch.zeros(1 << 20, dtype=torch.uint8, device="cuda")
    pinned = torch.zeros(1 << 20, dtype=torch.uint8, pin_memory=True)
    raw = np.zeros((4 << 20) + 4096, np.uint8)
    off = (-raw.ctypes.data) % 4096
    reg = raw[off:off + (4 << 20)]
    heap = np.zeros(1 << 20, np.uint8)
    rl = ra.RecordLayer(bytes(16), bytes(12))
    rl.register(reg)
    _with_report_path(log)
    try:
        for p in (d.data_ptr() + 4096, pinned.data_ptr() + 4096, reg.ctypes.data + 8192, heap.ctypes.data + 4096):
            ra.fault_journal_report(p, 0x1)
        text = open(log).read()
    finally:
        _with_report_path(os.environ["RAPIDO_FAULT_LOG"])
        rl.unregister(reg)
        rl.close()
    reports = text.split("=== end of fault journal ===")[:4]
    first = [next(ln for ln in r.splitlines() if "fault VA" in ln) for r in reports]
    assert "HSA allocation" in first[0], first[0]
    assert "HSA allocation" in first[1] or "locked" in first[1], first[1]
    assert "unknown to the runtime" in first[2] or "locked host range" in first[2], first[2]
    assert "unknown to the runtime" in first[3], first[3]
    held = [ln.strip() for ln in reports[2].splitlines() if "HOLDS THE FAULTING ADDRESS" in ln]
    # the record layer's registration table names it (and the journal's registration event)
    assert any(ln.startswith("host ") and "+ 4194304" in ln for ln in held), reports[2]
    assert "[heap]" in reports[3] or "maps: " in reports[3]
    assert ra.fault_journal_faults() == 0  # reports on request are not faults
