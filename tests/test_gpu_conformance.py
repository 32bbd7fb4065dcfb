"""The engine through the reference's own picotls.c code and inline dispatchers, cross-checked in
one process against the reference fusion engine (oracle/slot_conformance.c, built in the container
that holds /root/reference into oracle/_ref/slot_conformance)."""
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu
EXE = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle", "_ref", "slot_conformance")


@pytest.mark.skipif(not os.path.exists(EXE), reason="conformance binary not built (needs /root/reference at build time)")
def test_slot_conformance_against_reference_picotls_and_fusion(gpu):
    r = subprocess.run([EXE, "500"], capture_output=True, text=True, timeout=600)
    print(r.stdout[-3000:])
    if r.returncode == 3:
        pytest.skip("host CPU lacks AES-NI (fusion cannot run)")
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-2000:]
    assert " 0 failed" in r.stdout
