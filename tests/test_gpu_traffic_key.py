"""The engine's record layer installed through the reference picotls' own-record-layer hook (update_traffic_key,
lib/picotls.c:1206-1211) and run against a reference picotls peer: oracle/ref_traffic_key_harness.c, built by
oracle/Makefile from the unmodified /root/reference/lib/picotls.c and the reference minicrypto AES-GCM.

The harness's callback is INTEGRATION.md section 5 as C: setup_traffic_protection (lib/picotls.c:1190-1225) hands it
each application traffic secret; it derives key and IV as rapido does (lib/rapido.c:135-150) and creates or rekeys a
ptls_mi355x_record_layer.  Scenario (all bytes checked): send windows accepted by the peer's ptls_receive, the peer's
ptls_send output opened by the layer, a peer-initiated KeyUpdate (the window stops at the handshake record,
open_record hands it to ptls_handle_message, the callback rekeys, the rest opens from seq 0), a layer-initiated
KeyUpdate, and the 2^24-record limit with the peer following across it -- on every transport."""
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HARNESS = os.path.join(ROOT, "oracle", "_ref", "ref_traffic_key_harness")


@pytest.mark.parametrize("keylen", [16, 32])
@pytest.mark.parametrize("transport", ["direct", "dma", "dma_in", "zero_copy", "copy"])
def test_update_traffic_key_against_picotls(gpu, transport, keylen):
    assert os.path.exists(HARNESS), "oracle/_ref/ref_traffic_key_harness not built (oracle/Makefile, needs /root/reference)"
    r = subprocess.run([HARNESS, transport, str(keylen)], capture_output=True, text=True, timeout=100)
    assert r.returncode == 0, r.stderr
    assert r.stdout.startswith("ok: 7 checks (5 scenarios)"), r.stdout
    assert "5 update_traffic_key callbacks" in r.stdout  # 2 installs, 1 peer-initiated and 2 own KeyUpdates


@pytest.mark.parametrize("transport,keylen", [("direct", 16), ("dma_in", 16), ("zero_copy", 16), ("direct", 32)])
def test_rapido_stream_through_the_hook(gpu, transport, keylen):
    """Scenario 6: rapido's 1 MB stream (t/rapido_tests.c:290-340) both ways through the layers the hook installed --
    send windows of 16 x 16 KiB fragments checked by the peer's ptls_receive, the peer's ptls_send output opened in
    receive windows of 32 records -- then the same stream, same key, IV and seq, through standalone layers and through
    the engine's AEAD slot (ptls_send / ptls_receive per record, as rapido protects records today), every output equal
    to the checked stream; the host-to-host rates of each are printed."""
    import json
    assert os.path.exists(HARNESS), "oracle/_ref/ref_traffic_key_harness not built (oracle/Makefile, needs /root/reference)"
    r = subprocess.run([HARNESS, transport, str(keylen), "transfer"], capture_output=True, text=True, timeout=200)
    assert r.returncode == 0, r.stderr
    lines = r.stdout.splitlines()
    assert lines[-1].startswith("ok: 9 checks (6 scenarios)"), r.stdout
    rates = json.loads([x for x in lines if x.startswith("rates ")][0][6:])
    print(json.dumps(rates))
    assert all(rates[k] > 0 for k in rates if k.endswith("MBps"))
