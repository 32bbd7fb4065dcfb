"""The REFERENCE caller, unchanged, over the engine's AEAD slot (north_star: "the TCPLS record-protection path in
lib/rapido.c / lib/picotls.c calls it unchanged").

oracle/ref_caller_harness.c compiles the unmodified /root/reference/lib/picotls.c and hands it the engine's exported
objects ptls_mi355x_aes128gcm / ptls_mi355x_aes256gcm with no adapter:

* as the traffic AEAD installed by ptls_set_traffic_protection (rapido's per-connection install, lib/rapido.c:135-200):
  the reference ptls_send (lib/picotls.c:4969-4988) must reproduce tests/golden/tls_records.json -- the wire bytes the
  reference record layer produced over the fusion core -- bit for bit, a minicrypto peer's ptls_receive must accept
  them, the reference ptls_receive over the engine must reproduce the fixture's receive cases (padding, all-zero,
  tamper -> PTLS_ALERT_BAD_RECORD_MAC) and open what minicrypto sends;
* as the AEAD of a negotiated TLS 1.3 cipher suite (ptls_handshake against a minicrypto peer): handshake records,
  application data both ways, KeyUpdates from both sides and in-flight tamper.
"""
import hashlib
import json
import os
import subprocess

import numpy as np
import pytest

from rapido_amd.records import xorshift64star


ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HARNESS = os.path.join(ROOT, "oracle", "_ref", "ref_caller_harness")
FIX = json.load(open(os.path.join(ROOT, "tests", "golden", "tls_records.json")))
BAD_RECORD_MAC = 20


def xs(seed, n):
    return xorshift64star(seed, n).tobytes()


def run(lines, timeout=300):
    assert os.path.exists(HARNESS), "oracle/_ref/ref_caller_harness not built (oracle/Makefile, needs /root/reference)"
    r = subprocess.run([HARNESS], input="\n".join(lines) + "\n", capture_output=True, text=True, timeout=timeout)
    out = r.stdout.strip().splitlines()
    assert r.returncode == 0 and all(o.startswith("ok ") for o in out), (r.stdout[-2000:], r.stderr[-2000:])
    assert len(out) == len(lines)
    return [o.split(" ") for o in out]


def h(b: bytes) -> str:
    return b.hex() if b else "-"


def unh(s: str) -> bytes:
    return b"" if s == "-" else bytes.fromhex(s)


def send_inputs(c):
    keylen, ln, seed = int(c["keylen"]), int(c["len"]), int(c["seed"])
    return keylen, xs(seed + 1, keylen), xs(seed + 2, 12), int(c["seq0"]), xs(seed, ln)


def test_harness_pinned_by_minicrypto_without_gpu():
    """The harness itself (CPU only): the reference ptls_send over minicrypto reproduces the fixture's wire bytes, and
    the reference ptls_receive over minicrypto its receive cases -- so the GPU tests below differ only in the AEAD."""
    if not os.path.exists(HARNESS):
        pytest.skip("oracle/_ref/ref_caller_harness not built (needs /root/reference)")
    cases = FIX["send"]
    res = run([f"send minicrypto {k} {key.hex()} {iv.hex()} {seq0} {h(data)}" for k, key, iv, seq0, data in
               map(send_inputs, cases)])
    for c, r in zip(cases, res):
        assert int(r[1]) == 0 and int(r[2]) == int(c["seq_after"])
        assert hashlib.sha256(unh(r[3])).hexdigest() == c["wire_sha256"]
    cases = FIX["receive"]
    res = run([f"recv minicrypto {len(bytes.fromhex(c['key']))} {c['key']} {c['iv']} {c['seq']} {c['wire']}" for c in cases])
    for c, r in zip(cases, res):
        assert int(r[1]) == int(c["rc"]) and unh(r[4]).hex() == c["plaintext"]
    (r,) = run(["handshake minicrypto-both 16 20000"])
    assert int(r[1]) == 10


@pytest.mark.gpu
def test_ptls_send_over_engine_reproduces_reference_wire(gpu):
    """ptls_send with the engine as the installed traffic AEAD == the reference record layer's wire bytes."""
    cases = FIX["send"]
    lines = []
    for c in cases:
        keylen, key, iv, seq0, data = send_inputs(c)
        lines.append(f"send engine {keylen} {key.hex()} {iv.hex()} {seq0} {h(data)}")
    res = run(lines)
    for c, r in zip(cases, res):
        rc, seq_after, wire = int(r[1]), int(r[2]), unh(r[3])
        assert rc == 0
        assert seq_after == int(c["seq_after"])
        assert len(wire) == int(c["wire_len"])
        assert hashlib.sha256(wire).hexdigest() == c["wire_sha256"]
        if "wire" in c:
            assert wire.hex() == c["wire"]


@pytest.mark.gpu
@pytest.mark.parametrize("engine_side", ["send", "recv"])
def test_engine_and_minicrypto_peers_interoperate(gpu, engine_side):
    """Engine-sealed wire opened by the reference ptls_receive over minicrypto, and minicrypto-sealed wire opened by
    the reference ptls_receive over the engine (every fixture send stream, sizes 1 B .. 40 000 B)."""
    cases = FIX["send"]
    s_impl, r_impl = ("engine", "minicrypto") if engine_side == "send" else ("minicrypto", "engine")
    sends = [f"send {s_impl} {k} {key.hex()} {iv.hex()} {seq0} {h(data)}"
             for k, key, iv, seq0, data in map(send_inputs, cases)]
    wires = [unh(r[3]) for r in run(sends)]
    recvs = [f"recv {r_impl} {k} {key.hex()} {iv.hex()} {seq0} {h(w)}"
             for (k, key, iv, seq0, _), w in zip(map(send_inputs, cases), wires)]
    for c, w, r in zip(cases, wires, run(recvs)):
        _, key_len, key, iv, seq0, data = (None,) + send_inputs(c)
        assert hashlib.sha256(w).hexdigest() == c["wire_sha256"]
        assert int(r[1]) == 0 and int(r[2]) == len(w) and int(r[3]) == int(c["seq_after"])
        assert unh(r[4]) == data


@pytest.mark.gpu
def test_ptls_receive_over_engine_matches_reference_receive_cases(gpu):
    """The fixture's receive cases (padding 0-384 B, all-zero plaintext, tamper) through the reference ptls_receive
    with the engine installed: the same return code and delivered plaintext as the reference record layer."""
    cases = FIX["receive"]
    lines = [f"recv engine {len(bytes.fromhex(c['key']))} {c['key']} {c['iv']} {c['seq']} {c['wire']}" for c in cases]
    for c, r in zip(cases, run(lines)):
        assert int(r[1]) == int(c["rc"]), c
        assert unh(r[4]).hex() == c["plaintext"], c


@pytest.mark.gpu
@pytest.mark.parametrize("keylen", [16, 32])
def test_tampered_records_rejected_through_the_record_layer(gpu, keylen):
    """Engine-sealed streams with one flipped bit in a record's ciphertext, content-type byte or tag: the
    reference ptls_receive over the engine returns PTLS_ALERT_BAD_RECORD_MAC and delivers nothing of that record."""
    rng = np.random.default_rng(keylen)
    key, iv = rng.bytes(keylen), rng.bytes(12)
    data = rng.bytes(20000)  # two records: 16384 + 3616
    (r,) = run([f"send engine {keylen} {key.hex()} {iv.hex()} 77 {data.hex()}"])
    wire = unh(r[3])
    assert len(wire) == 20000 + 2 * 22
    lines, where = [], []
    for pos in (5 + 100, 5 + 16385 - 1, 16400, 16406 + 5 + 3000, len(wire) - 1):  # ciphertext, type byte, tag
        w = bytearray(wire)
        w[pos] ^= 0x01
        lines.append(f"recv engine {keylen} {key.hex()} {iv.hex()} 77 {bytes(w).hex()}")
        where.append(pos)
    for pos, r in zip(where, run(lines)):
        rc, consumed, pt = int(r[1]), int(r[2]), unh(r[4])
        assert rc == BAD_RECORD_MAC, pos
        first_bad = 0 if pos < 16406 else 1
        assert consumed == 16406 * first_bad
        assert pt == data[:16384 * first_bad]


@pytest.mark.gpu
@pytest.mark.parametrize("keylen", [16, 32])
@pytest.mark.parametrize("mode", ["engine-client", "engine-server", "engine-both"])
def test_tls13_handshake_with_engine_cipher_suite(gpu, mode, keylen):
    """A full TLS 1.3 handshake of the reference picotls with {TLS_AES_*_GCM_SHA*, ptls_mi355x_aes*gcm} as the cipher
    suite on one or both sides (the other side minicrypto), then application data, KeyUpdates and tamper."""
    (r,) = run([f"handshake {mode} {keylen} 50000"])
    assert int(r[1]) == 10
    assert r[2] == ("TLS_AES_256_GCM_SHA384" if keylen == 32 else "TLS_AES_128_GCM_SHA256")
    assert r[3] == ("AES256-GCM" if keylen == 32 else "AES128-GCM")


RAPIDO = os.path.join(ROOT, "oracle", "_ref", "ref_rapido_harness")


def test_rapido_harness_pinned_by_minicrypto_without_gpu():
    """oracle/ref_rapido_harness.c itself (CPU only): lib/rapido.c sessions over loopback TCP with minicrypto as the
    record AEAD pass every check, so the GPU run below differs only in the cipher suite's AEAD."""
    if not os.path.exists(RAPIDO):
        pytest.skip("oracle/_ref/ref_rapido_harness not built (needs /root/reference)")
    r = subprocess.run([RAPIDO, "16", "minicrypto"], capture_output=True, text=True, timeout=110)
    assert r.returncode == 0 and r.stdout.startswith("ok 61 checks"), (r.stdout[-2000:], r.stderr[-2000:])


@pytest.mark.gpu
@pytest.mark.parametrize("keylen", [16, 32])
def test_rapido_sessions_over_engine_cipher_suite(gpu, keylen):
    """rapido (lib/rapido.c, unmodified) with the engine as its context's only cipher suite: handshakes over loopback
    TCP, 1 MB stream transfers each way (t/rapido_tests.c:290-340), a joined second connection carrying the stream
    under its own IV (t/rapido_tests.c:347-420), and engine <-> minicrypto sessions in both roles."""
    assert os.path.exists(RAPIDO), "oracle/_ref/ref_rapido_harness not built (oracle/Makefile, needs /root/reference)"
    r = subprocess.run([RAPIDO, str(keylen)], capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-3000:])
    want = "TLS_AES_256_GCM_SHA384 (AES256-GCM)" if keylen == 32 else "TLS_AES_128_GCM_SHA256 (AES128-GCM)"
    assert r.stdout.startswith("ok 61 checks, rapido over " + want), r.stdout
