"""Every kernel family against the reference engine's own outputs, directly: tests/golden/fusion_random.json (192
random AES-GCM cases) and fusion_large.json (TLS-size records up to 64 KiB, as SHA-256 of the ciphertext + tag), both
produced by /root/reference/lib/fusion.c compiled unmodified (tests/golden/gen_golden.py).  No oracle in the loop:
the fixtures themselves are the expected bytes.  Each case is sealed and opened as a batch of one (nonce = the case's
IV: static IV = IV, seq 0)."""
import hashlib
import json
import os

import numpy as np
import pytest

import rapido_amd as ra
from conftest import FAMILIES, kernel_family
from rapido_amd import records
from test_gpu_parity import run_batch

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def golden(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)["cases"]


@pytest.fixture(params=FAMILIES)
def family(request, gpu):
    with kernel_family(request.param, framing=False):
        yield request.param


def seal_open_one(key, iv, aad, pt):
    """-> (ciphertext || tag, opened plaintext, open status) through the batch C-ABI"""
    recs, src_bytes, aad_bytes = records.layout(np.array([len(pt) + 16], np.uint64), np.array([len(aad)], np.uint64))
    recs["len"] = len(pt)
    recs["seq"] = 0
    src = np.zeros(src_bytes, np.uint8)
    a = int(recs[0]["src"])
    src[a:a + len(pt)] = np.frombuffer(pt, np.uint8)
    aadbuf = np.zeros(max(aad_bytes, 1), np.uint8)
    aadbuf[int(recs[0]["aad"]):int(recs[0]["aad"]) + len(aad)] = np.frombuffer(aad, np.uint8)
    eng = ra.Engine(key)
    try:
        ct, _ = run_batch(eng, True, iv, recs, src, src_bytes, aadbuf)
        d = int(recs[0]["dst"])
        sealed = ct[d:d + len(pt) + 16].tobytes()
        got, st = run_batch(eng, False, iv, recs, ct, src_bytes, aadbuf)
        return sealed, got[d:d + len(pt)].tobytes(), int(st[0])
    finally:
        eng.close()


def test_fusion_random_fixtures(family):
    for i, c in enumerate(golden("fusion_random.json")):
        key, iv, aad, pt = (bytes.fromhex(c[k]) for k in ("key", "iv", "aad", "pt"))
        sealed, opened, st = seal_open_one(key, iv, aad, pt)
        assert sealed.hex() == c["ct"], f"case {i}: len {len(pt)}, aad {len(aad)}"
        assert opened == pt and st == len(pt), f"case {i}"


def test_fusion_large_fixtures(family):
    for c in golden("fusion_large.json"):
        s = c["seed"]
        key = records.xorshift64star(s + 1, c["keylen"]).tobytes()
        iv = records.xorshift64star(s + 2, 12).tobytes()
        aad = records.xorshift64star(s + 3, c["aadlen"]).tobytes()
        pt = records.xorshift64star(s, c["len"]).tobytes()
        sealed, opened, st = seal_open_one(key, iv, aad, pt)
        assert hashlib.sha256(sealed[:c["len"]]).hexdigest() == c["ct_sha256"], f"len {c['len']} key {c['keylen']}"
        assert sealed[c["len"]:].hex() == c["tag"]
        assert opened == pt and st == c["len"]
