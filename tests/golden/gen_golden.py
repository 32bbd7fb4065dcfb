"""Generates the golden fixtures under tests/golden/ from the REFERENCE engine.

Run in the container that holds /root/reference (the reference is never present on the
GPU box): `python tests/golden/gen_golden.py`.  It drives the unmodified reference
lib/fusion.c + lib/picotls.c, compiled by oracle/Makefile into oracle/_ref/libref_fusion.so,
through oracle/ref_fusion_harness.c:

* fusion_random.json   -- 192 random AES-128/256-GCM cases (key, nonce, aad <= 64 B,
                          payload <= 1 KiB) with the full ciphertext || tag from the direct
                          core API ptls_fusion_aesgcm_encrypt (lib/fusion.c:239-495), plus
                          the open result of ptls_fusion_aesgcm_decrypt.
* fusion_large.json    -- (keylen, len, aadlen, seed) -> SHA-256(ciphertext) and tag for
                          TLS-sized records (1400 B, 16 KiB, 16 KiB + 1, ...); payload bytes
                          are rapido_amd.records.xorshift64star(seed, len).
* fusion_slot.json     -- TLS-framed records sealed through the AEAD slot exactly as the
                          record layer calls it (ptls_aead_new_direct + ptls_aead_xor_iv for
                          rapido's connection-id IV + ptls_aead_encrypt, lib/picotls.c:630-643,
                          lib/rapido.c:127-133), below fusion's slot capacity.
* fusion_supp.json     -- supplementary (header-protection) outputs, lib/fusion.c:472-487.
* tls_records.json     -- the reference TLS record layer (ptls_send / ptls_receive of
                          lib/picotls.c, driven by oracle/ref_record_harness.c over the fusion
                          core): send = wire bytes (SHA-256, full hex when small) for a stream of
                          xorshift64star(seed, len) application data from seq0; receive = the
                          reference's return code and plaintext for padded / tampered / all-zero
                          records (their wire bytes built by oracle.tls_seal_record).

The known-answer vectors transcribed from the reference's own tests (t/fusion.c,
t/picotls.c, deps/cifra/src/testmodes.c) are data inlined in tests/test_oracle.py and
tests/test_gpu_cipher.py, not generated here.
"""
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

import oracle  # noqa: E402


def xorshift_bytes(seed, n):
    from rapido_amd.records import xorshift64star
    return xorshift64star(seed, n).tobytes()


def main():
    oracle.build()
    ref = oracle.Reference()
    assert ref.supported(), "this CPU lacks AES-NI/PCLMUL/AVX2; fusion cannot run"
    rng = np.random.default_rng(20240807)

    cases = []
    for i in range(192):
        keylen = 16 if i % 2 == 0 else 32
        key = rng.integers(0, 256, keylen, dtype=np.uint8).tobytes()
        iv = rng.integers(0, 256, 12, dtype=np.uint8).tobytes()
        aad = rng.integers(0, 256, int(rng.integers(0, 65)), dtype=np.uint8).tobytes()
        ln = [0, 1, 15, 16, 17, 31, 32, 33][i] if i < 8 else int(rng.integers(0, 1025))
        pt = rng.integers(0, 256, ln, dtype=np.uint8).tobytes()
        ct = ref.seal(key, iv, aad, pt)
        assert ref.open_(key, iv, aad, ct) == pt
        cases.append({"key": key.hex(), "iv": iv.hex(), "aad": aad.hex(), "pt": pt.hex(), "ct": ct.hex()})
    with open(os.path.join(HERE, "fusion_random.json"), "w") as f:
        json.dump({"source": "reference lib/fusion.c direct API via oracle/_ref", "cases": cases}, f, indent=0)

    large = []
    for keylen in (16, 32):
        for ln, aadlen in ((1400, 5), (1500, 32), (4096, 5), (16383, 5), (16384, 5), (16385, 5), (16384, 13),
                           (65536, 5)):
            seed = 1000 + ln + keylen
            key = xorshift_bytes(seed + 1, keylen)
            iv = xorshift_bytes(seed + 2, 12)
            aad = xorshift_bytes(seed + 3, aadlen)
            pt = xorshift_bytes(seed, ln)
            ct = ref.seal(key, iv, aad, pt)
            large.append({"keylen": keylen, "len": ln, "aadlen": aadlen, "seed": seed,
                          "ct_sha256": hashlib.sha256(ct[:ln]).hexdigest(), "tag": ct[ln:].hex()})
    with open(os.path.join(HERE, "fusion_large.json"), "w") as f:
        json.dump({"source": "reference lib/fusion.c direct API via oracle/_ref",
                   "inputs": "key=xorshift64star(seed+1,keylen) iv=xorshift64star(seed+2,12) "
                             "aad=xorshift64star(seed+3,aadlen) pt=xorshift64star(seed,len)",
                   "cases": large}, f, indent=1)

    slot = []
    for i in range(48):
        keylen = 16 if i % 3 else 32
        key = rng.integers(0, 256, keylen, dtype=np.uint8).tobytes()
        static_iv = rng.integers(0, 256, 12, dtype=np.uint8).tobytes()
        conn_id = int(rng.integers(0, 2 ** 32))
        xor_iv = conn_id.to_bytes(4, "big")  # rapido derive_connection_aead_iv: iv[0..3] ^= BE32(id)
        data_len = int(rng.integers(0, 1300)) if i else 1399
        inner = rng.integers(0, 256, data_len, dtype=np.uint8).tobytes() + b"\x17"
        hdr = bytes([0x17, 0x03, 0x03, (len(inner) + 16) >> 8, (len(inner) + 16) & 0xFF])
        seq = int(rng.integers(0, 2 ** 24))
        ct = ref.slot_seal(key, static_iv, seq, hdr, inner, xor_iv=xor_iv)
        assert ref.slot_open(key, static_iv, seq, hdr, ct, xor_iv=xor_iv) == inner
        slot.append({"key": key.hex(), "static_iv": static_iv.hex(), "xor_iv": xor_iv.hex(), "seq": seq,
                     "aad": hdr.hex(), "pt": inner.hex(), "ct": ct.hex()})
    with open(os.path.join(HERE, "fusion_slot.json"), "w") as f:
        json.dump({"source": "reference ptls_fusion_aes{128,256}gcm through ptls_aead_encrypt", "cases": slot}, f,
                  indent=0)

    supp = []
    for i in range(16):
        keylen = 16 if i % 2 == 0 else 32
        key = rng.integers(0, 256, keylen, dtype=np.uint8).tobytes()
        skey = rng.integers(0, 256, keylen, dtype=np.uint8).tobytes()
        iv = rng.integers(0, 256, 12, dtype=np.uint8).tobytes()
        aad = rng.integers(0, 256, 20, dtype=np.uint8).tobytes()
        ln = int(rng.integers(20, 200))
        pt = rng.integers(0, 256, ln, dtype=np.uint8).tobytes()
        off = int(rng.integers(0, ln))  # the 16-byte sample may cover the tag
        ct, so = ref.seal_supp(key, iv, aad, pt, skey, off)
        supp.append({"key": key.hex(), "supp_key": skey.hex(), "iv": iv.hex(), "aad": aad.hex(), "pt": pt.hex(),
                     "ct": ct.hex(), "sample_off": off, "supp_out": so.hex()})
    with open(os.path.join(HERE, "fusion_supp.json"), "w") as f:
        json.dump({"source": "reference ptls_fusion_aesgcm_encrypt with supp", "cases": supp}, f, indent=0)
    tls = {"send": [], "receive": []}
    trng = np.random.default_rng(8446)
    for keylen in (16, 32):
        for ln in (1, 15, 16, 17, 255, 1400, 16383, 16384, 16385, 40000):
            seed = 5000 + ln + keylen
            key, iv = xorshift_bytes(seed + 1, keylen), xorshift_bytes(seed + 2, 12)
            seq0 = int(trng.integers(0, 2 ** 20))
            data = xorshift_bytes(seed, ln)
            wire, seq_after = ref.tls_send(key, iv, seq0, data)
            rc, pt, used, _ = ref.tls_receive(key, iv, seq0, wire)
            assert rc == 0 and pt == data and used == len(wire)
            case = {"keylen": keylen, "len": ln, "seed": seed, "seq0": seq0, "seq_after": seq_after,
                    "wire_len": len(wire), "wire_sha256": hashlib.sha256(wire).hexdigest()}
            if len(wire) <= 128:
                case["wire"] = wire.hex()
            tls["send"].append(case)
    for i, (ln, ctype, pad, tamper) in enumerate([(50, 23, 0, False), (50, 23, 1, False), (50, 23, 15, False),
                                                  (50, 23, 16, False), (0, 23, 40, False), (300, 23, 333, False),
                                                  (16000, 23, 384, False), (10, 23, 0, True), (0, 0, 7, False),
                                                  (0, 0, 0, False)]):
        keylen = 16 if i % 2 == 0 else 32
        key = trng.integers(0, 256, keylen, dtype=np.uint8).tobytes()
        iv = trng.integers(0, 256, 12, dtype=np.uint8).tobytes()
        seq = int(trng.integers(0, 2 ** 24))
        frag = trng.integers(1, 256, ln, dtype=np.uint8).tobytes()
        wire = bytearray(oracle.tls_seal_record(key, iv, seq, ctype, frag, pad))
        if tamper:
            wire[-1] ^= 0x80
        rc, pt, used, _ = ref.tls_receive(key, iv, seq, bytes(wire))
        tls["receive"].append({"key": key.hex(), "iv": iv.hex(), "seq": seq, "wire": bytes(wire).hex(), "rc": rc,
                               "plaintext": pt.hex()})
    with open(os.path.join(HERE, "tls_records.json"), "w") as f:
        json.dump({"source": "reference lib/picotls.c ptls_send / ptls_receive via oracle/ref_record_harness.c",
                   "inputs": "send: key=xorshift64star(seed+1,keylen) iv=xorshift64star(seed+2,12) "
                             "data=xorshift64star(seed,len); receive: wire from oracle.tls_seal_record",
                   "rc": "0 ok, 20 PTLS_ALERT_BAD_RECORD_MAC, 10 PTLS_ALERT_UNEXPECTED_MESSAGE", **tls}, f, indent=0)
    print("golden fixtures written to", HERE)


if __name__ == "__main__":
    main()
