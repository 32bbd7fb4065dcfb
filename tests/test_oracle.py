"""Pins the CPU oracle (oracle/aesgcm_oracle.c) to the reference's own known answers and to
golden vectors produced by the reference engine (tests/golden/, see gen_golden.py).  CPU only."""
import hashlib
import json
import os

import pytest

import oracle

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def golden(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def test_ecb_kats():
    # t/fusion.c:71-85 (zero key, "hello world!!!!!") and t/picotls.c:290-304 (FIPS-197 C.1 / C.3)
    assert oracle.ecb(bytes(16), b"hello world!!!!!").hex() == "172afecb50b5f1237814b2f7cb51d0f7"
    assert oracle.ecb(bytes(32), b"hello world!!!!!").hex() == "2a033f0627b3554aa4fe5786550736ff"
    pt = bytes.fromhex("00112233445566778899aabbccddeeff")
    assert oracle.ecb(bytes(range(16)), pt).hex() == "69c4e0d86a7b0430d8cdb78070b4c55a"
    assert oracle.ecb(bytes(range(32)), pt).hex() == "8ea2b7ca516745bfeafc49904b496089"


def test_ecb_decrypt_kats():
    # t/picotls.c:266-307 test_ecb: the ciphertext decrypts back to the FIPS-197 C.1 / C.3 plaintext
    pt = bytes.fromhex("00112233445566778899aabbccddeeff")
    for key, ct in ((bytes(range(16)), "69c4e0d86a7b0430d8cdb78070b4c55a"),
                    (bytes(range(32)), "8ea2b7ca516745bfeafc49904b496089")):
        assert oracle.ecb_blocks(key, bytes.fromhex(ct), encrypt=False) == pt
        assert oracle.ecb_blocks(key, pt * 3, encrypt=True) == bytes.fromhex(ct) * 3
    # t/fusion.c:71-85 vectors backwards
    assert oracle.ecb_blocks(bytes(16), bytes.fromhex("172afecb50b5f1237814b2f7cb51d0f7"), False) == b"hello world!!!!!"
    assert oracle.ecb_blocks(bytes(32), bytes.fromhex("2a033f0627b3554aa4fe5786550736ff"), False) == b"hello world!!!!!"


@pytest.mark.skipif(not os.path.exists(os.path.join(os.path.dirname(oracle.__file__), "_ref", "libref_fusion.so")),
                    reason="reference build (oracle/_ref) not present")
def test_ecb_decrypt_vs_reference_cifra():
    """The oracle's InvCipher against the reference's own minicrypto AES decryption (deps/cifra/src/aes.c,
    lib/cifra/aes-common.h:48-53), and its Cipher against fusion's aesecb_encrypt, on random keys and blocks."""
    import numpy as np
    ref = oracle.Reference()
    rng = np.random.default_rng(5)
    for i in range(300):
        kl = 16 if i % 2 else 32
        key = rng.integers(0, 256, kl, dtype=np.uint8).tobytes()
        blk = rng.integers(0, 256, 16, dtype=np.uint8).tobytes()
        assert oracle.ecb_blocks(key, blk, encrypt=False) == ref.ecb_decrypt(key, blk)
        if ref.supported():
            assert oracle.ecb_blocks(key, blk, encrypt=True) == ref.ecb(key, blk)


def test_ctr_kat():
    # t/picotls.c:312-321: AES128-CTR keystream block = AES-ECB(iv)
    key = bytes.fromhex("2b7e151628aed2a6abf7158809cf4f3c")
    iv = bytes.fromhex("6bc1bee22e409f96e93d7e117393172a")
    assert oracle.ecb(key, iv).hex() == "3ad77bb40d7a3660a89ecaf32466ef97"


MV = [  # McGrew-Viega GCM test cases 1-4, deps/cifra/src/testmodes.c:395-440 (AES-128, 96-bit IV)
    ("00" * 16, "", "", "00" * 12, "", "58e2fccefa7e3061367f1d57a4e7455a"),
    ("00" * 16, "00" * 16, "", "00" * 12, "0388dace60b6a392f328c2b971b2fe78", "ab6e47d42cec13bdf53a67b21257bddf"),
    ("feffe9928665731c6d6a8f9467308308",
     "d9313225f88406e5a55909c5aff5269a86a7a9531534f7da2e4c303d8a318a721c3c0c95956809532fcf0e2449a6b525"
     "b16aedf5aa0de657ba637b391aafd255", "", "cafebabefacedbaddecaf888",
     "42831ec2217774244b7221b784d0d49ce3aa212f2c02a4e035c17e2329aca12e21d514b25466931c7d8f6a5aac84aa05"
     "1ba30b396a0aac973d58e091473f5985", "4d5c2af327cd64a62cf35abd2ba6fab4"),
    ("feffe9928665731c6d6a8f9467308308",
     "d9313225f88406e5a55909c5aff5269a86a7a9531534f7da2e4c303d8a318a721c3c0c95956809532fcf0e2449a6b525"
     "b16aedf5aa0de657ba637b39", "feedfacedeadbeeffeedfacedeadbeefabaddad2", "cafebabefacedbaddecaf888",
     "42831ec2217774244b7221b784d0d49ce3aa212f2c02a4e035c17e2329aca12e21d514b25466931c7d8f6a5aac84aa05"
     "1ba30b396a0aac973d58e091", "5bc94fbc3221a5db94fae95ae7121a47"),
]


# AES-256 test cases 13-16 of the GCM specification (McGrew & Viega, "The Galois/Counter Mode of Operation",
# Appendix B): not in the reference (cifra's list stops at AES-192); published known answers, which the oracle pinned
# by the reference engine's own outputs reproduces.  (key, plaintext, aad, iv, ciphertext prefix, tag)
MV256 = [
    ("00" * 32, "", "", "00" * 12, "", "530f8afbc74536b9a963b4f1c4cb738b"),
    ("00" * 32, "00" * 16, "", "00" * 12, "cea7403d4d606b6e074ec5d3baf39d18", "d0d1c8a799996bf0265b98b5d48ab919"),
    ("feffe9928665731c6d6a8f9467308308" * 2, MV[2][1], "", "cafebabefacedbaddecaf888",
     "522dc1f099567d07f47f37a32a84427d", "b094dac5d93471bdec1a502270e3cc6c"),
    ("feffe9928665731c6d6a8f9467308308" * 2, MV[3][1], MV[3][2], "cafebabefacedbaddecaf888",
     "522dc1f099567d07f47f37a32a84427d", "76fc6ece0f4e1768cddf8853bb2d551b"),
]


@pytest.mark.parametrize("key,pt,aad,iv,ct,tag", MV256)
def test_gcm_spec_aes256(key, pt, aad, iv, ct, tag):
    out = oracle.seal(bytes.fromhex(key), bytes.fromhex(iv), bytes.fromhex(aad), bytes.fromhex(pt)).hex()
    assert out.startswith(ct) and out.endswith(tag) and len(out) == len(pt) + 32


@pytest.mark.parametrize("key,pt,aad,iv,ct,tag", MV)
def test_mcgrew_viega(key, pt, aad, iv, ct, tag):
    out = oracle.seal(bytes.fromhex(key), bytes.fromhex(iv), bytes.fromhex(aad), bytes.fromhex(pt))
    assert out.hex() == ct + tag
    assert oracle.open_(bytes.fromhex(key), bytes.fromhex(iv), bytes.fromhex(aad), out) == bytes.fromhex(pt)


def test_fusion_kats():
    from test_gpu_parity import GCM_VECTORS, HELLO, HELLO_EXPECTED, HELLO_KEY
    # gcm_basic (t/fusion.c:89-126), gcm_capacity (:128-139), gcm_test_vectors (:161-183), gcm_iv96 (:197-231)
    assert oracle.seal(bytes(16), bytes(12), b"hello", bytes(16)).hex() == \
        "0388dace60b6a392f328c2b971b2fe78973fbca65477bf4785b0d561f7e3fd6c"
    assert oracle.seal(bytes(16), bytes(12), b"a", b"X").hex() == "5b27215ed81a702e3941c80577d52fcb57"
    for aadlen, ptlen, tag in GCM_VECTORS:
        assert oracle.seal(bytes(16), bytes(12), bytes(aadlen), bytes(ptlen))[ptlen:].hex() == tag
    assert oracle.seal(HELLO_KEY, bytes(range(20, 32)), bytes(range(20)), HELLO).hex() == HELLO_EXPECTED
    iv96 = bytes(a ^ b for a, b in zip(bytes([20, 20, 20, 20]) + bytes(range(24, 32)), bytes([0, 1, 2, 3]) + bytes(8)))
    assert oracle.seal(HELLO_KEY, iv96, bytes(range(20)), HELLO).hex() == HELLO_EXPECTED
    bad = bytearray(oracle.seal(HELLO_KEY, iv96, bytes(range(20)), HELLO))
    bad[-1] ^= 1
    assert oracle.open_(HELLO_KEY, iv96, bytes(range(20)), bytes(bad)) is None
    assert oracle.open_(HELLO_KEY, iv96, b"", b"short") is None  # inlen < 16 -> SIZE_MAX


def test_supplementary_kats():
    # t/fusion.c:161-191 supp column: AES-ECB(key 0x01*16, ciphertext bytes 2..17)
    for aadlen, ptlen, want in ((13, 17, "4576f18ef3ae9dfd37cf72c4592da874"), (13, 32, "a062016e90dcc316d061fde5424cf34f")):
        ct = oracle.seal(bytes(16), bytes(12), bytes(aadlen), bytes(ptlen))
        assert oracle.ecb(bytes([1] * 16), ct[2:18]).hex() == want


def test_golden_random():
    for c in golden("fusion_random.json")["cases"]:
        key, iv, aad, pt = (bytes.fromhex(c[k]) for k in ("key", "iv", "aad", "pt"))
        assert oracle.seal(key, iv, aad, pt).hex() == c["ct"]
        assert oracle.open_(key, iv, aad, bytes.fromhex(c["ct"])) == pt


def test_golden_large():
    from rapido_amd.records import xorshift64star
    for c in golden("fusion_large.json")["cases"]:
        s = c["seed"]
        key = xorshift64star(s + 1, c["keylen"]).tobytes()
        iv = xorshift64star(s + 2, 12).tobytes()
        aad = xorshift64star(s + 3, c["aadlen"]).tobytes()
        pt = xorshift64star(s, c["len"]).tobytes()
        out = oracle.seal(key, iv, aad, pt)
        assert hashlib.sha256(out[:c["len"]]).hexdigest() == c["ct_sha256"]
        assert out[c["len"]:].hex() == c["tag"]


def test_golden_slot_records():
    """TLS-framed records through the reference AEAD slot (with rapido's connection-id IV xor)."""
    for c in golden("fusion_slot.json")["cases"]:
        key, siv, xiv = bytes.fromhex(c["key"]), bytes.fromhex(c["static_iv"]), bytes.fromhex(c["xor_iv"])
        siv = bytes(a ^ b for a, b in zip(siv, xiv + bytes(12 - len(xiv))))
        nonce = oracle.build_iv(siv, c["seq"])
        assert oracle.seal(key, nonce, bytes.fromhex(c["aad"]), bytes.fromhex(c["pt"])).hex() == c["ct"]


def test_golden_supp():
    for c in golden("fusion_supp.json")["cases"]:
        key, iv, aad, pt = (bytes.fromhex(c[k]) for k in ("key", "iv", "aad", "pt"))
        ct = oracle.seal(key, iv, aad, pt)
        assert ct.hex() == c["ct"]
        off = c["sample_off"]
        assert oracle.ecb(bytes.fromhex(c["supp_key"]), ct[off:off + 16]).hex() == c["supp_out"]


def test_build_iv():
    # lib/picotls.c:5291-5305
    siv = bytes(range(12))
    got = oracle.build_iv(siv, 0x0102030405060708)
    assert got == bytes([0, 1, 2, 3, 4 ^ 1, 5 ^ 2, 6 ^ 3, 7 ^ 4, 8 ^ 5, 9 ^ 6, 10 ^ 7, 11 ^ 8])


@pytest.mark.skipif(not os.path.exists(os.path.join(os.path.dirname(oracle.__file__), "_ref", "libref_fusion.so")),
                    reason="reference build (oracle/_ref) not present")
def test_oracle_vs_reference_engine_random():
    """Cross-check against lib/fusion.c itself (needs an AES-NI host)."""
    import numpy as np
    ref = oracle.Reference()
    if not ref.supported():
        pytest.skip("host CPU lacks AES-NI/PCLMUL/AVX2")
    rng = np.random.default_rng(99)
    for i in range(200):
        kl = 16 if i % 2 else 32
        key = rng.integers(0, 256, kl, dtype=np.uint8).tobytes()
        iv = rng.integers(0, 256, 12, dtype=np.uint8).tobytes()
        aad = rng.integers(0, 256, int(rng.integers(0, 50)), dtype=np.uint8).tobytes()
        pt = rng.integers(0, 256, int(rng.integers(0, 3000)), dtype=np.uint8).tobytes()
        assert oracle.seal(key, iv, aad, pt) == ref.seal(key, iv, aad, pt)
