"""CPU checkers for the AES-GCM engine -- TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg import this package, and only to check or to time a CPU baseline.  The
product (``rapido_amd``) never imports it.

* :func:`seal` / :func:`open_` / :func:`ecb` / :func:`batch` -- the CPU
  restatement in ``aesgcm_oracle.c`` (FIPS-197 + SP 800-38D, byte oriented),
  which follows the reference's ``lib/fusion.c:239-679`` semantics.
* :class:`Reference` -- the reference engine itself (``/root/reference/lib/fusion.c``
  compiled unmodified into ``oracle/_ref/libref_fusion.so`` by ``oracle/Makefile``).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
_ORACLE_SO = os.path.join(HERE, "_build", "liboracle.so")
_REF_SO = os.path.join(HERE, "_ref", "libref_fusion.so")
SIZE_MAX = (1 << 64) - 1

_lib = None


def build(quiet: bool = True) -> None:
    """Build the checkers (make -C oracle); the reference part only where /root/reference exists."""
    out = subprocess.run(["make", "-C", HERE], capture_output=True, text=True)
    if out.returncode != 0:
        raise RuntimeError("oracle build failed:\n" + out.stdout + out.stderr)
    if not quiet:
        print(out.stdout)


def _load():
    global _lib
    if _lib is None:
        if not os.path.exists(_ORACLE_SO):
            build()
        lib = C.CDLL(_ORACLE_SO)
        vp, sz = C.c_void_p, C.c_size_t
        lib.oracle_gcm_seal.argtypes = [vp, sz, vp, vp, sz, vp, sz, vp]
        lib.oracle_gcm_seal.restype = C.c_int
        lib.oracle_gcm_open.argtypes = [vp, sz, vp, vp, sz, vp, sz, vp]
        lib.oracle_gcm_open.restype = C.c_size_t
        lib.oracle_aes_ecb_encrypt.argtypes = [vp, sz, vp, vp]
        lib.oracle_aes_ecb_encrypt.restype = C.c_int
        lib.oracle_aes_ecb_encrypt_n.argtypes = [vp, sz, vp, vp, sz]
        lib.oracle_aes_ecb_encrypt_n.restype = C.c_int
        lib.oracle_aes_ecb_decrypt.argtypes = [vp, sz, vp, vp, sz]
        lib.oracle_aes_ecb_decrypt.restype = C.c_int
        lib.oracle_build_iv.argtypes = [vp, C.c_uint64, vp]
        lib.oracle_gf128_mul.argtypes = [vp, vp, vp]
        lib.oracle_gcm_batch.argtypes = [C.c_int, vp, sz, vp, vp, sz, vp, vp, vp, vp, C.c_int]
        lib.oracle_gcm_batch.restype = C.c_int
        lib.oracle_tls_seal_record.argtypes = [vp, sz, vp, C.c_uint64, C.c_uint8, vp, sz, sz, vp]
        lib.oracle_tls_seal_record.restype = C.c_size_t
        lib.oracle_tls_open_record.argtypes = [vp, sz, vp, C.c_uint64, vp, vp, vp]
        lib.oracle_tls_open_record.restype = C.c_size_t
        _lib = lib
    return _lib


def _buf(b: bytes):
    return C.create_string_buffer(bytes(b), max(len(b), 1))


def build_iv(static_iv: bytes, seq: int) -> bytes:
    """nonce = static_iv XOR (0^32 || BE64(seq)) -- lib/picotls.c:5291-5305."""
    out = C.create_string_buffer(12)
    _load().oracle_build_iv(_buf(static_iv), seq, out)
    return out.raw


def seal(key: bytes, iv: bytes, aad: bytes, pt: bytes) -> bytes:
    """AES-GCM seal with a 96-bit nonce: returns ciphertext || tag (16 B)."""
    out = C.create_string_buffer(len(pt) + 16)
    rc = _load().oracle_gcm_seal(_buf(key), len(key), _buf(iv), _buf(aad), len(aad), _buf(pt), len(pt), out)
    if rc != 0:
        raise ValueError("bad key size")
    return out.raw


def open_(key: bytes, iv: bytes, aad: bytes, ct_tag: bytes):
    """Returns the plaintext, or None where the reference returns SIZE_MAX."""
    out = C.create_string_buffer(max(len(ct_tag), 1))
    r = _load().oracle_gcm_open(_buf(key), len(key), _buf(iv), _buf(aad), len(aad), _buf(ct_tag), len(ct_tag), out)
    if r == SIZE_MAX:
        return None
    return out.raw[:r]


def ecb(key: bytes, block: bytes) -> bytes:
    out = C.create_string_buffer(16)
    if _load().oracle_aes_ecb_encrypt(_buf(key), len(key), _buf(block), out) != 0:
        raise ValueError("bad key size")
    return out.raw


def ecb_blocks(key: bytes, data: bytes, encrypt: bool = True) -> bytes:
    """AES-ECB over len(data) // 16 blocks: FIPS-197 Cipher (encrypt) or InvCipher (decrypt)."""
    assert len(data) % 16 == 0
    out = C.create_string_buffer(max(len(data), 1))
    f = _load().oracle_aes_ecb_encrypt_n if encrypt else _load().oracle_aes_ecb_decrypt
    if f(_buf(key), len(key), _buf(data), out, len(data) // 16) != 0:
        raise ValueError("bad key size")
    return out.raw[:len(data)]


def gf128_mul(x: bytes, y: bytes) -> bytes:
    out = C.create_string_buffer(16)
    _load().oracle_gf128_mul(_buf(x), _buf(y), out)
    return out.raw


def batch(is_seal: bool, key: bytes, static_iv: bytes, recs, src, dst, aad, status=None, nthreads: int = 8) -> None:
    """Batch seal/open over numpy arrays laid out like the engine's batch API.

    ``recs`` is a numpy structured array with the ptls_mi355x_record_t layout
    (see rapido_amd.RECORD_DTYPE); src/dst/aad are uint8 numpy arrays; status a
    uint32 numpy array (open only)."""
    import numpy as np

    lib = _load()
    st = status.ctypes.data if status is not None else None
    rc = lib.oracle_gcm_batch(1 if is_seal else 0, _buf(key), len(key), _buf(static_iv), recs.ctypes.data, len(recs),
                              src.ctypes.data, dst.ctypes.data, aad.ctypes.data if aad.size else _buf(b"\0"), st,
                              int(nthreads))
    if rc != 0:
        raise ValueError("oracle batch failed")
    del np


TLS_BAD_MAC = 2 ** 64 - 1  # oracle_tls_open_record: SIZE_MAX -> PTLS_ALERT_BAD_RECORD_MAC
TLS_NO_TYPE = 2 ** 64 - 2  # all-zero inner plaintext -> PTLS_ALERT_UNEXPECTED_MESSAGE


def tls_seal_record(key: bytes, static_iv: bytes, seq: int, content_type: int, fragment: bytes, pad: int = 0) -> bytes:
    """One TLS 1.3 record: header || seal(fragment || type || 0^pad) (lib/picotls.c:621-684)."""
    lib = _load()
    out = C.create_string_buffer(5 + len(fragment) + 1 + pad + 16)
    n = lib.oracle_tls_seal_record(key, len(key), static_iv, seq, content_type, _buf(fragment), len(fragment), pad, out)
    assert n == len(out.raw)
    return out.raw


def tls_open_record(key: bytes, static_iv: bytes, seq: int, wire: bytes):
    """-> (inner plaintext, content type) or TLS_BAD_MAC / TLS_NO_TYPE (lib/picotls.c:645-654,4779-4791)."""
    lib = _load()
    L = (wire[3] << 8) | wire[4]
    out = C.create_string_buffer(max(L, 1))
    t = C.c_uint8()
    n = lib.oracle_tls_open_record(key, len(key), static_iv, seq, _buf(wire), out, C.byref(t))
    if n in (TLS_BAD_MAC, TLS_NO_TYPE):
        return n
    return out.raw[:n], t.value


class Reference:
    """The reference lib/fusion.c engine (oracle/_ref), for golden vectors and the CPU baseline."""

    def __init__(self):
        if not os.path.exists(_REF_SO):
            raise FileNotFoundError(_REF_SO + " (built by oracle/Makefile where /root/reference exists)")
        lib = C.CDLL(_REF_SO)
        vp, sz = C.c_void_p, C.c_size_t
        lib.ref_supported.restype = C.c_int
        lib.ref_seal.argtypes = [vp, sz, vp, vp, sz, vp, sz, vp]
        lib.ref_open.argtypes = [vp, sz, vp, vp, sz, vp, sz, vp, vp]
        lib.ref_seal_supp.argtypes = [vp, sz, vp, vp, sz, vp, sz, vp, vp, sz, vp]
        lib.ref_slot_seal.argtypes = [vp, sz, vp, vp, sz, C.c_uint64, vp, sz, vp, sz, vp]
        lib.ref_slot_open.argtypes = [vp, sz, vp, vp, sz, C.c_uint64, vp, sz, vp, sz, vp]
        lib.ref_slot_open.restype = C.c_size_t
        lib.ref_ecb.argtypes = [vp, sz, vp, vp]
        lib.ref_ecb_decrypt.argtypes = [vp, sz, vp, vp]
        lib.ref_bench.argtypes = [sz, sz, sz, sz, C.c_int, C.POINTER(C.c_double)]
        lib.ref_bench.restype = C.c_int
        lib.ref_tls_send.argtypes = [vp, sz, vp, C.c_uint64, vp, sz, vp, sz, C.POINTER(C.c_size_t),
                                     C.POINTER(C.c_uint64)]
        lib.ref_tls_send.restype = C.c_int
        lib.ref_tls_receive.argtypes = [vp, sz, vp, C.c_uint64, vp, sz, vp, sz, C.POINTER(C.c_size_t),
                                        C.POINTER(C.c_size_t), C.POINTER(C.c_uint64)]
        lib.ref_tls_receive.restype = C.c_int
        self.lib = lib

    def supported(self) -> bool:
        return bool(self.lib.ref_supported())

    def seal(self, key, iv, aad, pt) -> bytes:
        out = C.create_string_buffer(len(pt) + 16)
        self.lib.ref_seal(_buf(key), len(key), _buf(iv), _buf(aad), len(aad), _buf(pt), len(pt), out)
        return out.raw

    def open_(self, key, iv, aad, ct_tag):
        n = len(ct_tag) - 16
        out = C.create_string_buffer(max(n, 1))
        ok = self.lib.ref_open(_buf(key), len(key), _buf(iv), _buf(aad), len(aad), _buf(ct_tag[:n]), n,
                               _buf(ct_tag[n:]), out)
        return out.raw[:n] if ok == 1 else None

    def seal_supp(self, key, iv, aad, pt, supp_key, supp_off):
        out = C.create_string_buffer(len(pt) + 16)
        so = C.create_string_buffer(16)
        self.lib.ref_seal_supp(_buf(key), len(key), _buf(iv), _buf(aad), len(aad), _buf(pt), len(pt), out,
                               _buf(supp_key), supp_off, so)
        return out.raw, so.raw

    def slot_seal(self, key, static_iv, seq, aad, pt, xor_iv=b""):
        out = C.create_string_buffer(len(pt) + 16)
        self.lib.ref_slot_seal(_buf(key), len(key), _buf(static_iv), _buf(xor_iv), len(xor_iv), seq, _buf(aad),
                               len(aad), _buf(pt), len(pt), out)
        return out.raw

    def slot_open(self, key, static_iv, seq, aad, ct_tag, xor_iv=b""):
        out = C.create_string_buffer(max(len(ct_tag), 1))
        r = self.lib.ref_slot_open(_buf(key), len(key), _buf(static_iv), _buf(xor_iv), len(xor_iv), seq, _buf(aad),
                                   len(aad), _buf(ct_tag), len(ct_tag), out)
        return None if r == SIZE_MAX else out.raw[:r]

    def ecb(self, key, block) -> bytes:
        out = C.create_string_buffer(16)
        self.lib.ref_ecb(_buf(key), len(key), _buf(block), out)
        return out.raw

    def ecb_decrypt(self, key, block) -> bytes:
        """cifra's cf_aes_decrypt (the reference minicrypto ECB decrypt, lib/cifra/aes-common.h:48-53)."""
        out = C.create_string_buffer(16)
        self.lib.ref_ecb_decrypt(_buf(key), len(key), _buf(block), out)
        return out.raw

    def tls_send(self, key, static_iv, seq0, data):
        """The reference ptls_send() (lib/picotls.c:4969-4988): -> (wire bytes, next seq)."""
        cap = len(data) + (len(data) // 16384 + 1) * 22 + 64
        out = C.create_string_buffer(cap)
        n, seq = C.c_size_t(), C.c_uint64()
        rc = self.lib.ref_tls_send(key, len(key), static_iv, seq0, _buf(data), len(data), out, cap, C.byref(n),
                                   C.byref(seq))
        if rc != 0:
            raise RuntimeError(f"ptls_send: {rc}")
        return out.raw[: n.value], seq.value

    def tls_receive(self, key, static_iv, seq0, wire):
        """The reference ptls_receive() over a whole buffer: -> (rc, plaintext, consumed, next seq)."""
        cap = len(wire) + 64
        out = C.create_string_buffer(cap)
        n, used, seq = C.c_size_t(), C.c_size_t(), C.c_uint64()
        rc = self.lib.ref_tls_receive(key, len(key), static_iv, seq0, _buf(wire), len(wire), out, cap, C.byref(n),
                                      C.byref(used), C.byref(seq))
        return rc, out.raw[: n.value], used.value, seq.value

    def bench(self, keylen: int, length: int, aadlen: int, nrec_per_thread: int, nthreads: int):
        """t/ptlsbench.c methodology; returns (seal B/s, open B/s, wall s, failed)."""
        res = (C.c_double * 4)()
        if self.lib.ref_bench(keylen, length, aadlen, nrec_per_thread, nthreads, res) != 0:
            raise ValueError("ref_bench: bad arguments")
        return res[0], res[1], res[2], bool(res[3])
