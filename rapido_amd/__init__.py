"""rapido_amd -- MI355X (gfx950) AES-GCM engine for picotls' AEAD slot.

The product is the C-ABI library ``rapido_amd/_lib/libptls_mi355x.so`` (HIP kernels +
host C adapter, declared in ``include/ptls_mi355x.h``).  This module is a thin ctypes
mirror used by the tests and the benchmark; it mirrors the reference's own entry points
so the parity tests read like the reference's tests:

* :func:`aead_new_direct` / :class:`Aead` -- ``ptls_aead_new_direct`` + the inline
  dispatchers ``ptls_aead_encrypt/_s/_decrypt/_xor_iv/_encrypt_init/_update/_final``
  (lib/picotls.c:5268-5289, include/picotls.h:1513-1564), called through the
  engine's exported ``ptls_aead_algorithm_t`` vtables exactly as picotls does.
* :func:`cipher_new` / :class:`Cipher` -- ``ptls_cipher_new/_init/_encrypt``.
* :class:`Engine` -- the direct engine API (mirror of ``ptls_fusion_aesgcm_*``,
  include/picotls/fusion.h:48-88) and the batch extension (the hot path).

There is no fallback: if the library is missing or no gfx950 GPU is present, the
calls fail loudly.
"""
from __future__ import annotations

import ctypes as C
import os
import weakref

try:  # load torch's bundled HIP runtime first: same SONAME, so one runtime serves both
    import torch as _torch  # noqa: F401
except Exception:  # pragma: no cover - torch is optional for the C-ABI itself
    _torch = None

import numpy as np

PKG = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("PTLS_MI355X_LIB") or os.path.join(PKG, "_lib", "libptls_mi355x.so")
SIZE_MAX = (1 << 64) - 1

#: numpy mirror of ptls_mi355x_record_t (include/ptls_mi355x.h)
RECORD_DTYPE = np.dtype([("src", "<u8"), ("dst", "<u8"), ("aad", "<u8"), ("seq", "<u8"), ("len", "<u4"),
                         ("aadlen", "<u4")])
assert RECORD_DTYPE.itemsize == 40

#: numpy mirror of ptls_mi355x_tls_record_t (include/ptls_mi355x.h section 4)
TLS_RECORD_DTYPE = np.dtype([("src", "<u8"), ("dst", "<u8"), ("seq", "<u8"), ("len", "<u4"), ("type", "<u4")])
#: ptls_mi355x_tls_deliver_t: one part of a delivery (slots, out, capacity, first record, records, any_type)
TLS_DELIVER_DTYPE = np.dtype([("slots", "<u8"), ("out", "<u8"), ("capacity", "<u8"), ("k0", "<u4"), ("n", "<u4"),
                              ("any_type", "<u4"), ("pad", "<u4")])
assert TLS_RECORD_DTYPE.itemsize == 32
TLS_HEADER_SIZE = 5
TLS_MAX_FRAGMENT = 16384
TLS_MAX_RECORD = 16384 + 256
TLS_OVERHEAD = 5 + 1 + 16
TLS_BAD_RECORD_MAC = 0xFFFFFFFF  # -> PTLS_ALERT_BAD_RECORD_MAC (20)
TLS_UNEXPECTED_MESSAGE = 0xFFFFFFFE  # -> PTLS_ALERT_UNEXPECTED_MESSAGE (10)
TLS_NOT_PROCESSED = 0xFFFFFFFD  # behind a failed record of its connection (OPEN_STOP_AT_FAILURE)
OPEN_STOP_AT_FAILURE = 1

#: every symbol include/ptls_mi355x.h declares
EXPORTED_FUNCTIONS = (
    "ptls_mi355x_is_supported", "ptls_mi355x_aesgcm_new", "ptls_mi355x_aesgcm_free", "ptls_mi355x_aesgcm_release",
    "ptls_mi355x_device_check", "ptls_mi355x_aesgcm_new_on", "ptls_mi355x_aesgcm_device",
    "ptls_mi355x_aesgcm_encrypt", "ptls_mi355x_aesgcm_decrypt", "ptls_mi355x_aesecb_encrypt",
    "ptls_mi355x_seal_batch", "ptls_mi355x_open_batch", "ptls_mi355x_order_by_length",
    "ptls_mi355x_seal_batch_ordered", "ptls_mi355x_open_batch_ordered", "ptls_mi355x_set_lanes_per_record",
    "ptls_mi355x_get_lanes_per_record", "ptls_mi355x_kernel_name", "ptls_mi355x_last_error",
    "ptls_mi355x_batch_ghash_reads", "ptls_mi355x_build_id",
    "ptls_mi355x_tls_seal_records", "ptls_mi355x_tls_open_records", "ptls_mi355x_tls_seal_records_multi",
    "ptls_mi355x_tls_open_records_multi", "ptls_mi355x_set_tls_window_records",
    "ptls_mi355x_set_aead_window_records", "ptls_mi355x_set_slot_zero_copy_bytes",
    "ptls_mi355x_set_work_ticket_origin", "ptls_mi355x_set_seg32_records", "ptls_mi355x_tls_plan_send",
    "ptls_mi355x_tls_parse_records", "ptls_mi355x_tls_open_records_ex", "ptls_mi355x_aes_new", "ptls_mi355x_aes_free",
    "ptls_mi355x_aes_ecb", "ptls_mi355x_aes_ecb_batch", "ptls_mi355x_set_win16_records",
    "ptls_mi355x_set_split_records", "ptls_mi355x_record_layer_new", "ptls_mi355x_record_layer_free",
    "ptls_mi355x_record_layer_get_seq", "ptls_mi355x_record_layer_set_seq", "ptls_mi355x_record_layer_seal",
    "ptls_mi355x_record_layer_open", "ptls_mi355x_record_layer_last_error", "ptls_mi355x_record_layer_register",
    "ptls_mi355x_record_layer_unregister", "ptls_mi355x_record_layer_set_zero_copy_bytes",
    "ptls_mi355x_record_layer_seal_multi", "ptls_mi355x_record_layer_open_multi",
    "ptls_mi355x_record_layer_open_record", "ptls_mi355x_record_layer_rekey", "ptls_mi355x_record_layer_seal_submit",
    "ptls_mi355x_record_layer_open_submit", "ptls_mi355x_record_layer_wait", "ptls_mi355x_record_layer_pending",
    "ptls_mi355x_record_layer_flush", "ptls_mi355x_record_layer_set_coalesce", "ptls_mi355x_record_layer_launches",
    "ptls_mi355x_record_layer_cork",
    "ptls_mi355x_record_layer_set_direct_dma", "ptls_mi355x_tls_deliver_records", "ptls_mi355x_prepare_copies",
    "ptls_mi355x_record_layer_reserve", "ptls_mi355x_fault_journal_install", "ptls_mi355x_fault_journal_installed",
    "ptls_mi355x_fault_journal_faults", "ptls_mi355x_fault_journal_report", "ptls_mi355x_fault_journal_note",
    "ptls_mi355x_slot_engine_errors", "ptls_mi355x_test_slot_without_engine", "ptls_mi355x_test_inject_engine_errors",
    "ptls_mi355x_seal_batch_multikey", "ptls_mi355x_open_batch_multikey", "ptls_mi355x_tls_seal_records_multikey",
    "ptls_mi355x_tls_open_records_multikey", "ptls_mi355x_kernel_name_multikey", "ptls_mi355x_order_by_key",
    "ptls_mi355x_seal_batch_multikey_ordered", "ptls_mi355x_open_batch_multikey_ordered",
)
EXPORTED_OBJECTS = ("ptls_mi355x_aes128gcm", "ptls_mi355x_aes256gcm", "ptls_mi355x_aes128ctr",
                    "ptls_mi355x_aes256ctr", "ptls_mi355x_aes128ecb", "ptls_mi355x_aes256ecb")

# ----------------------------------------------------------------- picotls ABI (ctypes) ---
vp, sz, u64 = C.c_void_p, C.c_size_t, C.c_uint64

_DISPOSE = C.CFUNCTYPE(None, vp)
_XOR_IV = C.CFUNCTYPE(None, vp, vp, sz)
_ENC_INIT = C.CFUNCTYPE(None, vp, u64, vp, sz)
_ENC_UPDATE = C.CFUNCTYPE(sz, vp, vp, vp, sz)
_ENC_FINAL = C.CFUNCTYPE(sz, vp, vp)
_ENCRYPT = C.CFUNCTYPE(None, vp, vp, vp, sz, u64, vp, sz, vp)
_DECRYPT = C.CFUNCTYPE(sz, vp, vp, vp, sz, u64, vp, sz)
_AEAD_SETUP = C.CFUNCTYPE(C.c_int, vp, C.c_int, vp, vp)
_CIPHER_SETUP = C.CFUNCTYPE(C.c_int, vp, C.c_int, vp)
_C_DISPOSE = C.CFUNCTYPE(None, vp)
_C_INIT = C.CFUNCTYPE(None, vp, vp)
_C_TRANSFORM = C.CFUNCTYPE(None, vp, vp, vp, sz)


class CipherContext(C.Structure):  # include/picotls.h:311-317
    _fields_ = [("algo", vp), ("do_dispose", _C_DISPOSE), ("do_init", _C_INIT), ("do_transform", _C_TRANSFORM)]


class CipherAlgorithm(C.Structure):  # include/picotls.h:322-329
    _fields_ = [("name", C.c_char_p), ("key_size", sz), ("block_size", sz), ("iv_size", sz), ("context_size", sz),
                ("setup_crypto", _CIPHER_SETUP)]


class SupplementaryEncryption(C.Structure):  # include/picotls.h:331-335
    _fields_ = [("ctx", vp), ("input", vp), ("output", C.c_uint8 * 16)]


class AeadContext(C.Structure):  # include/picotls.h:341-353
    _fields_ = [("algo", vp), ("dispose_crypto", _DISPOSE), ("do_xor_iv", _XOR_IV), ("do_encrypt_init", _ENC_INIT),
                ("do_encrypt_update", _ENC_UPDATE), ("do_encrypt_final", _ENC_FINAL), ("do_encrypt", _ENCRYPT),
                ("do_decrypt", _DECRYPT)]


class AeadAlgorithm(C.Structure):  # include/picotls.h:358-400
    _fields_ = [("name", C.c_char_p), ("confidentiality_limit", u64), ("integrity_limit", u64),
                ("ctr_cipher", C.POINTER(CipherAlgorithm)), ("ecb_cipher", C.POINTER(CipherAlgorithm)),
                ("key_size", sz), ("iv_size", sz), ("tag_size", sz), ("context_size", sz),
                ("setup_crypto", _AEAD_SETUP)]


_lib = None


def lib() -> C.CDLL:
    """The engine library (built by rapido_amd.build); raises if it is missing."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} not built: run `python -m rapido_amd.build` (or __graft_entry__.build())")
        L = C.CDLL(LIB_PATH)
        L.ptls_mi355x_is_supported.restype = C.c_int
        L.ptls_mi355x_aesgcm_new.argtypes = [vp, sz, sz]
        L.ptls_mi355x_aesgcm_new.restype = vp
        L.ptls_mi355x_aesgcm_free.argtypes = [vp]
        if hasattr(L, "ptls_mi355x_aesgcm_release"):  # (absent from older builds used in A/B timing runs)
            L.ptls_mi355x_aesgcm_release.argtypes = [vp]
            L.ptls_mi355x_device_check.argtypes = []
            L.ptls_mi355x_aesgcm_new_on.argtypes = [C.c_int, vp, sz, sz]
            L.ptls_mi355x_aesgcm_new_on.restype = vp
        L.ptls_mi355x_aesgcm_device.argtypes = [vp]
        L.ptls_mi355x_aesgcm_encrypt.argtypes = [vp, vp, vp, sz, vp, vp, sz]
        L.ptls_mi355x_aesgcm_decrypt.argtypes = [vp, vp, vp, sz, vp, vp, sz, vp]
        L.ptls_mi355x_aesecb_encrypt.argtypes = [vp, vp, vp, sz]
        L.ptls_mi355x_seal_batch.argtypes = [vp, vp, vp, sz, vp, vp, vp, vp]
        L.ptls_mi355x_open_batch.argtypes = [vp, vp, vp, sz, vp, vp, vp, vp, vp]
        L.ptls_mi355x_order_by_length.argtypes = [vp, vp, sz, vp, vp]
        L.ptls_mi355x_seal_batch_ordered.argtypes = [vp, vp, vp, vp, sz, vp, vp, vp, vp]
        L.ptls_mi355x_open_batch_ordered.argtypes = [vp, vp, vp, vp, sz, vp, vp, vp, vp, vp]
        L.ptls_mi355x_set_lanes_per_record.argtypes = [C.c_int]
        L.ptls_mi355x_kernel_name.argtypes = [C.c_int, sz, sz, C.c_int]
        L.ptls_mi355x_kernel_name.restype = C.c_char_p
        L.ptls_mi355x_last_error.restype = C.c_char_p
        L.ptls_mi355x_build_id.restype = C.c_char_p
        L.ptls_mi355x_tls_seal_records.argtypes = [vp, vp, vp, sz, vp, vp, vp]
        L.ptls_mi355x_tls_open_records.argtypes = [vp, vp, vp, sz, vp, vp, vp, vp, vp]
        L.ptls_mi355x_tls_seal_records_multi.argtypes = [vp, vp, vp, vp, sz, vp, vp, vp]
        L.ptls_mi355x_set_tls_window_records.argtypes = [sz]
        L.ptls_mi355x_set_tls_window_records.restype = sz
        L.ptls_mi355x_set_aead_window_records.argtypes = [sz]
        L.ptls_mi355x_set_aead_window_records.restype = sz
        L.ptls_mi355x_set_slot_zero_copy_bytes.argtypes = [sz]
        L.ptls_mi355x_set_slot_zero_copy_bytes.restype = sz
        L.ptls_mi355x_set_work_ticket_origin.argtypes = [C.c_uint32]
        L.ptls_mi355x_set_seg32_records.argtypes = [sz]
        L.ptls_mi355x_set_seg32_records.restype = sz
        L.ptls_mi355x_set_work_ticket_origin.restype = C.c_uint32
        L.ptls_mi355x_tls_open_records_multi.argtypes = [vp, vp, vp, vp, sz, vp, vp, vp, vp, vp]
        if hasattr(L, "ptls_mi355x_record_layer_new"):  # (absent from older builds used in A/B timing runs)
            L.ptls_mi355x_record_layer_new.argtypes = [vp, sz, vp, u64]
            L.ptls_mi355x_record_layer_new.restype = vp
            L.ptls_mi355x_record_layer_free.argtypes = [vp]
            L.ptls_mi355x_record_layer_get_seq.argtypes = [vp]
            L.ptls_mi355x_record_layer_get_seq.restype = u64
            L.ptls_mi355x_record_layer_set_seq.argtypes = [vp, u64]
            L.ptls_mi355x_record_layer_seal.argtypes = [vp, vp, sz, C.c_uint8, vp, sz, C.POINTER(sz), C.POINTER(sz)]
            L.ptls_mi355x_record_layer_open.argtypes = [vp, vp, sz, C.POINTER(sz), vp, sz, C.POINTER(sz), C.POINTER(sz)]
            L.ptls_mi355x_record_layer_last_error.restype = C.c_char_p
            L.ptls_mi355x_record_layer_register.argtypes = [vp, vp, sz]
            L.ptls_mi355x_record_layer_unregister.argtypes = [vp, vp]
            L.ptls_mi355x_record_layer_set_zero_copy_bytes.argtypes = [vp, sz]
            L.ptls_mi355x_record_layer_set_zero_copy_bytes.restype = sz
            L.ptls_mi355x_record_layer_seal_multi.argtypes = [vp, sz, vp, vp, C.c_uint8, vp, vp, vp, vp]
            L.ptls_mi355x_record_layer_open_multi.argtypes = [vp, sz, vp, vp, vp, vp, vp, vp, vp, vp]
        if hasattr(L, "ptls_mi355x_record_layer_rekey"):
            L.ptls_mi355x_record_layer_open_record.argtypes = [vp, vp, sz, C.POINTER(sz), vp, sz, C.POINTER(sz),
                                                               C.POINTER(C.c_uint8)]
            L.ptls_mi355x_record_layer_rekey.argtypes = [vp, vp, sz, vp]
            L.ptls_mi355x_record_layer_seal_submit.argtypes = [vp, sz, vp, vp, C.c_uint8, vp, vp, C.POINTER(u64)]
            L.ptls_mi355x_record_layer_open_submit.argtypes = [vp, sz, vp, vp, vp, vp, vp, C.POINTER(u64)]
            L.ptls_mi355x_record_layer_wait.argtypes = [vp, u64, vp, vp, vp, vp]
            L.ptls_mi355x_record_layer_pending.argtypes = [vp]
            L.ptls_mi355x_record_layer_pending.restype = sz
            L.ptls_mi355x_record_layer_flush.argtypes = [vp]
            L.ptls_mi355x_record_layer_set_coalesce.argtypes = [vp, sz]
            L.ptls_mi355x_record_layer_set_coalesce.restype = sz
            L.ptls_mi355x_record_layer_launches.argtypes = [vp]
            L.ptls_mi355x_record_layer_launches.restype = u64
            L.ptls_mi355x_record_layer_cork.argtypes = [vp, C.c_int]
            L.ptls_mi355x_record_layer_set_direct_dma.argtypes = [vp, C.c_int]
            if hasattr(L, "ptls_mi355x_record_layer_reserve"):
                L.ptls_mi355x_record_layer_reserve.argtypes = [vp, sz, sz]
        for name in ("ptls_mi355x_set_win16_records", "ptls_mi355x_set_split_records"):
            if hasattr(L, name):  # (absent from older builds used in A/B timing runs)
                getattr(L, name).argtypes = [sz]
                getattr(L, name).restype = sz
        if hasattr(L, "ptls_mi355x_aes_new"):  # (absent from older builds used in A/B timing runs)
            L.ptls_mi355x_tls_open_records_ex.argtypes = [vp, vp, vp, vp, sz, vp, vp, vp, vp, C.c_int, vp]
            L.ptls_mi355x_aes_new.argtypes = [vp, sz]
            L.ptls_mi355x_aes_new.restype = vp
            L.ptls_mi355x_aes_free.argtypes = [vp]
            L.ptls_mi355x_aes_ecb.argtypes = [vp, C.c_int, vp, vp, sz]
            L.ptls_mi355x_aes_ecb_batch.argtypes = [vp, C.c_int, vp, vp, sz, vp]
        if hasattr(L, "ptls_mi355x_tls_deliver_records"):
            L.ptls_mi355x_tls_deliver_records.argtypes = [vp, vp, vp, vp, vp, sz, sz, vp]
        if hasattr(L, "ptls_mi355x_prepare_copies"):
            L.ptls_mi355x_prepare_copies.argtypes = []
        L.ptls_mi355x_tls_plan_send.argtypes = [sz, C.c_uint32, C.POINTER(u64), u64, u64, vp, sz, C.POINTER(sz)]
        L.ptls_mi355x_tls_plan_send.restype = sz
        L.ptls_mi355x_tls_parse_records.argtypes = [vp, sz, u64, C.POINTER(u64), u64, vp, sz, C.POINTER(sz),
                                                    C.POINTER(sz)]
        L.ptls_mi355x_tls_parse_records.restype = C.c_int
        if hasattr(L, "ptls_mi355x_fault_journal_install"):
            L.ptls_mi355x_fault_journal_install.argtypes = [C.c_char_p]
            L.ptls_mi355x_fault_journal_faults.restype = C.c_ulong
            L.ptls_mi355x_fault_journal_report.argtypes = [u64, C.c_uint32]
            L.ptls_mi355x_fault_journal_note.argtypes = [C.c_char_p, vp, sz]
            L.ptls_mi355x_slot_engine_errors.restype = C.c_ulong
            L.ptls_mi355x_test_slot_without_engine.argtypes = [C.c_int]
            L.ptls_mi355x_test_inject_engine_errors.argtypes = [C.c_uint]
            L.ptls_mi355x_test_inject_engine_errors.restype = C.c_uint
        if hasattr(L, "ptls_mi355x_seal_batch_multikey"):
            L.ptls_mi355x_seal_batch_multikey.argtypes = [vp, vp, sz, vp, vp, sz, vp, vp, vp, vp]
            L.ptls_mi355x_open_batch_multikey.argtypes = [vp, vp, sz, vp, vp, sz, vp, vp, vp, vp, vp]
            L.ptls_mi355x_tls_seal_records_multikey.argtypes = [vp, vp, sz, vp, vp, vp, sz, vp, vp, vp]
            L.ptls_mi355x_tls_open_records_multikey.argtypes = [vp, vp, sz, vp, vp, vp, sz, vp, vp, vp, vp, C.c_int, vp]
            L.ptls_mi355x_kernel_name_multikey.argtypes = [C.c_int, sz, sz, C.c_int]
            L.ptls_mi355x_kernel_name_multikey.restype = C.c_char_p
            L.ptls_mi355x_order_by_key.argtypes = [vp, vp, sz, sz, vp, vp]
            L.ptls_mi355x_seal_batch_multikey_ordered.argtypes = [vp, vp, sz, vp, vp, vp, sz, vp, vp, vp, vp]
            L.ptls_mi355x_open_batch_multikey_ordered.argtypes = [vp, vp, sz, vp, vp, vp, sz, vp, vp, vp, vp, vp]
            global FAULT_JOURNAL_STATUS
            if os.environ.get("RAPIDO_FAULT_JOURNAL", "1") != "0":
                # before the first HIP call of the process where possible (tests/conftest.py sets the path)
                path = os.environ.get("RAPIDO_FAULT_LOG")
                FAULT_JOURNAL_STATUS = L.ptls_mi355x_fault_journal_install(path.encode() if path else None)
        _lib = L
    return _lib


#: status of the fault journal's installation at load (0: the memory-fault observer is registered; else the HSA status,
#: e.g. no GPU in this process; None: not attempted).  See include/ptls_mi355x.h "fault attribution".
FAULT_JOURNAL_STATUS = None


def fault_journal_report(va: int, reason_mask: int = 1) -> None:
    """Writes the fault journal's report for a fault at `va` (what the memory-fault handler writes; diagnostics)."""
    lib().ptls_mi355x_fault_journal_report(va, reason_mask)


def fault_journal_note(what: bytes, ptr: int, length: int) -> None:
    lib().ptls_mi355x_fault_journal_note(what, ptr, length)


def fault_journal_faults() -> int:
    """Memory-fault events the journal's handler has received in this process."""
    return int(lib().ptls_mi355x_fault_journal_faults())


def last_error() -> str:
    return lib().ptls_mi355x_last_error().decode()


def device_check() -> None:
    """Synchronises the current device and raises if any GPU work faulted, or a free path met an error, since the
    previous check (ptls_mi355x_device_check).  The GPU tests run it after every test (tests/conftest.py)."""
    if lib().ptls_mi355x_device_check():
        raise RuntimeError("device check: " + last_error())


#: errors raised by close() inside a finalizer (__del__ cannot raise): reported, and collected for the test suite (the
#: most recent FINALIZER_ERRORS_KEEP; FINALIZER_ERROR_COUNT counts them all)
FINALIZER_ERRORS: list = []
FINALIZER_ERRORS_KEEP = 256
FINALIZER_ERROR_COUNT = 0


def _finalize(obj, method: str = "close") -> None:
    """obj.close() (or .free()) from __del__: an error is printed and kept in FINALIZER_ERRORS, never dropped."""
    try:
        getattr(obj, method)()
    except Exception as e:  # noqa: BLE001 - __del__ must not raise; report instead
        msg = f"{type(obj).__name__}.__del__: {e}"
        global FINALIZER_ERROR_COUNT
        FINALIZER_ERROR_COUNT += 1
        FINALIZER_ERRORS.append(msg)
        if len(FINALIZER_ERRORS) > FINALIZER_ERRORS_KEEP:  # a long-running process keeps only the recent ones
            del FINALIZER_ERRORS[: len(FINALIZER_ERRORS) - FINALIZER_ERRORS_KEEP]
        import sys
        print("rapido_amd: " + msg, file=sys.stderr)


def build_id() -> str:
    """The source hash the loaded library was built from (ptls_mi355x_build_id, rapido_amd/build.py)."""
    return lib().ptls_mi355x_build_id().decode()


def source_build_id() -> str:
    """The same hash over this tree's sources: equal to build_id() iff the library was built from them."""
    from rapido_amd import build as _b
    return _b.source_build_id()


def is_supported() -> bool:
    return bool(lib().ptls_mi355x_is_supported())


def require_gpu() -> None:
    if not is_supported():
        raise RuntimeError("ptls_mi355x: no gfx950 (MI355X) device visible -- the engine has no CPU fallback")


def algorithm(name: str):
    """Pointer to one of the exported algorithm objects, e.g. 'aes128gcm' or 'aes256ctr'."""
    sym = "ptls_mi355x_" + name
    typ = AeadAlgorithm if name.endswith("gcm") else CipherAlgorithm
    return typ.in_dll(lib(), sym)


def _cbuf(b: bytes):
    return C.create_string_buffer(bytes(b), max(len(b), 1))


# ------------------------------------------------------------------ picotls API mirror ----
class Aead:
    """An AEAD context created exactly like ptls_aead_new_direct (lib/picotls.c:5268-5283)."""

    def __init__(self, algo: AeadAlgorithm, is_enc: bool, key: bytes, iv: bytes):
        self.algo = algo
        self._mem = C.create_string_buffer(algo.context_size)  # zeroed: *ctx = (ptls_aead_context_t){aead}
        self.ctx = AeadContext.from_buffer(self._mem)
        self.ctx.algo = C.cast(C.pointer(algo), vp)
        self._key, self._iv = _cbuf(key), _cbuf(iv)
        rc = algo.setup_crypto(C.addressof(self._mem), 1 if is_enc else 0, self._key, self._iv)
        if rc != 0:
            raise RuntimeError(f"setup_crypto failed ({rc:#x}): {last_error()}")
        self.tag_size = algo.tag_size

    @property
    def ptr(self) -> int:
        return C.addressof(self._mem)

    def free(self) -> None:  # ptls_aead_free (lib/picotls.c:5285-5289)
        if self._mem is not None:
            self.ctx.dispose_crypto(self.ptr)
            self._mem = None

    def xor_iv(self, b: bytes) -> None:
        self.ctx.do_xor_iv(self.ptr, _cbuf(b), len(b))

    def encrypt(self, pt: bytes, seq: int, aad: bytes = b"", supp: SupplementaryEncryption | None = None,
                inplace: bool = False) -> bytes:
        out = C.create_string_buffer(len(pt) + self.tag_size)
        if inplace:
            C.memmove(out, bytes(pt), len(pt))
            src = out
        else:
            src = _cbuf(pt)
        self.ctx.do_encrypt(self.ptr, out, src, len(pt), seq, _cbuf(aad) if aad else None, len(aad),
                            C.byref(supp) if supp is not None else None)
        return out.raw

    def decrypt(self, ct: bytes, seq: int, aad: bytes = b""):
        out = C.create_string_buffer(max(len(ct), 1))
        n = self.ctx.do_decrypt(self.ptr, out, _cbuf(ct), len(ct), seq, _cbuf(aad) if aad else None, len(aad))
        return None if n == SIZE_MAX else out.raw[:n]

    # streaming trio (include/picotls.h:1531-1544)
    def encrypt_init(self, seq: int, aad: bytes = b"") -> None:
        self._aad_keep = _cbuf(aad) if aad else None
        self.ctx.do_encrypt_init(self.ptr, seq, self._aad_keep, len(aad))

    def encrypt_update(self, out, out_off: int, data: bytes) -> int:
        return self.ctx.do_encrypt_update(self.ptr, C.addressof(out) + out_off, _cbuf(data), len(data))

    def encrypt_final(self, out, out_off: int) -> int:
        return self.ctx.do_encrypt_final(self.ptr, C.addressof(out) + out_off)

    def __del__(self):
        _finalize(self, "free")


def aead_new_direct(name_or_algo, is_enc: bool, key: bytes, iv: bytes) -> Aead:
    algo = algorithm(name_or_algo) if isinstance(name_or_algo, str) else name_or_algo
    return Aead(algo, is_enc, key, iv)


class Cipher:
    """ptls_cipher_new / ptls_cipher_init / ptls_cipher_encrypt / ptls_cipher_free."""

    def __init__(self, algo: CipherAlgorithm, is_enc: bool, key: bytes):
        self._mem = C.create_string_buffer(algo.context_size)
        self.ctx = CipherContext.from_buffer(self._mem)
        self.ctx.algo = C.cast(C.pointer(algo), vp)
        rc = algo.setup_crypto(C.addressof(self._mem), 1 if is_enc else 0, _cbuf(key))
        if rc != 0:
            raise RuntimeError(f"cipher setup failed ({rc:#x}): {last_error()}")

    @property
    def ptr(self) -> int:
        return C.addressof(self._mem)

    def init(self, iv: bytes) -> None:
        self._iv = _cbuf(iv)
        self.ctx.do_init(self.ptr, self._iv)

    def encrypt(self, data: bytes) -> bytes:
        out = C.create_string_buffer(max(len(data), 1))
        self.ctx.do_transform(self.ptr, out, _cbuf(data), len(data))
        return out.raw[:len(data)]

    def free(self) -> None:
        if self._mem is not None:
            self.ctx.do_dispose(self.ptr)
            self._mem = None

    def __del__(self):
        _finalize(self, "free")


def cipher_new(name: str, is_enc: bool, key: bytes) -> Cipher:
    return Cipher(algorithm(name), is_enc, key)


# ------------------------------------------------------------------ direct + batch API -----
#: every Engine not yet closed (tests/conftest.py closes the ones a test leaves open, before its device check)
LIVE_ENGINES: "weakref.WeakSet" = weakref.WeakSet()


class Engine:
    """ptls_mi355x_aesgcm_context_t: the device-resident key image + batch launches.  close() (or a with-block) releases
    it deterministically; the finalizer is the fallback."""

    def __init__(self, key: bytes, capacity: int = 16384, device: int | None = None):
        """device: the HIP ordinal to create the context on (ptls_mi355x_aesgcm_new_on); None: the current device."""
        if len(key) not in (16, 32):
            raise ValueError("key must be 16 or 32 bytes")
        self.key_size = len(key)
        self.handle = None
        if device is None:
            self.handle = lib().ptls_mi355x_aesgcm_new(_cbuf(key), len(key), capacity)
        else:
            self.handle = lib().ptls_mi355x_aesgcm_new_on(device, _cbuf(key), len(key), capacity)
        if not self.handle:
            raise RuntimeError("ptls_mi355x_aesgcm_new failed: " + last_error())
        LIVE_ENGINES.add(self)

    def __enter__(self) -> "Engine":
        return self

    def __exit__(self, *exc) -> None:
        self.close()

    def close(self) -> None:
        """ptls_mi355x_aesgcm_release: waits for the context's launches, clears and frees its key image; raises if
        that met an error (an asynchronous fault of earlier GPU work surfaces at its synchronisation)."""
        if self.handle:
            h, self.handle = self.handle, None
            L = lib()
            if not hasattr(L, "ptls_mi355x_aesgcm_release"):  # older builds (A/B timing runs): free reports nothing
                L.ptls_mi355x_aesgcm_free(h)
            elif L.ptls_mi355x_aesgcm_release(h):
                raise RuntimeError("ptls_mi355x_aesgcm_release: " + last_error())

    def __del__(self):
        _finalize(self)

    @property
    def device(self) -> int:
        return lib().ptls_mi355x_aesgcm_device(self.handle)

    def encrypt(self, nonce: bytes, aad: bytes, pt: bytes) -> bytes:
        out = C.create_string_buffer(len(pt) + 16)
        if lib().ptls_mi355x_aesgcm_encrypt(self.handle, out, _cbuf(pt), len(pt), _cbuf(nonce), _cbuf(aad), len(aad)):
            raise RuntimeError("encrypt failed: " + last_error())
        return out.raw

    def decrypt(self, nonce: bytes, aad: bytes, ct: bytes, tag: bytes):
        out = C.create_string_buffer(max(len(ct), 1))
        r = lib().ptls_mi355x_aesgcm_decrypt(self.handle, out, _cbuf(ct), len(ct), _cbuf(nonce), _cbuf(aad), len(aad),
                                             _cbuf(tag))
        if r < 0:
            raise RuntimeError("decrypt failed: " + last_error())
        return out.raw[:len(ct)] if r == 1 else None

    def ecb(self, blocks: bytes) -> bytes:
        assert len(blocks) % 16 == 0
        out = C.create_string_buffer(max(len(blocks), 1))
        if lib().ptls_mi355x_aesecb_encrypt(self.handle, out, _cbuf(blocks), len(blocks) // 16):
            raise RuntimeError("ecb failed: " + last_error())
        return out.raw[:len(blocks)]

    # batch: all pointers are device addresses (ints), stream a hipStream_t handle (int) or 0
    def seal_batch(self, static_iv: bytes, recs_ptr: int, n: int, src_ptr: int, dst_ptr: int, aad_ptr: int,
                   stream: int = 0) -> None:
        if lib().ptls_mi355x_seal_batch(self.handle, _cbuf(static_iv), recs_ptr, n, src_ptr, dst_ptr, aad_ptr,
                                        stream or None):
            raise RuntimeError("seal_batch failed: " + last_error())

    def order_by_length(self, recs_ptr: int, n: int, order_ptr: int, stream: int = 0) -> None:
        if lib().ptls_mi355x_order_by_length(self.handle, recs_ptr, n, order_ptr, stream or None):
            raise RuntimeError("order_by_length failed: " + last_error())

    def seal_batch_ordered(self, static_iv: bytes, recs_ptr: int, order_ptr: int, n: int, src_ptr: int, dst_ptr: int,
                           aad_ptr: int, stream: int = 0) -> None:
        if lib().ptls_mi355x_seal_batch_ordered(self.handle, _cbuf(static_iv), recs_ptr, order_ptr, n, src_ptr, dst_ptr,
                                                aad_ptr, stream or None):
            raise RuntimeError("seal_batch_ordered failed: " + last_error())

    def open_batch_ordered(self, static_iv: bytes, recs_ptr: int, order_ptr: int, n: int, src_ptr: int, dst_ptr: int,
                           aad_ptr: int, status_ptr: int, stream: int = 0) -> None:
        if lib().ptls_mi355x_open_batch_ordered(self.handle, _cbuf(static_iv), recs_ptr, order_ptr, n, src_ptr, dst_ptr,
                                                aad_ptr, status_ptr, stream or None):
            raise RuntimeError("open_batch_ordered failed: " + last_error())

    def open_batch(self, static_iv: bytes, recs_ptr: int, n: int, src_ptr: int, dst_ptr: int, aad_ptr: int,
                   status_ptr: int, stream: int = 0) -> None:
        if lib().ptls_mi355x_open_batch(self.handle, _cbuf(static_iv), recs_ptr, n, src_ptr, dst_ptr, aad_ptr,
                                        status_ptr, stream or None):
            raise RuntimeError("open_batch failed: " + last_error())


    # TLS 1.3 record framing in the batch (include/ptls_mi355x.h section 4)
    # conn_ptr: optional device array of per-record rapido connection ids (the *_multi entry points)
    def tls_seal_records(self, static_iv: bytes, recs_ptr: int, n: int, src_ptr: int, dst_ptr: int,
                         stream: int = 0, conn_ptr: int = 0) -> None:
        if lib().ptls_mi355x_tls_seal_records_multi(self.handle, _cbuf(static_iv), recs_ptr, conn_ptr or None, n,
                                                    src_ptr, dst_ptr, stream or None):
            raise RuntimeError("tls_seal_records failed: " + last_error())

    def tls_open_records(self, static_iv: bytes, recs_ptr: int, n: int, src_ptr: int, dst_ptr: int, status_ptr: int,
                         types_ptr: int, stream: int = 0, conn_ptr: int = 0, flags: int = 0) -> None:
        """flags: OPEN_STOP_AT_FAILURE -- records behind a connection's first failure become TLS_NOT_PROCESSED."""
        if lib().ptls_mi355x_tls_open_records_ex(self.handle, _cbuf(static_iv), recs_ptr, conn_ptr or None, n,
                                                 src_ptr, dst_ptr, status_ptr, types_ptr, flags, stream or None):
            raise RuntimeError("tls_open_records failed: " + last_error())


# ------------------------------------------------------------------ multi-key batches -----
# The records of many sessions in one launch (include/ptls_mi355x.h, "Multi-key batches"): engines[k] and static_ivs[k]
# are key k's context and IV, key_idx_ptr a device uint32 array of each record's key.
class MultiKey:
    """The contexts and IVs of a multi-key launch, marshalled once (a server re-sends its sessions' batches)."""

    def __init__(self, engines, static_ivs):
        if len(engines) != len(static_ivs) or not engines:
            raise ValueError("one static IV per engine, at least one")
        self.engines = list(engines)  # kept alive while the launches may run
        self.ctxs = (C.c_void_p * len(engines))(*[e.handle for e in engines])
        self.ivs = C.create_string_buffer(b"".join(bytes(iv) for iv in static_ivs), 12 * len(engines))
        if any(len(iv) != 12 for iv in static_ivs):
            raise ValueError("static IVs are 12 bytes")

    def __len__(self) -> int:
        return len(self.engines)

    def seal_batch(self, recs_ptr, key_idx_ptr, n, src_ptr, dst_ptr, aad_ptr, stream: int = 0) -> None:
        if lib().ptls_mi355x_seal_batch_multikey(self.ctxs, self.ivs, len(self), recs_ptr, key_idx_ptr, n, src_ptr,
                                                 dst_ptr, aad_ptr, stream or None):
            raise RuntimeError("seal_batch_multikey failed: " + last_error())

    def open_batch(self, recs_ptr, key_idx_ptr, n, src_ptr, dst_ptr, aad_ptr, status_ptr, stream: int = 0) -> None:
        if lib().ptls_mi355x_open_batch_multikey(self.ctxs, self.ivs, len(self), recs_ptr, key_idx_ptr, n, src_ptr,
                                                 dst_ptr, aad_ptr, status_ptr, stream or None):
            raise RuntimeError("open_batch_multikey failed: " + last_error())

    def order_by_key(self, key_idx_ptr, n, order_ptr, stream: int = 0) -> None:
        """The records sorted by key once, for several _ordered launches (ptls_mi355x_order_by_key)."""
        if lib().ptls_mi355x_order_by_key(self.ctxs[0], key_idx_ptr, n, len(self), order_ptr, stream or None):
            raise RuntimeError("order_by_key failed: " + last_error())

    def seal_batch_ordered(self, recs_ptr, key_idx_ptr, order_ptr, n, src_ptr, dst_ptr, aad_ptr, stream: int = 0):
        if lib().ptls_mi355x_seal_batch_multikey_ordered(self.ctxs, self.ivs, len(self), recs_ptr, key_idx_ptr, order_ptr,
                                                         n, src_ptr, dst_ptr, aad_ptr, stream or None):
            raise RuntimeError("seal_batch_multikey_ordered failed: " + last_error())

    def open_batch_ordered(self, recs_ptr, key_idx_ptr, order_ptr, n, src_ptr, dst_ptr, aad_ptr, status_ptr,
                           stream: int = 0):
        if lib().ptls_mi355x_open_batch_multikey_ordered(self.ctxs, self.ivs, len(self), recs_ptr, key_idx_ptr, order_ptr,
                                                         n, src_ptr, dst_ptr, aad_ptr, status_ptr, stream or None):
            raise RuntimeError("open_batch_multikey_ordered failed: " + last_error())

    def tls_seal_records(self, recs_ptr, key_idx_ptr, n, src_ptr, dst_ptr, stream: int = 0, conn_ptr: int = 0) -> None:
        if lib().ptls_mi355x_tls_seal_records_multikey(self.ctxs, self.ivs, len(self), recs_ptr, key_idx_ptr,
                                                       conn_ptr or None, n, src_ptr, dst_ptr, stream or None):
            raise RuntimeError("tls_seal_records_multikey failed: " + last_error())

    def tls_open_records(self, recs_ptr, key_idx_ptr, n, src_ptr, dst_ptr, status_ptr, types_ptr, stream: int = 0,
                         conn_ptr: int = 0, flags: int = 0) -> None:
        if lib().ptls_mi355x_tls_open_records_multikey(self.ctxs, self.ivs, len(self), recs_ptr, key_idx_ptr,
                                                       conn_ptr or None, n, src_ptr, dst_ptr, status_ptr, types_ptr,
                                                       flags, stream or None):
            raise RuntimeError("tls_open_records_multikey failed: " + last_error())


def kernel_name_multikey(is_seal: bool, key_size: int, n: int, framing: bool) -> str:
    return lib().ptls_mi355x_kernel_name_multikey(int(is_seal), key_size, n, int(framing)).decode()


def prepare_copies() -> None:
    """Has the HIP runtime set up its copy machinery on the current device now rather than inside a later window
    (include/ptls_mi355x.h; record layers call it before their first copy)."""
    if lib().ptls_mi355x_prepare_copies():
        raise RuntimeError("prepare_copies failed: " + last_error())


class AesKeys:
    """ptls_mi355x_aes_context_t: round keys only (the ECB/CTR ciphers), on the current device."""

    def __init__(self, key: bytes):
        if len(key) not in (16, 32):
            raise ValueError("key must be 16 or 32 bytes")
        self.handle = lib().ptls_mi355x_aes_new(_cbuf(key), len(key))
        if not self.handle:
            raise RuntimeError("ptls_mi355x_aes_new failed: " + last_error())

    def ecb(self, data: bytes, encrypt: bool = True) -> bytes:
        assert len(data) % 16 == 0
        out = C.create_string_buffer(max(len(data), 1))
        if lib().ptls_mi355x_aes_ecb(self.handle, 1 if encrypt else 0, out, _cbuf(data), len(data) // 16):
            raise RuntimeError("aes_ecb failed: " + last_error())
        return out.raw[:len(data)]

    def ecb_batch(self, dst_ptr: int, src_ptr: int, nblocks: int, encrypt: bool = True, stream: int = 0) -> None:
        if lib().ptls_mi355x_aes_ecb_batch(self.handle, 1 if encrypt else 0, dst_ptr, src_ptr, nblocks, stream or None):
            raise RuntimeError("aes_ecb_batch failed: " + last_error())

    def close(self) -> None:
        if self.handle:
            lib().ptls_mi355x_aes_free(self.handle)
            self.handle = None

    def __del__(self):
        _finalize(self)


class _IoVec(C.Structure):
    _fields_ = [("base", C.c_void_p), ("len", C.c_size_t)]


RECORD_LAYER_SEQ_LIMIT = 1 << 24  # ptls_send's key-update threshold (lib/picotls.c:4976-4977)
RECORD_LAYER_KEY_UPDATE = 1
RECORD_LAYER_STALE = -2
RECORD_LAYER_DMA_IN = 2  # set_direct_dma: the inputs by DMA, the outputs written in place


class RecordLayer:
    """ptls_mi355x_record_layer_t: one traffic direction of a connection, windows of records between host memory
    and the GPU (include/ptls_mi355x.h section 5)."""

    def __init__(self, key: bytes, static_iv: bytes, seq: int = 0):
        assert len(static_iv) == 12
        self._registered = {}
        self.handle = lib().ptls_mi355x_record_layer_new(_cbuf(key), len(key), _cbuf(static_iv), seq)
        if not self.handle:
            raise RuntimeError("ptls_mi355x_record_layer_new failed: " + lib().ptls_mi355x_record_layer_last_error().decode())

    @property
    def seq(self) -> int:
        return lib().ptls_mi355x_record_layer_get_seq(self.handle)

    @seq.setter
    def seq(self, v: int) -> None:
        lib().ptls_mi355x_record_layer_set_seq(self.handle, v)

    def seal(self, fragments, content_type: int = 23, capacity: int = None):
        """-> (wire bytes, record count); every fragment framed as records of <= 16384 bytes.  self.key_update is set
        when the window stopped at the 2^24-record limit (RECORD_LAYER_KEY_UPDATE)."""
        bufs = [_cbuf(f) for f in fragments]
        iov = (_IoVec * max(len(fragments), 1))()
        for i, (b, f) in enumerate(zip(bufs, fragments)):
            iov[i].base = C.cast(b, C.c_void_p)
            iov[i].len = len(f)
        if capacity is None:
            capacity = sum(len(f) + (len(f) + 16383) // 16384 * TLS_OVERHEAD for f in fragments)
        out = C.create_string_buffer(max(capacity, 1))
        olen, nrec = sz(), sz()
        rc = lib().ptls_mi355x_record_layer_seal(self.handle, iov, len(fragments), content_type, out, capacity,
                                                 C.byref(olen), C.byref(nrec))
        if rc not in (0, RECORD_LAYER_KEY_UPDATE):
            raise RuntimeError("record_layer_seal failed: " + lib().ptls_mi355x_record_layer_last_error().decode())
        self.key_update = rc == RECORD_LAYER_KEY_UPDATE
        return out.raw[:olen.value], nrec.value

    def open(self, wire: bytes, capacity: int = None):
        """-> (return code: 0 or a TLS alert, plaintext, wire bytes consumed, record count)."""
        if capacity is None:
            capacity = len(wire)
        out = C.create_string_buffer(max(capacity, 1))
        cons, olen, nrec = sz(), sz(), sz()
        rc = lib().ptls_mi355x_record_layer_open(self.handle, _cbuf(wire), len(wire), C.byref(cons), out, capacity,
                                                 C.byref(olen), C.byref(nrec))
        if rc < 0:
            raise RuntimeError("record_layer_open failed: " + lib().ptls_mi355x_record_layer_last_error().decode())
        return rc, out.raw[:olen.value], cons.value, nrec.value

    def set_direct_dma(self, on) -> int:
        """Registered windows by DMA to and from device memory (True / 1), read in place by the kernels (False / 0,
        default), or the inputs by DMA with the outputs written in place (RECORD_LAYER_DMA_IN).  Returns the previous
        mode."""
        mode = on if on == RECORD_LAYER_DMA_IN else (1 if on else 0)
        return lib().ptls_mi355x_record_layer_set_direct_dma(self.handle, mode)

    def reserve(self, window_bytes: int, windows_per_launch: int = 1) -> None:
        """Sets up every launch slot now (stream, engine context, staging and device buffers for windows_per_launch
        windows of window_bytes each) instead of at each slot's first window (ptls_mi355x_record_layer_reserve)."""
        self._check(lib().ptls_mi355x_record_layer_reserve(self.handle, window_bytes, windows_per_launch), "reserve")

    def set_zero_copy_bytes(self, n: int) -> int:
        """Windows of at most n staged bytes run zero-copy on the pinned staging (0: DMA copies); -> previous."""
        return lib().ptls_mi355x_record_layer_set_zero_copy_bytes(self.handle, n)

    def register(self, buf: np.ndarray) -> None:
        """Registers a long-lived host buffer (a uint8 numpy array) for direct calls: seal_into / open_into on
        views of registered buffers run with no copy (ptls_mi355x_record_layer_register)."""
        self._check(lib().ptls_mi355x_record_layer_register(self.handle, buf.ctypes.data, buf.nbytes), "register")
        self._registered[buf.ctypes.data] = buf  # keeps the memory alive while registered

    def unregister(self, buf: np.ndarray) -> None:
        self._check(lib().ptls_mi355x_record_layer_unregister(self.handle, buf.ctypes.data), "unregister")
        self._registered.pop(buf.ctypes.data, None)

    def _check(self, rc: int, what: str) -> None:
        if rc != 0:
            raise RuntimeError(f"record_layer_{what} failed: " + lib().ptls_mi355x_record_layer_last_error().decode())

    def seal_into(self, fragments, out: np.ndarray, content_type: int = 23):
        """seal with the fragments (uint8 numpy views) and the output written in place -> (wire bytes, records)."""
        iov = (_IoVec * max(len(fragments), 1))()
        for i, f in enumerate(fragments):
            iov[i].base = C.c_void_p(f.ctypes.data)
            iov[i].len = f.nbytes
        olen, nrec = sz(), sz()
        rc = lib().ptls_mi355x_record_layer_seal(self.handle, iov, len(fragments), content_type, out.ctypes.data,
                                                 out.nbytes, C.byref(olen), C.byref(nrec))
        if rc != RECORD_LAYER_KEY_UPDATE:
            self._check(rc, "seal")
        self.key_update = rc == RECORD_LAYER_KEY_UPDATE
        return olen.value, nrec.value

    def open_into(self, wire: np.ndarray, out: np.ndarray):
        """open of the records in `wire` (a uint8 numpy view) into `out` -> (rc, plaintext bytes, consumed, records)."""
        cons, olen, nrec = sz(), sz(), sz()
        rc = lib().ptls_mi355x_record_layer_open(self.handle, wire.ctypes.data, wire.nbytes, C.byref(cons),
                                                 out.ctypes.data, out.nbytes, C.byref(olen), C.byref(nrec))
        if rc < 0:
            self._check(rc, "open")
        return rc, olen.value, cons.value, nrec.value

    def open_record(self, wire: bytes, capacity: int = None):
        """ONE record of any inner content type (ptls_mi355x_record_layer_open_record)
        -> (rc: 0 or a TLS alert, plaintext, wire bytes consumed, content type)."""
        if capacity is None:
            capacity = len(wire)
        out = C.create_string_buffer(max(capacity, 1))
        cons, olen, ty = sz(), sz(), C.c_uint8()
        rc = lib().ptls_mi355x_record_layer_open_record(self.handle, _cbuf(wire), len(wire), C.byref(cons), out,
                                                        capacity, C.byref(olen), C.byref(ty))
        if rc < 0:
            self._check(rc, "open_record")
        return rc, out.raw[:olen.value], cons.value, ty.value

    def rekey(self, key: bytes, static_iv: bytes) -> None:
        """A new traffic key and IV for this direction; seq restarts at 0 (ptls_mi355x_record_layer_rekey)."""
        assert len(static_iv) == 12
        self._check(lib().ptls_mi355x_record_layer_rekey(self.handle, _cbuf(key), len(key), _cbuf(static_iv)), "rekey")

    @property
    def pending(self) -> int:
        return lib().ptls_mi355x_record_layer_pending(self.handle)

    def flush(self) -> None:
        """Launches the queued (coalesced) windows now (ptls_mi355x_record_layer_flush)."""
        self._check(lib().ptls_mi355x_record_layer_flush(self.handle), "flush")

    @property
    def launches(self) -> int:
        """Launches this layer has led (ptls_mi355x_record_layer_launches)."""
        return lib().ptls_mi355x_record_layer_launches(self.handle)

    def cork(self, on: bool) -> None:
        """Queue every window until uncorked (launched together), the first wait or a full queue."""
        self._check(lib().ptls_mi355x_record_layer_cork(self.handle, 1 if on else 0), "cork")

    def set_coalesce(self, windows: int) -> int:
        """At most `windows` queued windows per launch (0/1: every window launches at its submit) -> previous."""
        return lib().ptls_mi355x_record_layer_set_coalesce(self.handle, windows)

    def seal_submit(self, fragments, out: np.ndarray, content_type: int = 23) -> int:
        """Asynchronous seal of the fragments (uint8 numpy views) into `out` -> ticket (wait() completes it)."""
        iov = (_IoVec * max(len(fragments), 1))()
        for i, f in enumerate(fragments):
            iov[i].base = C.c_void_p(f.ctypes.data)
            iov[i].len = f.nbytes
        frag_ptrs = (C.c_void_p * 1)(C.cast(iov, C.c_void_p))
        nfr, outp, cap, t = (sz * 1)(len(fragments)), (C.c_void_p * 1)(out.ctypes.data), (sz * 1)(out.nbytes), u64()
        handles = (C.c_void_p * 1)(self.handle)
        self._check(lib().ptls_mi355x_record_layer_seal_submit(handles, 1, frag_ptrs, nfr, content_type, outp, cap,
                                                               C.byref(t)), "seal_submit")
        return t.value

    def open_submit(self, wire: np.ndarray, out: np.ndarray):
        """Asynchronous open of the records in `wire` into `out` -> (ticket, wire bytes parsed into the window)."""
        inp, inl = (C.c_void_p * 1)(wire.ctypes.data), (sz * 1)(wire.nbytes)
        outp, cap, parsed, t = (C.c_void_p * 1)(out.ctypes.data), (sz * 1)(out.nbytes), (sz * 1)(), u64()
        handles = (C.c_void_p * 1)(self.handle)
        self._check(lib().ptls_mi355x_record_layer_open_submit(handles, 1, inp, inl, outp, cap, parsed, C.byref(t)),
                    "open_submit")
        return t.value, parsed[0]

    def wait(self, ticket: int):
        """Completes the oldest window -> (outlen, records, consumed, alert); seal: consumed = fragments sealed,
        alert = RECORD_LAYER_KEY_UPDATE at the limit; open: alert = a TLS alert or RECORD_LAYER_STALE."""
        olen, nrec, cons, al = (sz * 1)(), (sz * 1)(), (sz * 1)(), (C.c_int * 1)()
        self._check(lib().ptls_mi355x_record_layer_wait(self.handle, ticket, olen, nrec, cons, al), "wait")
        return olen[0], nrec[0], cons[0], al[0]

    def wait_multi(self, ticket: int, nlayers: int):
        """Completes the oldest window of a submit over `nlayers` layers led by this one -> per layer (outlen, records,
        consumed, alert)."""
        olen, nrec, cons, al = (sz * nlayers)(), (sz * nlayers)(), (sz * nlayers)(), (C.c_int * nlayers)()
        self._check(lib().ptls_mi355x_record_layer_wait(self.handle, ticket, olen, nrec, cons, al), "wait")
        return [(olen[i], nrec[i], cons[i], al[i]) for i in range(nlayers)]

    def close(self) -> None:
        if self.handle:
            lib().ptls_mi355x_record_layer_free(self.handle)  # unregisters its ranges
            self._registered.clear()
            self.handle = None

    def __del__(self):
        _finalize(self)


def record_layer_seal_multi(layers, windows, content_type: int = 23, outs=None):
    """One launch for the send windows of several connections of a session (ptls_mi355x_record_layer_seal_multi):
    windows[l] is a list of fragments for layers[l], bytes or uint8 numpy views (for direct calls, with `outs` a
    list of uint8 numpy output buffers) -> [(wire bytes, record count)] per layer (wire length with `outs`)."""
    n = len(layers)
    keep, iov_arrays = [], []
    for frags in windows:
        iov = (_IoVec * max(len(frags), 1))()
        for i, f in enumerate(frags):
            if isinstance(f, np.ndarray):
                iov[i].base = C.c_void_p(f.ctypes.data)
                iov[i].len = f.nbytes
            else:
                b = _cbuf(f)
                keep.append(b)
                iov[i].base = C.cast(b, C.c_void_p)
                iov[i].len = len(f)
        iov_arrays.append(iov)
    frag_ptrs = (C.c_void_p * n)(*[C.cast(a, C.c_void_p) for a in iov_arrays])
    nfr = (sz * n)(*[len(w) for w in windows])
    if outs is None:
        caps = [sum(len(f) + (len(f) + 16383) // 16384 * TLS_OVERHEAD for f in w) for w in windows]
        bufs = [C.create_string_buffer(max(c, 1)) for c in caps]
        out_ptrs = (C.c_void_p * n)(*[C.cast(o, C.c_void_p) for o in bufs])
    else:
        caps = [o.nbytes for o in outs]
        out_ptrs = (C.c_void_p * n)(*[o.ctypes.data for o in outs])
    capv = (sz * n)(*caps)
    olen, nrec, cons, alerts = (sz * n)(), (sz * n)(), (sz * n)(), (C.c_int * n)()
    handles = (C.c_void_p * n)(*[lr.handle for lr in layers])
    # the synchronous call as its submit + wait, for the wait's per-layer alerts: layers[l].key_update is set when its
    # window stopped at the 2^24-record limit (send the KeyUpdate, rekey, seal the rest)
    if any(lib().ptls_mi355x_record_layer_pending(lr.handle) for lr in layers):
        raise RuntimeError("record_layer_seal_multi failed: asynchronous windows outstanding (wait for them first)")
    ticket = C.c_uint64()
    if lib().ptls_mi355x_record_layer_seal_submit(handles, n, frag_ptrs, nfr, content_type, out_ptrs, capv,
                                                  C.byref(ticket)) or \
            lib().ptls_mi355x_record_layer_wait(layers[0].handle, ticket.value, olen, nrec, cons, alerts):
        raise RuntimeError("record_layer_seal_multi failed: " + lib().ptls_mi355x_record_layer_last_error().decode())
    for lr in layers:
        lr.key_update = False
    for i in range(n):
        layers[i].key_update = layers[i].key_update or alerts[i] == RECORD_LAYER_KEY_UPDATE
    if outs is None:
        return [(bufs[i].raw[:olen[i]], nrec[i]) for i in range(n)]
    return [(olen[i], nrec[i]) for i in range(n)]


def record_layer_seal_submit_multi(layers, windows, outs, content_type: int = 23) -> int:
    """Asynchronous seal over several layers of a session (ptls_mi355x_record_layer_seal_submit): windows[l] lists
    uint8 numpy fragments for layers[l], outs[l] its output -> ticket of layers[0] (layers[0].wait_multi)."""
    n = len(layers)
    iovs = []
    for frags in windows:
        iov = (_IoVec * max(len(frags), 1))()
        for i, f in enumerate(frags):
            iov[i].base = C.c_void_p(f.ctypes.data)
            iov[i].len = f.nbytes
        iovs.append(iov)
    frag_ptrs = (C.c_void_p * n)(*[C.cast(a, C.c_void_p) for a in iovs])
    nfr = (sz * n)(*[len(w) for w in windows])
    out_ptrs, caps = (C.c_void_p * n)(*[o.ctypes.data for o in outs]), (sz * n)(*[o.nbytes for o in outs])
    handles, t = (C.c_void_p * n)(*[lr.handle for lr in layers]), C.c_uint64()
    if lib().ptls_mi355x_record_layer_seal_submit(handles, n, frag_ptrs, nfr, content_type, out_ptrs, caps, C.byref(t)):
        raise RuntimeError("seal_submit failed: " + lib().ptls_mi355x_record_layer_last_error().decode())
    return t.value


def record_layer_open_submit_multi(layers, wires, outs):
    """Asynchronous open over several layers of a session (ptls_mi355x_record_layer_open_submit): wires[l] / outs[l]
    uint8 numpy arrays -> (ticket of layers[0], wire bytes parsed per layer)."""
    n = len(layers)
    in_ptrs, inl = (C.c_void_p * n)(*[w.ctypes.data for w in wires]), (sz * n)(*[w.nbytes for w in wires])
    out_ptrs, caps = (C.c_void_p * n)(*[o.ctypes.data for o in outs]), (sz * n)(*[o.nbytes for o in outs])
    handles, parsed, t = (C.c_void_p * n)(*[lr.handle for lr in layers]), (sz * n)(), C.c_uint64()
    if lib().ptls_mi355x_record_layer_open_submit(handles, n, in_ptrs, inl, out_ptrs, caps, parsed, C.byref(t)):
        raise RuntimeError("open_submit failed: " + lib().ptls_mi355x_record_layer_last_error().decode())
    return t.value, list(parsed)


def record_layer_open_multi(layers, wires):
    """One launch for the receive windows of several connections of a session (ptls_mi355x_record_layer_open_multi):
    wires[l] (bytes) for layers[l] -> [(alert, plaintext, wire bytes consumed, record count)] per layer."""
    n = len(layers)
    bufs = [_cbuf(w) for w in wires]
    in_ptrs = (C.c_void_p * n)(*[C.cast(b, C.c_void_p) for b in bufs])
    inl = (sz * n)(*[len(w) for w in wires])
    outs = [C.create_string_buffer(max(len(w), 1)) for w in wires]
    out_ptrs = (C.c_void_p * n)(*[C.cast(o, C.c_void_p) for o in outs])
    caps = (sz * n)(*[len(w) for w in wires])
    cons, olen, nrec, alerts = (sz * n)(), (sz * n)(), (sz * n)(), (C.c_int * n)()
    handles = (C.c_void_p * n)(*[lr.handle for lr in layers])
    if lib().ptls_mi355x_record_layer_open_multi(handles, n, in_ptrs, inl, cons, out_ptrs, caps, olen, nrec, alerts):
        raise RuntimeError("record_layer_open_multi failed: " + lib().ptls_mi355x_record_layer_last_error().decode())
    return [(alerts[i], outs[i].raw[:olen[i]], cons[i], nrec[i]) for i in range(n)]


def tls_plan_send(length: int, seq: int, content_type: int = 23, src_off: int = 0, dst_off: int = 0):
    """Descriptors for sending `length` bytes as records (buffer_push_encrypted_records, lib/picotls.c:664-684).
    -> (TLS_RECORD_DTYPE array, wire bytes, next seq)."""
    L = lib()
    s = u64(seq)
    wire = sz()
    n = L.ptls_mi355x_tls_plan_send(length, content_type, C.byref(s), src_off, dst_off, None, 0, C.byref(wire))
    recs = np.zeros(n, TLS_RECORD_DTYPE)
    got = L.ptls_mi355x_tls_plan_send(length, content_type, C.byref(s), src_off, dst_off, recs.ctypes.data, n,
                                      C.byref(wire))
    assert got == n
    return recs, wire.value, s.value


def tls_parse_records(wire: bytes, seq: int, src_off: int = 0, dst_off: int = 0, max_records: int = 1 << 20):
    """Descriptors for the complete type-23 records at the start of `wire` (parse_record, lib/picotls.c:4243-4268).
    -> (rc, TLS_RECORD_DTYPE array, bytes consumed, next seq); rc 50 = PTLS_ALERT_DECODE_ERROR."""
    L = lib()
    cap = min(max_records, len(wire) // TLS_HEADER_SIZE + 1)
    recs = np.zeros(cap, TLS_RECORD_DTYPE)
    s, n, used = u64(seq), sz(), sz()
    buf = np.frombuffer(wire, np.uint8) if wire else np.zeros(1, np.uint8)
    rc = L.ptls_mi355x_tls_parse_records(buf.ctypes.data, len(wire), src_off, C.byref(s), dst_off, recs.ctypes.data,
                                         cap, C.byref(n), C.byref(used))
    return rc, recs[: n.value].copy(), used.value, s.value


def set_lanes_per_record(k: int) -> int:
    prev = lib().ptls_mi355x_set_lanes_per_record(k)
    if prev < 0:
        raise ValueError("lanes per record must be 1, 2, 4 or 8")
    return prev


def set_tls_window_records(n: int) -> int:
    """Framing batches of at most n records run on the window kernels (0: never); returns the previous value."""
    return lib().ptls_mi355x_set_tls_window_records(n)


def set_aead_window_records(n: int) -> int:
    """AEAD batches (and single-record slot calls) of at most n records run on the window kernels (0: never)."""
    return lib().ptls_mi355x_set_aead_window_records(n)


def set_slot_zero_copy_bytes(n: int) -> int:
    """Slot calls staging at most n bytes run zero-copy (the kernel reads/writes pinned host memory); returns the
    previous limit."""
    return lib().ptls_mi355x_set_slot_zero_copy_bytes(n)


SEG32_AUTO = (1 << 64) - 1  # SIZE_MAX: the device's CU count


def set_seg32_records(n: int) -> int:
    """Window batches of at most n records use 32-position segments (0: never; SEG32_AUTO: one per CU)."""
    return lib().ptls_mi355x_set_seg32_records(n)


def set_win16_records(n: int) -> int:
    """Window batches of at most n records use the 16-lane single-record kernels (0: never; SEG32_AUTO: one per
    CU); they take precedence over set_seg32_records."""
    L = lib()
    if not hasattr(L, "ptls_mi355x_set_win16_records"):
        return 0
    return L.ptls_mi355x_set_win16_records(n)


def set_split_records(n: int) -> int:
    """Window batches of at most n records use the split kernels (runs of 8 segments on separate CUs; 0: never;
    SEG32_AUTO: a fifth of the CUs); they take precedence over set_win16_records."""
    L = lib()
    if not hasattr(L, "ptls_mi355x_set_split_records"):
        return 0
    return L.ptls_mi355x_set_split_records(n)


def set_work_ticket_origin(origin: int) -> int:
    """Contexts created afterwards start their batch work counters at `origin` (diagnostics: the 2^32 wrap)."""
    return lib().ptls_mi355x_set_work_ticket_origin(origin & 0xFFFFFFFF)


def batch_ghash_reads(k: int = 0) -> int:
    """ds_read_b128 per block of the batch kernels' Horner multiply at k lanes per record (0: the current setting)."""
    return int(lib().ptls_mi355x_batch_ghash_reads(int(k or lib().ptls_mi355x_get_lanes_per_record())))


def kernel_name(is_seal: bool, key_size: int, n: int, framing: bool = False) -> str:
    """The kernel a launch of n records runs on (the selection launch_batch makes on the current device)."""
    return lib().ptls_mi355x_kernel_name(1 if is_seal else 0, key_size, n, 1 if framing else 0).decode()
