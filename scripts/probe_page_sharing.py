"""How does the HIP runtime treat host ranges that share a page without sharing bytes? (diagnostic only: no kernels,
no copies, nothing here can fault the GPU)

Two socket buffers from malloc can share a page.  If hipHostRegister answers "already registered" for the second
(because its first page is mapped for the first), the record layer takes it for the application's registration and
uses the first range's mapping -- which goes when the first range is unregistered.  This registers byte ranges of one
page-aligned buffer in several arrangements and reports the runtime's answers, the device pointers, and what is left
mapped after unregistering.

    python scripts/probe_page_sharing.py      (GPU box)  -> one JSON line
"""
import ctypes as C
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import rapido_amd as ra  # noqa: E402


class Attr(C.Structure):  # hipPointerAttribute_t (hip_runtime_api.h, ROCm 7)
    _fields_ = [("type", C.c_int), ("device", C.c_int), ("devicePointer", C.c_void_p), ("hostPointer", C.c_void_p),
                ("isManaged", C.c_int), ("allocationFlags", C.c_uint)]


def main():
    hip = C.CDLL("libamdhip64.so")
    hip.hipHostRegister.argtypes = [C.c_void_p, C.c_size_t, C.c_uint]
    hip.hipHostUnregister.argtypes = [C.c_void_p]
    hip.hipHostGetDevicePointer.argtypes = [C.POINTER(C.c_void_p), C.c_void_p, C.c_uint]
    hip.hipPointerGetAttributes.argtypes = [C.POINTER(Attr), C.c_void_p]
    hip.hipGetLastError.restype = C.c_int
    ra.require_gpu()
    raw = np.zeros(5 * 4096, np.uint8)
    p = raw.ctypes.data + (-raw.ctypes.data) % 4096  # page-aligned, 4 pages

    def reg(off, n):
        rc = hip.hipHostRegister(C.c_void_p(p + off), n, 1)  # hipHostRegisterMapped
        hip.hipGetLastError()
        d = C.c_void_p()
        rc2 = hip.hipHostGetDevicePointer(C.byref(d), C.c_void_p(p + off), 0)
        hip.hipGetLastError()
        return {"range": [hex(off), hex(off + n)], "register": rc, "devptr_rc": rc2,
                "dev_minus_host": (d.value - (p + off)) if d.value else None}

    def unreg(off):
        rc = hip.hipHostUnregister(C.c_void_p(p + off))
        hip.hipGetLastError()
        return rc

    def ask(off):
        a = Attr()
        rc = hip.hipPointerGetAttributes(C.byref(a), C.c_void_p(p + off))
        hip.hipGetLastError()
        return {"at": hex(off), "rc": rc, "type": a.type, "mapped": bool(a.devicePointer)}

    out = {}
    # 1. A and B share page 0 but no byte; then A goes
    out["A"] = reg(0x100, 0x800)
    out["B_same_page_disjoint"] = reg(0xa00, 0x700)
    out["C_inside_A"] = reg(0x200, 0x100)
    out["D_straddles_A_end"] = reg(0x800, 0x200)
    out["E_next_page_only"] = reg(0x1100, 0x100)
    out["before_unregister_A"] = [ask(0x100), ask(0xa00), ask(0x1050), ask(0x1100)]
    out["unregister_A"] = unreg(0x100)
    out["after_unregister_A"] = [ask(0x100), ask(0xa00), ask(0x1050), ask(0x1100)]
    for off in (0xa00, 0x200, 0x800, 0x1100):
        out[f"unregister_{off:#x}"] = unreg(off)
    out["after_all"] = [ask(0x100), ask(0xa00), ask(0x1100)]
    # 2. the same through two record layers: layer 1 registers A, layer 2 registers B; layer 1 closes
    tx, rx = ra.RecordLayer(bytes(16), bytes(12)), ra.RecordLayer(bytes(16), bytes(12))
    a = np.frombuffer((C.c_uint8 * 0x800).from_address(p + 0x100), np.uint8)
    b = np.frombuffer((C.c_uint8 * 0x700).from_address(p + 0xa00), np.uint8)
    res = {}
    try:
        tx.register(a)
        res["layer1_A"] = "ok"
    except RuntimeError as e:
        res["layer1_A"] = str(e)
    try:
        rx.register(b)
        res["layer2_B"] = "ok"
    except RuntimeError as e:
        res["layer2_B"] = str(e)
    res["before_close"] = ask(0xa00)
    tx.close()
    res["after_layer1_close"] = ask(0xa00)
    rx.close()
    res["after_both"] = ask(0xa00)
    out["layers"] = res
    print(json.dumps(out))


if __name__ == "__main__":
    main()
