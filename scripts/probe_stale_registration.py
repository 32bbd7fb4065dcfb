"""Does a host range stay known to the HIP runtime after the record layer unregistered it? (diagnostic only: no
kernels, no copies, so nothing here can fault the GPU)

The round-4 and round-5 GPU suites each failed once with an illegal address surfacing at the first host-to-device
copy of tests/test_gpu_tls.py::test_multi_connection_windows, after the record-layer tests had registered and
unregistered many page buffers (hipHostRegister / hipHostUnregister) that Python then freed; the per-test device check
after the previous test had passed.  If the runtime kept a registration past hipHostUnregister, a later pageable copy
from a new buffer at a reused address would run through the stale mapping.  This asks the runtime, with
hipPointerGetAttributes, about buffers at reused addresses after such cycles.

    python scripts/probe_stale_registration.py      (GPU box)  -> one JSON line
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


def page_buffer(n):
    raw = np.zeros(n + 4096, np.uint8)
    off = (-raw.ctypes.data) % 4096
    return raw, raw[off:off + n]


def main():
    hip = C.CDLL("libamdhip64.so")
    hip.hipPointerGetAttributes.argtypes = [C.POINTER(Attr), C.c_void_p]
    hip.hipGetLastError.restype = C.c_int
    ra.require_gpu()

    def ask(p):
        a = Attr()
        rc = hip.hipPointerGetAttributes(C.byref(a), C.c_void_p(p))
        hip.hipGetLastError()
        return {"rc": rc, "type": a.type, "dev": a.devicePointer or 0}

    key, iv = bytes(16), bytes(12)
    out = {"cycles": [], "after": []}
    seen = []
    for cycle in range(40):  # the campaign's pattern: an 8 MiB page buffer registered by two layers, closed, freed
        raw, buf = page_buffer(8 << 20)
        base = buf.ctypes.data
        tx, rx = ra.RecordLayer(key, iv), ra.RecordLayer(key, iv)
        tx.register(buf)
        rx.register(buf)
        during = ask(base)
        tx.close()
        rx.close()
        after = ask(base)
        out["cycles"].append({"base": hex(base), "during": during, "after_unregister": after})
        seen.append(base)
        del tx, rx, buf, raw
    # new buffers of other sizes, some at reused addresses: what does the runtime say about them?
    for n in (1 << 20, 1611110, 4 << 20, 8 << 20, 16 << 20):
        a = np.zeros(n, np.uint8)
        p = a.ctypes.data
        out["after"].append({"size": n, "ptr": hex(p), "inside_an_old_range": any(b <= p < b + (8 << 20) for b in seen),
                             "attrs": ask(p), "attrs_mid": ask(p + n // 2)})
        del a
    stale = [c for c in out["cycles"] if c["after_unregister"]["rc"] == 0 and c["after_unregister"]["dev"]]
    stale += [x for x in out["after"] if x["attrs"]["rc"] == 0 and x["attrs"]["dev"]]
    out["stale"] = len(stale)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
