"""Synchronous record-layer opens by window size (measurement only): rapido's receive windows of 8 / 16 / 32 records of
16 KiB (lib/rapido.c:2030), registered buffers in place (direct, the delivery kernel) and zero-copy staging; median
microseconds per window over 20 windows after 4 untimed ones.

    python scripts/rl_open_sizes.py   (GPU)  -> one JSON line
"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import rapido_amd as ra  # noqa: E402
from rapido_amd.records import xorshift64star  # noqa: E402


def page_buffer(nbytes):
    raw = np.zeros(nbytes + 4096, np.uint8)
    off = (-raw.ctypes.data) % 4096
    return raw[off:off + nbytes]


def main():
    key, iv = bytes(range(16)), bytes(range(12))
    res = {}
    for transport in ("direct", "zero_copy"):
        for nrec in (8, 16, 32):
            frags = [xorshift64star(100 + i, 16384) for i in range(nrec)]
            tx = ra.RecordLayer(key, iv)
            wire_b, n = tx.seal([f.tobytes() for f in frags])
            assert n == nrec
            tx.close()
            buf = page_buffer(4 << 20)
            wire = buf[:len(wire_b)]
            wire[:] = np.frombuffer(wire_b, np.uint8)
            out = buf[2 << 20:(2 << 20) + nrec * 16384 + 64]
            rx = ra.RecordLayer(key, iv)
            if transport == "direct":
                rx.register(buf)
            ts = []
            for w in range(24):
                rx.seq = 0
                t0 = time.perf_counter()
                rc, plen, cons, k = rx.open_into(wire, out)
                ts.append(time.perf_counter() - t0)
                assert (rc, k, cons, plen) == (0, nrec, len(wire_b), nrec * 16384)
            assert out[:plen].tobytes() == b"".join(f.tobytes() for f in frags)
            rx.close()
            us = float(np.median(ts[4:])) * 1e6
            res[f"{transport}_{nrec}"] = {"us_per_window": round(us, 1), "MBps": round(nrec * 16384 / us, 1)}
            print(transport, nrec, res[f"{transport}_{nrec}"], flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
