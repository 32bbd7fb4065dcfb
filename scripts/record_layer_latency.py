"""Host-to-host latency of the batched record layer (include/ptls_mi355x.h section 5): one rapido send window
(16 records of 16 KiB, lib/rapido.c:2115-2126) sealed from host memory into host memory, and the same window opened
back, through ptls_mi355x_record_layer_seal / _open (pinned staging, one H2D copy, one launch, one D2H copy).

    python scripts/record_layer_latency.py [--reps 50] [--records 16] [--size 16384]

Prints one JSON line: median microseconds per window for seal and open, and the payload rate.
"""
import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

import rapido_amd as ra  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--records", type=int, default=16)
    ap.add_argument("--size", type=int, default=16384)
    ap.add_argument("--keylen", type=int, default=16)
    a = ap.parse_args()
    rng = np.random.default_rng(1)
    key = rng.integers(0, 256, a.keylen, dtype=np.uint8).tobytes()
    iv = rng.integers(0, 256, 12, dtype=np.uint8).tobytes()
    frags = [rng.integers(0, 256, a.size, dtype=np.uint8).tobytes() for _ in range(a.records)]
    tx, rx = ra.RecordLayer(key, iv), ra.RecordLayer(key, iv)
    seal_us, open_us = [], []
    for i in range(a.reps + 5):
        t0 = time.perf_counter()
        wire, n = tx.seal(frags)
        t1 = time.perf_counter()
        rc, pt, consumed, m = rx.open(wire)
        t2 = time.perf_counter()
        assert rc == 0 and m == n == a.records and consumed == len(wire)
        if i >= 5:
            seal_us.append((t1 - t0) * 1e6)
            open_us.append((t2 - t1) * 1e6)
    assert pt == b"".join(frags)
    s, o = statistics.median(seal_us), statistics.median(open_us)
    payload = a.records * a.size
    print(json.dumps({"what": f"record layer, {a.records} x {a.size} B window, host buffers in and out (median of "
                              f"{a.reps}, us, including the Python binding's buffer copies)",
                      "kernel": ra.kernel_name(True, a.keylen, a.records, framing=True),
                      "seal_us": round(s, 1), "open_us": round(o, 1),
                      "seal_gibps": round(payload / 2 ** 30 / (s / 1e6), 2),
                      "open_gibps": round(payload / 2 ** 30 / (o / 1e6), 2)}))


if __name__ == "__main__":
    main()
