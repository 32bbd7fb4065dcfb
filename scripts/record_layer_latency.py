"""Host-to-host latency of the batched record layer (include/ptls_mi355x.h section 5): one rapido send window
(16 records of 16 KiB, lib/rapido.c:2115-2126) sealed from host memory into host memory, and the same window opened
back, through ptls_mi355x_record_layer_seal / _open, for each way the bytes can travel (record_layer.c):
  copy      -- the Python bytes go through the layer's pinned staging, one H2D and one D2H DMA copy;
  zero_copy -- the same staging, read and written by the kernel over PCIe (the default up to 4 MiB);
  direct    -- fragments, wire and plaintext in registered host buffers, no copy at all (seal_into / open_into).

    python scripts/record_layer_latency.py [--reps 50] [--records 16] [--size 16384]

Prints one JSON line per mode: median microseconds per window for seal and open, and the payload rate.
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
    payload = a.records * a.size
    for mode in ("copy", "zero_copy", "direct"):
        tx, rx = ra.RecordLayer(key, iv), ra.RecordLayer(key, iv)
        if mode == "copy":
            tx.set_zero_copy_bytes(0)
            rx.set_zero_copy_bytes(0)
        if mode == "direct":
            send = np.frombuffer(b"".join(frags), np.uint8).copy()
            views = [send[i * a.size:(i + 1) * a.size] for i in range(a.records)]
            wirebuf = np.zeros(payload + a.records * 64, np.uint8)
            ptbuf = np.zeros(payload + a.records * 64, np.uint8)
            tx.register(send)
            tx.register(wirebuf)
            rx.register(wirebuf)
            rx.register(ptbuf)
        seal_us, open_us = [], []
        for i in range(a.reps + 5):
            if mode == "direct":
                t0 = time.perf_counter()
                wlen, n = tx.seal_into(views, wirebuf)
                t1 = time.perf_counter()
                rc, olen, consumed, m = rx.open_into(wirebuf[:wlen], ptbuf)
                t2 = time.perf_counter()
                assert rc == 0 and m == n == a.records and consumed == wlen and olen == payload
            else:
                t0 = time.perf_counter()
                wire, n = tx.seal(frags)
                t1 = time.perf_counter()
                rc, pt, consumed, m = rx.open(wire)
                t2 = time.perf_counter()
                assert rc == 0 and m == n == a.records and consumed == len(wire)
            rx.seq = tx.seq
            if i >= 5:
                seal_us.append((t1 - t0) * 1e6)
                open_us.append((t2 - t1) * 1e6)
        got = ptbuf[:payload].tobytes() if mode == "direct" else pt
        assert got == b"".join(frags)
        s, o = statistics.median(seal_us), statistics.median(open_us)
        print(json.dumps({"what": f"record layer, {a.records} x {a.size} B window, host buffers in and out (median of "
                                  f"{a.reps}, us, including the Python binding)", "mode": mode,
                          "kernel": ra.kernel_name(True, a.keylen, a.records, framing=True),
                          "seal_us": round(s, 1), "open_us": round(o, 1),
                          "seal_gibps": round(payload / 2 ** 30 / (s / 1e6), 2),
                          "open_gibps": round(payload / 2 ** 30 / (o / 1e6), 2)}), flush=True)
        tx.close()
        rx.close()
    # the send windows of C connections of one session: one seal_multi launch vs C seal calls, on registered buffers
    # (direct) and through the zero-copy staging
    for conns in (4, 8):
        for direct in (True, False):
            ivs = [bytes([i]) + iv[1:] for i in range(conns)]
            layers = [ra.RecordLayer(key, v) for v in ivs]
            if direct:
                send = np.frombuffer(b"".join(frags), np.uint8).copy()
                wins = [[send[i * a.size:(i + 1) * a.size] for i in range(a.records)]] * conns
                per = payload + a.records * 64
                wirebuf = np.zeros(conns * per, np.uint8)
                outs = [wirebuf[c * per:(c + 1) * per] for c in range(conns)]
                for lr in layers:  # the first registers, the others find the ranges already registered
                    lr.register(send)
                    lr.register(wirebuf)
            else:
                wins, outs = [frags] * conns, None
            one, each = [], []
            for i in range(a.reps + 5):
                t0 = time.perf_counter()
                res = ra.record_layer_seal_multi(layers, wins, outs=outs)
                t1 = time.perf_counter()
                for c, (lr, w) in enumerate(zip(layers, wins)):
                    if direct:
                        ra.record_layer_seal_multi([lr], [w], outs=[outs[c]])
                    else:
                        lr.seal(w)
                t2 = time.perf_counter()
                assert all(n == a.records for _, n in res)
                if i >= 5:
                    one.append((t1 - t0) * 1e6)
                    each.append((t2 - t1) * 1e6)
            s1, s2 = statistics.median(one), statistics.median(each)
            print(json.dumps({"what": f"{conns} connections x {a.records} x {a.size} B send windows, host buffers in and "
                                      f"out (median of {a.reps}, us, Python binding, "
                                      f"{'registered buffers (direct)' if direct else 'zero-copy staging'})",
                              "mode": "seal_multi" + ("_direct" if direct else ""), "one_launch_us": round(s1, 1),
                              "per_connection_calls_us": round(s2, 1),
                              "one_launch_gibps": round(conns * payload / 2 ** 30 / (s1 / 1e6), 2),
                              "per_connection_calls_gibps": round(conns * payload / 2 ** 30 / (s2 / 1e6), 2)}),
                  flush=True)
            for lr in layers[::-1]:  # layers[0] owns the registrations: it goes last
                lr.close()


if __name__ == "__main__":
    main()
