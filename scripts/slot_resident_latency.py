"""Latency of the synchronous AEAD slot (ptls_aead_encrypt / _decrypt through the exported ptls_aead_algorithm_t, as
picotls' record layer calls it, one record per call): a launch + stream synchronisation per call against a job of
the resident grid (ptls_mi355x_set_slot_resident).  Measurement only.

    python scripts/slot_resident_latency.py [--reps 300]
"""
import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=300)
    a = ap.parse_args()
    import torch  # noqa: F401  (one HIP runtime for torch and the engine)

    import rapido_amd as ra
    ra.require_gpu()
    key, iv = bytes(range(16)), bytes(range(12))
    enc = ra.aead_new_direct("aes128gcm", True, key, iv)
    dec = ra.aead_new_direct("aes128gcm", False, key, iv)
    out = {"what": "one record per call through the AEAD slot, host buffers, median us", "reps": a.reps}
    for L in (64, 1400, 16384):
        pt = bytes(i & 0xFF for i in range(L))
        aad = bytes([0x17, 3, 3, (L + 16) >> 8, (L + 16) & 0xFF])
        row = {}
        for mode in ("launch", "resident", "launch", "resident"):
            ra.set_slot_resident(mode == "resident")
            for _ in range(20):
                ct = enc.encrypt(pt, 1, aad)
                assert dec.decrypt(ct, 1, aad) == pt
            te, td = [], []
            for i in range(a.reps):
                t0 = time.perf_counter()
                ct = enc.encrypt(pt, i, aad)
                t1 = time.perf_counter()
                assert dec.decrypt(ct, i, aad) == pt
                t2 = time.perf_counter()
                te.append((t1 - t0) * 1e6)
                td.append((t2 - t1) * 1e6)
            row[mode] = {"encrypt_us": round(statistics.median(te), 2), "decrypt_us": round(statistics.median(td), 2)}
        out[str(L)] = row
        print(json.dumps({L: row}), flush=True)
    ra.set_slot_resident(False)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
