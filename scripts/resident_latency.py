"""Latency of one rapido send window (16 x 16 KiB TLS records) sealed by a kernel launch + synchronisation against a
job of the resident grid (include/ptls_mi355x.h section 6) + its completion poll, with the records in device memory
and in pinned host memory read and written in place.  Measurement only.

    python scripts/resident_latency.py [--reps 300] [--workers 128]
"""
import argparse
import json
import os
import statistics
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=300)
    ap.add_argument("--workers", type=int, default=0)
    ap.add_argument("--records", type=int, default=16)
    ap.add_argument("--len", type=int, default=16384)
    a = ap.parse_args()
    import torch
    import rapido_amd as ra
    ra.require_gpu()
    if a.workers:
        ra.set_resident_workers(a.workers)
    rng = np.random.default_rng(1)
    key, iv = rng.integers(0, 256, 16, dtype=np.uint8).tobytes(), rng.integers(0, 256, 12, dtype=np.uint8).tobytes()
    n, ln = a.records, a.len
    trecs = np.zeros(n, ra.TLS_RECORD_DTYPE)
    for i in range(n):
        trecs[i] = (i * ln, i * (ln + 22), i, ln, 23)
    eng = ra.Engine(key)
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")

    def devptr(t):
        """the GPU's address of a pinned host tensor (hipHostGetDevicePointer), or the device tensor's own"""
        if not t.is_pinned():
            return t.data_ptr()
        p = ctypes.c_void_p()
        assert hip.hipHostGetDevicePointer(ctypes.byref(p), ctypes.c_void_p(t.data_ptr()), 0) == 0
        return p.value

    keep = []

    def registered(a_np):
        """a page-aligned host copy of a_np, hipHostRegister'ed (mapped) as the record layer registers ranges"""
        buf = np.zeros(a_np.nbytes + 8192, np.uint8)
        off = (-buf.ctypes.data) % 4096
        view = buf[off: off + a_np.nbytes]
        view[:] = a_np.view(np.uint8).reshape(-1)
        assert hip.hipHostRegister(ctypes.c_void_p(view.ctypes.data), ctypes.c_size_t(view.nbytes), 2) == 0
        p = ctypes.c_void_p()
        assert hip.hipHostGetDevicePointer(ctypes.byref(p), ctypes.c_void_p(view.ctypes.data), 0) == 0
        keep.append((buf, view))
        return view, p.value

    out = {"window": f"{n} x {ln} B TLS records, AES-128", "reps": a.reps}
    for where in ("device", "host", "registered"):
        pin = where == "host"
        src_np = rng.integers(0, 256, n * ln, dtype=np.uint8)
        if where == "registered":
            src, p_src = registered(src_np)
            dst, p_dst = registered(np.zeros(n * (ln + 22), np.uint8))
            recs, p_recs = registered(trecs.view(np.uint8).copy())
            dst = torch.from_numpy(dst)
        else:
            src = torch.from_numpy(src_np)
            src = src.pin_memory() if pin else src.cuda()
            dst = torch.zeros(n * (ln + 22), dtype=torch.uint8)
            dst = dst.pin_memory() if pin else dst.cuda()
            recs = torch.from_numpy(trecs.view(np.uint8).copy())
            recs = recs.pin_memory() if pin else recs.cuda()
            p_src, p_dst, p_recs = devptr(src), devptr(dst), devptr(recs)
        torch.cuda.synchronize()
        res = {}
        for mode in ("launch", "resident", "launch", "resident"):
            ts, tl = [], []
            for r in range(a.reps + 20):
                t0 = time.perf_counter()
                if mode == "launch":
                    eng.tls_seal_records(iv, p_recs, n, p_src, p_dst)
                    torch.cuda.synchronize()
                else:
                    job = eng.resident_tls_seal_records(iv, p_recs, n, p_src, p_dst)
                    eng.resident_wait(job)
                    if r >= 20:
                        tl.append(eng.resident_job_times(job))
                if r >= 20:
                    ts.append((time.perf_counter() - t0) * 1e6)
            res[mode] = round(statistics.median(ts), 2)  # (the second pass of each mode is kept)
            if tl:
                res["timeline_us"] = {k: round(statistics.median(x[i] for x in tl) / 1e3, 2) for i, k in
                                      enumerate(("pickup", "units", "finish", "gpu_total"))}
        ref = dst.cpu().numpy().tobytes()
        eng.tls_seal_records(iv, p_recs, n, p_src, p_dst)
        torch.cuda.synchronize()
        assert dst.cpu().numpy().tobytes() == ref
        out[where] = {"launch_sync_us": res["launch"], "resident_us": res["resident"],
                      "resident_timeline_us": res["timeline_us"]}
        print(json.dumps({where: out[where]}), flush=True)
    out["resident_launches"] = ra.resident_launches(0)
    print(json.dumps(out), flush=True)
    ra.resident_stop(0)


if __name__ == "__main__":
    main()
