"""Framing kernels at rapido's window sizes: where launch latency, not the kernel, decides.

    python scripts/window_bench.py [--out profiles/r01c_windows.json]

- send window: 16 TLS records of 16384-B fragments (rapido_send_on_connection, lib/rapido.c:2115-2126), one
  ptls_mi355x_tls_seal_records launch per window: latency per launch, eager and replayed from a hipGraph;
- receive window: 32 records (rapido_read_connection's recv() of 32 x 16406 B, lib/rapido.c:2030-2032), one
  ptls_mi355x_tls_open_records launch;
- C connections' send windows in ONE launch (tls_seal_records_multi, per-connection IVs): GiB/s vs C.
Device-resident buffers, HIP events on the launch stream.
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="")
    ap.add_argument("--reps", type=int, default=200)
    ap.add_argument("--seg32", type=int, default=-1,
                    help="window batches of at most this many records use 32-position segments (-1: default, 1 per CU)")
    args = ap.parse_args()
    import torch

    import rapido_amd as ra
    ra.require_gpu()
    if args.seg32 >= 0:
        ra.set_seg32_records(args.seg32)
    dev = torch.device("cuda:0")
    key, iv = bytes(range(16)), bytes(range(40, 52))
    eng = ra.Engine(key)
    stream = torch.cuda.current_stream(dev)
    sh = stream.cuda_stream
    FRAG, WIN = 16384, 16

    def plan(nconn):
        n = nconn * WIN
        t = np.zeros(n, ra.TLS_RECORD_DTYPE)
        t["src"] = np.arange(n, dtype=np.uint64) * FRAG
        t["dst"] = np.arange(n, dtype=np.uint64) * (FRAG + 22)
        t["seq"] = np.tile(np.arange(WIN, dtype=np.uint64), nconn)
        t["len"] = FRAG
        t["type"] = 23
        conn = np.repeat(np.arange(nconn, dtype=np.uint32), WIN)
        return t, conn

    def timed(fn, reps):
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ev[0].record(stream)
        for _ in range(reps):
            fn()
        ev[1].record(stream)
        torch.cuda.synchronize()
        return ev[0].elapsed_time(ev[1]) / reps  # ms per call

    res = {"window": f"{WIN} records x {FRAG} B", "send": {}, "receive": {}, "multi_connection": [],
           "note": "send/receive: default dispatch (window kernels up to 16384 records)"}
    # one send window per launch
    t, conn = plan(1)
    d_t = torch.from_numpy(t.view(np.uint8)).to(dev)
    d_src = torch.randint(0, 256, (WIN * FRAG,), dtype=torch.uint8, device=dev)
    d_wire = torch.zeros(WIN * (FRAG + 22), dtype=torch.uint8, device=dev)

    def send():
        eng.tls_seal_records(iv, d_t.data_ptr(), WIN, d_src.data_ptr(), d_wire.data_ptr(), sh)

    ms = timed(send, args.reps)
    res["send"]["eager_us"] = round(ms * 1e3, 2)
    res["send"]["eager_gibps"] = round(WIN * FRAG / (ms * 1e-3) / 2 ** 30, 2)
    g = torch.cuda.CUDAGraph()
    cap = torch.cuda.Stream(dev)
    cap.wait_stream(stream)
    with torch.cuda.stream(cap):
        send_cap = lambda: eng.tls_seal_records(iv, d_t.data_ptr(), WIN, d_src.data_ptr(), d_wire.data_ptr(),
                                                cap.cuda_stream)
        send_cap()
        torch.cuda.synchronize()
        with torch.cuda.graph(g, stream=cap):
            send_cap()
    torch.cuda.synchronize()
    ms = timed(g.replay, args.reps)
    res["send"]["graph_us"] = round(ms * 1e3, 2)
    res["send"]["graph_gibps"] = round(WIN * FRAG / (ms * 1e-3) / 2 ** 30, 2)

    # one receive window (32 records) per launch
    RW = 32
    t2, _ = plan(2)
    d_t2 = torch.from_numpy(t2.view(np.uint8)).to(dev)
    d_src2 = torch.randint(0, 256, (RW * FRAG,), dtype=torch.uint8, device=dev)
    d_wire2 = torch.zeros(RW * (FRAG + 22), dtype=torch.uint8, device=dev)
    eng.tls_seal_records(iv, d_t2.data_ptr(), RW, d_src2.data_ptr(), d_wire2.data_ptr(), sh)
    o = t2.copy()
    # plaintext slots hold fragment + content type (FRAG + 1 bytes): 16-byte aligned, FRAG + 16 apart
    o["src"], o["len"], o["dst"] = t2["dst"], FRAG + 17, np.arange(RW, dtype=np.uint64) * (FRAG + 16)
    d_o = torch.from_numpy(o.view(np.uint8)).to(dev)
    d_pt = torch.zeros(RW * (FRAG + 16), dtype=torch.uint8, device=dev)
    d_st = torch.zeros(RW, dtype=torch.int32, device=dev)
    d_ty = torch.zeros(RW, dtype=torch.uint8, device=dev)

    def recv():
        eng.tls_open_records(iv, d_o.data_ptr(), RW, d_wire2.data_ptr(), d_pt.data_ptr(), d_st.data_ptr(),
                             d_ty.data_ptr(), sh)

    ms = timed(recv, args.reps)
    torch.cuda.synchronize()
    assert (d_st.cpu().numpy() == FRAG).all()
    res["receive"] = {"records": RW, "eager_us": round(ms * 1e3, 2),
                      "eager_gibps": round(RW * FRAG / (ms * 1e-3) / 2 ** 30, 2)}

    # C connections' windows in one launch, on the window kernels and on the batch kernels
    for nconn in (1, 4, 16, 64, 256, 1024, 4096):
      for mode in ("window", "batch"):
        ra.set_tls_window_records(1 << 30 if mode == "window" else 0)
        t, conn = plan(nconn)
        n = len(t)
        d_t = torch.from_numpy(t.view(np.uint8)).to(dev)
        d_c = torch.from_numpy(conn.view(np.int32)).to(dev)
        d_src = torch.randint(0, 256, (n * FRAG,), dtype=torch.uint8, device=dev)
        d_wire = torch.zeros(n * (FRAG + 22), dtype=torch.uint8, device=dev)

        def sendm():
            eng.tls_seal_records(iv, d_t.data_ptr(), n, d_src.data_ptr(), d_wire.data_ptr(), sh, conn_ptr=d_c.data_ptr())

        ms = timed(sendm, max(5, args.reps // max(1, nconn // 16)))
        res["multi_connection"].append({"connections": nconn, "records": n, "kernels": mode,
                                        "us_per_launch": round(ms * 1e3, 1), "gibps": round(n * FRAG / (ms * 1e-3) / 2 ** 30, 1)})
        del d_t, d_c, d_src, d_wire
    ra.set_tls_window_records(16384)

    # AEAD batches (ptls_mi355x_seal_batch, 5-byte AAD): where the window kernels stop paying off
    from rapido_amd import records
    res["aead_batches"] = []
    for length in (1400, 16384):
        for n in (16, 256, 768, 1024, 4096, 16384):
            recs, src_bytes, aad_bytes = records.layout(np.full(n, length, np.uint64), np.full(n, 5, np.uint64), align=256)
            d_r = torch.from_numpy(recs.view(np.uint8)).to(dev)
            d_s = torch.randint(0, 256, (src_bytes,), dtype=torch.uint8, device=dev)
            d_o = torch.zeros_like(d_s)
            d_a = torch.zeros(aad_bytes, dtype=torch.uint8, device=dev)
            for mode in ("window", "batch"):
                ra.set_aead_window_records(1 << 30 if mode == "window" else 0)
                ms = timed(lambda: eng.seal_batch(iv, d_r.data_ptr(), n, d_s.data_ptr(), d_o.data_ptr(), d_a.data_ptr(), sh),
                           max(5, args.reps // max(1, n // 64)))
                res["aead_batches"].append({"record_bytes": length, "records": n, "kernels": mode,
                                            "us_per_launch": round(ms * 1e3, 1),
                                            "gibps": round(n * length / (ms * 1e-3) / 2 ** 30, 1)})
            del d_r, d_s, d_o, d_a
    ra.set_aead_window_records(2048)
    eng.close()
    line = json.dumps(res)
    print(line)
    if args.out:
        with open(args.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
