"""Do split-kernel windows on separate streams (one engine context each) run concurrently?  Device-resident
16 x 16 KiB send windows, `depth` streams round-robin, vs one stream; and the same with the window's input and
output in host memory (registered, mapped: the record layer's direct transport).  Measurement, not product.

    python scripts/concurrency_probe.py      (GPU)
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import rapido_amd as ra  # noqa: E402

WIN, FRAG = 16, 16384


def run(depth, host, nwin=96):
    dev = torch.device("cuda:0")
    engines = [ra.Engine(bytes(range(16))) for _ in range(depth)]
    streams = [torch.cuda.Stream(dev) for _ in range(depth)]
    t = np.zeros(WIN, ra.TLS_RECORD_DTYPE)
    t["src"] = np.arange(WIN, dtype=np.uint64) * FRAG
    t["dst"] = np.arange(WIN, dtype=np.uint64) * (FRAG + 22)
    t["seq"] = np.arange(WIN, dtype=np.uint64)
    t["len"], t["type"] = FRAG, 23
    d_t = torch.from_numpy(t.view(np.uint8)).to(dev)
    if host:
        src = [torch.zeros(WIN * FRAG, dtype=torch.uint8).pin_memory() for _ in range(depth)]
        dst = [torch.zeros(WIN * (FRAG + 22), dtype=torch.uint8).pin_memory() for _ in range(depth)]
    else:
        src = [torch.randint(0, 256, (WIN * FRAG,), dtype=torch.uint8, device=dev) for _ in range(depth)]
        dst = [torch.zeros(WIN * (FRAG + 22), dtype=torch.uint8, device=dev) for _ in range(depth)]
    iv = bytes(12)

    def go():
        for w in range(nwin):
            i = w % depth
            engines[i].tls_seal_records(iv, d_t.data_ptr(), WIN, src[i].data_ptr(), dst[i].data_ptr(),
                                        streams[i].cuda_stream)
    go()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    go()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    for e in engines:
        e.close()
    return round(dt / nwin * 1e6, 2)


res = {}
for host in (False, True):
    for depth in (1, 2, 4):
        res[f"{'host' if host else 'device'}_streams{depth}_us_per_window"] = run(depth, host)
        print(json.dumps(res), flush=True)
