"""Seal-only launches at several record lengths, for PMC passes (WRITE_SIZE / FETCH_SIZE per length).

    rocprofv3 --pmc WRITE_SIZE --kernel-trace -d DIR -o run --output-format csv -- python scripts/pmc_lengths.py

Prints one line per length: algorithmic read/write bytes per launch and the launch time, so the
counter rows (in launch order) can be matched to lengths.
"""
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402  (first: one HIP runtime)

import rapido_amd as ra  # noqa: E402
from rapido_amd import records  # noqa: E402

LENGTHS = [int(x) for x in os.environ.get("PMC_LENGTHS", "1392,1400,1408,1424,16384,16368").split(",")]
TOTAL = int(os.environ.get("PMC_BYTES", str(1 << 30)))
ALIGN = int(os.environ.get("PMC_ALIGN", "256"))
LANES = [int(x) for x in os.environ.get("PMC_LANES", "4").split(",")]

out = []
for K, L in [(k, l) for k in LANES for l in LENGTHS]:
    ra.set_lanes_per_record(K)
    n = max(1, TOTAL // L)
    lengths = np.full(n, L, dtype=np.uint64)
    recs, src_bytes, aad_bytes = records.layout(lengths, np.full(n, 5, dtype=np.uint64), align=ALIGN)
    aad = np.zeros(aad_bytes, dtype=np.uint8)
    aad[: 5 * n] = records.tls_aad(lengths)
    d_src = torch.randint(0, 256, (src_bytes,), dtype=torch.uint8, device="cuda")
    d_dst = torch.zeros_like(d_src)
    d_recs = torch.from_numpy(recs.view(np.uint8)).cuda()
    d_aad = torch.from_numpy(aad).cuda()
    eng = ra.Engine(bytes(range(16)))
    iv = bytes(12)
    for _ in range(2):
        eng.seal_batch(iv, d_recs.data_ptr(), n, d_src.data_ptr(), d_dst.data_ptr(), d_aad.data_ptr())
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    eng.seal_batch(iv, d_recs.data_ptr(), n, d_src.data_ptr(), d_dst.data_ptr(), d_aad.data_ptr())
    ev[1].record()
    torch.cuda.synchronize()
    ms = ev[0].elapsed_time(ev[1])
    out.append({"lanes": K, "len": L, "n": n, "read": n * (L + 5 + 40), "write": n * (L + 16), "ms": round(ms, 4),
                "gibps": round(n * L / 2 ** 30 / (ms / 1e3), 1), "launches": 3})
    del d_src, d_dst, d_recs, d_aad
    eng.close()
    print(json.dumps(out[-1]), flush=True)
