"""Drives scripts/probe_gh8.hip (a measurement probe, not the product): GHASH from 8-bit latin tables (16
conflict-free ds_read_b128 per multiply) against the nibble tables (32), inside the batch kernels' AES-CTR,
compute-only.

    python scripts/probe_gh8.py build     # CPU: hipcc -> scripts/_build/libprobe_gh8.so
    python scripts/probe_gh8.py run       # GPU: GH8 Horner chains bit-exact against the nibble tables, then the
                                          # throughput of each mode (GB/s of 16-B blocks)

    PROBE_MODES (default 0,2,1,3,4,5; see the .hip header), PROBE_KEYS (16,32), PROBE_REPS, PROBE_UNITS_PER_WAVE.
"""
import ctypes as C
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SO = os.path.join(ROOT, "scripts", "_build", "libprobe_gh8.so")
NAMES = {0: "aes4_only", 1: "aes2k_only", 2: "aes4+nibble (shipped)", 3: "aes2k+nibble", 4: "aes2k+gh8",
         5: "aes2+gh8"}


def build():
    os.makedirs(os.path.dirname(SO), exist_ok=True)
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
                    *os.environ.get("PROBE_FLAGS", "").split(), os.path.join(ROOT, "scripts", "probe_gh8.hip"), "-o",
                    SO], check=True)
    print("built", SO)


def run():
    import torch
    lib = C.CDLL(SO)
    vp, u32 = C.c_void_p, C.c_uint32
    lib.probe_key.argtypes = [vp, u32, vp, vp, vp]
    lib.probe_key_image_size.restype = C.c_size_t
    lib.probe_run.argtypes = [C.c_int, C.c_int, vp, u32, u32, vp, vp, vp]
    lib.probe_check.argtypes = [vp, vp, u32, vp, vp]
    lib.probe_err.restype = C.c_char_p
    dev = torch.device("cuda:0")
    stream = torch.cuda.current_stream(dev).cuda_stream
    ncu = torch.cuda.get_device_properties(dev).multi_processor_count

    def ok(rc):
        if rc != 0:
            raise SystemExit(lib.probe_err(rc).decode())

    results = {}
    for keylen in [int(x) for x in os.environ.get("PROBE_KEYS", "16,32").split(",")]:
        key = bytes(range(3, 3 + keylen))
        d_key = torch.tensor(list(key), dtype=torch.uint8, device=dev)
        d_ki = torch.zeros(lib.probe_key_image_size(), dtype=torch.uint8, device=dev)
        d_rc = torch.zeros(1, dtype=torch.int32, device=dev)
        ok(lib.probe_key(d_key.data_ptr(), keylen, d_ki.data_ptr(), d_rc.data_ptr(), stream))
        # correctness: 64 lanes x 5 chained multiplies by H^4, GH8 against the nibble tables
        rng = np.random.default_rng(5 + keylen)
        S = 5
        data = rng.integers(0, 256, S * 64 * 16, dtype=np.uint8)
        d_data = torch.from_numpy(data).to(dev)
        d_out = torch.zeros(2 * 64 * 16, dtype=torch.uint8, device=dev)
        ok(lib.probe_check(d_ki.data_ptr(), d_data.data_ptr(), S, d_out.data_ptr(), stream))
        torch.cuda.synchronize()
        got = d_out.cpu().numpy()
        if not np.array_equal(got[:1024], got[1024:]) or not got[:1024].any():
            raise SystemExit(f"GH8 Horner chains differ from the nibble tables (key {keylen} B)")
        print(f"GH8 multiply bit-exact against the nibble tables: 64 lanes x {S} chained steps, key {keylen} B",
              flush=True)
        nr = 10 if keylen == 16 else 14
        nunits = ncu * 16 * int(os.environ.get("PROBE_UNITS_PER_WAVE", "48"))
        d_work = torch.zeros(1, dtype=torch.int32, device=dev)
        d_o = torch.zeros(ncu * 1024, dtype=torch.int32, device=dev)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        res = {}
        for mode in [int(m) for m in os.environ.get("PROBE_MODES", "0,2,1,3,4,5").split(",")]:
            ts = []
            for rep in range(int(os.environ.get("PROBE_REPS", "4"))):
                d_work.zero_()
                ev[0].record()
                ok(lib.probe_run(nr, mode, d_ki.data_ptr(), nunits, ncu, d_work.data_ptr(), d_o.data_ptr(), stream))
                ev[1].record()
                torch.cuda.synchronize()
                if rep:
                    ts.append(ev[0].elapsed_time(ev[1]))
            ms = sorted(ts)[len(ts) // 2]
            gbps = nunits * 16 * 128 * 16 / (ms * 1e-3) / 1e9
            res[NAMES[mode]] = round(gbps, 1)
            print(f"AES-{8 * keylen} {NAMES[mode]:22s}: {ms:8.3f} ms  {gbps:8.1f} GB/s of 16-B blocks", flush=True)
        results[f"aes{8 * keylen}"] = res
    print(json.dumps(results))


if __name__ == "__main__":
    build() if sys.argv[1] == "build" else run()
