"""Drives scripts/probe_bs.hip (a measurement probe, not the product).

    python scripts/probe_bs.py build      # CPU: hipcc -> scripts/_build/libprobe_bs.so
    python scripts/probe_bs.py run        # GPU: correctness of the bitsliced keystream, then the wave-mix sweep

Sweep: per AES key size, the number of T-table waves per 16-wave workgroup (the rest run the bitsliced
AES); prints AES-CTR+GHASH throughput in GB/s of 16-byte blocks, no HBM traffic involved.
"""
import ctypes as C
import json
import os
import struct
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
SO = os.path.join(ROOT, "scripts", "_build", os.environ.get("PROBE_SO", "libprobe_bs.so"))


def build():
    os.makedirs(os.path.dirname(SO), exist_ok=True)
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
                    *os.environ.get("PROBE_FLAGS", "").split(), os.path.join(ROOT, "scripts", "probe_bs.hip"), "-o",
                    SO], check=True)
    print("built", SO)


def run():
    import numpy as np
    import torch

    import oracle
    lib = C.CDLL(SO)
    vp, u32 = C.c_void_p, C.c_uint32
    lib.probe_key.argtypes = [vp, u32, vp, vp, vp]
    lib.probe_key_image_size.restype = C.c_size_t
    lib.probe_run.argtypes = [vp, C.c_int, u32, u32, u32, vp, vp, vp, u32]
    lib.probe_check_run.argtypes = [vp, u32, u32, u32, u32, vp, vp]
    dev = torch.device("cuda:0")
    ncu = torch.cuda.get_device_properties(dev).multi_processor_count
    stream = torch.cuda.current_stream(dev).cuda_stream
    results = {}
    for keylen in [int(x) for x in os.environ.get("PROBE_KEYS", "16,32").split(",")]:
        key = bytes(range(3, 3 + keylen))
        d_key = torch.tensor(list(key), dtype=torch.uint8, device=dev)
        d_ki = torch.zeros(lib.probe_key_image_size(), dtype=torch.uint8, device=dev)
        d_rc = torch.zeros(1, dtype=torch.int32, device=dev)
        assert lib.probe_key(d_key.data_ptr(), keylen, d_ki.data_ptr(), d_rc.data_ptr(), stream) == 0
        torch.cuda.synchronize()
        assert int(d_rc.item()) == 0
        # correctness: 128 consecutive counter blocks, crossing a 2^8 and a 2^32 boundary
        nonce = bytes(range(0x40, 0x4C))
        n0, n1, n2 = struct.unpack("<III", nonce)
        for ctr0 in (0xF0, 0xFFFFFFC0):
            d_out = torch.zeros(128 * 16, dtype=torch.uint8, device=dev)
            assert lib.probe_check_run(d_ki.data_ptr(), n0, n1, n2, ctr0, d_out.data_ptr(), stream) == 0
            torch.cuda.synchronize()
            got = d_out.cpu().numpy().tobytes()
            want = b"".join(oracle.ecb(key, nonce + struct.pack(">I", (ctr0 + i) & 0xFFFFFFFF)) for i in range(128))
            if got != want:
                raise SystemExit(f"bitsliced keystream mismatch (AES-{8 * keylen}, ctr0={ctr0:#x})")
        print(f"AES-{8 * keylen}: bitsliced keystream on the GPU matches the oracle (256 blocks)", flush=True)

        nr = 10 if keylen == 16 else 14
        nunits = ncu * 16 * 96 * int(os.environ.get("PROBE_UNITS_MULT", "1"))
        d_work = torch.zeros(1, dtype=torch.int32, device=dev)
        d_out = torch.zeros(ncu * 1024, dtype=torch.int32, device=dev)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        res = {}
        threads = int(os.environ.get("PROBE_THREADS", "1024"))
        for n_tt in [int(x) for x in os.environ.get("PROBE_NTT", "16,14,13,12,11,10,8,6,4,0").split(",")]:
            ts = []
            for rep in range(int(os.environ.get("PROBE_REPS", "4"))):
                d_work.zero_()
                ev[0].record()
                assert lib.probe_run(d_ki.data_ptr(), nr, n_tt, nunits, ncu, d_work.data_ptr(), d_out.data_ptr(),
                                     stream, threads) == 0
                ev[1].record()
                torch.cuda.synchronize()
                if rep:
                    ts.append(ev[0].elapsed_time(ev[1]))
            ms = sorted(ts)[len(ts) // 2]
            gbps = nunits * 64 * 16 / (ms * 1e-3) / 1e9
            res[n_tt] = round(gbps, 1)
            print(f"AES-{8 * keylen} [{threads // 64} waves/CU] T-table waves {min(n_tt, threads // 64):2d}: {ms:7.3f} ms  {gbps:8.1f} GB/s", flush=True)
        results[f"aes{8 * keylen}"] = res
    print(json.dumps(results))


if __name__ == "__main__":
    build() if sys.argv[1] == "build" else run()
