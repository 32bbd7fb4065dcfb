"""Drives scripts/lds_bench.hip: sustained LDS read rate for the kernels' access patterns.
    python scripts/lds_bench.py build | run"""
import ctypes as C
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SO = os.path.join(ROOT, "scripts", "_build", "liblds_bench.so")


def build():
    os.makedirs(os.path.dirname(SO), exist_ok=True)
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
                    os.path.join(ROOT, "scripts", "lds_bench.hip"), "-o", SO], check=True)


def run():
    import torch
    lib = C.CDLL(SO)
    lib.lds_bench_run.argtypes = [C.c_int, C.c_uint32, C.c_uint32, C.c_uint32, C.c_void_p, C.c_void_p]
    dev = torch.device("cuda:0")
    ncu = torch.cuda.get_device_properties(dev).multi_processor_count
    out = torch.zeros(ncu * 1024, dtype=torch.int32, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    iters = 4096
    for mode, name in ((0, "ds_read_b32 (T-table pattern)"), (1, "ds_read_b128 (GHASH pattern)"), (2, "mix 4:1"),
                       (3, "ds_read_b64 (T-table, 8-B slots)"), (4, "mix64 4:1")):
        for threads in (int(t) for t in os.environ.get("LDS_THREADS", "1024").split(",")):
            ts = []
            for rep in range(4):
                ev[0].record()
                assert lib.lds_bench_run(mode, iters, ncu, threads, out.data_ptr(), s) == 0
                ev[1].record()
                torch.cuda.synchronize()
                if rep:
                    ts.append(ev[0].elapsed_time(ev[1]))
            ms = sorted(ts)[1]
            waves = ncu * threads // 64
            n32 = 16 * iters if mode != 1 else 0  # b32 or b64 lookups (2 array cycles each)
            n128 = 16 * iters if mode == 1 else (16 * iters // 4 if mode in (2, 4) else 0)
            arr = (2 * n32 + 4 * n128) * waves / ncu  # LDS array cycles per CU (MI355X_MICROARCH.md LDS table)
            print(f"{name:32s} {threads // 64:2d} waves/CU: {ms:7.3f} ms; array cycles/CU {arr / 1e6:.2f} M -> "
                  f"{arr / (ms * 1e-3) / 1e9:.2f} G array-cycles/s per CU", flush=True)


if __name__ == "__main__":
    build() if sys.argv[1] == "build" else run()
