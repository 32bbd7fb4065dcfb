"""Drives scripts/lds_ceiling.hip: the measured LDS ceiling of the batch kernels' read mix (measurement only).

    python scripts/lds_ceiling.py build            (here: hipcc into scripts/_build/liblds_ceiling.so)
    python scripts/lds_ceiling.py run [out.json]   (GPU)

Each mode runs back to back for >= 2 s first (the clock settles: MI355X_MICROARCH.md, DVFS item 6), then 5 timed
launches; per launch the in-kernel clock (delta s_memtime / delta s_memrealtime x 100 MHz, median over workgroups) and
the LDS cycles one wave step of 64 blocks costs (delta s_memtime / (16 waves x blocks per lane)).  The ceiling of a mix
is its measured cycles per 64 blocks: at a clock f, a CU can take at most f / (cycles / 64) blocks per second from the
LDS, whatever else the kernel does.  `nominal` is the 2 / 4 clk per b32 / b128 read model (MI355X_MICROARCH.md LDS
table); `sustained_frac` = nominal / measured."""
import ctypes as C
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SO = os.path.join(ROOT, "scripts", "_build", "liblds_ceiling.so")
MODES = {0: ("aes128_gh8", 133, 16), 1: ("aes256_gh8", 197, 16), 2: ("b32_only", 133, 0), 3: ("b128_only", 0, 16)}


def build():
    os.makedirs(os.path.dirname(SO), exist_ok=True)
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
                    os.path.join(ROOT, "scripts", "lds_ceiling.hip"), "-o", SO], check=True)


def run(out_path=None):
    import numpy as np
    import torch
    lib = C.CDLL(SO)
    lib.lds_ceiling_run.argtypes = [C.c_int, C.c_uint32, C.c_uint32, C.c_void_p, C.c_void_p, C.c_void_p]
    dev = torch.device("cuda:0")
    ncu = torch.cuda.get_device_properties(dev).multi_processor_count
    out = torch.zeros(ncu * 1024, dtype=torch.int32, device=dev)
    st = torch.zeros(2 * ncu, dtype=torch.int64, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    blocks = 2048
    res = {"cus": ncu, "waves_per_cu": 16, "blocks_per_lane": blocks, "modes": {}}
    for mode, (name, b32, b128) in MODES.items():
        t0 = time.time()
        while time.time() - t0 < 2.0:  # settle the clock under this load
            assert lib.lds_ceiling_run(mode, blocks, ncu, out.data_ptr(), st.data_ptr(), s) == 0
            torch.cuda.synchronize()
        runs = []
        for _ in range(5):
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            ev[0].record()
            assert lib.lds_ceiling_run(mode, blocks, ncu, out.data_ptr(), st.data_ptr(), s) == 0
            ev[1].record()
            torch.cuda.synchronize()
            v = st.cpu().numpy().reshape(-1, 2).astype(np.float64)
            ghz = float(np.median(v[:, 0] / v[:, 1] * 0.1))
            cyc = float(np.median(v[:, 0])) / (16.0 * blocks)  # LDS-bound cycles per wave step (64 blocks) per CU
            runs.append({"ms": round(ev[0].elapsed_time(ev[1]), 3), "clock_ghz": round(ghz, 4),
                         "cycles_per_64_blocks": round(cyc, 2)})
        nominal = 2.0 * b32 + 4.0 * b128
        cyc = float(np.median([r["cycles_per_64_blocks"] for r in runs]))
        ghz = float(np.median([r["clock_ghz"] for r in runs]))
        res["modes"][name] = {"b32_per_block": b32, "b128_per_block": b128, "nominal_cycles_per_64_blocks": nominal,
                              "measured_cycles_per_64_blocks": round(cyc, 2),
                              "sustained_frac": round(nominal / cyc, 4) if nominal else None,
                              "clock_ghz": round(ghz, 4),
                              "payload_gbps_at_probe_clock": round(ncu * ghz * 1e9 / (cyc / 64.0) * 16 / 1e9, 1),
                              "runs": runs}
        print(name, json.dumps(res["modes"][name]), flush=True)
    if out_path:
        with open(out_path, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    if sys.argv[1] == "build":
        build()
    else:
        run(sys.argv[2] if len(sys.argv) > 2 else None)
