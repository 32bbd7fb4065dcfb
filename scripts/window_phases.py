"""Where a window launch's time goes: phase timestamps inside the window kernels (measurement build).

    python scripts/window_phases.py build        # CPU: engine variant with -DGCM_WIN_TIMING=1
    python scripts/window_phases.py run          # GPU: one 16 x 16 KiB send window, repeated
    python scripts/window_phases.py run NREC FRAG [NREC FRAG ...]   # other windows, one JSON line each

The variant library stamps s_memrealtime (100 MHz) in workgroup 0 at kernel entry, after the LDS fill,
after the first pass's walk (wave 0), after the pass barrier (all waves), after the join and at the
end of the pass.  The launch's total comes from HIP events on the stream; the part before the first
stamp and after the last one is launch and completion overhead.
"""
import ctypes as C
import json
import os
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
SO = os.environ.get("WINTIMING_SO") or os.path.join(ROOT, "rapido_amd", "_lib", "variants", "wintiming.so")


def build(extra=()):
    """extra: -D flags of a variant (WINTIMING_SO names its library)"""
    from rapido_amd import build as b
    os.makedirs(os.path.dirname(SO), exist_ok=True)
    obj = SO[:-3] + ".o"
    b.build_engine()
    subprocess.run([b.HIPCC, f"--offload-arch={b.ARCH}", "-O3", "-std=c++17", "-fPIC", "-DGCM_WIN_TIMING=1", *extra, "-c",
                    os.path.join(b.CSRC, "gcm_engine.hip"), "-o", obj], check=True)
    subprocess.run([b.HIPCC, f"--offload-arch={b.ARCH}", "-shared", "-fPIC", "-o", SO, obj] + b.C_OBJS, check=True)
    print("built", SO)


def run(reps=50, nrec=16, frag=16384, family="win16"):
    import numpy as np
    import torch

    import rapido_amd as ra
    L = C.CDLL(SO, mode=C.RTLD_LOCAL)
    vp, sz = C.c_void_p, C.c_size_t
    L.ptls_mi355x_aesgcm_new.argtypes = [vp, sz, sz]
    L.ptls_mi355x_aesgcm_new.restype = vp
    L.ptls_mi355x_tls_seal_records.argtypes = [vp, vp, vp, sz, vp, vp, vp]
    L.ptls_mi355x_debug_window_times.argtypes = [vp]
    key = C.create_string_buffer(bytes(range(16)), 16)
    iv = C.create_string_buffer(bytes(range(12)), 12)
    ctx = L.ptls_mi355x_aesgcm_new(key, 16, 0)
    auto = C.c_size_t(-1).value
    for name, on in (("ptls_mi355x_set_win16_records", family == "win16"), ("ptls_mi355x_set_split_records", family == "split")):
        if hasattr(L, name):
            getattr(L, name).argtypes = [sz]
            getattr(L, name).restype = sz
            getattr(L, name)(auto if on else 0)
    t = np.zeros(nrec, ra.TLS_RECORD_DTYPE)
    t["src"] = np.arange(nrec, dtype=np.uint64) * frag
    t["dst"] = np.arange(nrec, dtype=np.uint64) * (frag + 22)
    t["seq"] = np.arange(nrec, dtype=np.uint64)
    t["len"] = frag
    t["type"] = 23
    dev = torch.device("cuda:0")
    d_t = torch.from_numpy(t.view(np.uint8)).to(dev)
    d_src = torch.randint(0, 256, (nrec * frag,), dtype=torch.uint8, device=dev)
    d_dst = torch.zeros(nrec * (frag + 22), dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream(dev)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    stamps = (C.c_uint64 * 16)()
    phases = {k: [] for k in ("fill", "walk", "barrier", "join", "epilogue", "in_kernel", "launch_total",
                              "walk_consts", "walk_step0", "walk_step1", "walk_step2", "walk_scale")}
    for i in range(reps + 5):
        ev[0].record(stream)
        assert L.ptls_mi355x_tls_seal_records(ctx, iv, d_t.data_ptr(), nrec, d_src.data_ptr(), d_dst.data_ptr(),
                                              stream.cuda_stream) == 0
        ev[1].record(stream)
        torch.cuda.synchronize()
        assert L.ptls_mi355x_debug_window_times(stamps) == 0
        if i < 5:
            continue
        s = [stamps[k] * 0.01 for k in range(6)]  # us
        phases["fill"].append(s[1] - s[0])
        phases["walk"].append(s[2] - s[1])
        phases["barrier"].append(s[3] - s[2])
        phases["join"].append(s[4] - s[3])
        phases["epilogue"].append(s[5] - s[4])
        phases["in_kernel"].append(s[5] - s[0])
        phases["launch_total"].append(ev[0].elapsed_time(ev[1]) * 1e3)
        # inside lane_walk (prefetching kernels only): stamps 8 (constants done) .. 13 (scaled)
        w = [stamps[k] * 0.01 for k in range(16)]
        if w[9] > w[1] > 0:
            phases["walk_consts"].append(w[8] - s[1])
            phases["walk_step0"].append(w[10] - w[9])
            phases["walk_step1"].append(w[11] - w[10])
            phases["walk_step2"].append(w[12] - w[11])
            phases["walk_scale"].append(w[13] - w[12])
    out = {k: round(statistics.median(v), 2) for k, v in phases.items() if v}
    out["window"] = f"{nrec} x {frag} B, AES-128 seal, window kernels (median of {reps} launches, us)"
    out["lib"] = os.path.basename(SO)
    out["kernels"] = {"split": "split (runs of 16 segments per workgroup; stamps of run 0 only)",
                      "win16": "16-lane (win16)", "win32": "8-lane 32-position (win32)"}[family]
    print(json.dumps(out))
    return out


if __name__ == "__main__":
    if sys.argv[1] == "build":
        build(sys.argv[2:])
    elif len(sys.argv) > 2:
        a = [int(x) for x in sys.argv[2:]]
        for nrec, frag in zip(a[0::2], a[1::2]):
            for fam in os.environ.get("WINTIMING_FAMILIES", "split,win16,win32").split(","):
                run(nrec=nrec, frag=frag, family=fam)
    else:
        run()
