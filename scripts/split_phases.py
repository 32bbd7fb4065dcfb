"""Where a split-window launch's time goes (measurement build of the split kernels).

    python scripts/split_phases.py build [BLOCK]   # CPU: engine variant, -DGCM_WIN_TIMING=1 -DGCM_STAMP_BLOCK=BLOCK
    python scripts/split_phases.py run [open]      # GPU: one 16 x 16 KiB send window (or its open), repeated

Workgroup BLOCK (3 r + k = run k of record r; default 2, the last run of record 0: 16 segments) stamps s_memrealtime
(100 MHz, one clock for the whole chip) at entry (0), after its LDS fill (1), in its walk (8: constants done; 9-11:
the two steps; 12: loop end; 13: lane scaling done), after the walk (2), after the segment sums (3), after the
local join (4) and at the arrival ticket (5); the run that finishes record 0 stamps its acquire (6) and its end (7).
Prints the median time of every stamp after stamp 0, in microseconds, and the launch total from HIP events.
"""
import ctypes as C
import json
import os
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
SO = os.path.join(ROOT, "rapido_amd", "_lib", "variants", "splittiming.so")


def build(block=2):
    from rapido_amd import build as b
    os.makedirs(os.path.dirname(SO), exist_ok=True)
    obj = SO[:-3] + ".o"
    b.build_engine()
    subprocess.run([b.HIPCC, f"--offload-arch={b.ARCH}", "-O3", "-std=c++17", "-fPIC", "-DGCM_WIN_TIMING=1",
                    f"-DGCM_STAMP_BLOCK={block}", "-c", os.path.join(b.CSRC, "gcm_engine.hip"), "-o", obj], check=True)
    subprocess.run([b.HIPCC, f"--offload-arch={b.ARCH}", "-shared", "-fPIC", "-o", SO, obj] + b.C_OBJS, check=True)
    print("built", SO)


def run(reps=50, nrec=16, frag=16384, is_open=False):
    import numpy as np
    import torch

    import rapido_amd as ra
    L = C.CDLL(SO, mode=C.RTLD_LOCAL)
    vp, sz = C.c_void_p, C.c_size_t
    L.ptls_mi355x_aesgcm_new.argtypes = [vp, sz, sz]
    L.ptls_mi355x_aesgcm_new.restype = vp
    L.ptls_mi355x_tls_seal_records.argtypes = [vp, vp, vp, sz, vp, vp, vp]
    L.ptls_mi355x_tls_open_records.argtypes = [vp, vp, vp, sz, vp, vp, vp, vp, vp]
    L.ptls_mi355x_debug_window_times.argtypes = [vp]
    key = C.create_string_buffer(bytes(range(16)), 16)
    iv = C.create_string_buffer(bytes(range(12)), 12)
    ctx = L.ptls_mi355x_aesgcm_new(key, 16, 0)
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
    if is_open:  # the window's wire records, sealed once, then opened repeatedly (plaintext slots of frag + 1 bytes)
        assert L.ptls_mi355x_tls_seal_records(ctx, iv, d_t.data_ptr(), nrec, d_src.data_ptr(), d_dst.data_ptr(),
                                              stream.cuda_stream) == 0
        o = np.zeros(nrec, ra.TLS_RECORD_DTYPE)
        o["src"] = t["dst"]
        o["dst"] = np.arange(nrec, dtype=np.uint64) * (frag + 1)
        o["seq"] = t["seq"]
        o["len"] = frag + 17
        d_o = torch.from_numpy(o.view(np.uint8)).to(dev)
        d_pt = torch.zeros(nrec * (frag + 1), dtype=torch.uint8, device=dev)
        d_st = torch.zeros(nrec, dtype=torch.int32, device=dev)
        d_ty = torch.zeros(nrec, dtype=torch.uint8, device=dev)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    stamps = (C.c_uint64 * 16)()
    rows = {i: [] for i in (1, 8, 9, 10, 11, 12, 13, 2, 3, 4, 5, 6, 7)}
    total = []
    for i in range(reps + 5):
        for k in range(16):
            stamps[k] = 0
        ev[0].record(stream)
        if is_open:
            assert L.ptls_mi355x_tls_open_records(ctx, iv, d_o.data_ptr(), nrec, d_dst.data_ptr(), d_pt.data_ptr(),
                                                  d_st.data_ptr(), d_ty.data_ptr(), stream.cuda_stream) == 0
        else:
            assert L.ptls_mi355x_tls_seal_records(ctx, iv, d_t.data_ptr(), nrec, d_src.data_ptr(), d_dst.data_ptr(),
                                                  stream.cuda_stream) == 0
        ev[1].record(stream)
        torch.cuda.synchronize()
        assert L.ptls_mi355x_debug_window_times(stamps) == 0
        if i < 5:
            continue
        for k in rows:
            rows[k].append((stamps[k] - stamps[0]) * 0.01)
        total.append(ev[0].elapsed_time(ev[1]) * 1e3)
    names = {1: "fill", 8: "consts", 9: "step0_start", 10: "step0_end", 11: "step1_end", 12: "loop_end", 13: "scaled",
             2: "walk_done", 3: "sums", 4: "local_join", 5: "ticket", 6: "last_acquire", 7: "finish_end"}
    if is_open:
        assert (d_st.cpu().numpy() == frag).all()
    print(json.dumps({"window": f"{nrec} x {frag} B, AES-128 {'open' if is_open else 'seal'}, split kernels, us after the stamped run's entry "
                                f"(median of {reps})",
                      **{names[k]: round(statistics.median(v), 2) for k, v in rows.items()},
                      "launch_total": round(statistics.median(total), 2)}))


if __name__ == "__main__":
    if sys.argv[1] == "build":
        build(int(sys.argv[2]) if len(sys.argv) > 2 else 2)
    else:
        run(is_open=len(sys.argv) > 2 and sys.argv[2] == "open")
