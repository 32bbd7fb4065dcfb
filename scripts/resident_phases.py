"""Where a resident job's time goes (measurement build of the resident grid).

    python scripts/resident_phases.py build [BLOCK]   # CPU: engine variant, -DGCM_WIN_TIMING=1 -DGCM_STAMP_BLOCK=BLOCK
    python scripts/resident_phases.py run [reps]      # GPU: one 16 x 16 KiB send window per job, device / pinned host

The grid runs with 80 workers, so a 16-record window's 80 run units land on the same workers every job and worker
BLOCK (default 3) always takes unit BLOCK - 1 (run k = (BLOCK - 1) % 5 of record (BLOCK - 1) // 5).  s_memrealtime
stamps (100 MHz, one clock for the chip): the dispatcher's publication (22); worker BLOCK's job read (16), its
system-scope acquire done (17), units start (18), the unit's own phases (split_body: 0 entry, 1 LDS fill, 2 walk, 3
sums, 4 local join, 5 ticket), units end (19), its system-scope release done (20), its done count added (21).  Prints
the median of each stamp after the publication, in microseconds, and the host-observed job time.
"""
import ctypes as C
import json
import os
import statistics
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
SO = os.path.join(ROOT, "scripts", "_build", "restiming.so")  # (travels to the GPU box; _lib/variants does not)


def build(block=3):
    from rapido_amd import build as b
    os.makedirs(os.path.dirname(SO), exist_ok=True)
    obj = SO[:-3] + ".o"
    b.build_engine()
    subprocess.run([b.HIPCC, f"--offload-arch={b.ARCH}", "-O3", "-std=c++17", "-fPIC", "-DGCM_WIN_TIMING=1",
                    f"-DGCM_STAMP_BLOCK={block}", "-c", os.path.join(b.CSRC, "gcm_engine.hip"), "-o", obj], check=True)
    subprocess.run([b.HIPCC, f"--offload-arch={b.ARCH}", "-shared", "-fPIC", "-o", SO, obj] + b.C_OBJS, check=True)
    print("built", SO)


def run(reps=200, nrec=16, frag=16384):
    import numpy as np
    import torch

    import rapido_amd as ra
    L = C.CDLL(SO, mode=C.RTLD_LOCAL)
    vp, sz, u64 = C.c_void_p, C.c_size_t, C.c_uint64
    L.ptls_mi355x_aesgcm_new.argtypes = [vp, sz, sz]
    L.ptls_mi355x_aesgcm_new.restype = vp
    L.ptls_mi355x_resident_tls_seal_records_multi.argtypes = [vp, vp, vp, vp, sz, vp, vp, C.POINTER(u64)]
    L.ptls_mi355x_resident_wait.argtypes = [vp, u64]
    L.ptls_mi355x_set_resident_workers.argtypes = [sz]
    L.ptls_mi355x_resident_stop.argtypes = [C.c_int]
    L.ptls_mi355x_debug_window_times.argtypes = [vp]
    L.ptls_mi355x_set_resident_workers(80)
    key = C.create_string_buffer(bytes(range(16)), 16)
    iv = C.create_string_buffer(bytes(range(12)), 12)
    ctx = L.ptls_mi355x_aesgcm_new(key, 16, 0)
    hip = C.CDLL("libamdhip64.so")

    def devptr(t):
        if not t.is_pinned():
            return t.data_ptr()
        p = C.c_void_p()
        assert hip.hipHostGetDevicePointer(C.byref(p), C.c_void_p(t.data_ptr()), 0) == 0
        return p.value

    t = np.zeros(nrec, ra.TLS_RECORD_DTYPE)
    t["src"] = np.arange(nrec, dtype=np.uint64) * frag
    t["dst"] = np.arange(nrec, dtype=np.uint64) * (frag + 22)
    t["seq"] = np.arange(nrec, dtype=np.uint64)
    t["len"] = frag
    t["type"] = 23
    names = {16: "job_read", 17: "acquired", 18: "units_start", 0: "unit_entry", 1: "unit_fill", 2: "unit_walk",
             3: "unit_sums", 4: "unit_join", 5: "unit_ticket", 19: "units_end", 20: "released", 21: "counted"}
    out = {"window": f"{nrec} x {frag} B, AES-128 seal, resident grid (80 workers), us after the dispatcher's "
                     f"publication (median of {reps})"}
    for where in ("device", "host"):
        src = torch.randint(0, 256, (nrec * frag,), dtype=torch.uint8)
        dst = torch.zeros(nrec * (frag + 22), dtype=torch.uint8)
        recs = torch.from_numpy(t.view(np.uint8).copy())
        if where == "device":
            src, dst, recs = src.cuda(), dst.cuda(), recs.cuda()
        else:
            src, dst, recs = src.pin_memory(), dst.pin_memory(), recs.pin_memory()
        torch.cuda.synchronize()
        stamps = (u64 * 32)()
        rows = {k: [] for k in names}
        host = []
        job = u64(0)
        for i in range(reps + 10):
            for k in range(32):
                stamps[k] = 0
            t0 = time.perf_counter()
            assert L.ptls_mi355x_resident_tls_seal_records_multi(ctx, iv, devptr(recs), None, nrec, devptr(src),
                                                                 devptr(dst), C.byref(job)) == 0
            assert L.ptls_mi355x_resident_wait(ctx, job.value) == 0
            host.append((time.perf_counter() - t0) * 1e6)
            # the stamps land before the job's completion word; read them once the grid has published them
            assert L.ptls_mi355x_debug_window_times(stamps) == 0
            if i < 10 or stamps[22] == 0 or stamps[21] == 0:
                continue
            for k in rows:
                rows[k].append((stamps[k] - stamps[22]) * 0.01)
        out[where] = {names[k]: round(statistics.median(v), 2) for k, v in rows.items() if v}
        out[where]["host_job_us"] = round(statistics.median(host[10:]), 2)
        print(json.dumps({where: out[where]}), flush=True)
    L.ptls_mi355x_resident_stop(0)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    if sys.argv[1] == "build":
        build(int(sys.argv[2]) if len(sys.argv) > 2 else 3)
    else:
        run(int(sys.argv[2]) if len(sys.argv) > 2 else 200)
