"""Kernel ablations / variants, timed in ONE process with interleaved rounds.

    python scripts/ablate.py build            # CPU: builds the variant libraries (hipcc)
    python scripts/ablate.py run [--workload 1400|16k-aes128] [--rounds 5]   # GPU

Each variant is the engine library compiled with extra -D flags (see VARIANTS).  Ablated
variants (no AES / no GHASH) produce wrong output; only their kernel times are used, to
locate the bottleneck (cdna_hip_programming.md sec. 7, "The diagnostic loop").
"""
import ctypes as C
import json
import os
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
# variant libraries: travel to the GPU box while they exist (delete the directory after an A/B: the round-end push
# should carry only the product library); the "head" source snapshot stays under rapido_amd/_lib/variants
VDIR = os.environ.get("ABLATE_VDIR") or os.path.join(ROOT, "scripts", "_abl")
HEAD_SRC = os.path.join(ROOT, "rapido_amd", "_lib", "variants", "src_head")

VARIANTS = {
    "base": [],
    "wg512": ["-DMI355X_WG_THREADS=512"],
    "wg768": ["-DMI355X_WG_THREADS=768"],
    "ilp": ["-mllvm", "--amdgpu-sched-strategy=iterative-ilp"],
    "noasm": ["-DGCM_ROUND_ASM=0"],
    "r1only": ["-DGCM_R2CACHE=0"],
    "noalign": ["-DGCM_ALIGN_OUTPUT=0"],
    "freealign": ["-DGCM_ALIGN_MIN_T=100000u"],
    "align8": ["-DGCM_ALIGN_MIN_T=8u"],
    "lanemajor": ["-DGCM_LANE_MAJOR=1"],
    "nohoist": ["-DGCM_HOIST_AAD=0"],
    "r01d": ["-DGCM_HOIST_AAD=0", "-DGCM_LANE_MAJOR=0"],  # the record walk before hoisting / j-major lanes
    "hoistonly": ["-DGCM_LANE_MAJOR=0"],
    "gh5": ["-DGCM_GH5=1", "-DGCM_GH8=0"],
    # r03: the nibble-table H^4 Horner (four T-table images) against the 8-bit latin tables (two T-table images)
    "nogh8": ["-DGCM_GH8=0"],
    "gh8": ["-DGCM_GH8=1"],
    "gh8pair": ["-DGCM_GH8=1", "-DGCM_PAIR_STORES=1"],
    "gh8nt": ["-DGCM_GH8=1", "-DGCM_NT_LOADS=1"],
    "pf3nt": ["-DGCM_NT_LOADS=1"],  # the default build (GH8, three-step prefetch) with non-temporal input loads
    "gh8pf3": ["-DGCM_GH8=1", "-DGCM_BATCH_PF=3"],  # batch loads three steps ahead (four buffers; the default)
    "gh8pf1": ["-DGCM_GH8=1", "-DGCM_BATCH_PF=1"],  # batch loads one step ahead (two buffers; before r03s)
    "nofast": ["-DGCM_FAST_STEP=0"],
    "scale0": ["-DGCM_SCALE_W=0"],  # closing multiply with compiler-paired reads (16 round trips; before r03)
    "scale2": ["-DGCM_SCALE_W=2"],  # closing multiply with all 32 reads in flight
    "vtmax": ["-DGCM_UNIFORM_TMAX=0"],  # the walk's trip count in a VGPR (exec-masked trip tests; before r03)
    "ntstore": ["-DGCM_NT_STORES=1"],  # the walk's output stores non-temporal (the default since r03zg)
    "tstore": ["-DGCM_NT_STORES=0"],  # the walk's output stores as plain (temporal) stores (before r03zg)
    "quarters": ["-DGCM_PASS_LANES=0"],  # K = 4: lane j = the wave quarter (two j per ds_read_b128 pass; before r03)
    "prio": ["-DGCM_ROUND_PRIO=1"],  # s_setprio 2 while a GH8 middle round issues its LDS reads (the default since r03zm)
    "noprio": ["-DGCM_ROUND_PRIO=0"],  # no wave-priority changes (before r03zm)
    "prio3": ["-DGCM_PRIO_LEVEL=3"],  # s_setprio 3 instead of 2
    "prio1": ["-DGCM_PRIO_LEVEL=1"],  # s_setprio 1 instead of 2
    "priolast": ["-DGCM_PRIO_LAST=1"],  # raised through the last round's S-box reads too
    "priogh8": ["-DGCM_PRIO_GH8=1"],  # raised already before the round's two GH8 reads
    "static": ["-DGCM_STATIC_GROUPS=1"],  # groups assigned round-robin to waves (no atomic; uniform batches only)
    "noscale": ["-DGCM_ABLATE_SCALE=1"],  # no closing H^(K-j) multiply (wrong tags: timing only)  # r03: every step through the per-lane flags (no interior fast path)
    "gh8sel": ["-DGCM_GH8=1", "-DGCM_GH8_LANESEL=1"],  # GH8 byte permutation folded into per-lane address selectors  # 5-bit ds_read_b64 GHASH tables for K = 4 (evaluated: 33% slower, bank conflicts)
    # "@src=DIR": compile gcm_engine.hip from DIR (e.g. a `git show` of an older revision) instead of csrc/
    "head": ["@src=" + HEAD_SRC],
    # r04: waves start their walks in four phases (wave w >> 2), GCM_STAGGER x s_sleep 127 apart
    "stagger2": ["-DGCM_STAGGER=2"],
    "stagger5": ["-DGCM_STAGGER=5"],
    "stagger10": ["-DGCM_STAGGER=10"],
    "no_ghash": ["-DGCM_ABLATE_GHASH=1"],
    "no_aes": ["-DGCM_ABLATE_AES=1"],
    "no_both": ["-DGCM_ABLATE_AES=1", "-DGCM_ABLATE_GHASH=1"],
    "fill16": ["-DGCM_WIN_FILL=16u"],
    "w32t1024": ["-DMI355X_WIN32_THREADS=1024"],
    # K = 4 walks storing whole 128-byte lines (lane_walk PAIRST, r02) vs one 64-byte piece per step
    "pair": ["-DGCM_PAIR_STORES=1"],
    "ntload": ["-DGCM_NT_LOADS=1"],
    "noglds": ["-DGCM_SPLIT_GLDS=0"],
    "nox2": ["-DGCM_SPLIT_X2=0"],  # split kernels: a segment's two steps one after the other (one AES chain each)  # split window kernels: register-staged LDS fill instead of LDS DMA  # non-temporal input loads (keep the half-written output lines in L2)
    # r02 experiments on the last AES round (last-round S-box lookups through the vector-memory path; two steps'
    # last rounds bitsliced on the VALU; T1 moved to image B): scripts/experiments/r02_last_round_vmem_pair_t1b.patch
    # holds the source, profiles/r02[c-e]_ablate_*.txt the measurements -- all slower, not in csrc/
}
if os.environ.get("ABLATE_VARIANTS"):
    VARIANTS = {k: v for k, v in VARIANTS.items() if k in os.environ["ABLATE_VARIANTS"].split(",")}


def build():
    from rapido_amd import build as b
    os.makedirs(VDIR, exist_ok=True)
    b.build_engine()
    for name, flags in VARIANTS.items():
        obj = os.path.join(VDIR, name + ".o")
        so = os.path.join(VDIR, name + ".so")
        srcdir = next((f[5:] for f in flags if f.startswith("@src=")), b.CSRC)
        if srcdir != b.CSRC and not os.path.isdir(srcdir):
            os.makedirs(srcdir)
            for f in ("gcm_engine.hip", "gcm_core.h"):
                with open(os.path.join(srcdir, f), "wb") as fh:
                    rev = os.environ.get("ABLATE_REV", "HEAD")  # e.g. an older commit to A/B against
                    fh.write(subprocess.run(["git", "-C", ROOT, "show", rev + ":rapido_amd/csrc/" + f],
                                            check=True, capture_output=True).stdout)
        flags = [f for f in flags if not f.startswith("@src=")]
        src = os.path.join(srcdir, "gcm_engine.hip")
        subprocess.run([b.HIPCC, f"--offload-arch={b.ARCH}", "-O3", "-std=c++17", "-fPIC", "-I" + b.CSRC, *flags, "-c",
                        src, "-o", obj], check=True)
        subprocess.run([b.HIPCC, f"--offload-arch={b.ARCH}", "-shared", "-fPIC", "-o", so, obj] + b.C_OBJS +
                       ["-L/opt/rocm/lib", "-lhsa-runtime64"], check=True)
        print("built", so)


def run(workload="1400", rounds=5, lanes=4):
    import numpy as np
    import torch
    from rapido_amd import records

    n, length, keylen = {"1400": (1 << 20, 1400, 16), "16k-aes128": (1 << 18, 16384, 16),
                         "16k": (1 << 18, 16384, 32)}[workload]
    lengths = np.full(n, length, dtype=np.uint64)
    recs, src_bytes, aad_bytes = records.layout(lengths, np.full(n, 5, dtype=np.uint64), align=256)
    aad = np.zeros(aad_bytes, dtype=np.uint8)
    aad[: 5 * n] = records.tls_aad(lengths)
    dev = torch.device("cuda:0")
    d_src = torch.randint(0, 256, (src_bytes,), dtype=torch.uint8, device=dev)
    d_ct, d_pt = torch.zeros_like(d_src), torch.zeros_like(d_src)
    d_recs = torch.from_numpy(recs.view(np.uint8)).to(dev)
    d_aad = torch.from_numpy(aad).to(dev)
    d_st = torch.zeros(n, dtype=torch.int32, device=dev)
    iv = C.create_string_buffer(bytes(range(12)), 12)
    key = C.create_string_buffer(bytes(range(keylen)), keylen)
    vp, sz = C.c_void_p, C.c_size_t
    libs = {}
    for name in VARIANTS:
        L = C.CDLL(os.path.join(VDIR, name + ".so"), mode=C.RTLD_LOCAL)
        L.ptls_mi355x_aesgcm_new.argtypes = [vp, sz, sz]
        L.ptls_mi355x_aesgcm_new.restype = vp
        L.ptls_mi355x_seal_batch.argtypes = [vp, vp, vp, sz, vp, vp, vp, vp]
        L.ptls_mi355x_open_batch.argtypes = [vp, vp, vp, sz, vp, vp, vp, vp, vp]
        L.ptls_mi355x_set_lanes_per_record(lanes)
        libs[name] = (L, L.ptls_mi355x_aesgcm_new(key, keylen, 0))
    stream = torch.cuda.current_stream().cuda_stream
    res = {name: {"seal": [], "open": []} for name in VARIANTS}
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    for r in range(rounds + 1):
        for name, (L, ctx) in libs.items():
            ev[0].record()
            L.ptls_mi355x_seal_batch(ctx, iv, d_recs.data_ptr(), n, d_src.data_ptr(), d_ct.data_ptr(), d_aad.data_ptr(),
                                     stream)
            ev[1].record()
            L.ptls_mi355x_open_batch(ctx, iv, d_recs.data_ptr(), n, d_ct.data_ptr(), d_pt.data_ptr(), d_aad.data_ptr(),
                                     d_st.data_ptr(), stream)
            ev[2].record()
            torch.cuda.synchronize()
            if r:  # round 0 is warmup
                res[name]["seal"].append(ev[0].elapsed_time(ev[1]))
                res[name]["open"].append(ev[1].elapsed_time(ev[2]))
    # outputs vs the first variant (ablated variants differ by design)
    ref = None
    same = {}
    for name, (L, ctx) in libs.items():
        d_ct.zero_()
        L.ptls_mi355x_seal_batch(ctx, iv, d_recs.data_ptr(), n, d_src.data_ptr(), d_ct.data_ptr(), d_aad.data_ptr(), stream)
        torch.cuda.synchronize()
        if ref is None:
            ref = d_ct.clone()
        same[name] = bool(torch.equal(d_ct, ref))
    out = {}
    for name, d in res.items():
        s, o = statistics.median(d["seal"]), statistics.median(d["open"])
        gib = n * length / 2 ** 30
        out[name] = {"seal_ms": round(s, 4), "open_ms": round(o, 4), "seal_gibps": round(gib / (s / 1e3), 1),
                     "open_gibps": round(gib / (o / 1e3), 1), "same_output": same[name]}
        print(f"{workload:10s} K={lanes} {name:12s} seal {s:7.3f} ms {gib / (s / 1e3):8.1f} GiB/s   open {o:7.3f} ms "
              f"{gib / (o / 1e3):8.1f} GiB/s  same={same[name]}", flush=True)
    return out


if __name__ == "__main__":
    if sys.argv[1] == "build":
        build()
    else:
        import argparse
        ap = argparse.ArgumentParser()
        ap.add_argument("cmd")
        ap.add_argument("--workload", default="1400")
        ap.add_argument("--rounds", type=int, default=5)
        ap.add_argument("--lanes", type=int, default=4)
        a = ap.parse_args()
        print(json.dumps(run(a.workload, a.rounds, a.lanes)))
