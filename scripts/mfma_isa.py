"""Drives scripts/mfma_isa.hip (a measurement probe, not the product).

    python scripts/mfma_isa.py build     # CPU: hipcc -> scripts/_build/libmfma_isa.so
    python scripts/mfma_isa.py run       # GPU: FP4 MFMA fragment layout check, then issue-rate / VALU-hold sweep

Layout: random e2m1 fragments and E8M0 scales through one v_mfma_scale_f32_{32x32x64,16x16x128}_f8f6f4; the host
evaluates candidate lane -> (row, k) maps and reports the one that reproduces C exactly.
Rate: cycles per MFMA (s_memtime) with NV independent v_bitop3 fillers after each MFMA, one wave per SIMD.
"""
import ctypes as C
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SO = os.path.join(ROOT, "scripts", "_build", "libmfma_isa.so")
FP4 = np.array([0, .5, 1, 1.5, 2, 3, 4, 6, -0., -.5, -1, -1.5, -2, -3, -4, -6])


def build():
    os.makedirs(os.path.dirname(SO), exist_ok=True)
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
                    os.path.join(ROOT, "scripts", "mfma_isa.hip"), "-o", SO], check=True)
    print("built", SO)


def nibbles(frag):
    """frag: (64, 4) uint32 -> (64, 32) element codes, element j = nibble j%8 of dword j//8"""
    j = np.arange(32)
    return (frag[:, j // 8] >> (4 * (j % 8)).astype(np.uint32)) & 0xF


def expand(frag, scale, M, K, kmap):
    """fragment (64 lanes x 32 elements) -> (M, K) matrix under kmap(lane, j) -> (row, k)"""
    mat = np.full((M, K), np.nan)
    el = FP4[nibbles(frag)] * (2.0 ** (scale.astype(np.int64) - 127))[:, None]
    for lane in range(64):
        for j in range(32):
            r, k = kmap(lane, j)
            mat[r, k] = el[lane, j]
    return mat


def cmaps(shape):
    if shape == 32:
        return {"32g+j": lambda l, j: (l % 32, 32 * (l // 32) + j),
                "g+2j": lambda l, j: (l % 32, (l // 32) + 2 * j),
                "32g+rev": lambda l, j: (l % 32, 32 * (l // 32) + 8 * (j // 8) + 7 - j % 8),
                "16-halves": lambda l, j: (l % 32, 32 * (j // 16) + 16 * (l // 32) + j % 16)}
    return {"32g+j": lambda l, j: (l % 16, 32 * (l // 16) + j),
            "g+4j": lambda l, j: (l % 16, (l // 16) + 4 * j),
            "32g+rev": lambda l, j: (l % 16, 32 * (l // 16) + 8 * (j // 8) + 7 - j % 8)}


def c_layout(c, shape):
    out = np.zeros((shape, shape))
    for lane in range(64):
        for reg in range(16 if shape == 32 else 4):
            if shape == 32:
                row, col = (reg & 3) + 8 * (reg >> 2) + 4 * (lane >> 5), lane & 31
            else:
                row, col = 4 * (lane >> 4) + reg, lane & 15
            out[row, col] = c[lane, reg]
    return out


def run():
    import torch  # first: the process then uses torch's HIP runtime for this library too
    lib = C.CDLL(SO)
    vp = C.c_void_p
    lib.run_layout.argtypes = [vp] * 7
    lib.run_rate.argtypes = [C.c_int, C.c_int, vp, vp, C.c_int, C.c_int]
    lib.err_str.restype = C.c_char_p
    dev = torch.device("cuda:0")
    rng = np.random.default_rng(5)
    report = {"layout": {}, "rate": {}}
    for trial in range(4 if os.environ.get("ISA_LAYOUT", "1") == "1" else 0):
        # codes 0..3 and 8..11 only (0, +-.5, +-1, +-1.5): exact small products
        a = rng.integers(0, 2**32, size=(64, 4), dtype=np.uint64).astype(np.uint32) & np.uint32(0xBBBBBBBB)
        b = rng.integers(0, 2**32, size=(64, 4), dtype=np.uint64).astype(np.uint32) & np.uint32(0xBBBBBBBB)
        sa = (127 + rng.integers(-2, 3, size=64)).astype(np.uint32) if trial >= 2 else np.full(64, 127, np.uint32)
        sb = (127 + rng.integers(-2, 3, size=64)).astype(np.uint32) if trial >= 3 else np.full(64, 127, np.uint32)
        t = [torch.from_numpy(x.view(np.int32)).to(dev) for x in (a.ravel(), b.ravel(), sa, sb)]
        c32 = torch.zeros(64 * 16, dtype=torch.float32, device=dev)
        c16 = torch.zeros(64 * 4, dtype=torch.float32, device=dev)
        c32u = torch.zeros(64 * 16, dtype=torch.float32, device=dev)
        rc = lib.run_layout(*(x.data_ptr() for x in t), c32.data_ptr(), c16.data_ptr(), c32u.data_ptr())
        assert rc == 0, lib.err_str(rc).decode()
        for shape, cc in ((32, c32), (16, c16)):
            got = c_layout(cc.cpu().numpy().reshape(64, -1), shape)
            K = 64 if shape == 32 else 128
            ok = []
            for name, km in cmaps(shape).items():
                try:
                    A = expand(a, sa, shape, K, km)
                    Bt = expand(b, sb, shape, K, km)  # B[k][col]: same lane map with col for row
                except IndexError:
                    continue
                if np.isnan(A).any() or np.isnan(Bt).any():
                    continue
                want = A @ Bt.T
                if np.array_equal(want, got):
                    ok.append(name)
            report["layout"].setdefault(f"{shape}x{shape}", []).append(ok)
            print(f"trial {trial} {shape}x{shape}: matching maps {ok}", flush=True)
        # the unscaled instruction (immediate zero scales): the plain product, no E8M0 factor
        km = cmaps(32)["32g+j"]
        gu = c_layout(c32u.cpu().numpy().reshape(64, -1), 32)
        one = np.full(64, 127, np.uint32)
        unscaled_ok = bool(np.array_equal(expand(a, one, 32, 64, km) @ expand(b, one, 32, 64, km).T, gu))
        report["layout"].setdefault("32x32_unscaled_is_plain_product", []).append(unscaled_ok)
        print(f"trial {trial} unscaled v_mfma_f32_32x32x64_f8f6f4 = plain product: {unscaled_ok}", flush=True)
        np.savez(os.path.join(ROOT, "gpurun_out", f"mfma_layout_{trial}.npz"), a=a, b=b, sa=sa, sb=sb,
                 c32=c32.cpu().numpy(), c16=c16.cpu().numpy())
    ncu = torch.cuda.get_device_properties(dev).multi_processor_count
    inp = torch.from_numpy(rng.integers(0, 2**31, size=4096).astype(np.int32) & 0x33333333).to(dev)
    iters = 2000
    for blocks in (1, ncu):
        out = torch.zeros(blocks * 4, dtype=torch.int64, device=dev)
        for m16, nvs in ((0, (0, 2, 4, 6, 8, 12, 16)), (1, (0, 2, 4, 6, 8)), (0, (-1,))):
            for nv in nvs:
                for n in (10, iters):
                    rc = lib.run_rate(nv, m16, inp.data_ptr(), out.data_ptr(), n, blocks)
                    assert rc == 0, lib.err_str(rc).decode()
                cyc = float(np.median(out.cpu().numpy()))
                per = cyc / (iters * (4 if nv >= 0 else 32))
                key = f"{'valu_only' if nv < 0 else ('16x16x128' if m16 else '32x32x64')}_nv{nv}_blocks{blocks}"
                report["rate"][key] = round(per, 2)
                print(f"{key}: {per:.2f} cycles per {'MFMA (+ fillers)' if nv >= 0 else 'v_bitop3'}", flush=True)
    lib.run_rate4.argtypes = [C.c_int, vp, vp, C.c_int, C.c_int]
    out = torch.zeros(ncu * 16, dtype=torch.int64, device=dev)
    for nv in (-1, 0, 4, 8, 12, 16, 24, 32, 1000, 1008, 1016, 1032):
        for n in (10, iters):
            rc = lib.run_rate4(nv, inp.data_ptr(), out.data_ptr(), n, ncu)
            assert rc == 0, lib.err_str(rc).decode()
        cyc = float(np.median(out.cpu().numpy()))
        per = cyc / (iters * (4 if nv >= 0 else 32))
        key = (f"4waves_per_simd_{'valu_only' if nv < 0 else '32x32x64'}_nv{nv}" if nv < 1000 else
               f"4waves_per_simd_32x32x64_unscaled_nv{nv - 1000}")
        report["rate"][key] = round(per, 2)
        print(f"{key}: {per:.2f} wave-cycles per {'MFMA (+ fillers)' if nv >= 0 else 'v_bitop3'}", flush=True)
    print(json.dumps(report))
    with open(os.path.join(ROOT, "gpurun_out", "mfma_isa.json"), "w") as f:
        json.dump(report, f, indent=1)


if __name__ == "__main__":
    build() if sys.argv[1] == "build" else run()
