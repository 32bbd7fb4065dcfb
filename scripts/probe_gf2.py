"""Drives scripts/probe_gf2.hip (a measurement probe, not the product): GHASH as a GF(2) GEMM on the FP4 matrix
cores against the nibble tables, inside the batch kernels' AES-CTR, compute-only.

    python scripts/probe_gf2.py build     # CPU: hipcc -> scripts/_build/libprobe_gf2.so
    python scripts/probe_gf2.py run       # GPU: MFMA GHASH bit-exact against the host GHASH, then the throughput
                                          # of AES only / AES + MFMA GHASH / AES + nibble GHASH (GB/s of blocks)

    PROBE_MODES (0 AES only, 1 MFMA v_perm pack, 3 MFMA v_alignbit pack, 2 nibble tables), PROBE_KEYS (16,32),
    PROBE_REPS: one mode under rocprofv3 --pmc, or many repetitions for amd-smi power samples
    (scripts/gpu_probe_gf2_pmc.sh).

W (128 x 512 bits of M(H^4) | M(H^3) | M(H^2) | M(H)) is laid out as the kernel's fragments: 32 KiB, fragment
(mt, t) = 1 KiB, lane l's 16 bytes = row 32 mt + l % 32, the 32 elements of K tile t of lane half l // 32.
"""
import ctypes as C
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
SO = os.path.join(ROOT, "scripts", "_build", "libprobe_gf2.so")


def build():
    os.makedirs(os.path.dirname(SO), exist_ok=True)
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
                    *os.environ.get("PROBE_FLAGS", "").split(), os.path.join(ROOT, "scripts", "probe_gf2.hip"), "-o",
                    SO], check=True)
    print("built", SO)


def gf_mul(x: bytes, y: bytes) -> bytes:
    """SP 800-38D Algorithm 1 (GCM bit order: bit 0 = MSB of byte 0)"""
    X, V, Z, R = int.from_bytes(x, "big"), int.from_bytes(y, "big"), 0, 0xE1 << 120
    for i in range(127, -1, -1):
        if (X >> i) & 1:
            Z ^= V
        V = (V >> 1) ^ R if V & 1 else V >> 1
    return Z.to_bytes(16, "big")


def dword_bits(block: bytes) -> np.ndarray:
    """128 bits in the kernel's order: bit p = bit p % 32 of little-endian dword p // 32"""
    v = np.frombuffer(block, "<u4")
    return np.array([(int(v[p // 32]) >> (p % 32)) & 1 for p in range(128)], np.uint8)


def mul_matrix(c: bytes) -> np.ndarray:
    """M[out_p][in_p] of y = x * c in the dword-bit order"""
    M = np.zeros((128, 128), np.uint8)
    for p in range(128):
        x = np.zeros(4, "<u4")
        x[p // 32] = np.uint32(1 << (p % 32))
        M[:, p] = dword_bits(gf_mul(x.tobytes(), c))
    return M


def build_w(H: bytes, pack: int = 0) -> np.ndarray:
    """pack 0: value i of M tile mt, lane half h -> Y' bit 64 h + 32 (mt >> 1) + 4 (mt & 1) + 8 (i & 3) + (i >> 2)
    (the v_perm gather); pack 1: -> bit 64 h + 32 (mt >> 1) + 16 (mt & 1) + i (the v_alignbit chain: the first of the
    32 values alignbit'ed into a dword ends at bit 0)"""
    powers = [H]
    for _ in range(3):
        powers.append(gf_mul(powers[-1], H))
    Ms = {k: mul_matrix(powers[k - 1]) for k in (1, 2, 3, 4)}
    code = {0: 0x4, 1: 0x2, 2: 0x1, 3: 0x4}  # e2m1 2.0 / 1.0 / 0.5 / 2.0: every product 0 or 1
    frag = np.zeros((4, 8, 64, 4), np.uint32)
    for mt in range(4):
        for lane in range(64):
            hh, r = lane // 32, lane % 32
            # row 32 mt + r is value i of lane half h' with r = (i & 3) + 8 (i >> 2) + 4 h'
            h_out, i = (r >> 2) & 1, (r & 3) + 4 * (r >> 3)
            if pack == 0:
                ybit = 64 * h_out + 32 * (mt >> 1) + 4 * (mt & 1) + 8 * (i & 3) + (i >> 2)
            else:
                ybit = 64 * h_out + 32 * (mt >> 1) + 16 * (mt & 1) + i
            for t in range(8):
                blk, dd = 2 * hh + (t >> 2), t & 3
                M = Ms[4 - blk]
                for j in range(32):
                    q, m = j // 8, j % 8
                    inbit = 32 * dd + 4 * m + q
                    if M[ybit, inbit]:
                        frag[mt, t, lane, q] |= np.uint32(code[q] << (4 * m))
    return frag.reshape(-1)


def ghash_ref(H: bytes, blocks) -> bytes:
    y = bytes(16)
    for b in blocks:
        y = gf_mul(bytes(a ^ c for a, c in zip(y, b)), H)
    return y


def run():
    import torch
    lib = C.CDLL(SO)
    vp, u32 = C.c_void_p, C.c_uint32
    lib.probe_key.argtypes = [vp, u32, vp, vp, vp]
    lib.probe_key_image_size.restype = C.c_size_t
    lib.probe_run.argtypes = [C.c_int, C.c_int, vp, vp, u32, u32, vp, vp, vp]
    lib.probe_check.argtypes = [vp, vp, u32, vp, vp, u32]
    lib.probe_err.restype = C.c_char_p
    dev = torch.device("cuda:0")
    stream = torch.cuda.current_stream(dev).cuda_stream
    ncu = torch.cuda.get_device_properties(dev).multi_processor_count

    def ok(rc):
        if rc != 0:
            raise SystemExit(lib.probe_err(rc).decode())

    # correctness: 3 chunks of 32 records x 4 blocks against Algorithm-1 GHASH, both packs
    rng = np.random.default_rng(17)
    H = rng.integers(0, 256, 16, dtype=np.uint8).tobytes()
    S = 3
    data = rng.integers(0, 256, S * 32 * 4 * 16, dtype=np.uint8)
    d_data = torch.from_numpy(data).to(dev)
    d_ws = {}
    for pack in (0, 1):
        w = build_w(H, pack)
        d_ws[pack] = d_w = torch.from_numpy(w.view(np.int32)).to(dev)
        d_y = torch.zeros(32 * 16, dtype=torch.uint8, device=dev)
        ok(lib.probe_check(d_w.data_ptr(), d_data.data_ptr(), S, d_y.data_ptr(), stream, pack))
        torch.cuda.synchronize()
        got = d_y.cpu().numpy().tobytes()
        for n in range(32):
            blocks = [data[((s * 32 + n) * 4 + j) * 16:((s * 32 + n) * 4 + j + 1) * 16].tobytes() for s in range(S)
                      for j in range(4)]
            if got[16 * n:16 * n + 16] != ghash_ref(H, blocks):
                raise SystemExit(f"MFMA GHASH (pack {pack}) differs from the reference GHASH for record {n}")
        print(f"MFMA GHASH (pack {pack}) bit-exact against Algorithm-1 GHASH: 32 records x 12 blocks", flush=True)

    results = {}
    for keylen in [int(x) for x in os.environ.get("PROBE_KEYS", "16,32").split(",")]:
        key = bytes(range(3, 3 + keylen))
        d_key = torch.tensor(list(key), dtype=torch.uint8, device=dev)
        d_ki = torch.zeros(lib.probe_key_image_size(), dtype=torch.uint8, device=dev)
        d_rc = torch.zeros(1, dtype=torch.int32, device=dev)
        ok(lib.probe_key(d_key.data_ptr(), keylen, d_ki.data_ptr(), d_rc.data_ptr(), stream))
        nr = 10 if keylen == 16 else 14
        nunits = ncu * 16 * int(os.environ.get("PROBE_UNITS_PER_WAVE", "48"))
        d_work = torch.zeros(1, dtype=torch.int32, device=dev)
        d_out = torch.zeros(ncu * 1024, dtype=torch.int32, device=dev)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        res = {}
        modes = [int(m) for m in os.environ.get("PROBE_MODES", "0,1,3,2").split(",")]
        for mode, name in ((0, "aes_only"), (1, "aes+mfma_ghash"), (3, "aes+mfma_ghash_alignbit"), (2, "aes+nibble_ghash")):
            if mode not in modes:
                continue
            d_w = d_ws[1 if mode == 3 else 0]
            ts = []
            for rep in range(int(os.environ.get("PROBE_REPS", "4"))):
                d_work.zero_()
                ev[0].record()
                ok(lib.probe_run(nr, mode, d_ki.data_ptr(), d_w.data_ptr(), nunits, ncu, d_work.data_ptr(),
                                 d_out.data_ptr(), stream))
                ev[1].record()
                torch.cuda.synchronize()
                if rep:
                    ts.append(ev[0].elapsed_time(ev[1]))
            ms = sorted(ts)[len(ts) // 2]
            gbps = nunits * 16 * 128 * 16 / (ms * 1e-3) / 1e9
            res[name] = round(gbps, 1)
            print(f"AES-{8 * keylen} {name:18s}: {ms:8.3f} ms  {gbps:8.1f} GB/s of 16-B blocks", flush=True)
        results[f"aes{8 * keylen}"] = res
    print(json.dumps(results))


if __name__ == "__main__":
    build() if sys.argv[1] == "build" else run()
