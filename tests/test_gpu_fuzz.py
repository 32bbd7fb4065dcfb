"""Randomised GPU parity sweep over the walk's parameter space, against the CPU oracle (bit-exact).

Each case draws record lengths 0..20000 B and AAD lengths 0..255 B (so the AAD is hoisted into the lanes'
starting accumulators when it spans <= K blocks and sits in the grid otherwise), places every record at an
arbitrary byte offset (unaligned loads/stores, every output alignment), and runs seal then open through
the C-ABI with K = 1, 2, 4, 8 lanes per record on both kernel families (window kernels, batch kernels).
Seeds are fixed, so a failure reproduces.
"""
import numpy as np
import pytest

import oracle
import rapido_amd as ra
from conftest import FAMILIES, kernel_family
from rapido_amd import RECORD_DTYPE
from rapido_amd.hostmem import to_cpu, to_gpu

pytestmark = pytest.mark.gpu


def make_batch(rng, n):
    lens = rng.integers(0, 20001, n)
    aadlens = rng.integers(0, 256, n)
    lens[:6] = [0, 1, 15, 16, 1400, 16384]
    aadlens[:6] = [0, 255, 64, 65, 5, 13]
    recs = np.zeros(n, RECORD_DTYPE)
    off = aoff = 0
    for i in range(n):
        off += int(rng.integers(0, 64))  # arbitrary byte offset before each record
        recs[i] = (off, off, aoff, int(rng.integers(0, 2 ** 63)), lens[i], aadlens[i])
        off += int(lens[i]) + 16
        aoff += int(aadlens[i]) + int(rng.integers(0, 8))
    src = rng.integers(0, 256, off + 64, dtype=np.uint8)
    aad = rng.integers(0, 256, aoff + 16, dtype=np.uint8)
    return recs, src, aad


@pytest.mark.parametrize("family", FAMILIES)
@pytest.mark.parametrize("lanes", [1, 2, 4, 8])
@pytest.mark.parametrize("keylen", [16, 32])
def test_fuzz_seal_open(gpu, family, lanes, keylen):
    import torch
    rng = np.random.default_rng(7000 + 10 * lanes + keylen + FAMILIES.index(family))
    recs, src, aad = make_batch(rng, 120)
    key = rng.integers(0, 256, keylen, dtype=np.uint8).tobytes()
    iv = rng.integers(0, 256, 12, dtype=np.uint8).tobytes()
    prev_k = ra.set_lanes_per_record(lanes)
    try:
        with kernel_family(family, framing=False):
            eng = ra.Engine(key)
            d_recs = to_gpu(recs.view(np.uint8))
            d_src = to_gpu(src)
            d_aad = to_gpu(aad)
            d_ct = torch.zeros_like(d_src)
            d_pt = torch.zeros_like(d_src)
            d_st = torch.zeros(len(recs), dtype=torch.int32, device="cuda")
            eng.seal_batch(iv, d_recs.data_ptr(), len(recs), d_src.data_ptr(), d_ct.data_ptr(), d_aad.data_ptr())
            eng.open_batch(iv, d_recs.data_ptr(), len(recs), d_ct.data_ptr(), d_pt.data_ptr(), d_aad.data_ptr(),
                           d_st.data_ptr())
            torch.cuda.synchronize()
            ct, pt, st = to_cpu(d_ct), to_cpu(d_pt), to_cpu(d_st).view(np.uint32)
            want = np.zeros_like(src)
            oracle.batch(True, key, iv, recs, src, want, aad)
            for i, r in enumerate(recs):
                a, n = int(r["dst"]), int(r["len"])
                assert bytes(ct[a: a + n + 16]) == bytes(want[a: a + n + 16]), (i, n, int(r["aadlen"]))
                assert bytes(pt[a: a + n]) == bytes(src[a: a + n]), (i, n)
            assert (st == recs["len"]).all()
            eng.close()
    finally:
        ra.set_lanes_per_record(prev_k)
