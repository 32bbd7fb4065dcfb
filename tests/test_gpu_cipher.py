"""GPU parity of the cold-path pieces through the C-ABI: the ECB cipher objects (encrypt AND decrypt, SURVEY.md
8(f) row 4), the round-keys-only AES context, the parallel key-image setup, kernel selection reporting, and the
batch kernels' work-counter ring under launches on several streams.  Bit-exact against the CPU oracle."""
import numpy as np
import pytest

import oracle
import rapido_amd as ra
from conftest import FAMILIES, kernel_family
from rapido_amd import records
from rapido_amd.hostmem import to_cpu, to_gpu

pytestmark = pytest.mark.gpu

FIPS_PT = bytes.fromhex("00112233445566778899aabbccddeeff")


@pytest.mark.parametrize("name,expected", [("aes128gcm", "69c4e0d86a7b0430d8cdb78070b4c55a"),
                                           ("aes256gcm", "8ea2b7ca516745bfeafc49904b496089")])
def test_ecb_cipher_of_aead_reference_test(gpu, name, expected):
    """t/picotls.c:266-307 test_ecb through aead->ecb_cipher: ptls_cipher_new(algo, 1, key) encrypts the FIPS-197
    plaintext to the expected block, ptls_cipher_new(algo, 0, key) decrypts it back (in place, as the test does)."""
    algo = ra.algorithm(name)
    ecb = algo.ecb_cipher.contents
    assert ecb.block_size == 16 and ecb.iv_size == 0 and ecb.key_size == algo.key_size
    key = bytes(range(32))[:algo.key_size]
    enc = ra.Cipher(ecb, True, key)
    actual = enc.encrypt(FIPS_PT)
    enc.free()
    assert actual.hex() == expected
    dec = ra.Cipher(ecb, False, key)
    assert dec.encrypt(actual) == FIPS_PT
    dec.free()


@pytest.mark.parametrize("keylen", [16, 32])
@pytest.mark.parametrize("nblocks", [1, 2, 255, 256, 257, 4099])
def test_ecb_many_blocks_both_directions(gpu, keylen, nblocks):
    """Many-block ECB through the cipher objects, host buffers, against the oracle's Cipher / InvCipher."""
    rng = np.random.default_rng(nblocks + keylen)
    key = rng.integers(0, 256, keylen, dtype=np.uint8).tobytes()
    data = rng.integers(0, 256, 16 * nblocks, dtype=np.uint8).tobytes()
    name = "aes128ecb" if keylen == 16 else "aes256ecb"
    enc = ra.cipher_new(name, True, key)
    ct = enc.encrypt(data)
    assert ct == oracle.ecb_blocks(key, data, True)
    dec = ra.cipher_new(name, False, key)
    assert dec.encrypt(ct) == data
    # decrypting arbitrary blocks: the oracle's InvCipher
    assert dec.encrypt(data) == oracle.ecb_blocks(key, data, False)


@pytest.mark.parametrize("keylen", [16, 32])
def test_aes_context_device_batch(gpu, keylen):
    """ptls_mi355x_aes_ecb_batch on device buffers (1 M blocks = 16 MiB, one launch each way), in place too."""
    import torch
    rng = np.random.default_rng(70 + keylen)
    key = rng.integers(0, 256, keylen, dtype=np.uint8).tobytes()
    n = 1 << 20
    data = rng.integers(0, 256, 16 * n, dtype=np.uint8)
    ks = ra.AesKeys(key)
    d_in = to_gpu(data)
    d_out = torch.zeros_like(d_in)
    ks.ecb_batch(d_out.data_ptr(), d_in.data_ptr(), n, encrypt=True)
    torch.cuda.synchronize()
    ct = to_cpu(d_out)
    # the oracle is byte-serial: check a spread sample of blocks, plus the round trip of the whole buffer
    idx = np.unique(np.concatenate([[0, 1, n - 1], rng.integers(0, n, 2000)]))
    for i in idx:
        blk = data[16 * i:16 * i + 16].tobytes()
        assert ct[16 * i:16 * i + 16].tobytes() == oracle.ecb_blocks(key, blk, True)
    ks.ecb_batch(d_out.data_ptr(), d_out.data_ptr(), n, encrypt=False)  # in place
    torch.cuda.synchronize()
    assert torch.equal(d_out, d_in)
    ks.close()


def test_ctr_cipher_256_and_repeated_init(gpu):
    """The CTR cipher (header-protection mask, lib/fusion.c:822-872) on the round-keys-only context: each init is
    one ECB block of the IV, AES-256 too."""
    rng = np.random.default_rng(3)
    for keylen, name in ((16, "aes128ctr"), (32, "aes256ctr")):
        key = rng.integers(0, 256, keylen, dtype=np.uint8).tobytes()
        c = ra.cipher_new(name, True, key)
        for _ in range(5):
            iv = rng.integers(0, 256, 16, dtype=np.uint8).tobytes()
            c.init(iv)
            data = rng.integers(0, 256, 13, dtype=np.uint8).tobytes()
            mask = oracle.ecb(key, iv)
            assert c.encrypt(data) == bytes(a ^ b for a, b in zip(data, mask))
        c.free()


@pytest.mark.parametrize("keylen", [16, 32])
def test_parallel_key_setup_all_tables(gpu, keylen):
    """Contexts built by the parallel setup kernel seal like the oracle on every kernel family, so every table of
    the key image is exercised: H^1..H^8 (K = 1, 2, 4, 8 batch kernels), H^32/H^64/H^128/H^256 (window joins)."""
    import torch
    rng = np.random.default_rng(keylen)
    key = rng.integers(0, 256, keylen, dtype=np.uint8).tobytes()
    iv = rng.integers(0, 256, 12, dtype=np.uint8).tobytes()
    lens = np.array([0, 1, 16, 100, 1400, 4097, 16384, 16399], dtype=np.uint64)
    recs, src_bytes, aad_bytes = records.layout(lens, np.full(len(lens), 13, np.uint64), align=16)
    recs["seq"] = rng.integers(0, 2 ** 63, len(lens), dtype=np.uint64)
    src = rng.integers(0, 256, src_bytes, dtype=np.uint8)
    aad = rng.integers(0, 256, aad_bytes, dtype=np.uint8)
    want = np.zeros_like(src)
    oracle.batch(True, key, iv, recs, src, want, aad)
    eng = ra.Engine(key)
    d_recs, d_src, d_aad = (to_gpu(a) for a in (recs.view(np.uint8), src, aad))
    configs = [("batch", k) for k in (1, 2, 4, 8)] + [(f, 4) for f in FAMILIES if f != "batch"]
    for family, k in configs:
        prev_k = ra.set_lanes_per_record(k)
        try:
            with kernel_family(family, framing=False):
                d_dst = torch.zeros_like(d_src)
                eng.seal_batch(iv, d_recs.data_ptr(), len(recs), d_src.data_ptr(), d_dst.data_ptr(), d_aad.data_ptr())
                torch.cuda.synchronize()
        finally:
            ra.set_lanes_per_record(prev_k)
        got = to_cpu(d_dst)
        for r in recs:
            a, n = int(r["dst"]), int(r["len"]) + 16
            assert np.array_equal(got[a:a + n], want[a:a + n]), (family, k, int(r["len"]))
    eng.close()


def test_kernel_name_reports_the_launched_family(gpu):
    """ptls_mi355x_kernel_name takes n and the framing flag and names the kernel launch_batch picks."""
    import torch
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    assert ra.kernel_name(True, 16, 1) == "mi355x_gcm_wins_seal_aes128"
    assert ra.kernel_name(False, 32, ncu // 5, framing=True) == "mi355x_tls_wins_open_aes256"  # 5 runs per record
    assert ra.kernel_name(False, 32, ncu, framing=True) == "mi355x_tls_win16_open_aes256"
    prevs = ra.set_split_records(0)
    try:
        assert ra.kernel_name(True, 16, 1) == "mi355x_gcm_win16_seal_aes128"
        prev16 = ra.set_win16_records(0)
        try:
            assert ra.kernel_name(True, 16, 1) == "mi355x_gcm_win32_seal_aes128"
            assert ra.kernel_name(False, 32, 1, framing=True) == "mi355x_tls_win32_open_aes256"
        finally:
            ra.set_win16_records(prev16)
    finally:
        ra.set_split_records(prevs)
    assert ra.kernel_name(True, 16, 16 * ncu, framing=True) == "mi355x_tls_winw_seal_aes128"
    assert ra.kernel_name(True, 16, 3 * ncu, framing=True) == "mi355x_tls_win_seal_aes128"
    assert ra.kernel_name(True, 16, 1 << 20) == "mi355x_gcm_seal_aes128_k4"
    assert ra.kernel_name(False, 32, 1 << 20) == "mi355x_gcm_open_aes256_k4"
    assert ra.kernel_name(True, 16, 1 << 20, framing=True) == "mi355x_tls_seal_aes128_k4"
    prev = ra.set_lanes_per_record(8)
    try:
        assert ra.kernel_name(True, 32, 1 << 20) == "mi355x_gcm_seal_aes256_k8"
    finally:
        ra.set_lanes_per_record(prev)


def test_work_slots_reused_across_streams(gpu):
    """More launches than work-counter slots (256), alternating between two streams with nothing synchronised in
    between: every launch seals all its records (a shared or out-of-step counter would make waves exit early)."""
    import torch
    rng = np.random.default_rng(9)
    n = 4096  # above the AEAD window threshold: the batch kernels and their work counters
    lens = np.full(n, 64, np.uint64)
    recs, src_bytes, aad_bytes = records.layout(lens, np.zeros(n, np.uint64), align=16)
    src = rng.integers(0, 256, src_bytes, dtype=np.uint8)
    key, iv = bytes(range(16)), bytes(12)
    want = np.zeros_like(src)
    oracle.batch(True, key, iv, recs, src, want, np.zeros(1, np.uint8))
    eng = ra.Engine(key)
    d_recs, d_src = to_gpu(recs.view(np.uint8)), to_gpu(src)
    d_aad = torch.zeros(1, dtype=torch.uint8, device="cuda")
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    outs = [torch.zeros_like(d_src) for _ in range(8)]
    torch.cuda.synchronize()
    for i in range(600):
        s = streams[i % 2]
        out = outs[i % 8]
        eng.seal_batch(iv, d_recs.data_ptr(), n, d_src.data_ptr(), out.data_ptr(), d_aad.data_ptr(), s.cuda_stream)
    torch.cuda.synchronize()
    for out in outs:
        assert np.array_equal(to_cpu(out), want)
    eng.close()


def test_shared_resources_across_destroyed_streams(gpu):
    """A context's work slots and sort scratch used from streams that are destroyed and replaced between uses (their
    handles may be reused): each use waits on the event recorded right after the previous one, never on a stored
    stream handle; ordered (ragged) seals through order_by_length on rotating streams stay bit-exact."""
    import torch
    rng = np.random.default_rng(19)
    n = 3000
    lens = rng.integers(0, 700, n).astype(np.uint64)
    recs, src_bytes, aad_bytes = records.layout(lens, np.zeros(n, np.uint64), align=16)
    src = rng.integers(0, 256, src_bytes, dtype=np.uint8)
    key, iv = bytes(range(16)), bytes(range(12))
    want = np.zeros_like(src)
    oracle.batch(True, key, iv, recs, src, want, np.zeros(1, np.uint8))
    eng = ra.Engine(key)
    d_recs, d_src = to_gpu(recs.view(np.uint8)), to_gpu(src)
    d_aad = torch.zeros(1, dtype=torch.uint8, device="cuda")
    d_order = torch.zeros(n, dtype=torch.int32, device="cuda")
    outs = [torch.zeros_like(d_src) for _ in range(4)]
    torch.cuda.synchronize()
    for i in range(40):
        s = torch.cuda.Stream()  # a fresh stream each time; the previous one is released
        eng.order_by_length(d_recs.data_ptr(), n, d_order.data_ptr(), s.cuda_stream)
        eng.seal_batch_ordered(iv, d_recs.data_ptr(), d_order.data_ptr(), n, d_src.data_ptr(), outs[i % 4].data_ptr(),
                               d_aad.data_ptr(), s.cuda_stream)
        del s
    torch.cuda.synchronize()
    for out in outs:
        assert np.array_equal(to_cpu(out), want)
    eng.close()
