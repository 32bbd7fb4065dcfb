"""GPU parity: the HIP engine (through the C-ABI) against the CPU oracle and the reference KATs.

Bar: bit-exact ciphertext, tags, plaintext and status (integer/byte work).
"""
import numpy as np
import pytest

import oracle
import rapido_amd as ra
from conftest import FAMILIES, kernel_family
from rapido_amd import records
from rapido_amd.hostmem import to_cpu, to_gpu

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True, params=FAMILIES)
def aead_kernels(request, engine_lib):
    """Every test here runs on each kernel family (conftest.FAMILIES): the window kernels with 64-block segments
    walked in parallel, the same with 32-block segments of 8 or of 16 lanes (the default up to one record per CU,
    so the slot calls), and the batch kernels (K lanes per record)."""
    with kernel_family(request.param, framing=False):
        yield request.param


def to_dev(a: np.ndarray):
    import torch
    return to_gpu(np.ascontiguousarray(a))


def run_batch(eng, is_seal, static_iv, recs, src, dst_size, aad, inplace=False):
    import torch
    d_recs = to_dev(recs.view(np.uint8))
    d_src = to_dev(src)
    d_dst = d_src if inplace else torch.zeros(dst_size, dtype=torch.uint8, device="cuda")
    d_aad = to_dev(aad)
    d_st = torch.zeros(max(len(recs), 1), dtype=torch.int32, device="cuda")
    if is_seal:
        eng.seal_batch(static_iv, d_recs.data_ptr(), len(recs), d_src.data_ptr(), d_dst.data_ptr(), d_aad.data_ptr())
    else:
        eng.open_batch(static_iv, d_recs.data_ptr(), len(recs), d_src.data_ptr(), d_dst.data_ptr(), d_aad.data_ptr(),
                       d_st.data_ptr())
    torch.cuda.synchronize()
    return to_cpu(d_dst), to_cpu(d_st).view(np.uint32)


def random_batch(rng, n, max_len=2000, max_aad=64, unaligned=True):
    lens = rng.integers(0, max_len, n).astype(np.uint64)
    aadlens = rng.integers(0, max_aad, n).astype(np.uint64)
    edge = [(0, 0), (1, 0), (15, 1), (16, 16), (17, 15), (31, 17), (32, 32), (33, 5), (64, 0), (0, 13)]
    for i, (l, a) in enumerate(edge[:n]):
        lens[i], aadlens[i] = l, a
    # 8 spare bytes per slot so the unaligned shift below never makes records overlap
    recs, src_bytes, aad_bytes = records.layout(lens + 8, aadlens, align=1 if unaligned else 16)
    recs["len"] = lens.astype(np.uint32)
    if unaligned:  # shift every record by a few bytes: exercises unaligned 16-byte accesses
        recs["src"] += np.arange(n, dtype=np.uint64) % 7
        recs["dst"] = recs["src"]
    recs["seq"] = rng.integers(0, 2 ** 63, n, dtype=np.uint64)
    src = rng.integers(0, 256, src_bytes, dtype=np.uint8)
    aad = rng.integers(0, 256, aad_bytes, dtype=np.uint8)
    return recs, src, aad


def slices(buf, recs, extra):
    return [bytes(buf[int(r["dst"]): int(r["dst"]) + int(r["len"]) + extra]) for r in recs]


@pytest.mark.parametrize("lanes", [1, 2, 4, 8])
@pytest.mark.parametrize("keylen", [16, 32])
def test_batch_vs_oracle(gpu, lanes, keylen):
    rng = np.random.default_rng(100 + lanes * 7 + keylen)
    n = 300
    recs, src, aad = random_batch(rng, n)
    key = rng.integers(0, 256, keylen, dtype=np.uint8).tobytes()
    iv = rng.integers(0, 256, 12, dtype=np.uint8).tobytes()
    prev = ra.set_lanes_per_record(lanes)
    try:
        eng = ra.Engine(key)
        got, _ = run_batch(eng, True, iv, recs, src, len(src), aad)
        want = np.zeros_like(src)
        oracle.batch(True, key, iv, recs, src, want, aad)
        assert slices(got, recs, 16) == slices(want, recs, 16)

        # open the GPU output; all verify and return the plaintext
        pt, st = run_batch(eng, False, iv, recs, got, len(src), aad)
        assert (st == recs["len"]).all()
        assert slices(pt, recs, 0) == [bytes(src[int(r["src"]): int(r["src"]) + int(r["len"])]) for r in recs]

        # tamper: one ciphertext bit, one tag bit, one AAD bit -> SIZE_MAX status, zeroed output
        bad = got.copy()
        bad[int(recs[11]["dst"])] ^= 1
        bad[int(recs[12]["dst"]) + int(recs[12]["len"]) + 3] ^= 0x80
        aad2 = aad.copy()
        aad2[int(recs[13]["aad"])] ^= 4
        assert recs[13]["aadlen"] > 0
        pt2, st2 = run_batch(eng, False, iv, recs, bad, len(src), aad2)
        assert st2[11] == 0xFFFFFFFF and st2[12] == 0xFFFFFFFF and st2[13] == 0xFFFFFFFF
        for i in (11, 12, 13):
            r = recs[i]
            assert not pt2[int(r["dst"]): int(r["dst"]) + int(r["len"])].any()
        ok = np.ones(n, bool)
        ok[[11, 12, 13]] = False
        assert (st2[ok] == recs["len"][ok]).all()
        eng.close()
    finally:
        ra.set_lanes_per_record(prev)


def test_inplace_and_zero_length(gpu):
    rng = np.random.default_rng(7)
    recs, src, aad = random_batch(rng, 64, max_len=300, unaligned=False)
    key, iv = bytes(range(16)), bytes(range(12))
    eng = ra.Engine(key)
    got, _ = run_batch(eng, True, iv, recs, src.copy(), len(src), aad, inplace=True)
    want = np.zeros_like(src)
    oracle.batch(True, key, iv, recs, src, want, aad)
    assert slices(got, recs, 16) == slices(want, recs, 16)
    pt, st = run_batch(eng, False, iv, recs, got.copy(), len(src), aad, inplace=True)
    assert (st == recs["len"]).all()
    assert slices(pt, recs, 0) == [bytes(src[int(r["src"]): int(r["src"]) + int(r["len"])]) for r in recs]


def test_direct_api_fusion_vectors(gpu):
    # t/fusion.c:89-97 gcm_basic (1): zero key/nonce, AAD "hello", 16 zero bytes
    eng = ra.Engine(bytes(16))
    out = eng.encrypt(bytes(12), b"hello", bytes(16))
    assert out.hex() == "0388dace60b6a392f328c2b971b2fe78973fbca65477bf4785b0d561f7e3fd6c"
    assert eng.decrypt(bytes(12), b"hello", out[:16], out[16:]) == bytes(16)
    # t/fusion.c:128-139 gcm_capacity: one byte
    out = eng.encrypt(bytes(12), b"a", b"X")
    assert out.hex() == "5b27215ed81a702e3941c80577d52fcb57"
    # t/fusion.c:71-85 ECB with a zero key
    assert eng.ecb(b"hello world!!!!!").hex() == "172afecb50b5f1237814b2f7cb51d0f7"
    assert ra.Engine(bytes(32)).ecb(b"hello world!!!!!").hex() == "2a033f0627b3554aa4fe5786550736ff"


GCM_VECTORS = [  # t/fusion.c:161-183: (aadlen, ptlen, tag) with zero key, nonce, aad and plaintext
    (13, 17, "1b4e515384e8aa5bb781ee12549a2ccf"), (13, 32, "84030586f55adf8ac3c145913c6fd0f8"),
    (13, 64, "66165d39739c50c90727e7d49127146b"), (13, 65, "eb3b75e1d4431e1bb67da46f6a1a0edd"),
    (13, 79, "8f4a96c7390c26bb15b68865e6a861b9"), (13, 80, "5cc2554857b19e7a9e18d015feac61fd"),
    (13, 81, "5a65f0d4db36c981bf7babd11691fe78"), (13, 95, "6a8a51152efe928999a610d8a7b1df9d"),
    (13, 96, "6b9c468e24ed96010687f3880a044d42"), (13, 97, "1b4eb785b884a7d4fdebaff81c1c12e8"),
    (22, 1328, "0507baaece8d573774c94e8103821316"), (21, 1329, "dd70d59030eadb6313e778046540a253"),
    (20, 1330, "f1b456b955afde7603188af0124a32ef"), (13, 1337, "a22deec51250a7eb1f4384dea5f2e890"),
    (12, 1338, "42102b0a499b2efa89702ece4b0c5789"), (11, 1339, "9827f0b34252160d0365ffaa9364bedc"),
    (0, 80, "98885a3a22bd4742fe7b72172193b163"), (0, 96, "afd649fc51e14f3966e4518ad53b9ddc"),
    (20, 85, "afe8b727057c804a0525c2914ef856b0"),
]


@pytest.mark.parametrize("aadlen,ptlen,tag", GCM_VECTORS)
def test_fusion_tag_vectors(gpu, aadlen, ptlen, tag):
    eng = ra.Engine(bytes(16))
    out = eng.encrypt(bytes(12), bytes(aadlen), bytes(ptlen))
    assert out[ptlen:].hex() == tag
    assert eng.decrypt(bytes(12), bytes(aadlen), out[:ptlen], out[ptlen:]) == bytes(ptlen)


HELLO = b"hello world\nhello world\nhello world\nhello world\nhello world\nhello world\nhello world\n\0"
HELLO_KEY = bytes([0x00, 0x11, 0x22, 0x33, 0x44, 0x55, 0x66, 0x77, 0x88, 0x99, 0xaa, 0xbb, 0xcc, 0xdd, 0xee, 0xff])
HELLO_EXPECTED = (  # t/fusion.c:110-116
    "d3a81d964c9b02d79ab041074c8ce2e02e83545245cbd468c84345ca91fba37a67ede8d75ee233d13ebf50c24b86835511bb"
    "174ff578b865eb9a2b8f7708a9601773c507f304c93f674d12a10293c23cd3f85933d501c3bbaae63fbb2366942628 43a5fd2f"
).replace(" ", "")


def test_slot_gcm_basic_and_iv96(gpu):
    aad = bytes(range(20))
    # t/fusion.c:99-125: through ptls_aead_new_direct / ptls_aead_encrypt / ptls_aead_decrypt
    a = ra.aead_new_direct("aes128gcm", False, HELLO_KEY, bytes(range(20, 32)))
    enc = a.encrypt(HELLO, 0, aad)
    assert enc.hex() == HELLO_EXPECTED
    assert a.decrypt(enc, 0, aad) == HELLO
    a.free()
    # t/fusion.c:197-231 gcm_iv96: xor_iv is persistent and applies to the leading IV bytes
    a = ra.aead_new_direct("aes128gcm", False, HELLO_KEY, bytes([20, 20, 20, 20]) + bytes(range(24, 32)))
    seq32, bad32 = bytes([0, 1, 2, 3]), bytes([0x89, 0xab, 0xcd, 0xef])
    a.xor_iv(seq32)
    enc = a.encrypt(HELLO, 0, aad)
    assert enc.hex() == HELLO_EXPECTED
    assert a.decrypt(enc, 0, aad) == HELLO
    a.xor_iv(seq32)
    a.xor_iv(bad32)
    assert a.decrypt(enc, 0, aad) is None
    a.xor_iv(bad32)
    a.xor_iv(seq32)
    assert a.decrypt(enc, 0, aad) == HELLO
    a.free()


@pytest.mark.parametrize("zero_copy", [True, False])
def test_slot_zero_copy_and_copied(gpu, zero_copy):
    """The slot's two staging paths (the kernel reading/writing pinned host memory, or DMA copies in and out) give
    the oracle's bytes for every size class, and a tampered tag fails without releasing plaintext."""
    prev = ra.set_slot_zero_copy_bytes(1 << 30 if zero_copy else 0)
    try:
        rng = np.random.default_rng(5 if zero_copy else 6)
        key, iv = rng.integers(0, 256, 16, dtype=np.uint8).tobytes(), rng.integers(0, 256, 12, dtype=np.uint8).tobytes()
        a = ra.aead_new_direct("aes128gcm", True, key, iv)
        d = ra.aead_new_direct("aes128gcm", False, key, iv)
        for n, alen in [(0, 0), (1, 5), (15, 13), (16, 0), (1400, 5), (4097, 33), (16384, 5), (20000, 100)]:
            pt = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
            aad = rng.integers(0, 256, alen, dtype=np.uint8).tobytes()
            seq = int(rng.integers(0, 2 ** 48))
            ct = a.encrypt(pt, seq, aad)
            assert ct == oracle.seal(key, oracle.build_iv(iv, seq), aad, pt), n
            assert d.decrypt(ct, seq, aad) == pt
            bad = bytearray(ct)
            bad[-1] ^= 1
            assert d.decrypt(bytes(bad), seq, aad) is None
        a.free()
        d.free()
    finally:
        ra.set_slot_zero_copy_bytes(prev)


@pytest.mark.parametrize("lanes", [1, 4, 8])
def test_gcm_spec_vectors_in_a_batch(gpu, lanes):
    """The GCM specification's test cases with 96-bit IVs (McGrew-Viega 1-4, AES-128, as cifra's testmodes.c; 13-16,
    AES-256, tests/test_oracle.py) in one batch per key, and the AES-256 ones through the slot: tags and
    ciphertext against the published values."""
    from test_oracle import MV, MV256
    prev = ra.set_lanes_per_record(lanes)
    try:
        for keyhex in sorted({v[0] for v in MV + MV256}):
            cases = [v for v in MV + MV256 if v[0] == keyhex]
            key = bytes.fromhex(keyhex)
            eng = ra.Engine(key)
            for _, pt, aad, iv, ct, tag in cases:  # one record per batch (the cases' IVs differ; the batch IV is static)
                ptb, aadb = bytes.fromhex(pt), bytes.fromhex(aad)
                recs = np.zeros(1, ra.RECORD_DTYPE)
                recs[0] = (0, 0, 0, 0, len(ptb), len(aadb))
                src = np.frombuffer(ptb + bytes(32), np.uint8).copy()
                out, _ = run_batch(eng, True, bytes.fromhex(iv), recs, src, len(src), np.frombuffer(aadb + bytes(16), np.uint8).copy())
                got = out[:len(ptb) + 16].tobytes().hex()
                assert got.startswith(ct) and got.endswith(tag), (keyhex[:8], len(ptb))
                back, st = run_batch(eng, False, bytes.fromhex(iv), recs, out, len(src), np.frombuffer(aadb + bytes(16), np.uint8).copy())
                assert st[0] == len(ptb) and back[:len(ptb)].tobytes() == ptb
            eng.close()
    finally:
        ra.set_lanes_per_record(prev)
    for key, pt, aad, iv, ct, tag in MV256:
        a = ra.aead_new_direct("aes256gcm", True, bytes.fromhex(key), bytes.fromhex(iv))
        got = a.encrypt(bytes.fromhex(pt), 0, bytes.fromhex(aad)).hex()  # seq 0: the nonce is the IV itself
        assert got.startswith(ct) and got.endswith(tag)
        a.free()


def test_slot_contexts_on_concurrent_threads(gpu):
    """picotls contexts are used by one thread each; a server runs one per connection on several threads.  Eight
    threads seal and open through their own slot contexts at once (the calls share the device's staging under its
    lock; ctypes releases the GIL, so they overlap), AES-128 and AES-256, every size class: the oracle's bytes."""
    from concurrent.futures import ThreadPoolExecutor

    def one(t):
        rng = np.random.default_rng(900 + t)
        keylen = 16 if t % 2 == 0 else 32
        algo = "aes128gcm" if keylen == 16 else "aes256gcm"
        key, iv = rng.integers(0, 256, keylen, dtype=np.uint8).tobytes(), rng.integers(0, 256, 12, dtype=np.uint8).tobytes()
        a, d = ra.aead_new_direct(algo, True, key, iv), ra.aead_new_direct(algo, False, key, iv)
        for i in range(24):
            n = int(rng.choice([0, 1, 15, 16, 17, 1400, 4097, 16384, 16401]))
            pt = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
            aad = rng.integers(0, 256, int(rng.integers(0, 40)), dtype=np.uint8).tobytes()
            ct = a.encrypt(pt, i, aad)
            assert ct == oracle.seal(key, oracle.build_iv(iv, i), aad, pt), (t, i, n)
            assert d.decrypt(ct, i, aad) == pt
        a.free()
        d.free()

    with ThreadPoolExecutor(8) as ex:
        for f in [ex.submit(one, t) for t in range(8)]:
            f.result()


@pytest.mark.parametrize("algo,keylen", [("aes128gcm", 16), ("aes256gcm", 32)])
def test_slot_streaming_and_record_layer(gpu, algo, keylen):
    """The TLS record-layer call sequence (lib/picotls.c:630-643) and t/picotls.c:161-198."""
    key, iv = bytes(range(1, keylen + 1)), bytes(range(40, 52))
    enc = ra.aead_new_direct(algo, True, key, iv)
    dec = ra.aead_new_direct(algo, False, key, iv)
    data = bytes(range(256)) * 5
    for seq, ln in enumerate([0, 1, 11, 1399, 16384]):
        d = (data * 20)[:ln]
        inner = d + b"\x17"  # content type appended as a second update
        hdr = bytes([0x17, 0x03, 0x03, (len(inner) + 16) >> 8, (len(inner) + 16) & 0xFF])
        import ctypes
        out = ctypes.create_string_buffer(len(inner) + 16)
        enc.encrypt_init(seq, hdr)
        off = enc.encrypt_update(out, 0, d)
        off += enc.encrypt_update(out, off, b"\x17")
        off += enc.encrypt_final(out, off)
        assert off == len(inner) + 16
        want = oracle.seal(key, oracle.build_iv(iv, seq), hdr, inner)
        assert out.raw == want
        assert dec.decrypt(out.raw, seq, hdr) == inner
        bad = bytearray(out.raw)
        bad[0 if ln else -1] ^= 1
        assert dec.decrypt(bytes(bad), seq, hdr) is None
    assert dec.decrypt(b"short", 0, b"") is None  # inlen < 16 -> SIZE_MAX


def test_slot_supplementary_encryption(gpu):
    """t/fusion.c:185-191: supp output = AES-ECB(supp key, sample of the written record)."""
    a = ra.aead_new_direct("aes128gcm", True, bytes(16), bytes(12))
    supp_cipher = ra.cipher_new("aes128ctr", True, bytes([1] * 16))
    want_tags = {17: "1b4e515384e8aa5bb781ee12549a2ccf", 32: "84030586f55adf8ac3c145913c6fd0f8"}
    want_supp = {17: "4576f18ef3ae9dfd37cf72c4592da874", 32: "a062016e90dcc316d061fde5424cf34f"}
    import ctypes
    for ptlen in (17, 32):
        out = ctypes.create_string_buffer(ptlen + 16)
        supp = ra.SupplementaryEncryption()
        supp.ctx = supp_cipher.ptr
        supp.input = ctypes.addressof(out) + 2
        a.ctx.do_encrypt(a.ptr, out, ctypes.create_string_buffer(ptlen), ptlen, 0,
                         ctypes.create_string_buffer(13), 13, ctypes.byref(supp))
        assert out.raw[ptlen:].hex() == want_tags[ptlen]
        assert bytes(supp.output).hex() == want_supp[ptlen]


def test_ctr_cipher_kat(gpu):
    """t/picotls.c:312-321: AES128-CTR of 16 zero bytes."""
    key = bytes.fromhex("2b7e151628aed2a6abf7158809cf4f3c")
    iv = bytes.fromhex("6bc1bee22e409f96e93d7e117393172a")
    c = ra.cipher_new("aes128ctr", True, key)
    c.init(iv)
    assert c.encrypt(bytes(16)).hex() == "3ad77bb40d7a3660a89ecaf32466ef97"


@pytest.mark.parametrize("lanes", [4, 8])
def test_ordered_ragged_batch(gpu, lanes):
    """ptls_mi355x_order_by_length + *_batch_ordered: descending work, every record sealed once, status per descriptor."""
    import torch
    rng = np.random.default_rng(55 + lanes)
    n = 2000
    lens = rng.integers(0, 5000, n).astype(np.uint64)
    recs, src_bytes, aad_bytes = records.layout(lens, rng.integers(0, 40, n).astype(np.uint64), align=16)
    recs["seq"] = rng.integers(0, 2 ** 63, n, dtype=np.uint64)
    src = rng.integers(0, 256, src_bytes, dtype=np.uint8)
    aad = rng.integers(0, 256, aad_bytes, dtype=np.uint8)
    key, iv = bytes(range(40, 56)), bytes(range(12))
    prev = ra.set_lanes_per_record(lanes)
    try:
        eng = ra.Engine(key)
        d_recs, d_src, d_aad = to_dev(recs.view(np.uint8)), to_dev(src), to_dev(aad)
        d_dst = torch.zeros_like(d_src)
        d_order = torch.zeros(n, dtype=torch.int32, device="cuda")
        eng.order_by_length(d_recs.data_ptr(), n, d_order.data_ptr())
        eng.seal_batch_ordered(iv, d_recs.data_ptr(), d_order.data_ptr(), n, d_src.data_ptr(), d_dst.data_ptr(),
                               d_aad.data_ptr())
        torch.cuda.synchronize()
        order = to_cpu(d_order).view(np.uint32)
        assert sorted(order.tolist()) == list(range(n))
        work = (recs["len"].astype(np.int64) + 15) // 16 + (recs["aadlen"].astype(np.int64) + 15) // 16
        assert (np.diff(work[order]) <= 0).all()
        want = np.zeros_like(src)
        oracle.batch(True, key, iv, recs, src, want, aad)
        got = to_cpu(d_dst)
        assert slices(got, recs, 16) == slices(want, recs, 16)
        d_pt = torch.zeros_like(d_src)
        d_st = torch.zeros(n, dtype=torch.int32, device="cuda")
        eng.open_batch_ordered(iv, d_recs.data_ptr(), d_order.data_ptr(), n, d_dst.data_ptr(), d_pt.data_ptr(),
                               d_aad.data_ptr(), d_st.data_ptr())
        torch.cuda.synchronize()
        assert (to_cpu(d_st).view(np.uint32) == recs["len"]).all()
        assert slices(to_cpu(d_pt), recs, 0) == [bytes(src[int(r["src"]): int(r["src"]) + int(r["len"])])
                                                        for r in recs]
    finally:
        ra.set_lanes_per_record(prev)


@pytest.mark.parametrize("lanes", [4, 8])
def test_record_beyond_2p16_blocks(gpu, lanes):
    """Counters past 2^16 (records > 1 MiB): round-1 constants are recomputed per 2^16 window."""
    lens = np.array([70000 * 16 + 5, 1400, 200000 * 16], dtype=np.uint64)
    recs, src, aad = records.tls_batch(lens, seed=21, align=256)
    key, iv = bytes(range(7, 39)), bytes(range(12))
    prev = ra.set_lanes_per_record(lanes)
    try:
        eng = ra.Engine(key)
        got, _ = run_batch(eng, True, iv, recs, src, len(src), aad)
        want = np.zeros_like(src)
        oracle.batch(True, key, iv, recs, src, want, aad)
        assert slices(got, recs, 16) == slices(want, recs, 16)
        pt, st = run_batch(eng, False, iv, recs, got, len(src), aad)
        assert (st == recs["len"]).all()
    finally:
        ra.set_lanes_per_record(prev)


def test_work_counter_wrap(gpu, aead_kernels):
    """The batch kernels' work counters are never reset (a launch starts at the ticket where the previous one
    on its ring slot ended, mod 2^32).  Start them 25 tickets below 2^32 so every launch's range (groups plus
    one exit ticket per wave) crosses the wrap, and check seal/open stay bit-exact."""
    if aead_kernels != "batch":
        pytest.skip("the window kernels use no work counter")
    rng = np.random.default_rng(77)
    recs, src, aad = random_batch(rng, 300)
    key = rng.integers(0, 256, 16, dtype=np.uint8).tobytes()
    iv = rng.integers(0, 256, 12, dtype=np.uint8).tobytes()
    prev = ra.set_work_ticket_origin(2 ** 32 - 25)
    try:
        eng = ra.Engine(key)
    finally:
        ra.set_work_ticket_origin(prev)
    want = np.zeros_like(src)
    oracle.batch(True, key, iv, recs, src, want, aad)
    for _ in range(3):  # later launches reuse nothing; each slot's first range crosses 2^32
        got, _ = run_batch(eng, True, iv, recs, src, len(src), aad)
        assert slices(got, recs, 16) == slices(want, recs, 16)
        pt, st = run_batch(eng, False, iv, recs, got, len(src), aad)
        assert (st == recs["len"]).all()
        assert slices(pt, recs, 0) == [bytes(src[int(r["src"]): int(r["src"]) + int(r["len"])]) for r in recs]
    eng.close()
