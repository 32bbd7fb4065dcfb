"""CPU execution of the kernels' own code (rapido_amd/csrc/gcm_core.h via tests/cpp/kernel_model.cpp)
against the oracle: T-table AES with bank-replicated v_perm addressing, nibble-table GHASH, the K-lane
record walk with front padding, software-pipelined Horner, tail handling.  No GPU needed."""
import ctypes as C
import os

import numpy as np
import pytest

import oracle
from rapido_amd import RECORD_DTYPE, records


@pytest.fixture(scope="module")
def model():
    from rapido_amd import build
    path = build.build_model()
    lib = C.CDLL(path)
    vp = C.c_void_p
    lib.model_batch.argtypes = [C.c_int, C.c_int, vp, C.c_size_t, vp, vp, C.c_size_t, vp, vp, vp, vp]
    lib.model_key_image.argtypes = [vp, C.c_size_t, vp, C.c_size_t]
    lib.model_key_image_size.restype = C.c_size_t
    return lib


def run(lib, is_seal, K, key, iv, recs, src, dst, aad, st):
    """K = "w4" / "w8": the window kernels' math (64-position segments of 4 / 8 lanes joined with H^64);
    else the K-lane batch walk."""
    if K in ("w16", "split"):  # the 16-lane latency kernels and the split kernels (32-position segments, 2 steps)
        lib.model_batch_win16.argtypes = [C.c_int, C.c_int, C.c_void_p, C.c_size_t, C.c_void_p, C.c_void_p,
                                          C.c_size_t, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
        rc = lib.model_batch_win16(1 if is_seal else 0, 1 if K == "split" else 0, key, len(key), iv, recs.ctypes.data,
                                   len(recs), src.ctypes.data, dst.ctypes.data, aad.ctypes.data, st.ctypes.data)
    elif isinstance(K, str):  # "w4", "w8", or "w8s32" (32-position segments: the single-record latency kernels)
        lanes, _, seglen = K[1:].partition("s")
        assert lib.model_set_window_lanes(int(lanes)) > 0
        assert lib.model_set_window_seglen(int(seglen or 64)) > 0
        lib.model_batch_window.argtypes = [C.c_int, C.c_void_p, C.c_size_t, C.c_void_p, C.c_void_p, C.c_size_t,
                                           C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
        rc = lib.model_batch_window(1 if is_seal else 0, key, len(key), iv, recs.ctypes.data, len(recs),
                                    src.ctypes.data, dst.ctypes.data, aad.ctypes.data, st.ctypes.data)
    else:
        rc = lib.model_batch(1 if is_seal else 0, K, key, len(key), iv, recs.ctypes.data, len(recs), src.ctypes.data,
                             dst.ctypes.data, aad.ctypes.data, st.ctypes.data)
    assert rc == 0


def batch(rng, n, max_len, max_aad, shift=True):
    lens = rng.integers(0, max_len, n).astype(np.uint64)
    aadlens = rng.integers(0, max_aad, n).astype(np.uint64)
    for i, (l, a) in enumerate([(0, 0), (1, 0), (15, 1), (16, 16), (17, 15), (31, 17), (32, 32), (33, 5), (0, 13)]):
        if i < n:
            lens[i], aadlens[i] = l, a
    recs, src_bytes, aad_bytes = records.layout(lens + 8, aadlens, align=1)
    recs["len"] = lens.astype(np.uint32)
    if shift:
        recs["src"] += np.arange(n, dtype=np.uint64) % 7
        recs["dst"] = recs["src"]
    recs["seq"] = rng.integers(0, 2 ** 63, n, dtype=np.uint64)
    return recs, rng.integers(0, 256, src_bytes, dtype=np.uint8), rng.integers(0, 256, aad_bytes, dtype=np.uint8)


def spans(buf, recs, extra):
    return [bytes(buf[int(r["dst"]): int(r["dst"]) + int(r["len"]) + extra]) for r in recs]


@pytest.mark.parametrize("K", [1, 2, 4, 8, "w4", "w8", "w8s32", "w16", "split"])
@pytest.mark.parametrize("keylen", [16, 32])
def test_model_matches_oracle(model, K, keylen):
    seed = K if isinstance(K, int) else {"w16": 9016, "split": 9017}.get(K) or 900 + int(K[1:].replace("s", ""))
    rng = np.random.default_rng(seed * 100 + keylen)
    recs, src, aad = batch(rng, 150, 700, 48)
    key = rng.integers(0, 256, keylen, dtype=np.uint8).tobytes()
    iv = rng.integers(0, 256, 12, dtype=np.uint8).tobytes()
    got, want = np.zeros_like(src), np.zeros_like(src)
    st = np.zeros(len(recs), np.uint32)
    run(model, True, K, key, iv, recs, src, got, aad, st)
    oracle.batch(True, key, iv, recs, src, want, aad)
    assert spans(got, recs, 16) == spans(want, recs, 16)
    pt = np.zeros_like(src)
    run(model, False, K, key, iv, recs, got, pt, aad, st)
    assert (st == recs["len"]).all()
    assert spans(pt, recs, 0) == [bytes(src[int(r["src"]): int(r["src"]) + int(r["len"])]) for r in recs]
    got[int(recs[20]["dst"]) + 1] ^= 0x40
    run(model, False, K, key, iv, recs, got, pt, aad, st)
    assert st[20] == 0xFFFFFFFF and (np.delete(st, 20) == np.delete(recs["len"], 20)).all()


@pytest.mark.parametrize("K", ["w16", "split"])
def test_model_long_records_16_lanes(model, K):
    """Records of 1..3 runs of 16 segments and beyond (walked whole): the 16-lane and split kernels' joins and the
    H^8 x H^(8 - j) lane scaling, seal and open against the oracle."""
    rng = np.random.default_rng(77 if K == "w16" else 78)
    lens = np.array([0, 15, 496, 497, 1000, 8150, 8190, 8200, 16383, 16384, 16385, 24000, 24560, 24600, 30000, 40000],
                    np.uint64)
    aadlens = np.array([0, 13, 5, 31, 16, 5, 17, 0, 5, 13, 5, 3, 16, 40, 5, 20], np.uint64)
    recs, src_bytes, aad_bytes = records.layout(lens, aadlens, align=16)
    recs["seq"] = rng.integers(0, 2 ** 63, len(lens), dtype=np.uint64)
    src = rng.integers(0, 256, src_bytes, dtype=np.uint8)
    aad = rng.integers(0, 256, aad_bytes, dtype=np.uint8)
    key = rng.integers(0, 256, 16, dtype=np.uint8).tobytes()
    iv = rng.integers(0, 256, 12, dtype=np.uint8).tobytes()
    got, want = np.zeros_like(src), np.zeros_like(src)
    st = np.zeros(len(recs), np.uint32)
    run(model, True, K, key, iv, recs, src, got, aad, st)
    oracle.batch(True, key, iv, recs, src, want, aad)
    assert spans(got, recs, 16) == spans(want, recs, 16)
    pt = np.zeros_like(src)
    run(model, False, K, key, iv, recs, got, pt, aad, st)
    assert (st == recs["len"]).all()


def test_model_tls_records_all_sizes(model):
    """Every TLS-ish length around block and lane boundaries, in place."""
    lens = np.array(list(range(0, 70)) + [1399, 1400, 1401, 4095, 4096, 4097, 16383, 16384, 16385], dtype=np.uint64)
    recs, src, aad = records.tls_batch(lens, seed=3, align=16)
    key, iv = bytes(range(16)), bytes(range(12))
    for K in (4, 8):
        got = src.copy()
        st = np.zeros(len(recs), np.uint32)
        run(model, True, K, key, iv, recs, got, got, aad, st)  # in place
        want = np.zeros_like(src)
        oracle.batch(True, key, iv, recs, src, want, aad)
        assert spans(got, recs, 16) == spans(want, recs, 16)


def test_key_image_tables(model):
    """The nibble tables in the key image equal H^p * (nibble basis element), via the oracle's multiply."""
    size = model.model_key_image_size()
    buf = C.create_string_buffer(size)
    key = bytes(range(3, 19))
    assert model.model_key_image(key, 16, buf, size) == 0
    raw = buf.raw
    H = raw[240 + 16: 240 + 32]
    assert H == oracle.ecb(key, bytes(16))
    gh = raw[272:]
    rng = np.random.default_rng(1)
    hp = H
    for p in range(1, 9):
        if p > 1:
            hp = oracle.gf128_mul(hp, H)
        tab = np.frombuffer(gh[(p - 1) * 8192: p * 8192], dtype=np.uint8).reshape(32, 16, 16)
        for _ in range(8):
            x = rng.integers(0, 256, 16, dtype=np.uint8)
            acc = np.zeros(16, np.uint8)
            words = x.view("<u4")
            for t in range(32):
                nib = (int(words[t // 8]) >> (4 * (t % 8))) & 0xF
                acc ^= tab[t, nib]
            assert acc.tobytes() == oracle.gf128_mul(x.tobytes(), hp)


def test_record_dtype_matches_header():
    hdr = open(os.path.join(os.path.dirname(os.path.dirname(__file__)), "include", "ptls_mi355x.h")).read()
    body = hdr[hdr.index("typedef struct st_ptls_mi355x_record_t"):]
    body = body[: body.index("}")]
    fields = [ln.split(";")[0].split()[-1] for ln in body.splitlines() if ";" in ln]
    assert fields == list(RECORD_DTYPE.names)


@pytest.mark.parametrize("K", [4, 8])
def test_model_record_beyond_2p16_blocks(model, K):
    """A 1.1 MB record: counters cross 2^16, so the hoisted round-1 constants must be recomputed."""
    lens = np.array([70000 * 16 + 5, 33], dtype=np.uint64)
    recs, src, aad = records.tls_batch(lens, seed=9, align=16)
    key, iv = bytes(range(1, 17)), bytes(range(12))
    got, want = np.zeros_like(src), np.zeros_like(src)
    st = np.zeros(len(recs), np.uint32)
    run(model, True, K, key, iv, recs, src, got, aad, st)
    oracle.batch(True, key, iv, recs, src, want, aad)
    assert spans(got, recs, 16) == spans(want, recs, 16)


def run_tls(lib, is_seal, key, iv, trecs, src, dst, st=None, ty=None, conn=None, window=False):
    """window = 4 / 8: the window kernels' math (64-position segments of that many lanes, joined with H^64)
    instead of the batch walk."""
    vp = C.c_void_p
    if window:  # 4 or 8 lanes per segment (the wide and the latency window kernels); "8s32": 32-position segments
        lanes, _, seglen = str(window).partition("s")
        assert lib.model_set_window_lanes(int(lanes)) > 0
        assert lib.model_set_window_seglen(int(seglen or 64)) > 0
    fn = lib.model_tls_window if window else lib.model_tls_batch
    fn.argtypes = [C.c_int, vp, C.c_size_t, vp, vp, C.c_size_t, vp, vp, vp, vp, vp]
    st = np.zeros(max(len(trecs), 1), np.uint32) if st is None else st
    ty = np.zeros(max(len(trecs), 1), np.uint8) if ty is None else ty
    rc = fn(1 if is_seal else 0, key, len(key), iv, trecs.ctypes.data, len(trecs), src.ctypes.data, dst.ctypes.data,
            st.ctypes.data, ty.ctypes.data, None if conn is None else conn.ctypes.data)
    assert rc == 0
    return st, ty


@pytest.mark.parametrize("window", [False, 4, 8, "8s32"])
@pytest.mark.parametrize("keylen", [16, 32])
def test_model_tls_framing(model, keylen, window):
    """The FRAME walk (header AAD in registers, content-type byte spliced into the tail block) vs the oracle's
    restatement of the picotls record layer, both directions, every fragment length around the block edges."""
    import rapido_amd as ra
    rng = np.random.default_rng(keylen)
    key, iv = rng.integers(0, 256, keylen, dtype=np.uint8).tobytes(), rng.integers(0, 256, 12, dtype=np.uint8).tobytes()
    lens = list(range(0, 40)) + [255, 256, 1399, 1400, 4095, 16383, 16384]
    trecs = np.zeros(len(lens), ra.TLS_RECORD_DTYPE)
    off = woff = 0
    for i, n in enumerate(lens):
        trecs[i] = (off, woff, 1000 + 3 * i, n, [23, 22, 21][i % 3])
        off += n + 3
        woff += n + 22 + 1
    src = rng.integers(0, 256, off + 16, dtype=np.uint8)
    wire = np.zeros(woff + 16, np.uint8)
    run_tls(model, True, key, iv, trecs, src, wire, window=window)
    for t in trecs:
        frag = bytes(src[int(t["src"]): int(t["src"]) + int(t["len"])])
        want = oracle.tls_seal_record(key, iv, int(t["seq"]), int(t["type"]), frag)
        assert bytes(wire[int(t["dst"]): int(t["dst"]) + len(want)]) == want, int(t["len"])
    # receive the same wire: descriptors from the host parser semantics (src = header, len = length field)
    orecs = trecs.copy()
    orecs["src"], orecs["len"] = trecs["dst"], trecs["len"] + 17
    orecs["dst"] = np.cumsum(np.concatenate([[0], (orecs["len"] - 16)[:-1].astype(np.int64)])).astype(np.uint64)
    pt = np.zeros(int(orecs["dst"][-1]) + int(orecs["len"][-1]), np.uint8)
    st, ty = run_tls(model, False, key, iv, orecs, wire, pt, window=window)
    assert list(st[: len(lens)]) == lens and list(ty[: len(lens)]) == list(trecs["type"])
    for t, o in zip(trecs, orecs):
        assert bytes(pt[int(o["dst"]): int(o["dst"]) + int(t["len"])]) == bytes(src[int(t["src"]): int(t["src"]) +
                                                                                    int(t["len"])])


@pytest.mark.parametrize("window", [False, 4, 8, "8s32"])
def test_model_tls_open_padding_and_failures(model, window):
    import rapido_amd as ra
    key, iv = bytes(range(16)), bytes(range(30, 42))
    cases = [(50, 23, 0), (50, 23, 1), (50, 23, 15), (50, 23, 16), (0, 23, 40), (300, 23, 333), (0, 0, 7)]
    wires = [oracle.tls_seal_record(key, iv, 77 + i, t, bytes(k % 255 + 1 for k in range(n)), p)
             for i, (n, t, p) in enumerate(cases)]
    bad = bytearray(oracle.tls_seal_record(key, iv, 99, 23, b"hello world")); bad[9] ^= 1
    short = b"\x17\x03\x03\x00\x0f" + bytes(15)
    wires += [bytes(bad), short]
    seqs = [77 + i for i in range(len(cases))] + [99, 5]
    buf = np.frombuffer(b"".join(wires), np.uint8).copy()
    orecs = np.zeros(len(wires), ra.TLS_RECORD_DTYPE)
    off = dst = 0
    for i, w in enumerate(wires):
        L = (w[3] << 8) | w[4]
        orecs[i] = (off, dst, seqs[i], L, 0)
        off += len(w)
        dst += max(L - 16, 0)
    pt = np.zeros(dst + 16, np.uint8)
    st, ty = run_tls(model, False, key, iv, orecs, buf, pt, window=window)
    for i, w in enumerate(wires):
        want = oracle.tls_open_record(key, iv, seqs[i], w)
        if want == oracle.TLS_BAD_MAC:
            assert st[i] == 0xFFFFFFFF
        elif want == oracle.TLS_NO_TYPE:
            assert st[i] == 0xFFFFFFFE
        else:
            assert st[i] == len(want[0]) and ty[i] == want[1]
            assert bytes(pt[int(orecs[i]["dst"]): int(orecs[i]["dst"]) + st[i]]) == want[0]


@pytest.mark.parametrize("K", [2, 4, 8])
def test_model_every_front_pad(model, K):
    """The same records at output offsets shifted by 0..K-1 blocks: make_walk picks every front padding
    (and trailing-pad chain ends with their H^(pad + g - q_last) scaling) for long and short records."""
    rng = np.random.default_rng(K)
    lens = np.array([0, 5, 16, 100, 1392, 1400, 1401, 4096, 16384, 16368], dtype=np.uint64)
    key, iv = bytes(range(16)), bytes(range(12))
    for shift in range(K):
        recs, src, aad = records.tls_batch(lens, seed=shift + 1, align=256)
        recs["dst"] = recs["dst"] + np.uint64(16 * shift)
        got = np.zeros(len(src) + 256, np.uint8)
        want = np.zeros_like(got)
        st = np.zeros(len(recs), np.uint32)
        run(model, True, K, key, iv, recs, src, got, aad, st)
        oracle.batch(True, key, iv, recs, src, want, aad)
        assert spans(got, recs, 16) == spans(want, recs, 16)
        opened = np.zeros_like(got)
        orecs = recs.copy()
        orecs["src"] = recs["dst"]
        run(model, False, K, key, iv, orecs, got, opened, aad, st)
        assert (st == recs["len"]).all()


@pytest.mark.parametrize("K", [1, 2, 4, 8])
def test_model_hoisted_aad(model, K):
    """AAD hoisting (make_walk): AADs of 0..7 blocks -- seeding the lanes' accumulators before step 0 when
    A <= K, in the grid otherwise -- in front of payloads of every length class, at every output offset
    modulo K blocks, sealed and opened, vs the oracle."""
    rng = np.random.default_rng(40 + K)
    key, iv = rng.integers(0, 256, 16, dtype=np.uint8).tobytes(), rng.integers(0, 256, 12, dtype=np.uint8).tobytes()
    aadlens = [0, 1, 5, 13, 16, 17, 31, 32, 33, 48, 63, 64, 65, 100, 112]
    lens = [0, 1, 15, 16, 17, 100, 1392, 1400, 4096]
    pairs = [(a, n) for a in aadlens for n in lens]
    for shift in range(K):
        recs, src_bytes, aad_bytes = records.layout(np.array([p[1] for p in pairs], np.uint64),
                                                    np.array([p[0] for p in pairs], np.uint64), align=256)
        recs["dst"] = recs["dst"] + np.uint64(16 * shift)  # slots keep >= 112 spare bytes
        recs["seq"] = rng.integers(0, 2 ** 63, len(recs), dtype=np.uint64)
        src = rng.integers(0, 256, src_bytes + 256, dtype=np.uint8)
        aad = rng.integers(0, 256, aad_bytes, dtype=np.uint8)
        got, want = np.zeros_like(src), np.zeros_like(src)
        st = np.zeros(len(recs), np.uint32)
        run(model, True, K, key, iv, recs, src, got, aad, st)
        oracle.batch(True, key, iv, recs, src, want, aad)
        assert spans(got, recs, 16) == spans(want, recs, 16), shift
        orecs = recs.copy()
        orecs["src"] = recs["dst"]
        opened = np.zeros_like(got)
        run(model, False, K, key, iv, orecs, got, opened, aad, st)
        assert (st == recs["len"]).all()
        assert spans(opened, orecs, 0) == [bytes(src[int(r["src"]): int(r["src"]) + int(r["len"])]) for r in recs]


@pytest.mark.parametrize("keylen", [16, 32])
def test_model_bitsliced_keystream(model, keylen):
    """The VALU engine of gcm_bitslice.h (quad layout: Boyar-Peralta S-box as 92 three-input LUTs, DPP
    MixColumns, plane transposes) for 8 counter blocks, against the oracle's AES, including a counter wrap."""
    import struct
    model.model_bs_keystream.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p, C.c_uint32, C.c_void_p]
    rng = np.random.default_rng(keylen + 5)
    for ctr0 in [0, 1, 0xF9, 0xFFFFFFFC] + [int(x) for x in rng.integers(0, 2 ** 32, 6)]:
        key = rng.integers(0, 256, keylen, dtype=np.uint8).tobytes()
        nonce = rng.integers(0, 256, 12, dtype=np.uint8).tobytes()
        out = C.create_string_buffer(128)
        assert model.model_bs_keystream(key, keylen, nonce, ctr0, out) == 0
        want = b"".join(oracle.ecb(key, nonce + struct.pack(">I", (ctr0 + b) & 0xFFFFFFFF)) for b in range(8))
        assert out.raw == want


def test_sbox_circuit_and_lut3_mapping():
    """The Boyar-Peralta circuit and its 3-input-LUT cover (the S-box of the VALU engine) on all 256 inputs."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(__file__))
    for script in ("sbox_circuit.py", "sbox_lut3.py"):
        r = subprocess.run([sys.executable, os.path.join(root, "scripts", script)], capture_output=True, text=True)
        assert r.returncode == 0, r.stdout + r.stderr


def conn_iv(iv: bytes, conn_id: int) -> bytes:
    """rapido's derive_connection_aead_iv (lib/rapido.c:127-133): IV bytes 0..3 ^= BE32(connection_id)."""
    head = (int.from_bytes(iv[:4], "big") ^ conn_id).to_bytes(4, "big")
    return head + iv[4:]


@pytest.mark.parametrize("window", [False, 4, 8, "8s32"])
def test_model_tls_multi_connection_window(model, window):
    """One batch holding the send windows of several connections of a session (same key, per-connection IV and
    seq), sealed and opened in one pass, against the oracle's record layer with each connection's derived IV."""
    import rapido_amd as ra
    key, iv = bytes(range(50, 66)), bytes(range(12))
    conns = [0, 1, 2, 7, 0xFFFFFFFF]
    lens = [16384, 1, 1399, 16384, 300]
    trecs = np.zeros(len(conns) * len(lens), ra.TLS_RECORD_DTYPE)
    conn = np.zeros(len(trecs), np.uint32)
    off = woff = 0
    for k, (c, n) in enumerate((c, n) for c in conns for n in lens):
        trecs[k] = (off, woff, 5 + k % len(lens), n, 23)
        conn[k] = c
        off += n
        woff += n + 22
    src = np.frombuffer(bytes((i * 7 + 3) & 0xFF for i in range(off + 16)), np.uint8).copy()
    wire = np.zeros(woff + 16, np.uint8)
    run_tls(model, True, key, iv, trecs, src, wire, conn=conn, window=window)
    for t, c in zip(trecs, conn):
        frag = bytes(src[int(t["src"]): int(t["src"]) + int(t["len"])])
        want = oracle.tls_seal_record(key, conn_iv(iv, int(c)), int(t["seq"]), 23, frag)
        assert bytes(wire[int(t["dst"]): int(t["dst"]) + len(want)]) == want
    orecs = trecs.copy()
    orecs["src"], orecs["len"] = trecs["dst"], trecs["len"] + 17
    orecs["dst"] = trecs["src"] + np.arange(len(trecs), dtype=np.uint64)  # slots of len + 1 (fragment + type)
    pt = np.zeros(off + len(trecs) + 16, np.uint8)
    st, ty = run_tls(model, False, key, iv, orecs, wire, pt, conn=conn, window=window)
    assert (st[: len(trecs)] == trecs["len"]).all() and (ty[: len(trecs)] == 23).all()
    for t, o in zip(trecs, orecs):
        n, d, s0 = int(t["len"]), int(o["dst"]), int(t["src"])
        assert bytes(pt[d:d + n]) == bytes(src[s0:s0 + n])
    # a record opened under another connection's IV fails
    wrong = conn.copy()
    wrong[3] ^= 1
    st, _ = run_tls(model, False, key, iv, orecs, wire, pt, conn=wrong, window=window)
    assert st[3] == 0xFFFFFFFF and (np.delete(st[: len(trecs)], 3) == np.delete(trecs["len"], 3)).all()


@pytest.mark.parametrize("kw", [4, 8, "8s32"])
def test_model_tls_window_oversized_record(model, kw):
    """A record above the largest TLS record (more than 17 segments) is walked whole by the window kernels' first
    slot: 20 000- and 70 000-byte fragments plus TLS-sized neighbours, against the oracle."""
    import rapido_amd as ra
    key, iv = bytes(range(16)), bytes(range(12))
    lens = [20000, 16384, 70000, 5]
    trecs = np.zeros(len(lens), ra.TLS_RECORD_DTYPE)
    off = woff = 0
    for i, n in enumerate(lens):
        trecs[i] = (off, woff, 9 + i, n, 23)
        off += n
        woff += n + 22
    src = np.frombuffer(bytes((i * 13 + 1) & 0xFF for i in range(off + 16)), np.uint8).copy()
    wire = np.zeros(woff + 16, np.uint8)
    run_tls(model, True, key, iv, trecs, src, wire, window=kw)
    for t in trecs:
        want = oracle.tls_seal_record(key, iv, int(t["seq"]), 23, bytes(src[int(t["src"]): int(t["src"]) + int(t["len"])]))
        assert bytes(wire[int(t["dst"]): int(t["dst"]) + len(want)]) == want


@pytest.mark.parametrize("kw", ["w4", "w8", "w8s32"])
def test_model_window_aead_edges(model, kw):
    """The window math for AEAD records: AAD of every length 0..40 in front of payloads around segment edges
    (so the short AAD sits in later steps of the first segment), records above 17 segments, vs the oracle."""
    rng = np.random.default_rng(31)
    pairs = [(a, l) for a in range(0, 41, 3) for l in (0, 1, 15, 16, 17, 1000, 1007, 1008, 1009, 16384)]
    pairs += [(5, 17 * 1024), (300, 16000), (13, 40000)]
    lens = np.array([p[1] for p in pairs], np.uint64)
    aadlens = np.array([p[0] for p in pairs], np.uint64)
    recs, src_bytes, aad_bytes = records.layout(lens, aadlens, align=16)
    recs["seq"] = rng.integers(0, 2 ** 63, len(recs), dtype=np.uint64)
    src = rng.integers(0, 256, src_bytes, dtype=np.uint8)
    aad = rng.integers(0, 256, aad_bytes, dtype=np.uint8)
    key, iv = bytes(range(16)), bytes(range(12))
    got, want = np.zeros_like(src), np.zeros_like(src)
    st = np.zeros(len(recs), np.uint32)
    run(model, True, kw, key, iv, recs, src, got, aad, st)
    oracle.batch(True, key, iv, recs, src, want, aad)
    assert spans(got, recs, 16) == spans(want, recs, 16)
    pt = np.zeros_like(src)
    run(model, False, kw, key, iv, recs, got, pt, aad, st)
    assert (st == recs["len"]).all()


@pytest.mark.parametrize("keylen", [16, 32])
def test_parallel_key_setup_matches_sequential(model, keylen):
    """mi355x_gcm_setup's steps (wave-parallel power chain, monomial products, table entries) give the key image
    build_key_image builds one bit at a time, byte for byte."""
    size = model.model_key_image_size()
    model.model_key_image_parallel.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t]
    for seed in range(3):
        key = np.random.default_rng(seed + 40).integers(0, 256, keylen, dtype=np.uint8).tobytes()
        a, b = C.create_string_buffer(size), C.create_string_buffer(size)
        assert model.model_key_image(key, keylen, a, size) == 0
        assert model.model_key_image_parallel(key, keylen, b, size) == 0
        assert a.raw == b.raw


def test_gf_mul_xpow_matches_oracle(model):
    """v * x^i for every i (the single-bit products of the key setup) against the oracle's Algorithm-1 multiply."""
    model.model_gf_mul_xpow.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p]
    rng = np.random.default_rng(7)
    for _ in range(4):
        v = rng.integers(0, 256, 16, dtype=np.uint8).tobytes()
        for i in range(128):
            xi = bytearray(16)
            xi[i // 8] = 0x80 >> (i % 8)  # the element x^i (GCM bit i)
            out = C.create_string_buffer(16)
            model.model_gf_mul_xpow(v, i, out)
            assert out.raw == oracle.gf128_mul(v, bytes(xi)), i


@pytest.mark.parametrize("keylen", [16, 32])
def test_model_ecb_block_both_directions(model, keylen):
    """aes_ecb_block (the ECB kernels' code) encrypts like the oracle's FIPS-197 Cipher and decrypts like its
    InvCipher, over random blocks and keys."""
    model.model_aes_ecb.argtypes = [C.c_void_p, C.c_size_t, C.c_int, C.c_void_p, C.c_size_t]
    rng = np.random.default_rng(keylen)
    for _ in range(8):
        key = rng.integers(0, 256, keylen, dtype=np.uint8).tobytes()
        data = rng.integers(0, 256, 16 * 37, dtype=np.uint8).tobytes()
        buf = C.create_string_buffer(data, len(data))
        assert model.model_aes_ecb(key, keylen, 1, buf, 37) == 0
        enc = buf.raw[:len(data)]
        assert enc == oracle.ecb_blocks(key, data, True)
        assert model.model_aes_ecb(key, keylen, 0, buf, 37) == 0
        assert buf.raw[:len(data)] == data
        assert oracle.ecb_blocks(key, enc, False) == data


def test_bitsliced_last_round_matches_sbox(model):
    """aes_last_round_bs2 (gcm_sbox.h: 8x8 bit transposes + the S-box circuit, two blocks per lane) equals
    SubBytes + ShiftRows + AddRoundKey computed byte by byte, on random states and keys."""
    sbox = [oracle.ecb(bytes(16), bytes(16))]  # warm the oracle build
    model.model_last_round_bs2.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
    rng = np.random.default_rng(21)
    # the S-box from the FIPS-197 definition: SubBytes(x) is the first byte of a one-round AES with zero keys
    # would need internals; use the table of the kernel model's own T0 (byte 1 of T0[x] = S[x]) via the oracle
    S = np.zeros(256, np.uint8)
    inv = np.zeros(256, np.uint8)
    for x in range(256):  # multiplicative inverse in GF(2^8), then the affine map (FIPS-197 5.1.1)
        if x:
            for y in range(1, 256):
                a, b, p = x, y, 0
                while b:
                    if b & 1:
                        p ^= a
                    a = ((a << 1) ^ (0x1B if a & 0x80 else 0)) & 0xFF
                    b >>= 1
                if p == 1:
                    inv[x] = y
                    break
        v = int(inv[x])
        r = v
        for k in range(1, 5):
            r ^= ((v << k) | (v >> (8 - k))) & 0xFF
        S[x] = r ^ 0x63
    for _ in range(200):
        a = rng.integers(0, 2 ** 32, 4, dtype=np.uint64).astype(np.uint32)
        b = rng.integers(0, 2 ** 32, 4, dtype=np.uint64).astype(np.uint32)
        k = rng.integers(0, 2 ** 32, 4, dtype=np.uint64).astype(np.uint32)
        want = []
        for st in (a, b):
            by = st.view(np.uint8)  # byte r of column c at 4c + r
            out = np.zeros(16, np.uint8)
            for c in range(4):
                for r in range(4):
                    out[4 * c + r] = S[by[4 * ((c + r) & 3) + r]]
            want.append(out.view(np.uint32) ^ k)
        ga, gb = a.copy(), b.copy()
        model.model_last_round_bs2(ga.ctypes.data, gb.ctypes.data, k.ctypes.data)
        assert (ga == want[0]).all() and (gb == want[1]).all()


@pytest.mark.parametrize("keylen", [16, 32])
def test_gh8_latin_tables_every_read_order(model, keylen):
    """GH8 (the K = 4 batch kernels' Horner multiply, Layout<4>::gh8): X * H^4 through the 8-bit latin table for all 16
    lane read orders (lane & 15: dword swaps and byte permutations) equals the nibble-table product and the oracle's
    Algorithm-1 multiply by H^4."""
    model.model_gh8_mul.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t, C.c_void_p]
    key = bytes(range(7, 7 + keylen))
    H = oracle.ecb(key, bytes(16))
    h4 = oracle.gf128_mul(oracle.gf128_mul(H, H), oracle.gf128_mul(H, H))
    rng = np.random.default_rng(keylen)
    xs = rng.integers(0, 256, (12, 16), dtype=np.uint8)
    xs[0] = 0
    xs[1] = 0xFF
    out = C.create_string_buffer(16 * 17 * len(xs))
    assert model.model_gh8_mul(key, keylen, xs.tobytes(), len(xs), out) == 0
    raw = out.raw
    for n, x in enumerate(xs):
        want = oracle.gf128_mul(x.tobytes(), h4)
        assert raw[16 * (16 * len(xs) + n):16 * (16 * len(xs) + n + 1)] == want
        for i in range(16):
            assert raw[16 * (16 * n + i):16 * (16 * n + i + 1)] == want, (n, i)


@pytest.mark.parametrize("K", [1, 2, 4, 8])
def test_walk_interior_is_exactly_the_whole_payload_steps(model, K):
    """walk_interior (the batch kernels' fast-path range, gcm_core.h) against the walk's own position map: step t of lane j
    is interior iff its position holds a whole payload block taken from the input (c = j + K t - pad - A, 0 <= c < len/16);
    every length, AAD length, output alignment and lane, plus the TLS seal case (GCM payload = fragment + type byte)."""
    fn = model.model_walk_interior
    fn.argtypes = [C.c_uint32] * 6 + [C.c_void_p]
    out = (C.c_uint32 * 6)()
    for frame in (False, True):
        for length in list(range(0, 70)) + [1399, 1400, 1401, 16383, 16384, 16385]:
            plen = length + 1 if frame else length
            for aadlen in ((5,) if frame else (0, 5, 13, 16, 17, 40, 64)):
                for out16 in range(K):
                    for j in range(K):
                        fn(plen, aadlen, K, out16, j, length, out)
                        A, Cn, T, pad, lo, hi = (int(v) for v in out)
                        pad = pad - (1 << 32) if pad >= 1 << 31 else pad
                        assert Cn == (plen + 15) // 16
                        for t in range(T + 2):
                            c = j + K * t - pad - A
                            whole = 0 <= c < length // 16 and t < T
                            assert whole == (lo <= t < hi), (frame, length, aadlen, out16, j, t, lo, hi)
