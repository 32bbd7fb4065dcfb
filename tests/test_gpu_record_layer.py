"""The batched record layer over host buffers (include/ptls_mi355x.h section 5, rapido_amd/csrc/record_layer.c)
against the oracle's TLS 1.3 record functions, which reproduce the reference ptls_send / ptls_receive outputs
(tests/test_tls_records.py, tests/golden/tls_records.json).

A rapido send window is up to 16 records of 16 KiB (lib/rapido.c:2115-2126), each record one cleartext that
rapido_prepare_record produced; a connection's key and IV come from the traffic secret (lib/rapido.c:135-150),
with the connection id XORed into the IV's first four bytes (derive_connection_aead_iv, lib/rapido.c:123-133)."""
import struct

import numpy as np
import pytest

import oracle
import rapido_amd as ra
from conftest import FAMILIES, kernel_family

pytestmark = pytest.mark.gpu


def conn_iv(iv: bytes, conn_id: int) -> bytes:
    """derive_connection_aead_iv (lib/rapido.c:123-133): BE32(first 4 IV bytes) ^ connection id."""
    msb = struct.unpack(">I", iv[:4])[0] ^ conn_id
    return struct.pack(">I", msb) + iv[4:]


def oracle_window(key, iv, seq, frags, ctype=23):
    out = b""
    for f in frags:
        for off in range(0, max(len(f), 1), 16384):
            if not f:
                break
            out += oracle.tls_seal_record(key, iv, seq, ctype, f[off:off + 16384])
            seq += 1
    return out, seq


@pytest.fixture(params=["split", "window16", "batch"])
def family(request, gpu):
    with kernel_family(request.param, framing=True):
        yield request.param


@pytest.fixture(params=["zero_copy", "copy"])
def transport(request, gpu):
    return request.param


def layer(transport, key, iv, seq=0):
    """A record layer whose windows go through the pinned staging zero-copy (the default) or by DMA copies."""
    rl = ra.RecordLayer(key, iv, seq=seq)
    if transport == "copy":
        rl.set_zero_copy_bytes(0)
    return rl


@pytest.mark.parametrize("keylen", [16, 32])
def test_send_window_matches_ptls_send(family, transport, keylen):
    rng = np.random.default_rng(keylen)
    key = rng.integers(0, 256, keylen, dtype=np.uint8).tobytes()
    iv = conn_iv(rng.integers(0, 256, 12, dtype=np.uint8).tobytes(), 3)
    frags = [rng.integers(0, 256, 16384, dtype=np.uint8).tobytes() for _ in range(16)]
    rl = layer(transport, key, iv, seq=41)
    wire, n = rl.seal(frags)
    want, seq = oracle_window(key, iv, 41, frags)
    assert n == 16 and rl.seq == seq == 57
    assert wire == want
    # ragged fragments, one over 16 KiB (two records), empty ones (no record), in the same call
    frags2 = [b"", rng.integers(0, 256, 1, dtype=np.uint8).tobytes(), rng.integers(0, 256, 40000, dtype=np.uint8).tobytes(),
              rng.integers(0, 256, 1399, dtype=np.uint8).tobytes(), b""]
    wire2, n2 = rl.seal(frags2)
    want2, seq2 = oracle_window(key, iv, 57, frags2)
    assert wire2 == want2 and n2 == 1 + 3 + 1 and rl.seq == seq2
    rl.close()


@pytest.mark.parametrize("keylen", [16, 32])
def test_receive_window_round_trip(family, transport, keylen):
    rng = np.random.default_rng(100 + keylen)
    key = rng.integers(0, 256, keylen, dtype=np.uint8).tobytes()
    iv = rng.integers(0, 256, 12, dtype=np.uint8).tobytes()
    frags = [rng.integers(0, 256, int(n), dtype=np.uint8).tobytes() for n in rng.integers(1, 16385, 32)]
    wire, _ = oracle_window(key, iv, 7, frags)
    rx = layer(transport, key, iv, seq=7)
    rc, pt, consumed, n = rx.open(wire)
    assert (rc, consumed, n) == (0, len(wire), 32)
    assert pt == b"".join(frags) and rx.seq == 39
    # a window that ends inside a record: the complete ones only
    wire2, _ = oracle_window(key, iv, 39, frags[:3])
    rc, pt, consumed, n = rx.open(wire2[:-10])
    assert (rc, n) == (0, 2) and consumed == len(oracle_window(key, iv, 39, frags[:2])[0])
    assert pt == frags[0] + frags[1] and rx.seq == 41
    rx.close()


def test_receive_stops_at_first_failure(family, transport):
    """picotls returns the alert of the first bad record and does not advance seq past it (lib/picotls.c:650-652);
    the records before it are delivered."""
    rng = np.random.default_rng(5)
    key, iv = bytes(range(16)), bytes(range(12))
    frags = [rng.integers(0, 256, 3000, dtype=np.uint8).tobytes() for _ in range(8)]
    wire = bytearray(oracle_window(key, iv, 0, frags)[0])
    rec = 5 + 3000 + 1 + 16
    wire[5 * rec + 100] ^= 1  # record 5's ciphertext
    rx = layer(transport, key, iv)
    rc, pt, consumed, n = rx.open(bytes(wire))
    assert rc == 20 and n == 5 and consumed == 5 * rec and pt == b"".join(frags[:5]) and rx.seq == 5
    # the window resent intact from record 5 on continues the stream
    rc, pt, consumed, n = rx.open(oracle_window(key, iv, 5, frags[5:])[0])
    assert rc == 0 and n == 3 and pt == b"".join(frags[5:]) and rx.seq == 8


def test_receive_leaves_other_content_types(family, transport):
    """A handshake record (post-handshake message, inner type 22) or an alert record (outer type 21) ends the
    delivered run: it is left, with its seq, for the caller's picotls path."""
    key, iv = bytes(range(32)), bytes(range(12))
    a, b, c = b"a" * 1000, b"b" * 2000, b"c" * 300
    w_a, s = oracle_window(key, iv, 0, [a])
    w_hs = oracle.tls_seal_record(key, iv, s, 22, b"\x04\x00\x00\x00")
    w_c, _ = oracle_window(key, iv, s + 1, [c])
    rx = layer(transport, key, iv)
    rc, pt, consumed, n = rx.open(w_a + w_hs + w_c)
    assert (rc, pt, consumed, n, rx.seq) == (0, a, len(w_a), 1, 1)
    alert = bytes([21, 3, 3, 0, 2, 2, 40])
    rx.seq = 0
    rc, pt, consumed, n = rx.open(w_a + alert + w_c)
    assert (rc, pt, consumed, n, rx.seq) == (0, a, len(w_a), 1, 1)
    # padding and the all-zero record (no content type: UNEXPECTED_MESSAGE)
    padded = oracle.tls_seal_record(key, iv, 1, 23, b, pad=100)
    nothing = oracle.tls_seal_record(key, iv, 2, 0, b"", pad=8)
    rx.seq = 1
    rc, pt, consumed, n = rx.open(padded + nothing)
    assert (rc, pt, n, rx.seq) == (10, b, 1, 2)


def test_capacity_and_errors(gpu):
    key, iv = bytes(16), bytes(12)
    rl = ra.RecordLayer(key, iv)
    with pytest.raises(RuntimeError):
        rl.seal([b"x" * 100], capacity=100)
    assert rl.seq == 0
    wire, n = rl.seal([b"x" * 100])
    assert n == 1 and len(wire) == 122
    rx = ra.RecordLayer(key, iv)
    with pytest.raises(RuntimeError):
        rx.open(wire, capacity=50)
    assert rx.seq == 0
    rc, pt, consumed, n = rx.open(wire[:3])
    assert (rc, pt, consumed, n) == (0, b"", 0, 0)
    rc, pt, consumed, n = rx.open(bytes([23, 3, 3, 0xff, 0xff]) + bytes(10))
    assert rc == 50 and n == 0  # DECODE_ERROR: length field above 16640


def page_buffer(nbytes: int) -> np.ndarray:
    """A page-aligned uint8 host buffer (a long-lived socket buffer to register)."""
    raw = np.zeros(nbytes + 4096, np.uint8)
    off = (-raw.ctypes.data) % 4096
    return raw[off:off + nbytes]


@pytest.mark.parametrize("keylen", [16, 32])
def test_direct_window_in_registered_buffers(family, keylen):
    """Fragments, wire and plaintext in registered host buffers: the kernels read and write them in place over
    PCIe (no staging copy); same bytes as ptls_send / ptls_receive."""
    rng = np.random.default_rng(200 + keylen)
    key = rng.integers(0, 256, keylen, dtype=np.uint8).tobytes()
    iv = conn_iv(rng.integers(0, 256, 12, dtype=np.uint8).tobytes(), 9)
    sizes = [16384] * 12 + [1, 40000, 1399, 0]
    sendbuf, wirebuf, ptbuf = page_buffer(sum(sizes) + 4096), page_buffer(1 << 20), page_buffer(1 << 20)
    frags, pos = [], 0
    for n in sizes:  # fragments scattered through the send buffer, out of order
        pos += int(rng.integers(0, 64))
        sendbuf[pos:pos + n] = rng.integers(0, 256, n, dtype=np.uint8)
        frags.append(sendbuf[pos:pos + n])
        pos += n
    frags = frags[::-1]
    tx, rx = ra.RecordLayer(key, iv, seq=3), ra.RecordLayer(key, iv, seq=3)
    for b in (sendbuf, wirebuf):
        tx.register(b)
    for b in (wirebuf, ptbuf):
        rx.register(b)
    out = wirebuf[100:]  # an unaligned start inside the registered range
    wlen, nrec = tx.seal_into(frags, out)
    want, seq = oracle_window(key, iv, 3, [f.tobytes() for f in frags])
    assert out[:wlen].tobytes() == want and nrec == seq - 3 and tx.seq == seq
    # open in place: the delivery kernel writes the plaintexts back to back at the start of ptbuf and nothing else
    ptbuf[:] = 0xee
    rc, olen, consumed, n = rx.open_into(out[:wlen], ptbuf)
    assert (rc, consumed, n) == (0, wlen, nrec) and rx.seq == seq
    assert ptbuf[:olen].tobytes() == b"".join(f.tobytes() for f in frags)
    assert (ptbuf[olen:] == 0xee).all()
    # a tampered record: the ones before it delivered, nothing of it or behind it left in the buffer
    rx.seq = 3
    wire = out[:wlen].copy()
    before, seq_before = oracle_window(key, iv, 3, [f.tobytes() for f in frags[:3]])
    tampered = wire.copy()
    tampered[len(before) + 10] ^= 0x80  # the tag of the record of frags[3] (1 byte)
    wirebuf[:wlen] = tampered
    ptbuf[:] = 0xee
    rc, olen, consumed, n = rx.open_into(wirebuf[:wlen], ptbuf)
    assert (rc, n, consumed, rx.seq) == (20, seq_before - 3, len(before), seq_before)
    assert ptbuf[:olen].tobytes() == b"".join(f.tobytes() for f in frags[:3])
    assert (ptbuf[olen:] == 0xee).all()
    # input and output outside the registered ranges: through the staging, same bytes
    plain = np.zeros(wlen, np.uint8)
    rx.seq = 3
    rc, olen2, consumed, n = rx.open_into(wire, plain)
    assert rc == 0 and plain[:olen2].tobytes() == b"".join(f.tobytes() for f in frags)
    tx.unregister(sendbuf)
    with pytest.raises(RuntimeError):
        tx.unregister(sendbuf)
    tx.close()
    rx.close()


@pytest.mark.parametrize("keylen", [16, 32])
def test_seal_multi_session_windows(family, transport, keylen):
    """The send windows of four connections of one session (session key, per-connection IV: the connection id in IV
    bytes 0..3, lib/rapido.c:123-133) sealed in one launch: every connection's wire bytes are its own ptls_send
    output, every seq advances by its record count."""
    rng = np.random.default_rng(300 + keylen)
    key = rng.integers(0, 256, keylen, dtype=np.uint8).tobytes()
    iv = rng.integers(0, 256, 12, dtype=np.uint8).tobytes()
    # (the last connection ends right below ptls_send's 2^24-record key-update limit: its 9 records all go out)
    cids, seqs = [0, 3, 7, 0x01020304], [5, 0, 1000, ra.RECORD_LAYER_SEQ_LIMIT - 9]
    layers = [layer(transport, key, conn_iv(iv, c), seq=s) for c, s in zip(cids, seqs)]
    windows = [[rng.integers(0, 256, 16384, dtype=np.uint8).tobytes() for _ in range(16)],
               [b"", rng.integers(0, 256, 40000, dtype=np.uint8).tobytes()],
               [],
               [rng.integers(0, 256, int(n), dtype=np.uint8).tobytes() for n in rng.integers(1, 3000, 9)]]
    got = ra.record_layer_seal_multi(layers, windows)
    for lr, c, s, w, (wire, n) in zip(layers, cids, seqs, windows, got):
        want, end = oracle_window(key, conn_iv(iv, c), s, w)
        assert wire == want and n == end - s and lr.seq == end
    # a layer of another session (another key) joins the same launch as a multi-key batch: its records are its own
    # ptls_send output under its key (round 6; it used to be refused)
    other = layer(transport, bytes(keylen), conn_iv(iv, 1), seq=9)
    before = [lr.seq for lr in layers[:2]]
    got = ra.record_layer_seal_multi(layers[:2] + [other], windows[:2] + [[b"x" * 10]])
    for lr, c, s, w, (wire, n) in zip(layers[:2], cids[:2], before, windows[:2], got[:2]):
        want, end = oracle_window(key, conn_iv(iv, c), s, w)
        assert wire == want and n == end - s and lr.seq == end
    assert got[2] == (oracle_window(bytes(keylen), conn_iv(iv, 1), 9, [b"x" * 10])[0], 1) and other.seq == 10
    # a layer of another key size cannot share a launch: refused, nothing advanced
    odd = layer(transport, bytes(48 - keylen), conn_iv(iv, 1), seq=9)
    before = [lr.seq for lr in layers]
    with pytest.raises(RuntimeError, match="another key size"):
        ra.record_layer_seal_multi(layers[:2] + [odd], windows[:2] + [[b"x" * 10]])
    assert [lr.seq for lr in layers] == before and odd.seq == 9
    for lr in layers + [other, odd]:
        lr.close()


@pytest.mark.parametrize("nsess", [2, 16])
def test_windows_of_many_sessions_in_one_launch(family, transport, nsess):
    """A server's connections of many sessions -- each session its own traffic key and IV, each connection its own
    IV bytes 0..3 -- sealed in ONE launch (a multi-key batch): every connection's wire bytes are
    its own ptls_send output; then the same windows, one tampered, opened in ONE launch: every connection gets what
    its own ptls_receive would deliver."""
    rng = np.random.default_rng(900 + nsess)
    keylen = 16 if nsess == 2 else 32
    keys = [rng.integers(0, 256, keylen, dtype=np.uint8).tobytes() for _ in range(nsess)]
    ivs = [rng.integers(0, 256, 12, dtype=np.uint8).tobytes() for _ in range(nsess)]
    conns = [(s, c) for s in range(nsess) for c in ((0, 5) if s % 3 == 0 else (1,))]
    rng.shuffle(conns)
    seqs = [int(x) for x in rng.integers(0, 1000, len(conns))]
    tx = [layer(transport, keys[s], conn_iv(ivs[s], c), seq=q) for (s, c), q in zip(conns, seqs)]
    windows = [[rng.integers(0, 256, int(n), dtype=np.uint8).tobytes() for n in rng.integers(0, 16385, k)]
               for k in rng.integers(0, 5, len(conns))]
    windows[0] = [rng.integers(0, 256, 1000, dtype=np.uint8).tobytes(), rng.integers(0, 256, 77, dtype=np.uint8).tobytes()]
    got = ra.record_layer_seal_multi(tx, windows)
    wires = []
    for lr, (s, c), q, w, (wire, n) in zip(tx, conns, seqs, windows, got):
        want, end = oracle_window(keys[s], conn_iv(ivs[s], c), q, w)
        assert wire == want and n == end - q and lr.seq == end, (s, c)
        wires.append(wire)
    rx = [layer(transport, keys[s], conn_iv(ivs[s], c), seq=q) for (s, c), q in zip(conns, seqs)]
    hit = 0
    bad = bytearray(wires[hit])
    first = 5 + len(windows[hit][0]) + 17
    bad[first + 5] ^= 8  # the second record's first ciphertext byte
    wires[hit] = bytes(bad)
    res = ra.record_layer_open_multi(rx, wires)
    for i, (lr, w, (alert, pt, cons, n)) in enumerate(zip(rx, windows, res)):
        if i == hit:
            assert (alert, pt, cons, n) == (20, w[0], first, 1) and lr.seq == seqs[i] + 1
        else:
            nrec = len([f for f in w if f])  # (an empty fragment makes no record)
            assert alert == 0 and pt == b"".join(w) and cons == len(wires[i]) and n == nrec, i
    for lr in tx + rx:
        lr.close()


def test_seal_multi_direct(family):
    """The same, direct: every connection's fragments and output in registered host buffers."""
    rng = np.random.default_rng(400)
    key, iv = rng.integers(0, 256, 16, dtype=np.uint8).tobytes(), rng.integers(0, 256, 12, dtype=np.uint8).tobytes()
    cids = [11, 12, 13]
    layers = [ra.RecordLayer(key, conn_iv(iv, c), seq=c) for c in cids]
    sendbuf, wirebuf = page_buffer(1 << 20), page_buffer(1 << 20)
    sendbuf[:] = rng.integers(0, 256, sendbuf.size, dtype=np.uint8)
    layers[0].register(sendbuf)
    layers[1].register(wirebuf)
    sizes = [[16384, 100, 0], [40000], [1, 2, 3, 16385]]
    windows, pos = [], 0
    for w in sizes:
        frags = []
        for n in w:
            frags.append(sendbuf[pos:pos + n])
            pos += n + 7
        windows.append(frags)
    outs = [wirebuf[300000:600000], wirebuf[17:200000], wirebuf[700000:]]  # out of order in the buffer
    got = ra.record_layer_seal_multi(layers, windows, outs=outs)
    for lr, c, w, o, (wlen, n) in zip(layers, cids, windows, outs, got):
        want, end = oracle_window(key, conn_iv(iv, c), c, [f.tobytes() for f in w])
        assert o[:wlen].tobytes() == want and lr.seq == end and n == end - c
    for lr in layers:
        lr.close()


def test_open_multi_session_windows(family, transport):
    """The receive windows of four connections of one session opened in one launch: each connection gets exactly
    what its own ptls_receive would have delivered, alerts and stops included, and only its seq advances."""
    rng = np.random.default_rng(500)
    key, iv = rng.integers(0, 256, 32, dtype=np.uint8).tobytes(), rng.integers(0, 256, 12, dtype=np.uint8).tobytes()
    cids, seqs = [2, 9, 0x7fffffff, 40], [0, 17, 5, 2 ** 33]
    layers = [layer(transport, key, conn_iv(iv, c), seq=s) for c, s in zip(cids, seqs)]
    frags = [[rng.integers(0, 256, int(n), dtype=np.uint8).tobytes() for n in rng.integers(1, 16385, k)]
             for k in (16, 3, 0, 5)]
    wires = [oracle_window(key, conn_iv(iv, c), s, f)[0] for c, s, f in zip(cids, seqs, frags)]
    # connection 1: its second record tampered (delivers the first, alert 20); connection 3: ends inside a record
    bad = bytearray(wires[1])
    first = 5 + len(frags[1][0]) + 17
    bad[first + 5] ^= 4  # the first ciphertext byte of record 2
    wires[1] = bytes(bad)
    wires[3] = wires[3][:-9]
    got = ra.record_layer_open_multi(layers, wires)
    assert got[0] == (0, b"".join(frags[0]), len(wires[0]), 16) and layers[0].seq == 16
    assert got[1] == (20, frags[1][0], first, 1) and layers[1].seq == 18
    assert got[2] == (0, b"", 0, 0) and layers[2].seq == 5
    whole4 = len(oracle_window(key, conn_iv(iv, 40), 2 ** 33, frags[3][:4])[0])
    assert got[3] == (0, b"".join(frags[3][:4]), whole4, 4) and layers[3].seq == 2 ** 33 + 4
    for lr in layers:
        lr.close()


def test_prepare_copies_then_copy_windows(gpu):
    """ptls_mi355x_prepare_copies is idempotent, and the copy windows after it are the oracle's (it only warms the
    runtime: DESIGN.md section 2, coalesced DMA streams)."""
    ra.prepare_copies()
    ra.prepare_copies()
    rng = np.random.default_rng(7)
    key = rng.integers(0, 256, 16, dtype=np.uint8).tobytes()
    iv = rng.integers(0, 256, 12, dtype=np.uint8).tobytes()
    frags = [rng.integers(0, 256, 16384, dtype=np.uint8).tobytes() for _ in range(8)]
    rl = layer("copy", key, iv)
    wire, n = rl.seal(frags)
    assert (wire, n) == (oracle_window(key, iv, 0, frags)[0], 8)
    rl.close()
