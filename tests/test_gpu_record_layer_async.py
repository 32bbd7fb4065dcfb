"""The record layer's asynchronous windows, the 2^24-record key-update limit, open_record and rekey
(include/ptls_mi355x.h section 5, rapido_amd/csrc/record_layer.c), on every transport: direct (registered host
buffers read and written in place by the kernels), direct_dma (moved by DMA to and from device memory), zero-copy
(pinned staging) and copy (staging + DMA).

Every wire byte is checked against the oracle's TLS 1.3 record functions, which reproduce the reference ptls_send /
ptls_receive (tests/test_tls_records.py, tests/golden/tls_records.json).  The limit follows ptls_send
(lib/picotls.c:4969-4988): a call starting at seq >= 2^24 first sends a KeyUpdate (update_send_key, :4949-4962,
sealed under the old key at that seq) and continues under the next key from seq 0; the check is at the start of a
call, so a fragment that starts below the limit is sealed whole."""
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

import oracle
import rapido_amd as ra
from conftest import kernel_family
from test_gpu_record_layer import conn_iv, oracle_window, page_buffer

pytestmark = pytest.mark.gpu

# direct: registered buffers read in place by the kernels, plaintexts written by the delivery kernel (the default);
# direct_dma: registered buffers moved by DMA around a device-resident launch; direct_dma_in: the inputs moved by DMA,
# the outputs written in place (seal's wire records, an open's delivery kernel); zero_copy / copy: the layer's staging
TRANSPORTS = ["direct", "direct_dma", "direct_dma_in", "zero_copy", "copy"]
LIMIT = ra.RECORD_LAYER_SEQ_LIMIT
KEY_UPDATE_MSG = bytes([24, 0, 0, 1, 0])  # handshake KeyUpdate, update_not_requested (RFC 8446 sec. 4.6.3)


class Host:
    """Host buffers for one transport: registered page-aligned ranges (direct) or plain arrays (staging)."""

    def __init__(self, transport, layers, nbytes):
        self.transport, self.layers = transport, layers
        self.buf = page_buffer(nbytes)
        self.pos = 0
        if transport.startswith("direct"):
            for rl in layers:
                rl.register(self.buf)
                rl.set_direct_dma(ra.RECORD_LAYER_DMA_IN if transport == "direct_dma_in" else transport == "direct_dma")
        for rl in layers:
            if transport == "copy":
                rl.set_zero_copy_bytes(0)

    def take(self, n, fill=None):
        """n bytes of the buffer (64-B aligned pieces, so windows do not share lines by accident)"""
        v = self.buf[self.pos:self.pos + n]
        self.pos += (n + 63) & ~63
        assert self.pos <= self.buf.size
        if fill is not None:
            v[:] = np.frombuffer(fill, np.uint8) if isinstance(fill, (bytes, bytearray)) else fill
        return v


def oracle_windows_parallel(key, iv, seq, windows):
    """oracle_window over many windows on 8 threads (the C oracle releases the GIL): wire bytes per window"""
    seqs, s = [], seq
    for w in windows:
        seqs.append(s)
        s += sum(max(1, -(-len(f) // 16384)) if f else 0 for f in w)
    with ThreadPoolExecutor(8) as ex:
        return list(ex.map(lambda a: oracle_window(key, iv, a[0], a[1])[0], zip(seqs, windows)))


@pytest.mark.parametrize("transport", TRANSPORTS)
def test_key_update_limit(gpu, transport):
    rng = np.random.default_rng(2024)
    key, key2 = rng.integers(0, 256, 16, dtype=np.uint8).tobytes(), rng.integers(0, 256, 16, dtype=np.uint8).tobytes()
    iv, iv2 = conn_iv(rng.integers(0, 256, 12, dtype=np.uint8).tobytes(), 5), rng.integers(0, 256, 12, dtype=np.uint8).tobytes()
    frags_b = [rng.integers(0, 256, 1000 + 37 * i, dtype=np.uint8).tobytes() for i in range(16)]
    tx, rx = ra.RecordLayer(key, iv, seq=LIMIT - 3), ra.RecordLayer(key, iv, seq=LIMIT - 3)
    h = Host(transport, [tx, rx], 1 << 21)
    frags = [h.take(len(f), f) for f in frags_b]
    # a 16-record window at 2^24 - 3: three fragments sealed, the window stops at the limit
    out = h.take(1 << 17)
    olen, nrec = tx.seal_into(frags, out)
    want3, _ = oracle_window(key, iv, LIMIT - 3, frags_b[:3])
    assert tx.key_update and nrec == 3 and out[:olen].tobytes() == want3 and tx.seq == LIMIT
    # nothing more of type 23 under this key
    out0 = h.take(1 << 12)
    assert tx.seal_into(frags[3:4], out0) == (0, 0) and tx.key_update and tx.seq == LIMIT
    # the KeyUpdate message itself goes out at 2^24 under the old key (update_send_key)
    ku = h.take(len(KEY_UPDATE_MSG), KEY_UPDATE_MSG)
    out_ku = h.take(64)
    olen_ku, n_ku = tx.seal_into([ku], out_ku, content_type=22)
    assert not tx.key_update and n_ku == 1 and tx.seq == LIMIT + 1
    assert out_ku[:olen_ku].tobytes() == oracle.tls_seal_record(key, iv, LIMIT, 22, KEY_UPDATE_MSG)
    # the next traffic key: seq restarts at 0, the rest of the window follows
    tx.rekey(key2, iv2)
    assert tx.seq == 0
    out2 = h.take(1 << 17)
    olen2, nrec2 = tx.seal_into(frags[3:], out2)
    want13, _ = oracle_window(key2, iv2, 0, frags_b[3:])
    assert not tx.key_update and nrec2 == 13 and out2[:olen2].tobytes() == want13 and tx.seq == 13
    # the receiver: three records, stop at the handshake record, open_record hands it over, rekey, the rest
    wire_b = out[:olen].tobytes() + out_ku[:olen_ku].tobytes() + out2[:olen2].tobytes()
    wire = h.take(len(wire_b), wire_b)
    pt = h.take(len(wire_b))
    rc, plen, cons, n = rx.open_into(wire, pt)
    assert (rc, n, cons) == (0, 3, olen) and pt[:plen].tobytes() == b"".join(frags_b[:3]) and rx.seq == LIMIT
    rc, msg, cons_ku, ctype = rx.open_record(wire_b[cons:])
    assert (rc, msg, cons_ku, ctype) == (0, KEY_UPDATE_MSG, olen_ku, 22) and rx.seq == LIMIT + 1
    rx.rekey(key2, iv2)
    rc, plen, cons2, n = rx.open_into(wire[cons + cons_ku:], pt)
    assert (rc, n, cons2) == (0, 13, olen2) and pt[:plen].tobytes() == b"".join(frags_b[3:]) and rx.seq == 13
    # ptls_send checks the limit at its start: a 40000-byte fragment starting at 2^24 - 1 is sealed whole
    tx.seq = LIMIT - 1
    tx.rekey(key, iv)
    tx.seq = LIMIT - 1
    big_b = rng.integers(0, 256, 40000, dtype=np.uint8).tobytes()
    big = h.take(len(big_b), big_b)
    out3 = h.take(1 << 16)
    olen3, nrec3 = tx.seal_into([big, frags[0]], out3)
    want_big, _ = oracle_window(key, iv, LIMIT - 1, [big_b])
    assert tx.key_update and nrec3 == 3 and out3[:olen3].tobytes() == want_big and tx.seq == LIMIT + 2
    for rl in (tx, rx):
        rl.close()


def test_key_update_limit_multi(gpu):
    """seal_multi: each connection stops at its own limit; the others seal their whole windows."""
    rng = np.random.default_rng(2025)
    key = rng.integers(0, 256, 32, dtype=np.uint8).tobytes()
    iv = rng.integers(0, 256, 12, dtype=np.uint8).tobytes()
    ivs = [conn_iv(iv, c) for c in range(3)]
    seqs = [LIMIT - 2, 7, LIMIT]
    layers = [ra.RecordLayer(key, ivs[c], seq=seqs[c]) for c in range(3)]
    windows = [[rng.integers(0, 256, 500 + 100 * i, dtype=np.uint8).tobytes() for i in range(4)] for _ in range(3)]
    got = ra.record_layer_seal_multi(layers, windows)
    assert got[0] == (oracle_window(key, ivs[0], LIMIT - 2, windows[0][:2])[0], 2) and layers[0].seq == LIMIT
    assert got[1] == (oracle_window(key, ivs[1], 7, windows[1])[0], 4) and layers[1].seq == 11
    assert got[2] == (b"", 0) and layers[2].seq == LIMIT
    for rl in layers:
        rl.close()


def _stream(transport, nwin, depth, key, iv, rng):
    """nwin windows of 16 x 16 KiB through seal_submit / wait and open_submit / wait, `depth` in flight"""
    WIN, FRAG = 16, 16384
    tx, rx = ra.RecordLayer(key, iv), ra.RecordLayer(key, iv)
    h = Host(transport, [tx, rx], nwin * WIN * (3 * FRAG + 192) + (1 << 20))
    frags_b = [[rng.integers(0, 256, FRAG, dtype=np.uint8).tobytes() for _ in range(WIN)] for _ in range(nwin)]
    frags = [[h.take(FRAG, f) for f in w] for w in frags_b]
    wire_win = WIN * (FRAG + ra.TLS_OVERHEAD)
    wires = [h.take(wire_win) for _ in range(nwin)]
    pts = [h.take(WIN * (FRAG + 1)) for _ in range(nwin)]
    tickets, done = [], []
    for w in range(nwin):
        if len(tickets) == depth:
            done.append(tx.wait(tickets.pop(0)))
        tickets.append(tx.seal_submit(frags[w], wires[w]))
        assert tx.seq == WIN * (w + 1) and tx.pending == len(tickets)
    done += [tx.wait(t) for t in tickets]
    assert done == [(wire_win, WIN, WIN, 0)] * nwin and tx.pending == 0
    want = oracle_windows_parallel(key, iv, 0, frags_b)
    for w in range(nwin):
        assert wires[w].tobytes() == want[w], f"window {w}"
    tickets, done = [], []
    for w in range(nwin):
        if len(tickets) == depth:
            done.append(rx.wait(tickets.pop(0)))
        t, parsed = rx.open_submit(wires[w], pts[w])
        assert parsed == wire_win
        tickets.append(t)
    done += [rx.wait(t) for t in tickets]
    assert done == [(WIN * FRAG, WIN, wire_win, 0)] * nwin and rx.seq == nwin * WIN
    for w in range(nwin):
        assert pts[w][:WIN * FRAG].tobytes() == b"".join(frags_b[w]), f"window {w}"
    tx.close()
    rx.close()


@pytest.mark.parametrize("transport", TRANSPORTS)
def test_async_stream_matches_oracle(gpu, transport):
    """64 back-to-back rapido send windows, 4 in flight, then their receive windows: every wire byte is
    ptls_send's, every plaintext comes back."""
    rng = np.random.default_rng(64)
    _stream(transport, 64, 4, rng.integers(0, 256, 16, dtype=np.uint8).tobytes(),
            rng.integers(0, 256, 12, dtype=np.uint8).tobytes(), rng)


def test_layers_on_concurrent_threads(gpu):
    """A layer is used by one thread at a time (include/ptls_mi355x.h section 5); four threads stream windows through
    their own layer pairs at once, one transport each (ctypes releases the GIL, so the calls overlap), sharing the
    process-wide registration table, the copy warm-up and the device: every wire byte and plaintext against the
    oracle."""
    def one(t):
        rng = np.random.default_rng(700 + t)
        _stream(["direct", "direct_dma_in", "zero_copy", "copy"][t], 12, 4,
                rng.integers(0, 256, 16 * (1 + t % 2), dtype=np.uint8).tobytes(),
                rng.integers(0, 256, 12, dtype=np.uint8).tobytes(), rng)
    with ThreadPoolExecutor(4) as ex:
        for f in [ex.submit(one, t) for t in range(4)]:
            f.result()


@pytest.mark.parametrize("family", ["split", "window16", "batch"])
def test_async_stream_families(gpu, family):
    rng = np.random.default_rng(65)
    with kernel_family(family, framing=True):
        _stream("direct", 6, 3, rng.integers(0, 256, 32, dtype=np.uint8).tobytes(),
                rng.integers(0, 256, 12, dtype=np.uint8).tobytes(), rng)


@pytest.mark.parametrize("coalesce", [0, 16])
@pytest.mark.parametrize("transport", TRANSPORTS)
def test_async_open_stale_after_failure(gpu, transport, coalesce):
    """Windows in flight behind a window that stops early (a bad record) complete STALE with nothing delivered;
    resubmitted from the stop they open normally.  Without coalescing, four launches are the limit."""
    rng = np.random.default_rng(99)
    key, iv = rng.integers(0, 256, 16, dtype=np.uint8).tobytes(), rng.integers(0, 256, 12, dtype=np.uint8).tobytes()
    rx = ra.RecordLayer(key, iv, seq=100)
    rx.set_coalesce(coalesce)
    h = Host(transport, [rx], 1 << 21)
    frags = [[rng.integers(0, 256, 700 + 13 * i, dtype=np.uint8).tobytes() for i in range(8)] for _ in range(4)]
    wires_b = oracle_windows_parallel(key, iv, 100, frags)
    rec_bounds = []  # wire offsets of window 1's records
    off = 0
    for f in frags[1]:
        rec_bounds.append(off)
        off += len(f) + ra.TLS_OVERHEAD
    bad = bytearray(wires_b[1])
    bad[rec_bounds[2] + 9] ^= 1  # ciphertext of record 2 of window 1
    wires = [h.take(len(w), w) for w in (wires_b[0], bytes(bad), wires_b[2], wires_b[3])]
    pts = [h.take(len(w)) for w in wires_b]
    tickets = [rx.open_submit(wires[w], pts[w])[0] for w in range(4)]
    if coalesce == 0:
        with pytest.raises(RuntimeError):
            rx.open_submit(wires[0], pts[0])  # all four launch slots in flight
    with pytest.raises(RuntimeError):
        rx.wait(tickets[1])  # completion is in submission order
    with pytest.raises(RuntimeError):
        rx.open(wires_b[0])  # a synchronous window behind asynchronous ones
    r0 = rx.wait(tickets[0])
    assert r0 == (sum(map(len, frags[0])), 8, len(wires_b[0]), 0) and pts[0][:r0[0]].tobytes() == b"".join(frags[0])
    r1 = rx.wait(tickets[1])
    assert r1 == (sum(map(len, frags[1][:2])), 2, rec_bounds[2], 20) and rx.seq == 110
    assert pts[1][:r1[0]].tobytes() == b"".join(frags[1][:2])
    for w in (2, 3):
        assert rx.wait(tickets[w]) == (0, 0, 0, ra.RECORD_LAYER_STALE)
    assert rx.seq == 110 and rx.pending == 0
    # resubmitted from the stop (the intact bytes of window 1 from record 2, then windows 2 and 3)
    tail = h.take(len(wires_b[1]) - rec_bounds[2], wires_b[1][rec_bounds[2]:])
    outs = [h.take(len(wires_b[1])) for _ in range(3)]
    tickets = [rx.open_submit(x, o)[0] for x, o in zip((tail, wires[2], wires[3]), outs)]
    res = [rx.wait(t) for t in tickets]
    assert [r[1] for r in res] == [6, 8, 8] and all(r[3] == 0 for r in res) and rx.seq == 132
    assert outs[0][:res[0][0]].tobytes() == b"".join(frags[1][2:])
    assert outs[2][:res[2][0]].tobytes() == b"".join(frags[3])
    rx.close()


def test_async_rekey_and_free_with_pending(gpu):
    rng = np.random.default_rng(7)
    key, iv = rng.integers(0, 256, 16, dtype=np.uint8).tobytes(), rng.integers(0, 256, 12, dtype=np.uint8).tobytes()
    tx = ra.RecordLayer(key, iv)
    h = Host("zero_copy", [tx], 1 << 20)
    f = h.take(5000, rng.integers(0, 256, 5000, dtype=np.uint8))
    t = tx.seal_submit([f], h.take(8192))
    with pytest.raises(RuntimeError):
        tx.rekey(key, iv)  # a window outstanding
    assert tx.wait(t)[:2] == (5000 + ra.TLS_OVERHEAD, 1)
    tx.rekey(key, iv)
    tx.seal_submit([f], h.take(8192))
    tx.close()  # frees with a window never waited for


@pytest.mark.parametrize("transport", ["direct", "direct_dma_in", "zero_copy"])
def test_one_connection_windows_in_one_launch(gpu, transport):
    """A layer given several times in one _multi call: its consecutive windows in one launch, each behind the one
    before (the same bytes as one seal after another); a receive window that stops early leaves the same
    connection's windows behind it STALE, the other connection's window unaffected."""
    rng = np.random.default_rng(31)
    key, iv = rng.integers(0, 256, 16, dtype=np.uint8).tobytes(), rng.integers(0, 256, 12, dtype=np.uint8).tobytes()
    iv0, iv1 = conn_iv(iv, 0), conn_iv(iv, 1)
    tx, other = ra.RecordLayer(key, iv0, seq=5), ra.RecordLayer(key, iv1, seq=70)
    h = Host(transport, [tx, other], 1 << 22)
    wins_b = [[rng.integers(0, 256, int(n), dtype=np.uint8).tobytes() for n in rng.integers(1, 16385, k)]
              for k in (16, 3, 9, 5)]
    wins = [[h.take(len(f), f) for f in w] for w in wins_b]
    outs = [h.take(sum(len(f) + ra.TLS_OVERHEAD for f in w)) for w in wins_b]
    layers = [tx, other, tx, tx]
    got = ra.record_layer_seal_multi(layers, wins, outs=outs)
    want0, s = oracle_window(key, iv0, 5, wins_b[0])
    want2, s = oracle_window(key, iv0, s, wins_b[2])
    want3, s = oracle_window(key, iv0, s, wins_b[3])
    want1, s1 = oracle_window(key, iv1, 70, wins_b[1])
    for o, (wlen, n), want, k in zip(outs, got, (want0, want1, want2, want3), (16, 3, 9, 5)):
        assert o[:wlen].tobytes() == want and n == k
    assert tx.seq == s == 5 + 30 and other.seq == s1
    # the receiver: window 0 of connection 0 has a bad record 4, so its windows 2 and 3 come back STALE
    rx, rx1 = ra.RecordLayer(key, iv0, seq=5), ra.RecordLayer(key, iv1, seq=70)
    bad = bytearray(want0)
    r4 = sum(len(f) + ra.TLS_OVERHEAD for f in wins_b[0][:4])
    bad[r4 + 7] ^= 2
    res = ra.record_layer_open_multi([rx, rx1, rx, rx], [bytes(bad), want1, want2, want3])
    assert res[0] == (20, b"".join(wins_b[0][:4]), r4, 4)
    assert res[1] == (0, b"".join(wins_b[1]), len(want1), 3) and rx1.seq == s1
    assert [r[0] for r in res[2:]] == [ra.RECORD_LAYER_STALE] * 2 and [r[3] for r in res[2:]] == [0, 0]
    assert rx.seq == 9
    # resent intact, the three windows of connection 0 in one launch
    rx.seq = 5
    res = ra.record_layer_open_multi([rx, rx, rx], [want0, want2, want3])
    assert [r[:2] for r in res] == [(0, b"".join(wins_b[k])) for k in (0, 2, 3)] and rx.seq == 35
    for rl in (tx, other, rx, rx1):
        rl.close()


@pytest.mark.parametrize("transport", ["direct", "direct_dma_in"])
def test_seal_output_over_its_fragments(gpu, transport):
    """A window sealed over its own fragments (the output range starts at the first fragment): direct mode takes the
    staging for it, DMA-in copies the fragments to the device first; both give ptls_send's bytes."""
    rng = np.random.default_rng(77)
    key, iv = rng.integers(0, 256, 16, dtype=np.uint8).tobytes(), rng.integers(0, 256, 12, dtype=np.uint8).tobytes()
    tx = ra.RecordLayer(key, iv, seq=11)
    h = Host(transport, [tx], 1 << 20)
    frags_b = [rng.integers(0, 256, n, dtype=np.uint8).tobytes() for n in (16384, 3000, 1, 16384)]
    region = h.take(sum(len(f) + ra.TLS_OVERHEAD for f in frags_b))
    frags, pos = [], 0
    for f in frags_b:
        region[pos:pos + len(f)] = np.frombuffer(f, np.uint8)
        frags.append(region[pos:pos + len(f)])
        pos += len(f)
    olen, nrec = tx.seal_into(frags, region)
    want, seq = oracle_window(key, iv, 11, frags_b)
    assert region[:olen].tobytes() == want and nrec == 4 and tx.seq == seq
    tx.close()


@pytest.mark.parametrize("transport", ["direct", "zero_copy"])
def test_free_and_rekey_of_a_layer_named_by_another_layers_window(gpu, transport):
    """A window led by layer A that also names layer B (a multi-layer submit): B cannot be rekeyed or used
    synchronously while it is in flight; B freed meanwhile (its registered range unregistered after the device has
    finished with it) completes STALE in A's wait, with A's part delivered and bit-exact."""
    rng = np.random.default_rng(404)
    key, iv = rng.integers(0, 256, 16, dtype=np.uint8).tobytes(), rng.integers(0, 256, 12, dtype=np.uint8).tobytes()
    a, b = ra.RecordLayer(key, conn_iv(iv, 0), seq=3), ra.RecordLayer(key, conn_iv(iv, 1), seq=40)
    h = Host(transport, [b, a], 1 << 21)  # direct: the range is B's own registration (A reuses it)
    wins_b = [[rng.integers(0, 256, n, dtype=np.uint8).tobytes() for n in (16384, 999, 5)] for _ in range(2)]
    wins = [[h.take(len(f), f) for f in w] for w in wins_b]
    outs = [h.take(sum(len(f) + ra.TLS_OVERHEAD for f in w)) for w in wins_b]
    t = ra.record_layer_seal_submit_multi([a, b], wins, outs)
    assert b.pending == 0  # the window is on A's queue ...
    with pytest.raises(RuntimeError):
        b.rekey(key, conn_iv(iv, 1))  # ... but names B
    with pytest.raises(RuntimeError):
        b.seal([wins_b[1][0]])
    b.close()
    res = a.wait_multi(t, 2)
    want, s = oracle_window(key, conn_iv(iv, 0), 3, wins_b[0])
    assert res[0][:2] == (len(want), 3) and outs[0][:len(want)].tobytes() == want and a.seq == s
    assert res[1] == (0, 0, 0, ra.RECORD_LAYER_STALE)
    a.close()


def test_open_windows_waited_out_of_order_across_leads(gpu):
    """Layer B's receive windows in two submits led by different layers, the later one waited first: it comes back
    STALE for B, the earlier one delivers, and B's next window opens normally (its speculative position resyncs once
    nothing names it in flight)."""
    rng = np.random.default_rng(505)
    key, iv = rng.integers(0, 256, 16, dtype=np.uint8).tobytes(), rng.integers(0, 256, 12, dtype=np.uint8).tobytes()
    ivs = [conn_iv(iv, c) for c in range(3)]
    frags = [[rng.integers(0, 256, n, dtype=np.uint8).tobytes() for n in (3000, 17, 16384)] for _ in range(4)]
    w_a, _ = oracle_window(key, ivs[0], 0, frags[0])
    w_b1, sb = oracle_window(key, ivs[1], 9, frags[1])
    w_b2, sb2 = oracle_window(key, ivs[1], sb, frags[2])
    w_c, _ = oracle_window(key, ivs[2], 0, frags[3])
    a, b, c = ra.RecordLayer(key, ivs[0]), ra.RecordLayer(key, ivs[1], seq=9), ra.RecordLayer(key, ivs[2])
    arr = [np.frombuffer(w, np.uint8).copy() for w in (w_a, w_b1, w_c, w_b2)]
    outs = [np.zeros(len(w), np.uint8) for w in arr]
    t1, _ = ra.record_layer_open_submit_multi([a, b], arr[:2], outs[:2])
    t2, _ = ra.record_layer_open_submit_multi([c, b], arr[2:], outs[2:])
    r2 = c.wait_multi(t2, 2)
    assert r2[0][3] == 0 and outs[2][:r2[0][0]].tobytes() == b"".join(frags[3])
    assert r2[1] == (0, 0, 0, ra.RECORD_LAYER_STALE)  # B's first window was not delivered yet
    r1 = a.wait_multi(t1, 2)
    assert r1[1][:2] == (sum(map(len, frags[1])), 3) and b.seq == sb
    # B's second window again, alone: delivered (before the fix its submits stayed STALE until set_seq)
    alert, pt, cons, n = ra.record_layer_open_multi([b], [w_b2])[0]
    assert (alert, n, cons) == (0, 3, len(w_b2)) and pt == b"".join(frags[2]) and b.seq == sb2
    for rl in (a, b, c):
        rl.close()


@pytest.mark.parametrize("transport", ["direct", "direct_dma_in", "zero_copy", "copy"])
def test_coalesced_windows_of_one_connection(gpu, transport):
    """One window per submit, 12 submits without a wait: the windows queued while the layer's launch runs go out
    together (fewer launches than windows), with every ticket's results, the wire bytes and seq exactly those of 12
    separate ptls_send windows; then opened the same way (one window per submit) back to their fragments; with
    coalescing off every window is a launch of its own."""
    rng = np.random.default_rng(808)
    key, iv = rng.integers(0, 256, 16, dtype=np.uint8).tobytes(), rng.integers(0, 256, 12, dtype=np.uint8).tobytes()
    nwin = 12
    wins_b = [[rng.integers(0, 256, int(n), dtype=np.uint8).tobytes() for n in rng.integers(0, 16385, 6)]
              for _ in range(nwin)]
    wants, s = [], 40
    for w in wins_b:
        want, s = oracle_window(key, iv, s, w)
        wants.append(want)
    for coalesce in (16, 0):
        tx, rx = ra.RecordLayer(key, iv, seq=40), ra.RecordLayer(key, iv, seq=40)
        for rl in (tx, rx):
            rl.set_coalesce(coalesce)
        h = Host(transport, [tx, rx], 1 << 23)
        wins = [[h.take(len(f), f) for f in w] for w in wins_b]
        outs = [h.take(len(want) + 64) for want in wants]
        l0 = tx.launches
        if coalesce:
            tx.cork(True)  # a burst known to follow: queued, then one launch (uncorked: queued while one runs)
            tickets = [tx.seal_submit(w, o) for w, o in zip(wins, outs)]
            assert tx.seq == s and tx.pending == nwin  # records take their seq at submit, queued or not
            tx.cork(False)
            res = [tx.wait(t) for t in tickets]
        else:  # a launch per window: at most four in flight
            res, tickets = [], []
            for w, o in zip(wins, outs):
                if len(tickets) == 4:
                    res.append(tx.wait(tickets.pop(0)))
                tickets.append(tx.seal_submit(w, o))
            res += [tx.wait(t) for t in tickets]
        for r, o, want, w in zip(res, outs, wants, wins_b):
            assert r == (len(want), sum(max(1, -(-len(f) // 16384)) if f else 0 for f in w), len(w), 0)
            assert o[:len(want)].tobytes() == want
        assert tx.launches - l0 == (nwin if coalesce == 0 else 1)
        wires = [h.take(len(want), want) for want in wants]
        pts = [h.take(len(want)) for want in wants]
        l0 = rx.launches
        pending = []

        def check(t, p, w, want):
            r = rx.wait(t)
            assert r == (sum(map(len, w)), sum(max(1, -(-len(f) // 16384)) if f else 0 for f in w), len(want), 0)
            assert p[:r[0]].tobytes() == b"".join(w)

        for x, p, w, want in zip(wires, pts, wins_b, wants):  # uncorked: queued only while a launch runs
            if coalesce == 0 and len(pending) == 4:
                check(*pending.pop(0))
            t, parsed = rx.open_submit(x, p)
            assert parsed == len(want)  # parsed at submit
            pending.append((t, p, w, want))
        for args in pending:
            check(*args)
        assert rx.seq == s and rx.pending == 0 and 1 <= rx.launches - l0 <= nwin
        tx.close()
        rx.close()


def test_coalesced_open_stops_and_flush(gpu):
    """Coalesced receive windows: a bad record in window 2 stops it (alert 20), windows 3.. come back STALE; the
    layer's queue can be launched early (flush), and windows resubmitted from the stop open normally."""
    rng = np.random.default_rng(909)
    key, iv = rng.integers(0, 256, 32, dtype=np.uint8).tobytes(), rng.integers(0, 256, 12, dtype=np.uint8).tobytes()
    frags = [[rng.integers(0, 256, n, dtype=np.uint8).tobytes() for n in (1000, 16384, 77)] for _ in range(6)]
    wires, s = [], 7
    for f in frags:
        w, s = oracle_window(key, iv, s, f)
        wires.append(w)
    rx = ra.RecordLayer(key, iv, seq=7)
    bad = bytearray(wires[2])
    bad[1022 + 300] ^= 4  # record 1 of window 2 (record 0: 5 + 1000 + 1 + 16 bytes)
    arr = [np.frombuffer(w, np.uint8).copy() for w in wires[:2] + [bytes(bad)] + wires[3:]]
    outs = [np.zeros(len(w), np.uint8) for w in wires]
    tickets = [rx.open_submit(a, o)[0] for a, o in zip(arr, outs)]
    rx.flush()
    res = [rx.wait(t) for t in tickets]
    assert [r[3] for r in res] == [0, 0, 20] + [ra.RECORD_LAYER_STALE] * 3
    assert res[2][:2] == (1000, 1) and outs[2][:1000].tobytes() == frags[2][0]
    assert rx.seq == 7 + 3 + 3 + 1 and rx.pending == 0
    # resubmitted from the stop: the rest of window 2, then windows 3..5
    rest = np.frombuffer(wires[2][1022:], np.uint8).copy()
    again = [rest] + arr[3:]
    outs2 = [np.zeros(len(a), np.uint8) for a in again]
    tickets = [rx.open_submit(a, o)[0] for a, o in zip(again, outs2)]
    res = [rx.wait(t) for t in tickets]
    assert all(r[3] == 0 for r in res) and rx.seq == 7 + 18
    assert outs2[0][:res[0][0]].tobytes() == b"".join(frags[2][1:])
    assert outs2[3][:res[3][0]].tobytes() == b"".join(frags[5])
    rx.close()


def test_coalesced_windows_at_the_key_update_limit(gpu):
    """Queued windows across the 2^24-record limit: the window that reaches it stops (KEY_UPDATE), the windows queued
    behind it seal nothing (as separate ptls_send calls would: every fragment starts at or past the limit)."""
    rng = np.random.default_rng(1001)
    key, iv = rng.integers(0, 256, 16, dtype=np.uint8).tobytes(), rng.integers(0, 256, 12, dtype=np.uint8).tobytes()
    tx = ra.RecordLayer(key, iv, seq=LIMIT - 5)
    wins = [[rng.integers(0, 256, 2000, dtype=np.uint8) for _ in range(3)] for _ in range(4)]
    outs = [np.zeros(3 * (2000 + ra.TLS_OVERHEAD), np.uint8) for _ in wins]
    tickets = [tx.seal_submit(w, o) for w, o in zip(wins, outs)]
    res = [tx.wait(t) for t in tickets]
    assert [r[1] for r in res] == [3, 2, 0, 0]
    assert [r[3] for r in res] == [0, ra.RECORD_LAYER_KEY_UPDATE, ra.RECORD_LAYER_KEY_UPDATE, ra.RECORD_LAYER_KEY_UPDATE]
    want0, s0 = oracle_window(key, iv, LIMIT - 5, [w.tobytes() for w in wins[0]])
    want1, s1 = oracle_window(key, iv, s0, [w.tobytes() for w in wins[1][:2]])
    assert outs[0][:len(want0)].tobytes() == want0 and outs[1][:len(want1)].tobytes() == want1
    assert tx.seq == LIMIT
    tx.close()


@pytest.mark.parametrize("transport", ["direct", "zero_copy"])
def test_coalesced_windows_of_mixed_content_types(gpu, transport):
    """Windows of other content types among queued application-data windows (a KeyUpdate or alert sealed
    while every launch slot is busy was appended to the queued type-23 group and sealed as type 23): a group never
    mixes types, so every window's records carry their own type and seq, as separate ptls_send calls would."""
    rng = np.random.default_rng(1212)
    key, iv = rng.integers(0, 256, 16, dtype=np.uint8).tobytes(), rng.integers(0, 256, 12, dtype=np.uint8).tobytes()
    types = [23] * 10 + [22] + [23] * 6 + [21, 21] + [23] * 9
    wins_b = [[rng.integers(0, 256, 16384, dtype=np.uint8).tobytes() for _ in range(4 if t == 23 else 1)]
              for t in types]
    tx = ra.RecordLayer(key, iv, seq=3)
    h = Host(transport, [tx], 1 << 23)
    wins = [[h.take(len(f), f) for f in w] for w in wins_b]
    wants, s = [], 3
    for t, w in zip(types, wins_b):
        want, s = oracle_window(key, iv, s, w, t)
        wants.append(want)
    outs = [h.take(len(want) + 64) for want in wants]
    tickets = []
    for t, w, o in zip(types, wins, outs):  # up to 24 outstanding: launches in flight while others queue
        if len(tickets) == 24:
            r = tx.wait(tickets.pop(0))
            assert r[3] == 0
        tickets.append(tx.seal_submit(w, o, content_type=t))
    for tk in tickets:
        assert tx.wait(tk)[3] == 0
    for i, (o, want) in enumerate(zip(outs, wants)):
        assert o[:len(want)].tobytes() == want, (i, types[i])
    assert tx.seq == s
    tx.close()


def test_shared_registration_outlives_its_first_layer(gpu):
    """Two layers (the two directions of a connection) register one socket buffer: the registration is shared and
    counted, so freeing the layer that registered it first leaves it mapped for the other one, whose windows keep
    reading and writing it in place (round 4 unmapped it under the second layer); the last one unmaps it."""
    rng = np.random.default_rng(1313)
    key, iv = rng.integers(0, 256, 16, dtype=np.uint8).tobytes(), rng.integers(0, 256, 12, dtype=np.uint8).tobytes()
    buf = page_buffer(1 << 21)
    frags_b = [rng.integers(0, 256, 16384, dtype=np.uint8).tobytes() for _ in range(8)]
    want, _ = oracle_window(key, iv, 0, frags_b)
    for first_closed in ("tx", "rx"):
        tx, rx = ra.RecordLayer(key, iv), ra.RecordLayer(key, iv)
        tx.register(buf)
        rx.register(buf)
        frags = []
        for i, f in enumerate(frags_b):
            v = buf[i * 16384:(i + 1) * 16384]
            v[:] = np.frombuffer(f, np.uint8)
            frags.append(v)
        wire = buf[1 << 19:(1 << 19) + len(want)]
        olen, n = tx.seal_into(frags, wire)
        assert wire[:olen].tobytes() == want and n == 8
        (tx if first_closed == "tx" else rx).close()
        ra.device_check()
        other = rx if first_closed == "tx" else tx
        pt = buf[1 << 20:(1 << 20) + len(want)]
        if other is rx:  # the surviving layer runs in place on the shared range
            rc, plen, cons, nrec = rx.open_into(wire, pt)
            assert (rc, cons, nrec) == (0, len(want), 8) and pt[:plen].tobytes() == b"".join(frags_b)
        else:
            olen2, _ = tx.seal_into(frags, pt)
            want2, _ = oracle_window(key, iv, 8, frags_b)
            assert pt[:olen2].tobytes() == want2
        ra.device_check()
        other.close()
    ra.device_check()


def test_registration_inside_a_shared_range_and_partial_overlaps(gpu):
    """A range inside one another layer mapped shares that mapping and counts on it: the enclosing range's layer is
    freed first and the inner range's windows still run in place on it (the 1 MiB mapping stays while the inner range
    holds it).  A range that overlaps a mapped one without lying inside it (only the mapped part would be reachable by
    the kernels) is refused, before and after; once the last holder lets go the whole buffer registers."""
    rng = np.random.default_rng(1515)
    key, iv = rng.integers(0, 256, 16, dtype=np.uint8).tobytes(), rng.integers(0, 256, 12, dtype=np.uint8).tobytes()
    buf = page_buffer(1 << 21)
    frags_b = [rng.integers(0, 256, 16384, dtype=np.uint8).tobytes() for _ in range(4)]
    want, _ = oracle_window(key, iv, 0, frags_b)
    outer, inner, other = ra.RecordLayer(key, iv), ra.RecordLayer(key, iv), ra.RecordLayer(key, iv)
    outer.register(buf[: 1 << 20])
    for bad in (buf[(1 << 20) - 4096:(1 << 20) + 4096], buf):  # straddles the end; encloses it
        with pytest.raises(RuntimeError, match="overlaps a registered range"):
            other.register(bad)
    inner_buf = buf[1 << 18:(1 << 18) + (1 << 19)]
    inner.register(inner_buf)
    outer.close()  # the mapping stays: the inner registration counts on it
    ra.device_check()
    frags = []
    for i, f in enumerate(frags_b):
        v = inner_buf[i * 16384:(i + 1) * 16384]
        v[:] = np.frombuffer(f, np.uint8)
        frags.append(v)
    wire = inner_buf[1 << 17:(1 << 17) + len(want)]
    olen, n = inner.seal_into(frags, wire)
    assert wire[:olen].tobytes() == want and n == 4
    with pytest.raises(RuntimeError, match="overlaps a registered range"):
        other.register(buf)  # the mapping kept for the inner range is still the enclosing 1 MiB one
    other.register(buf[:1 << 20])  # inside it: shared
    inner.close()
    other.close()
    ra.device_check()
    last = ra.RecordLayer(key, iv)
    last.register(buf)  # nothing mapped over it any more
    last.close()
    ra.device_check()


@pytest.mark.parametrize("transport", ["direct", "copy"])
def test_reserved_layer_across_a_rekey(gpu, transport):
    """ptls_mi355x_record_layer_reserve sets up every launch slot before the first window (streams, contexts, staging
    for rapido's windows); windows on all four slots, a rekey (every slot's context re-created under the new key), and
    more windows -- every record against the oracle under its key and seq."""
    rng = np.random.default_rng(1414)
    key, key2 = rng.integers(0, 256, 16, dtype=np.uint8).tobytes(), rng.integers(0, 256, 16, dtype=np.uint8).tobytes()
    iv, iv2 = rng.integers(0, 256, 12, dtype=np.uint8).tobytes(), rng.integers(0, 256, 12, dtype=np.uint8).tobytes()
    tx = ra.RecordLayer(key, iv, seq=9)
    h = Host(transport, [tx], 1 << 23)
    tx.reserve(16 * (16384 + ra.TLS_OVERHEAD), 1)
    for k, v, s0 in ((key, iv, 9), (key2, iv2, 0)):
        if k is key2:
            tx.rekey(key2, iv2)
            assert tx.seq == 0
        wins_b = [[rng.integers(0, 256, int(n), dtype=np.uint8).tobytes() for n in rng.integers(1, 16385, 5)]
                  for _ in range(6)]
        wins = [[h.take(len(f), f) for f in w] for w in wins_b]
        wants, s = [], s0
        for w in wins_b:
            want, s = oracle_window(k, v, s, w)
            wants.append(want)
        outs = [h.take(len(x) + 64) for x in wants]
        tickets = []
        for w, o in zip(wins, outs):
            if len(tickets) == 4:
                assert tx.wait(tickets.pop(0))[3] == 0
            tickets.append(tx.seal_submit(w, o))
        for t in tickets:
            assert tx.wait(t)[3] == 0
        for o, want in zip(outs, wants):
            assert o[:len(want)].tobytes() == want
    tx.close()


@pytest.mark.parametrize("transport", ["direct", "zero_copy"])
def test_sessions_in_one_async_launch(gpu, transport):
    """Round 6: the windows of three sessions (each its own key and IV) in one asynchronous launch each way.  Sealed
    bytes per session against the oracle; on the receive side session B's window stops at a bad record (alert 20, its
    next window in the following launch completes STALE) while sessions A and C deliver in both launches; a session
    layer named by an in-flight launch cannot be rekeyed."""
    rng = np.random.default_rng(606)
    keys = [rng.integers(0, 256, 16, dtype=np.uint8).tobytes() for _ in range(3)]
    ivs = [rng.integers(0, 256, 12, dtype=np.uint8).tobytes() for _ in range(3)]
    seqs = [5, 70, 0]
    tx = [ra.RecordLayer(k, v, seq=s) for k, v, s in zip(keys, ivs, seqs)]
    rx = [ra.RecordLayer(k, v, seq=s) for k, v, s in zip(keys, ivs, seqs)]
    h = Host(transport, tx + rx, 1 << 22)
    frags = [[[rng.integers(0, 256, n, dtype=np.uint8).tobytes() for n in (16384, 1400, 3, 9000)] for _ in range(3)]
             for _ in range(2)]  # [launch][session] -> fragments
    # seal: two launches of one window per session, both in flight
    tickets = []
    for L in range(2):
        wins = [[h.take(len(f), f) for f in frags[L][s]] for s in range(3)]
        outs = [h.take(sum(len(f) + ra.TLS_OVERHEAD for f in frags[L][s])) for s in range(3)]
        tickets.append((ra.record_layer_seal_submit_multi(tx, wins, outs), outs))
    with pytest.raises(RuntimeError):
        tx[2].rekey(keys[2], ivs[2])  # named by a launch in flight
    wires, run = [[None] * 3 for _ in range(2)], list(seqs)
    for L, (t, outs) in enumerate(tickets):
        res = tx[0].wait_multi(t, 3)
        for s in range(3):
            want, run[s] = oracle_window(keys[s], ivs[s], run[s], frags[L][s])
            assert res[s][:2] == (len(want), 4) and outs[s][:len(want)].tobytes() == want, (L, s)
            wires[L][s] = want
    assert [t.seq for t in tx] == run
    # open: session B's first window has a bad ciphertext byte in its third record
    bad = bytearray(wires[0][1])
    third = len(frags[0][1][0]) + len(frags[0][1][1]) + 2 * ra.TLS_OVERHEAD
    bad[third + 9] ^= 4
    tickets = []
    for L in range(2):
        ws = [bytes(bad) if (L, s) == (0, 1) else wires[L][s] for s in range(3)]
        ins = [h.take(len(w), w) for w in ws]
        outs = [h.take(len(w)) for w in ws]
        tickets.append((ra.record_layer_open_submit_multi(rx, ins, outs)[0], outs))
    r0 = rx[0].wait_multi(tickets[0][0], 3)
    r1 = rx[0].wait_multi(tickets[1][0], 3)
    for s in (0, 2):
        for L, r in ((0, r0), (1, r1)):
            n = sum(map(len, frags[L][s]))
            assert r[s][:2] == (n, 4) and r[s][3] == 0 and tickets[L][1][s][:n].tobytes() == b"".join(frags[L][s])
    assert r0[1][1] == 2 and r0[1][3] == 20  # two records delivered, then BAD_RECORD_MAC
    assert tickets[0][1][1][:r0[1][0]].tobytes() == b"".join(frags[0][1][:2])
    assert r1[1] == (0, 0, 0, ra.RECORD_LAYER_STALE)
    assert rx[1].seq == seqs[1] + 2 and rx[0].seq == seqs[0] + 8 and rx[2].seq == seqs[2] + 8
    for rl in tx + rx:
        rl.close()
