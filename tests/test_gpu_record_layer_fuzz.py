"""Randomised record-layer sessions against the oracle (include/ptls_mi355x.h section 5, rapido_amd/csrc/record_layer.c).

Each case draws a session (key size, connections, seqs, some right below ptls_send's 2^24-record limit), a launch of
windows over those connections (a connection may appear several times: its consecutive windows), ragged fragments
(empty, 1 byte, exactly 16 KiB, over 16 KiB), a transport, and damage on the receive side (a flipped ciphertext or
tag bit, a truncated tail).  The expected bytes come from a plain model of ptls_send / ptls_receive over the oracle's
TLS 1.3 record functions (lib/picotls.c:4969-4988 for the limit, :650-652 for the stop at the first failure), which
tests/test_tls_records.py pins to the reference's own outputs.  Since round 6 a third of the sessions give every
connection a session (key and IV) of its own, so their launches carry several keys."""
import numpy as np
import pytest

import oracle
import rapido_amd as ra
from test_gpu_record_layer import conn_iv
from test_gpu_record_layer_async import Host

pytestmark = pytest.mark.gpu
LIMIT = ra.RECORD_LAYER_SEQ_LIMIT
MAXREC = 16384


def model_seal(key, iv, seq, frags):
    """ptls_send per fragment: the limit is checked at each fragment's start -> (wire, records, next seq)"""
    wire, n = b"", 0
    for f in frags:
        if seq >= LIMIT:
            break
        for off in range(0, len(f), MAXREC):
            wire += oracle.tls_seal_record(key, iv, seq, 23, f[off:off + MAXREC])
            seq += 1
            n += 1
    return wire, n, seq


def record_spans(wire):
    """(offset, total length) of the complete records at the start of wire"""
    spans, off = [], 0
    while off + 5 <= len(wire):
        ln = int.from_bytes(wire[off + 3:off + 5], "big")
        if off + 5 + ln > len(wire):
            break
        spans.append((off, 5 + ln))
        off += 5 + ln
    return spans


def model_open(key, iv, seq, wire):
    """ptls_receive over a window: the complete application_data records in order, stopping at the first that fails
    -> (alert, plaintext, consumed, records).  A header is judged as soon as its 5 bytes are there: a length past
    2^14 + 256 is DECODE_ERROR even before the record is complete (parse_record_header, lib/picotls.c:4243-4254); a
    record of another outer type is left to picotls (open_record)."""
    pt, cons, n, off = b"", 0, 0, 0
    while off + 5 <= len(wire):
        ln = int.from_bytes(wire[off + 3:off + 5], "big")
        if wire[off] != 23:
            break
        if ln > 16640:
            return 50, pt, cons, n
        if off + 5 + ln > len(wire):  # incomplete: wait for more bytes
            break
        got = oracle.tls_open_record(key, iv, seq, wire[off:off + 5 + ln])
        if isinstance(got, int):  # TLS_BAD_MAC -> bad_record_mac, TLS_NO_TYPE -> unexpected_message
            return (20 if got == oracle.TLS_BAD_MAC else 10), pt, cons, n
        inner, ctype = got
        if ctype != 23:
            break
        pt += inner
        cons += 5 + ln
        off += 5 + ln
        n += 1
        seq += 1
    return 0, pt, cons, n


def draw_frags(rng, k):
    sizes = rng.choice([0, 1, 15, 16, 17, 1399, 1400, 4096, 16383, 16384, 16385, 40000], size=k)
    return [rng.integers(0, 256, int(n), dtype=np.uint8).tobytes() for n in sizes]


TRANSPORTS = ["direct", "direct_dma", "direct_dma_in", "zero_copy", "copy"]


@pytest.mark.parametrize("case", range(24))
def test_random_session(gpu, case):
    random_session(np.random.default_rng(1000 + case), TRANSPORTS[case % 5], 16 if case % 3 else 32, f"case {case}")


def test_record_layer_campaign(gpu):
    """Random sessions as above, each with a fresh seed, transport and key size: 1000 from a fixed seed by default (the
    same sessions on every box), or time-boxed with RAPIDO_RL_FUZZ_SECONDS (RAPIDO_FUZZ_SEED as in
    test_gpu_fuzz_campaign.py; RAPIDO_FUZZ_LOG gets a summary line)."""
    import json
    import os
    import time
    timed = "RAPIDO_RL_FUZZ_SECONDS" in os.environ  # else the gate: 1000 sessions from the fixed seed on every box
    budget = float(os.environ.get("RAPIDO_RL_FUZZ_SECONDS", "0"))
    seed = os.environ.get("RAPIDO_FUZZ_SEED", "31337")
    base = int(time.time()) & 0xFFFFFFF if seed == "random" else int(seed)
    stats = {"what": "record layer sessions", "seed_base": base, "sessions": 0, "transports": {}}
    t0 = last = time.time()
    while (time.time() - t0 < budget) if timed else stats["sessions"] < 1000:
        rng = np.random.default_rng(base + stats["sessions"])
        transport, keylen = TRANSPORTS[int(rng.integers(0, 5))], int(rng.choice([16, 32]))
        random_session(rng, transport, keylen, f"seed {base + stats['sessions']}")
        stats["sessions"] += 1
        stats["transports"][transport] = stats["transports"].get(transport, 0) + 1
        if time.time() - last > 30:
            last = time.time()
            print("progress", json.dumps(stats), flush=True)
    stats["seconds"] = round(time.time() - t0, 1)
    print(json.dumps(stats))
    if os.environ.get("RAPIDO_FUZZ_LOG"):
        with open(os.environ["RAPIDO_FUZZ_LOG"], "a") as f:
            f.write(json.dumps(stats) + "\n")
    assert stats["sessions"] > 0


def random_session(rng, transport, keylen, case):
    key = rng.integers(0, 256, keylen, dtype=np.uint8).tobytes()
    iv = rng.integers(0, 256, 12, dtype=np.uint8).tobytes()
    nconn = int(rng.integers(1, 4))
    cids = [int(c) for c in rng.choice(1 << 16, nconn, replace=False)]
    seqs = [int(LIMIT - rng.integers(1, 6)) if rng.random() < 0.3 else int(rng.integers(0, 1 << 20)) for _ in cids]
    # round 6: in a third of the sessions every connection is a session of its own (its own key and IV, one key
    # size), so the launches below carry several keys (the multi-key framing kernels)
    own = rng.random() < 1 / 3
    keys = [rng.integers(0, 256, keylen, dtype=np.uint8).tobytes() if own and c else key for c in range(nconn)]
    sivs = [rng.integers(0, 256, 12, dtype=np.uint8).tobytes() if own and c else iv for c in range(nconn)]
    civ = [conn_iv(sivs[c], cids[c]) for c in range(nconn)]
    tx = [ra.RecordLayer(keys[c], civ[c], seq=seqs[c]) for c in range(nconn)]
    rx = [ra.RecordLayer(keys[c], civ[c], seq=seqs[c]) for c in range(nconn)]
    h = Host(transport, tx + rx, 1 << 23)
    # the launch: windows over the connections, some connections more than once
    order = [int(c) for c in rng.integers(0, nconn, int(rng.integers(1, 6)))]
    windows_b = [draw_frags(rng, int(rng.integers(0, 7))) for _ in order]
    windows = [[h.take(len(f), f) for f in w] for w in windows_b]
    outs = [h.take(sum(len(f) + (len(f) + MAXREC - 1) // MAXREC * ra.TLS_OVERHEAD for f in w) + 64) for w in windows_b]
    got = ra.record_layer_seal_multi([tx[c] for c in order], windows, outs=outs)
    run_seq = list(seqs)
    wires = []
    for c, w, o, (wlen, n) in zip(order, windows_b, outs, got):
        want, wn, run_seq[c] = model_seal(keys[c], civ[c], run_seq[c], w)
        assert o[:wlen].tobytes() == want and n == wn, f"{case} ({transport}): seal window of connection {c}"
        wires.append(want)
    assert [t.seq for t in tx] == run_seq
    # the receive side: damage some windows, open them all in one launch (staging) and model the outcome
    damaged = []
    for w in wires:
        w = bytearray(w)
        r = rng.random()
        if w and r < 0.25:
            w[int(rng.integers(5, len(w)))] ^= 1 << int(rng.integers(0, 8))  # a header, ciphertext or tag bit
        elif w and r < 0.45:
            w = w[:len(w) - int(rng.integers(1, min(len(w), 30) + 1))]  # a truncated tail
        damaged.append(bytes(w))
    res = ra.record_layer_open_multi([rx[c] for c in order], damaged)
    # per connection: "ok"; "stale" behind a window that stopped early (the layer knows); "lost" behind a window
    # whose stream the damage broke without a stop (a truncated record, a flipped header): the next records carry
    # seqs the receiver has not reached, so nothing more is delivered
    exp_seq, state = list(seqs), ["ok"] * nconn
    for c, w, r in zip(order, damaged, res):
        if state[c] == "stale":
            assert r[0] == ra.RECORD_LAYER_STALE and r[3] == 0, f"{case}: window behind a stop"
            continue
        if state[c] == "lost":
            assert r[1] == b"" and r[3] == 0, f"{case}: window behind a broken stream"
            continue
        spans = record_spans(w)
        # the parser reads a header's type and length; the legacy version bytes are neither checked nor authenticated
        # (build_aad writes 03 03 itself, lib/picotls.c:621-628), so a flipped version bit leaves the stream intact
        hdr_ok = all(w[o] == 23 and 17 <= ln - 5 <= 16640 for o, ln in spans)
        if not hdr_ok:  # a flipped type or length bit: the layer's parser decides; only the delivered prefix is checked
            assert r[1] == model_open(keys[c], civ[c], exp_seq[c], w[:r[2]])[1]
            exp_seq[c] += r[3]
            state[c] = "lost"
            continue
        want = model_open(keys[c], civ[c], exp_seq[c], w)
        assert r == want, f"{case}: open window of connection {c}"
        exp_seq[c] += want[3]
        if want[3] < len(spans):
            state[c] = "stale"
        elif (spans[-1][0] + spans[-1][1] if spans else 0) < len(w):
            state[c] = "lost"
    assert [x.seq for x in rx] == exp_seq
    for rl in tx + rx:
        rl.close()


@pytest.mark.parametrize("transport", ["direct", "direct_dma_in", "zero_copy"])
def test_random_async_stream(gpu, transport):
    """A random stream of windows of one connection through submit / wait, up to four in flight, a bad record in
    one of them: the windows behind it STALE, then resubmitted from the stop."""
    rng = np.random.default_rng(4242)
    key, iv = rng.integers(0, 256, 16, dtype=np.uint8).tobytes(), rng.integers(0, 256, 12, dtype=np.uint8).tobytes()
    tx, rx = ra.RecordLayer(key, iv, seq=3), ra.RecordLayer(key, iv, seq=3)
    h = Host(transport, [tx, rx], 1 << 24)
    wins_b = [draw_frags(rng, int(rng.integers(1, 9))) for _ in range(12)]
    tickets, sealed = [], []
    outs = [h.take(sum(len(f) + (len(f) + MAXREC - 1) // MAXREC * ra.TLS_OVERHEAD for f in w) + 64) for w in wins_b]
    for w, o in zip(wins_b, outs):
        if len(tickets) == 4:
            sealed.append(tx.wait(tickets.pop(0)))
        tickets.append(tx.seal_submit([h.take(len(f), f) for f in w], o))
    sealed += [tx.wait(t) for t in tickets]
    seq, wires = 3, []
    for w, o, (olen, nrec, nfr, al) in zip(wins_b, outs, sealed):
        want, n, seq = model_seal(key, iv, seq, w)
        assert (o[:olen].tobytes(), nrec, al) == (want, n, 0)
        wires.append(want)
    bad = int(rng.integers(2, 8))
    while not wires[bad]:
        bad += 1
    dmg = bytearray(wires[bad])
    dmg[len(dmg) - 3] ^= 0x40  # the last record's tag
    ins = [h.take(len(w), w) for w in wires[:bad] + [bytes(dmg)] + wires[bad + 1:]]
    pts = [h.take(len(w) + 16) for w in wires]
    tickets, res = [], []
    for x, p in zip(ins, pts):
        if len(tickets) == 4:
            res.append(rx.wait(tickets.pop(0)))
        tickets.append(rx.open_submit(x, p)[0])
    res += [rx.wait(t) for t in tickets]
    seq = 3
    for i, (w, p, r) in enumerate(zip(wires, pts, res)):
        if i < bad:
            a, pt, cons, n = model_open(key, iv, seq, w)
            assert r == (len(pt), n, cons, a) and p[:len(pt)].tobytes() == pt
            seq += n
        elif i == bad:
            a, pt, cons, n = model_open(key, iv, seq, bytes(dmg))
            assert a == 20 and r == (len(pt), n, cons, 20) and p[:len(pt)].tobytes() == pt
            seq += n
        elif r[3] != ra.RECORD_LAYER_STALE:  # windows submitted after the stop was known (none in flight): empty
            assert r[:2] == (0, 0)
        else:
            assert r[:3] == (0, 0, 0)
    assert rx.seq == seq
    tx.close()
    rx.close()
