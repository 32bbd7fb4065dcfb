"""GPU parity of the TLS 1.3 record-framing kernels (include/ptls_mi355x.h section 4, SURVEY.md 8(f)
rows 1-3) through the C-ABI: against the reference record layer's own outputs
(tests/golden/tls_records.json: ptls_send / ptls_receive of lib/picotls.c) and the oracle's
restatement of it.  Bit-exact wire bytes, plaintext, status and content types."""
import hashlib
import json
import os

import numpy as np
import pytest

import oracle
import rapido_amd as ra
from conftest import FAMILIES, kernel_family
from rapido_amd.records import xorshift64star
from rapido_amd.hostmem import to_cpu, to_gpu

pytestmark = pytest.mark.gpu
GOLDEN = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "tls_records.json")))


@pytest.fixture(autouse=True, params=FAMILIES)
def framing_kernels(request, engine_lib):
    """Every framing test runs on each kernel family (conftest.FAMILIES): the window kernels (64-block segments in
    parallel), the same with 32-block segments, with 32-block segments of 16 lanes (the default up to one record
    per CU) and the batch kernels (4 lanes per record)."""
    with kernel_family(request.param, framing=True):
        yield request.param


def dev(a):
    import torch
    return to_gpu(np.array(a, copy=True))


def seal(eng, iv, trecs, src, wire_size, dst=None):
    import torch
    d_src = dev(src)
    d_dst = torch.zeros(wire_size, dtype=torch.uint8, device="cuda") if dst is None else dst
    d_recs = dev(trecs.view(np.uint8))
    eng.tls_seal_records(iv, d_recs.data_ptr(), len(trecs), d_src.data_ptr(), d_dst.data_ptr())
    torch.cuda.synchronize()
    return to_cpu(d_dst)


def open_(eng, iv, orecs, wire, pt_size, inplace=False):
    import torch
    d_wire = dev(wire)
    d_pt = d_wire if inplace else torch.zeros(max(pt_size, 1), dtype=torch.uint8, device="cuda")
    d_recs = dev(orecs.view(np.uint8))
    d_st = torch.zeros(max(len(orecs), 1), dtype=torch.int32, device="cuda")
    d_ty = torch.zeros(max(len(orecs), 1), dtype=torch.uint8, device="cuda")
    eng.tls_open_records(iv, d_recs.data_ptr(), len(orecs), d_wire.data_ptr(), d_pt.data_ptr(), d_st.data_ptr(),
                         d_ty.data_ptr())
    torch.cuda.synchronize()
    return to_cpu(d_pt), to_cpu(d_st).view(np.uint32), to_cpu(d_ty)


def xs(seed, n):
    return xorshift64star(seed, n).tobytes()


@pytest.mark.parametrize("case", GOLDEN["send"], ids=lambda c: f"aes{c['keylen'] * 8}-{c['len']}")
def test_send_matches_reference_ptls_send(gpu, case):
    """ptls_send's wire bytes (lib/picotls.c:4969-4988) from one framing launch per stream."""
    key, iv = xs(case["seed"] + 1, case["keylen"]), xs(case["seed"] + 2, 12)
    data = np.frombuffer(xs(case["seed"], case["len"]), np.uint8)
    trecs, wire_len, seq = ra.tls_plan_send(case["len"], case["seq0"])
    assert wire_len == case["wire_len"] and seq == case["seq_after"]
    eng = ra.Engine(key)
    wire = seal(eng, iv, trecs, data, wire_len).tobytes()
    assert hashlib.sha256(wire).hexdigest() == case["wire_sha256"]
    if "wire" in case:
        assert wire.hex() == case["wire"]
    # and back: parse the wire on the host, open every record in one launch
    rc, orecs, used, seq2 = ra.tls_parse_records(wire, case["seq0"])
    assert rc == 0 and used == len(wire) and seq2 == seq
    pt, st, ty = open_(eng, iv, orecs, np.frombuffer(wire, np.uint8), case["len"] + 16 * len(orecs))
    assert list(st[: len(orecs)]) == list(trecs["len"]) and (ty[: len(orecs)] == 23).all()
    got = b"".join(pt[int(o["dst"]): int(o["dst"]) + int(s)].tobytes() for o, s in zip(orecs, st))
    assert got == data.tobytes()


@pytest.mark.parametrize("i", range(len(GOLDEN["receive"])))
def test_receive_matches_reference_ptls_receive(gpu, i):
    """Padding strip, content-type pop, bad MAC and no-content-type verdicts of handle_input_tls13."""
    c = GOLDEN["receive"][i]
    key, iv, wire = bytes.fromhex(c["key"]), bytes.fromhex(c["iv"]), bytes.fromhex(c["wire"])
    rc, orecs, used, _ = ra.tls_parse_records(wire, c["seq"])
    assert rc == 0 and len(orecs) == 1
    with ra.Engine(key) as eng:
        pt, st, ty = open_(eng, iv, orecs, np.frombuffer(wire, np.uint8), int(orecs[0]["len"]))
    if c["rc"] == 20:
        assert st[0] == ra.TLS_BAD_RECORD_MAC and not pt.any()
    elif c["rc"] == 10:
        assert st[0] == ra.TLS_UNEXPECTED_MESSAGE
    else:
        assert pt[: st[0]].tobytes() == bytes.fromhex(c["plaintext"]) and ty[0] == 23


@pytest.mark.parametrize("keylen", [16, 32])
def test_framing_edges_vs_oracle(gpu, keylen):
    """Every fragment length around the block edges, three content types, unaligned offsets, both ways."""
    rng = np.random.default_rng(100 + keylen)
    key, iv = rng.integers(0, 256, keylen, dtype=np.uint8).tobytes(), rng.integers(0, 256, 12, dtype=np.uint8).tobytes()
    lens = list(range(0, 70)) + [255, 256, 1399, 1400, 1401, 4095, 16383, 16384] + list(rng.integers(0, 16385, 60))
    n = len(lens)
    trecs = np.zeros(n, ra.TLS_RECORD_DTYPE)
    off = woff = 0
    for i, ln in enumerate(lens):
        trecs[i] = (off, woff, int(rng.integers(0, 2 ** 48)), ln, [23, 22, 21, 0x40][i % 4])
        off += int(ln) + 3
        woff += int(ln) + 22 + (i % 5)
    src = rng.integers(0, 256, off + 16, dtype=np.uint8)
    eng = ra.Engine(key)
    wire = seal(eng, iv, trecs, src, woff + 16)
    for t in trecs:
        frag = src[int(t["src"]): int(t["src"]) + int(t["len"])].tobytes()
        want = oracle.tls_seal_record(key, iv, int(t["seq"]), int(t["type"]), frag)
        assert wire[int(t["dst"]): int(t["dst"]) + len(want)].tobytes() == want, int(t["len"])
    orecs = trecs.copy()
    orecs["src"], orecs["len"] = trecs["dst"], trecs["len"] + 17
    orecs["dst"] = np.concatenate([[0], np.cumsum((orecs["len"] - 16).astype(np.uint64))[:-1]]).astype(np.uint64)
    pt, st, ty = open_(eng, iv, orecs, wire, int(orecs["dst"][-1]) + int(orecs["len"][-1]))
    assert list(st[:n]) == lens and list(ty[:n]) == list(trecs["type"])
    for t, o in zip(trecs, orecs):
        assert pt[int(o["dst"]): int(o["dst"]) + int(t["len"])].tobytes() == \
            src[int(t["src"]): int(t["src"]) + int(t["len"])].tobytes()


def test_open_padding_tamper_short(gpu):
    key, iv = bytes(range(16)), bytes(range(30, 42))
    cases = [(50, 23, 0), (50, 23, 1), (50, 23, 15), (50, 23, 16), (0, 23, 40), (300, 23, 333), (0, 0, 7),
             (1000, 22, 2000), (15, 21, 17)]
    wires = [oracle.tls_seal_record(key, iv, 77 + i, t, bytes(k % 255 + 1 for k in range(n)), p)
             for i, (n, t, p) in enumerate(cases)]
    seqs = [77 + i for i in range(len(cases))]
    for k in (1, 9, -3):  # the header's version byte (not in the AAD: build_aad uses 03 03), ciphertext, tag
        w = bytearray(oracle.tls_seal_record(key, iv, 1, 23, bytes(range(100))))
        w[k] ^= 1
        wires.append(bytes(w))
        seqs.append(1)
    w = bytearray(oracle.tls_seal_record(key, iv, 1, 23, bytes(range(100))))
    wires.append(bytes(w)); seqs.append(2)  # wrong seq
    wires.append(b"\x17\x03\x03\x00\x0f" + bytes(15)); seqs.append(3)  # shorter than a tag
    wires.append(b"\x17\x03\x03\x00\x10" + bytes(16)); seqs.append(4)  # empty ciphertext, wrong tag
    buf = b"".join(wires)
    rc, orecs, used, _ = ra.tls_parse_records(buf, 0)
    assert rc == 0 and len(orecs) == len(wires) and used == len(buf)
    orecs["seq"] = seqs
    with ra.Engine(key) as eng:
        pt, st, ty = open_(eng, iv, orecs, np.frombuffer(buf, np.uint8), int(orecs["dst"][-1]) + int(orecs["len"][-1]))
    for i, w in enumerate(wires):
        want = oracle.tls_open_record(key, iv, seqs[i], w)
        o = orecs[i]
        if want == oracle.TLS_BAD_MAC:
            assert st[i] == ra.TLS_BAD_RECORD_MAC, i
            assert not pt[int(o["dst"]): int(o["dst"]) + max(int(o["len"]) - 16, 0)].any()
        elif want == oracle.TLS_NO_TYPE:
            assert st[i] == ra.TLS_UNEXPECTED_MESSAGE, i
        else:
            assert st[i] == len(want[0]) and ty[i] == want[1], i
            assert pt[int(o["dst"]): int(o["dst"]) + int(st[i])].tobytes() == want[0]


def test_rapido_windows_and_retransmission(gpu):
    """rapido's send window (16 x 16406-B records, lib/rapido.c:2083-2126) sealed in one launch, a recv()
    window of 32 records (:2030) opened in one launch, and the retransmission path (:1555-1590): a
    non-contiguous subset of the sent records re-opened with their stored sequence numbers."""
    key, iv = bytes(range(7, 23)), bytes(range(12))
    data = xorshift64star(11, 16 * 16384).tobytes()
    trecs, wire_len, seq = ra.tls_plan_send(len(data), 1000)
    assert len(trecs) == 16 and wire_len == 16 * 16406
    eng = ra.Engine(key)
    wire = seal(eng, iv, trecs, np.frombuffer(data, np.uint8), wire_len)
    # recv window of 32 records: two send windows back to back
    wire2 = np.concatenate([wire, seal(eng, iv, ra.tls_plan_send(len(data), seq)[0], np.frombuffer(data, np.uint8),
                                       wire_len)])
    rc, orecs, used, _ = ra.tls_parse_records(wire2.tobytes(), 1000)
    assert rc == 0 and len(orecs) == 32 and used == len(wire2)
    pt, st, ty = open_(eng, iv, orecs, wire2, 32 * 16401)
    assert (st[:32] == 16384).all() and (ty[:32] == 23).all()
    assert b"".join(pt[int(o["dst"]): int(o["dst"]) + 16384].tobytes() for o in orecs) == data + data
    # retransmission: records 1, 4, 5, 9, 15 of the first window, stored (offset, ciphertext_len, seq)
    pick = [1, 4, 5, 9, 15]
    rrecs = np.zeros(len(pick), ra.TLS_RECORD_DTYPE)
    for k, i in enumerate(pick):
        rrecs[k] = (int(trecs[i]["dst"]), k * 16401, int(trecs[i]["seq"]), 16384 + 17, 0)
    pt, st, ty = open_(eng, iv, rrecs, wire, len(pick) * 16401)
    assert (st[: len(pick)] == 16384).all()
    for k, i in enumerate(pick):
        assert pt[k * 16401: k * 16401 + 16384].tobytes() == data[i * 16384: (i + 1) * 16384]


def test_in_place(gpu):
    """Seal a fragment already placed 5 bytes into its record slot, and open a record in place (plaintext
    over its own header + ciphertext, dst = src + 5), as picotls's buffer_encrypt_record does in its buffer."""
    import torch
    key, iv = bytes(range(16)), bytes(range(12))
    lens = [0, 1, 16, 100, 1400, 16384]
    slots = [ln + 22 for ln in lens]
    base = np.cumsum([0] + slots[:-1])
    buf = np.zeros(sum(slots) + 16, np.uint8)
    trecs = np.zeros(len(lens), ra.TLS_RECORD_DTYPE)
    frags = []
    for i, ln in enumerate(lens):
        f = xorshift64star(20 + i, ln).tobytes()
        frags.append(f)
        buf[base[i] + 5: base[i] + 5 + ln] = np.frombuffer(f, np.uint8)
        trecs[i] = (base[i] + 5, base[i], 50 + i, ln, 23)
    eng = ra.Engine(key)
    d, d_recs = dev(buf), dev(trecs.view(np.uint8))  # descriptors held until the launch completes
    eng.tls_seal_records(iv, d_recs.data_ptr(), len(trecs), d.data_ptr(), d.data_ptr())
    torch.cuda.synchronize()
    wire = to_cpu(d)
    for i, ln in enumerate(lens):
        assert wire[base[i]: base[i] + ln + 22].tobytes() == oracle.tls_seal_record(key, iv, 50 + i, 23, frags[i])
    orecs = trecs.copy()
    orecs["src"], orecs["dst"], orecs["len"] = base, base + 5, np.array(lens) + 17
    pt, st, ty = open_(eng, iv, orecs, wire, 0, inplace=True)
    eng.close()  # explicitly, after its launches' results are read back (not at a later collection)
    assert list(st[: len(lens)]) == lens
    for i, ln in enumerate(lens):
        assert pt[base[i] + 5: base[i] + 5 + ln].tobytes() == frags[i]


def conn_iv(iv: bytes, conn_id: int) -> bytes:
    """rapido's derive_connection_aead_iv (lib/rapido.c:127-133): IV bytes 0..3 ^= BE32(connection_id)."""
    return (int.from_bytes(iv[:4], "big") ^ conn_id).to_bytes(4, "big") + iv[4:]


@pytest.mark.parametrize("keylen", [16, 32])
def test_multi_connection_windows(gpu, keylen):
    """The 16-record send windows of several TCPLS connections of one session (same key; per-connection IV and
    seq, lib/rapido.c:135-200) sealed in ONE launch through tls_seal_records_multi, then received in one
    tls_open_records_multi launch; every record matches the oracle's record layer under its connection's IV,
    and a record opened under the wrong connection id fails alone."""
    import torch
    key = bytes(range(90, 90 + keylen))
    iv = bytes(range(200, 212))
    conns = [0, 1, 2, 3, 5, 0x01020304, 0xFFFFFFFF]
    lens = [16384] * 14 + [1, 777]
    trecs = np.zeros(len(conns) * len(lens), ra.TLS_RECORD_DTYPE)
    conn = np.zeros(len(trecs), np.uint32)
    off = woff = 0
    k = 0
    for ci, c in enumerate(conns):
        for j, n in enumerate(lens):
            trecs[k] = (off, woff, 1000 * ci + j, n, 23 if j % 5 else 22)
            conn[k] = c
            off += n
            woff += n + 22
            k += 1
    src = np.frombuffer(xs(33, off + 16), np.uint8)
    d_src, d_recs, d_conn = dev(src), dev(trecs.view(np.uint8)), dev(conn.view(np.int32))
    d_wire = torch.zeros(woff + 16, dtype=torch.uint8, device="cuda")
    eng = ra.Engine(key)
    eng.tls_seal_records(iv, d_recs.data_ptr(), len(trecs), d_src.data_ptr(), d_wire.data_ptr(), conn_ptr=d_conn.data_ptr())
    torch.cuda.synchronize()
    wire = to_cpu(d_wire)
    for t, c in zip(trecs, conn):
        frag = bytes(src[int(t["src"]): int(t["src"]) + int(t["len"])])
        want = oracle.tls_seal_record(key, conn_iv(iv, int(c)), int(t["seq"]), int(t["type"]), frag)
        assert bytes(wire[int(t["dst"]): int(t["dst"]) + len(want)]) == want
    # receive: plaintext slots of len + 1 bytes each (fragment + type), back to back
    orecs = trecs.copy()
    orecs["src"], orecs["len"] = trecs["dst"], trecs["len"] + 17
    orecs["dst"] = np.concatenate([[0], np.cumsum(trecs["len"].astype(np.int64) + 1)[:-1]]).astype(np.uint64)
    pt_size = int(orecs["dst"][-1]) + int(trecs["len"][-1]) + 1

    def receive(conn_ids):
        d_pt = torch.zeros(pt_size, dtype=torch.uint8, device="cuda")
        d_st = torch.zeros(len(orecs), dtype=torch.int32, device="cuda")
        d_ty = torch.zeros(len(orecs), dtype=torch.uint8, device="cuda")
        d_orecs, d_ids = dev(orecs.view(np.uint8)), dev(conn_ids.view(np.int32))  # held until the launch completes
        eng.tls_open_records(iv, d_orecs.data_ptr(), len(orecs), d_wire.data_ptr(), d_pt.data_ptr(), d_st.data_ptr(),
                             d_ty.data_ptr(), conn_ptr=d_ids.data_ptr())
        torch.cuda.synchronize()
        return to_cpu(d_pt), to_cpu(d_st).view(np.uint32), to_cpu(d_ty)

    pt, st, ty = receive(conn)
    assert (st == trecs["len"]).all() and (ty == trecs["type"]).all()
    for t, o in zip(trecs, orecs):
        assert bytes(pt[int(o["dst"]): int(o["dst"]) + int(t["len"])]) == bytes(src[int(t["src"]): int(t["src"]) +
                                                                                  int(t["len"])])
    wrong = conn.copy()
    wrong[20] ^= 0x10
    _, st, _ = receive(wrong)
    assert st[20] == 0xFFFFFFFF
    assert (np.delete(st, 20) == np.delete(trecs["len"], 20)).all()
    eng.close()


def test_many_windows_one_launch(gpu, framing_kernels):
    """1200 framed records of random lengths in one launch each way: above 3 records per CU, so the window path
    takes its persistent 1024-thread kernels (15 records per pass); every record vs the oracle's record layer."""
    import torch
    rng = np.random.default_rng(4242)
    n = 1200
    lens = rng.integers(0, 16385, n)
    lens[:5] = [0, 1, 16383, 16384, 15]
    trecs = np.zeros(n, ra.TLS_RECORD_DTYPE)
    conn = rng.integers(0, 2 ** 32, n, dtype=np.uint64).astype(np.uint32)
    off = woff = 0
    for i, ln in enumerate(lens):
        trecs[i] = (off, woff, int(rng.integers(0, 2 ** 40)), int(ln), int(rng.choice([21, 22, 23])))
        off += int(ln)
        woff += int(ln) + 22
    key, iv = bytes(range(7, 23)), bytes(range(60, 72))
    src = np.frombuffer(xs(77, off + 16), np.uint8)
    d_src, d_recs, d_conn = dev(src), dev(trecs.view(np.uint8)), dev(conn.view(np.int32))
    d_wire = torch.zeros(woff + 16, dtype=torch.uint8, device="cuda")
    eng = ra.Engine(key)
    eng.tls_seal_records(iv, d_recs.data_ptr(), n, d_src.data_ptr(), d_wire.data_ptr(), conn_ptr=d_conn.data_ptr())
    torch.cuda.synchronize()
    wire = to_cpu(d_wire)
    for i in range(n):
        t = trecs[i]
        frag = bytes(src[int(t["src"]): int(t["src"]) + int(t["len"])])
        civ = (int.from_bytes(iv[:4], "big") ^ int(conn[i])).to_bytes(4, "big") + iv[4:]
        want = oracle.tls_seal_record(key, civ, int(t["seq"]), int(t["type"]), frag)
        assert bytes(wire[int(t["dst"]): int(t["dst"]) + len(want)]) == want, i
    orecs = trecs.copy()
    orecs["src"], orecs["len"] = trecs["dst"], trecs["len"] + 17
    orecs["dst"] = np.concatenate([[0], np.cumsum(trecs["len"].astype(np.int64) + 1)[:-1]]).astype(np.uint64)
    d_orecs = dev(orecs.view(np.uint8))
    d_pt = torch.zeros(int(orecs["dst"][-1]) + int(trecs["len"][-1]) + 17, dtype=torch.uint8, device="cuda")
    d_st = torch.zeros(n, dtype=torch.int32, device="cuda")
    d_ty = torch.zeros(n, dtype=torch.uint8, device="cuda")
    eng.tls_open_records(iv, d_orecs.data_ptr(), n, d_wire.data_ptr(), d_pt.data_ptr(), d_st.data_ptr(), d_ty.data_ptr(),
                         conn_ptr=d_conn.data_ptr())
    torch.cuda.synchronize()
    st, ty, pt = to_cpu(d_st).view(np.uint32), to_cpu(d_ty), to_cpu(d_pt)
    assert (st == trecs["len"]).all() and (ty == trecs["type"]).all()
    for i in range(n):
        a, b = int(orecs["dst"][i]), int(trecs["src"][i])
        assert bytes(pt[a: a + int(lens[i])]) == bytes(src[b: b + int(lens[i])]), i
    eng.close()


@pytest.mark.parametrize("multi", [False, True])
def test_open_stop_at_first_failure(gpu, multi):
    """PTLS_MI355X_OPEN_STOP_AT_FAILURE: ptls_receive stops at the first record that fails and does not advance seq
    (lib/picotls.c:650-652, 4790), so records of the same connection behind it are never delivered.  The batch open
    marks them TLS_NOT_PROCESSED with a zeroed plaintext slot; records before the failure, and every record of the
    other connections, are opened as usual.  Without the flag every record is verified independently."""
    import torch
    key, iv = bytes(range(16)), bytes(range(12))
    nconn, per = (3, 6) if multi else (1, 10)
    conns = [7, 1, 0xABCDEF01][:nconn]
    trecs = np.zeros(nconn * per, ra.TLS_RECORD_DTYPE)
    conn = np.zeros(len(trecs), np.uint32)
    lens = [100, 1400, 16384, 0, 17, 300, 5000, 64, 1, 2000]
    frags, off, wire_off = [], 0, 0
    for ci, c in enumerate(conns):
        for k in range(per):
            i = ci * per + k
            ln = lens[k]
            trecs[i] = (off, wire_off, 500 + k, ln, 23)
            conn[i] = c if multi else 0
            frags.append(xorshift64star(300 + i, ln).tobytes())
            off += ln
            wire_off += ln + 22
    src = np.frombuffer(b"".join(frags), np.uint8) if off else np.zeros(1, np.uint8)
    d_src, d_recs, d_conn = dev(src), dev(trecs.view(np.uint8)), dev(conn.view(np.int32))
    d_wire = torch.zeros(wire_off, dtype=torch.uint8, device="cuda")
    eng = ra.Engine(key)
    eng.tls_seal_records(iv, d_recs.data_ptr(), len(trecs), d_src.data_ptr(), d_wire.data_ptr(),
                         conn_ptr=d_conn.data_ptr() if multi else 0)
    torch.cuda.synchronize()
    wire = to_cpu(d_wire).copy()
    orecs = trecs.copy()
    orecs["src"] = trecs["dst"]
    orecs["len"] = trecs["len"] + 17
    orecs["dst"] = np.cumsum([0] + [ln + 1 for ln in trecs["len"][:-1]]).astype(np.uint64)
    # connection 0: record 3 tampered; connection 1 (multi): record 1 and 4 tampered; connection 2: none
    bad = {3} if not multi else {3, per + 1, per + 4}
    for i in bad:
        wire[int(orecs[i]["src"]) + 5] ^= 0x40
    pt_size = int(orecs["dst"][-1]) + int(orecs["len"][-1])
    for flags in (0, ra.OPEN_STOP_AT_FAILURE):
        d_w, d_o, d_ids = dev(wire), dev(orecs.view(np.uint8)), dev(conn.view(np.int32))
        d_pt = torch.full((pt_size,), 0xAA, dtype=torch.uint8, device="cuda")
        d_st = torch.zeros(len(orecs), dtype=torch.int32, device="cuda")
        d_ty = torch.zeros(len(orecs), dtype=torch.uint8, device="cuda")
        eng.tls_open_records(iv, d_o.data_ptr(), len(orecs), d_w.data_ptr(), d_pt.data_ptr(), d_st.data_ptr(),
                             d_ty.data_ptr(), conn_ptr=d_ids.data_ptr() if multi else 0, flags=flags)
        torch.cuda.synchronize()
        st, ty, pt = to_cpu(d_st).view(np.uint32), to_cpu(d_ty), to_cpu(d_pt)
        for ci in range(nconn):
            first_bad = min([i for i in bad if ci * per <= i < (ci + 1) * per], default=None)
            for i in range(ci * per, (ci + 1) * per):
                a, n = int(orecs[i]["dst"]), int(trecs[i]["len"])
                if flags and first_bad is not None and i > first_bad:  # never reached by ptls_receive
                    assert st[i] == ra.TLS_NOT_PROCESSED and ty[i] == 0, (flags, i, st[i])
                    assert not pt[a:a + n + 1].any(), (flags, i)
                elif i in bad:
                    assert st[i] == ra.TLS_BAD_RECORD_MAC, (flags, i)
                else:
                    assert st[i] == n and ty[i] == 23, (flags, i, st[i])
                    assert pt[a:a + n].tobytes() == frags[i], (flags, i)
    eng.close()


def test_open_stop_at_failure_two_streams(gpu):
    """Two STOP_AT_FAILURE opens from one context on two streams, the second launched while the first still runs: each
    stops at its own first failure (the per-context scratch of the stop pass is ordered across streams)."""
    import torch
    key, iv = bytes(range(16)), bytes(range(12))
    eng = ra.Engine(key)

    def batch(n, ln, bad, seed):
        trecs = np.zeros(n, ra.TLS_RECORD_DTYPE)
        trecs["src"] = np.arange(n, dtype=np.uint64) * ln
        trecs["dst"] = np.arange(n, dtype=np.uint64) * (ln + 22)
        trecs["seq"] = np.arange(n, dtype=np.uint64) + seed
        trecs["len"] = ln
        trecs["type"] = 23
        src = xorshift64star(seed, n * ln)
        d_wire = torch.zeros(n * (ln + 22), dtype=torch.uint8, device="cuda")
        d_recs, d_src = dev(trecs.view(np.uint8)), dev(src)  # alive until the seal has run
        eng.tls_seal_records(iv, d_recs.data_ptr(), n, d_src.data_ptr(), d_wire.data_ptr())
        torch.cuda.synchronize()
        wire = to_cpu(d_wire).copy()
        wire[bad * (ln + 22) + 9] ^= 0x10
        orecs = trecs.copy()
        orecs["src"], orecs["dst"], orecs["len"] = trecs["dst"], np.arange(n, dtype=np.uint64) * (ln + 1), ln + 17
        return orecs, dev(wire), src

    jobs = [batch(60000, 1400, 41000, 1), batch(500, 1400, 37, 900000)]
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    outs = []
    for (orecs, d_w, _), s in zip(jobs, streams):
        n = len(orecs)
        d_o = dev(orecs.view(np.uint8))
        d_pt = torch.full((n * 1401,), 0xAA, dtype=torch.uint8, device="cuda")
        d_st = torch.zeros(n, dtype=torch.int32, device="cuda")
        d_ty = torch.zeros(n, dtype=torch.uint8, device="cuda")
        torch.cuda.synchronize()
        outs.append((d_o, d_pt, d_st, d_ty))
    for (orecs, d_w, _), (d_o, d_pt, d_st, d_ty), s in zip(jobs, outs, streams):  # back to back, no sync between
        eng.tls_open_records(iv, d_o.data_ptr(), len(orecs), d_w.data_ptr(), d_pt.data_ptr(), d_st.data_ptr(),
                             d_ty.data_ptr(), stream=s.cuda_stream, flags=ra.OPEN_STOP_AT_FAILURE)
    torch.cuda.synchronize()
    for (orecs, _, src), (_, d_pt, d_st, _), bad in zip(jobs, outs, (41000, 37)):
        st = to_cpu(d_st).view(np.uint32)
        assert (st[:bad] == 1400).all() and st[bad] == ra.TLS_BAD_RECORD_MAC
        assert (st[bad + 1:] == ra.TLS_NOT_PROCESSED).all()
        pt = to_cpu(d_pt).reshape(-1, 1401)
        assert pt[:bad, :1400].tobytes() == src[:bad * 1400].tobytes()
        assert not pt[bad + 1:].any()
    eng.close()
