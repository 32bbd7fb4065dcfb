"""GPU parity of the resident window engine (include/ptls_mi355x.h section 6): the split runs and the delivery
executed as jobs of the persistent grid must give exactly the bytes of the stream launches (themselves pinned to the
reference's ptls_send / ptls_receive by tests/test_gpu_tls.py) and of the oracle; plus the grid's own mechanics --
many jobs in flight past the ring's size, contexts freed and recreated under a running grid (key images at reused
addresses), dependent delivery jobs, the idle exit and the relaunch."""
import time

import numpy as np
import pytest

import oracle
import rapido_amd as ra

pytestmark = pytest.mark.gpu


def dev(a):
    import torch
    return torch.from_numpy(np.array(a, copy=True)).cuda()


def window(rng, lens, types=(23,)):
    """TLS records of the given fragment lengths, back to back, with their seal and open descriptors."""
    n = len(lens)
    trecs = np.zeros(n, ra.TLS_RECORD_DTYPE)
    off = woff = 0
    for i, ln in enumerate(lens):
        trecs[i] = (off, woff, int(rng.integers(0, 2 ** 40)), ln, types[i % len(types)])
        off += int(ln)
        woff += int(ln) + 22
    src = rng.integers(0, 256, max(off, 1), dtype=np.uint8)
    orecs = trecs.copy()
    orecs["src"], orecs["len"] = trecs["dst"], trecs["len"] + 17
    # the plaintext slots of an open: each record's len - 16 bytes (fragment + type byte), back to back
    orecs["dst"] = np.concatenate([[0], np.cumsum(trecs["len"].astype(np.uint64) + 1)[:-1]]) if n else []
    return trecs, orecs, src, woff


def seal_resident(eng, iv, trecs, src, wire_size, conn=None):
    import torch
    d_src, d_recs = dev(src), dev(trecs.view(np.uint8))
    d_dst = torch.zeros(max(wire_size, 1), dtype=torch.uint8, device="cuda")
    d_conn = dev(conn) if conn is not None else None
    torch.cuda.synchronize()
    job = eng.resident_tls_seal_records(iv, d_recs.data_ptr(), len(trecs), d_src.data_ptr(), d_dst.data_ptr(),
                                        d_conn.data_ptr() if d_conn is not None else 0)
    eng.resident_wait(job)
    assert eng.resident_done(job)
    return d_dst.cpu().numpy()


def seal_stream(eng, iv, trecs, src, wire_size, conn=None):
    import torch
    d_src, d_recs = dev(src), dev(trecs.view(np.uint8))
    d_dst = torch.zeros(max(wire_size, 1), dtype=torch.uint8, device="cuda")
    d_conn = dev(conn) if conn is not None else None
    eng.tls_seal_records(iv, d_recs.data_ptr(), len(trecs), d_src.data_ptr(), d_dst.data_ptr(),
                         conn_ptr=d_conn.data_ptr() if d_conn is not None else 0)
    torch.cuda.synchronize()
    return d_dst.cpu().numpy()


def open_resident(eng, iv, orecs, wire, pt_size):
    import torch
    d_wire, d_recs = dev(wire), dev(orecs.view(np.uint8))
    d_pt = torch.zeros(max(pt_size, 1), dtype=torch.uint8, device="cuda")
    d_st = torch.zeros(max(len(orecs), 1), dtype=torch.int32, device="cuda")
    d_ty = torch.zeros(max(len(orecs), 1), dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    job = eng.resident_tls_open_records(iv, d_recs.data_ptr(), len(orecs), d_wire.data_ptr(), d_pt.data_ptr(),
                                        d_st.data_ptr(), d_ty.data_ptr())
    eng.resident_wait(job)
    return d_pt.cpu().numpy(), d_st.cpu().numpy().view(np.uint32)[: len(orecs)], d_ty.cpu().numpy()[: len(orecs)]


def open_stream(eng, iv, orecs, wire, pt_size):
    import torch
    d_wire, d_recs = dev(wire), dev(orecs.view(np.uint8))
    d_pt = torch.zeros(max(pt_size, 1), dtype=torch.uint8, device="cuda")
    d_st = torch.zeros(max(len(orecs), 1), dtype=torch.int32, device="cuda")
    d_ty = torch.zeros(max(len(orecs), 1), dtype=torch.uint8, device="cuda")
    eng.tls_open_records(iv, d_recs.data_ptr(), len(orecs), d_wire.data_ptr(), d_pt.data_ptr(), d_st.data_ptr(),
                         d_ty.data_ptr())
    torch.cuda.synchronize()
    return d_pt.cpu().numpy(), d_st.cpu().numpy().view(np.uint32)[: len(orecs)], d_ty.cpu().numpy()[: len(orecs)]


def edge_lens(rng):
    return list(range(0, 40)) + [255, 256, 1399, 1400, 1401, 4095, 16383, 16384] + \
        [int(x) for x in rng.integers(0, 16385, 24)]


@pytest.mark.parametrize("keylen", [16, 32])
def test_resident_seal_and_open_match_the_oracle(gpu, keylen):
    """Every length around the block edges up to a full record, four content types: wire bytes against the
    oracle's ptls_send restatement; the open back: plaintext, inner type and status."""
    rng = np.random.default_rng(7000 + keylen)
    key, iv = rng.integers(0, 256, keylen, dtype=np.uint8).tobytes(), rng.integers(0, 256, 12, dtype=np.uint8).tobytes()
    trecs, orecs, src, wsize = window(rng, edge_lens(rng), types=(23, 22, 21, 0x40))
    eng = ra.Engine(key)
    wire = seal_resident(eng, iv, trecs, src, wsize)
    for t in trecs:
        frag = src[int(t["src"]): int(t["src"]) + int(t["len"])].tobytes()
        want = oracle.tls_seal_record(key, iv, int(t["seq"]), int(t["type"]), frag)
        assert wire[int(t["dst"]): int(t["dst"]) + len(want)].tobytes() == want, int(t["len"])
    pt, st, ty = open_resident(eng, iv, orecs, wire, int(orecs["len"].astype(np.int64).sum()))
    assert list(st) == list(trecs["len"]) and list(ty) == list(trecs["type"])
    for t, o in zip(trecs, orecs):
        assert pt[int(o["dst"]): int(o["dst"]) + int(t["len"])].tobytes() == \
            src[int(t["src"]): int(t["src"]) + int(t["len"])].tobytes()
    eng.close()


@pytest.mark.parametrize("keylen", [16, 32])
def test_resident_equals_stream_launches(gpu, keylen):
    """The same window (16 full records, per-record connection ids) through the stream kernels and the resident
    grid: identical wire bytes; a tampered record fails alone, its plaintext zeroed, identically."""
    rng = np.random.default_rng(7100 + keylen)
    key, iv = rng.integers(0, 256, keylen, dtype=np.uint8).tobytes(), rng.integers(0, 256, 12, dtype=np.uint8).tobytes()
    trecs, orecs, src, wsize = window(rng, [16384] * 15 + [1000])
    conn = rng.integers(0, 2 ** 32, len(trecs), dtype=np.uint64).astype(np.uint32)
    eng = ra.Engine(key)
    a = seal_stream(eng, iv, trecs, src, wsize, conn)
    b = seal_resident(eng, iv, trecs, src, wsize, conn)
    assert a.tobytes() == b.tobytes()
    wire = seal_stream(eng, iv, trecs, src, wsize)
    bad = wire.copy()
    bad[int(trecs[3]["dst"]) + 100] ^= 1
    pts = int(orecs["len"].astype(np.int64).sum())
    p1, s1, t1 = open_stream(eng, iv, orecs, bad, pts)
    p2, s2, t2 = open_resident(eng, iv, orecs, bad, pts)
    assert s2[3] == ra.TLS_BAD_RECORD_MAC and list(s1) == list(s2)
    assert p1.tobytes() == p2.tobytes() and t1.tobytes() == t2.tobytes()
    eng.close()


def test_resident_many_jobs_in_flight_past_the_ring(gpu):
    """260 windows of 260 contexts (a context's run jobs go one at a time) posted before any wait: the ring holds 256,
    so the last posts wait for the oldest entries; two keys taking turns, each window checked against the oracle."""
    import torch
    rng = np.random.default_rng(7200)
    keys = [rng.integers(0, 256, 16, dtype=np.uint8).tobytes(), rng.integers(0, 256, 32, dtype=np.uint8).tobytes()]
    iv = rng.integers(0, 256, 12, dtype=np.uint8).tobytes()
    nwin = 260
    engs = [ra.Engine(keys[i % 2]) for i in range(nwin)]
    wins = []
    for w in range(nwin):
        trecs, _, src, wsize = window(rng, [int(x) for x in rng.integers(0, 2000, 4)])
        wins.append((trecs, src, dev(src), dev(trecs.view(np.uint8)),
                     torch.zeros(max(wsize, 1), dtype=torch.uint8, device="cuda")))
    torch.cuda.synchronize()
    jobs = [engs[w].resident_tls_seal_records(iv, d_recs.data_ptr(), len(trecs), d_src.data_ptr(), d_dst.data_ptr())
            for w, (trecs, _, d_src, d_recs, d_dst) in enumerate(wins)]
    assert jobs == list(range(jobs[0], jobs[0] + nwin))
    for w, (trecs, src, _, _, d_dst) in enumerate(wins):
        engs[w].resident_wait(jobs[w])
        wire = d_dst.cpu().numpy()
        for t in trecs:
            frag = src[int(t["src"]): int(t["src"]) + int(t["len"])].tobytes()
            want = oracle.tls_seal_record(keys[w % 2], iv, int(t["seq"]), int(t["type"]), frag)
            assert wire[int(t["dst"]): int(t["dst"]) + len(want)].tobytes() == want
    for e in engs:
        e.close()


def test_resident_new_keys_at_reused_addresses(gpu):
    """Contexts freed and created again while the grid runs (their key images land at addresses the grid has read
    before): every window seals under its own context's key."""
    rng = np.random.default_rng(7300)
    iv = rng.integers(0, 256, 12, dtype=np.uint8).tobytes()
    for _ in range(12):
        key = rng.integers(0, 256, 16, dtype=np.uint8).tobytes()
        eng = ra.Engine(key)
        trecs, _, src, wsize = window(rng, [int(x) for x in rng.integers(1, 3000, 3)])
        wire = seal_resident(eng, iv, trecs, src, wsize)
        for t in trecs:
            frag = src[int(t["src"]): int(t["src"]) + int(t["len"])].tobytes()
            want = oracle.tls_seal_record(key, iv, int(t["seq"]), int(t["type"]), frag)
            assert wire[int(t["dst"]): int(t["dst"]) + len(want)].tobytes() == want
        eng.close()


def test_resident_delivery_follows_its_open(gpu):
    """An open job and the delivery job behind it, posted back to back: the delivered plaintexts are those of the
    stream delivery (stop at the tampered record, the non-application-data record, the capacity)."""
    import torch
    rng = np.random.default_rng(7400)
    key, iv = rng.integers(0, 256, 16, dtype=np.uint8).tobytes(), rng.integers(0, 256, 12, dtype=np.uint8).tobytes()
    eng = ra.Engine(key)
    parts_spec = [(list(range(100, 116)), None, None, 1 << 20),   # all delivered
                  ([3000] * 8, 5, None, 1 << 20),                 # stops at the tampered 6th record
                  ([500] * 6, None, 2, 1 << 20),                  # stops at the handshake record (3rd)
                  ([4000] * 5, None, None, 9000)]                 # capacity: two records
    lens, types, tamper = [], [], []
    for ls, bad, hs, _ in parts_spec:
        for i, ln in enumerate(ls):
            lens.append(ln)
            types.append(22 if hs is not None and i == hs else 23)
            tamper.append(bad is not None and i == bad)
    trecs, orecs, src, wsize = window(rng, lens)
    trecs["type"] = types
    wire = seal_stream(eng, iv, trecs, src, wsize)
    for i, t in enumerate(trecs):
        if tamper[i]:
            wire[int(t["dst"]) + 7] ^= 0x80
    # slots 16-aligned, as the record layer lays them out for the delivery kernel
    slot = [(int(t["len"]) + 1 + 15) // 16 * 16 for t in trecs]
    orecs["dst"] = np.concatenate([[0], np.cumsum(slot)[:-1]])
    d_wire, d_orecs = dev(wire), dev(orecs.view(np.uint8))
    d_slots = torch.zeros(sum(slot), dtype=torch.uint8, device="cuda")
    d_st = torch.zeros(len(orecs), dtype=torch.int32, device="cuda")
    d_ty = torch.zeros(len(orecs), dtype=torch.uint8, device="cuda")
    outs_a = [torch.zeros(cap, dtype=torch.uint8, device="cuda") for *_, cap in parts_spec]
    outs_b = [torch.zeros(cap, dtype=torch.uint8, device="cuda") for *_, cap in parts_spec]

    def parts_of(outs):
        p = np.zeros(len(parts_spec), ra.TLS_DELIVER_DTYPE)
        k0 = 0
        for i, ((ls, *_), o) in enumerate(zip(parts_spec, outs)):
            p[i] = (d_slots.data_ptr(), o.data_ptr(), o.numel(), k0, len(ls), 0, 0)
            k0 += len(ls)
        return dev(p.view(np.uint8))

    maxp = max(len(p[0]) for p in parts_spec)
    # stream: open + delivery
    eng.tls_open_records(iv, d_orecs.data_ptr(), len(orecs), d_wire.data_ptr(), d_slots.data_ptr(), d_st.data_ptr(),
                         d_ty.data_ptr())
    pa = parts_of(outs_a)
    assert ra.lib().ptls_mi355x_tls_deliver_records(eng.handle, d_orecs.data_ptr(), d_st.data_ptr(), d_ty.data_ptr(),
                                                    pa.data_ptr(), len(parts_spec), maxp, None) == 0
    torch.cuda.synchronize()
    st_a = d_st.cpu().numpy().copy()
    d_slots.zero_()
    d_st.zero_()
    d_ty.zero_()
    pb = parts_of(outs_b)
    torch.cuda.synchronize()
    j1 = eng.resident_tls_open_records(iv, d_orecs.data_ptr(), len(orecs), d_wire.data_ptr(), d_slots.data_ptr(),
                                       d_st.data_ptr(), d_ty.data_ptr())
    j2 = eng.resident_tls_deliver_records(d_orecs.data_ptr(), d_st.data_ptr(), d_ty.data_ptr(), pb.data_ptr(),
                                          len(parts_spec), maxp)
    assert j2 > j1
    eng.resident_wait(j2)
    assert eng.resident_done(j1)
    assert (d_st.cpu().numpy() == st_a).all()
    for a, b in zip(outs_a, outs_b):
        assert a.cpu().numpy().tobytes() == b.cpu().numpy().tobytes()
    # and the delivered bytes are the fragments, up to each part's stop
    k0 = 0
    for (ls, bad, hs, cap), o in zip(parts_spec, outs_b):
        stop = min(x for x in (bad, hs, len(ls)) if x is not None)
        want, tot = b"", 0
        for i in range(stop):
            t = trecs[k0 + i]
            if tot + int(t["len"]) > cap:
                break
            want += src[int(t["src"]): int(t["src"]) + int(t["len"])].tobytes()
            tot += int(t["len"])
        assert o.cpu().numpy()[: len(want)].tobytes() == want
        k0 += len(ls)
    eng.close()


def test_resident_idle_exit_and_relaunch(gpu):
    """A grid with a 2 ms idle time leaves after it; the next job starts a new one (launch count + 1) and completes;
    ptls_mi355x_resident_stop ends it and a later job creates the engine again."""
    rng = np.random.default_rng(7500)
    key, iv = rng.integers(0, 256, 16, dtype=np.uint8).tobytes(), rng.integers(0, 256, 12, dtype=np.uint8).tobytes()
    ra.resident_stop(0)
    prev_idle = ra.set_resident_idle_us(2000)
    try:
        eng = ra.Engine(key)
        trecs, _, src, wsize = window(rng, [1400] * 4)
        w1 = seal_resident(eng, iv, trecs, src, wsize)
        n1 = ra.resident_launches(0)
        assert n1 >= 1
        time.sleep(0.05)  # well past the idle time: the grid has left
        w2 = seal_resident(eng, iv, trecs, src, wsize)
        assert ra.resident_launches(0) == n1 + 1
        assert w1.tobytes() == w2.tobytes()
        ra.resident_stop(0)
        assert ra.resident_launches(0) == 0  # the engine is gone; the next job makes a new one
        w3 = seal_resident(eng, iv, trecs, src, wsize)
        assert w3.tobytes() == w1.tobytes() and ra.resident_launches(0) == 1
        eng.close()
    finally:
        ra.resident_stop(0)
        ra.set_resident_idle_us(prev_idle)


def test_resident_then_stream_on_one_context(gpu):
    """A context alternating between resident jobs and stream launches of the split kernels (they share its
    tickets): every window correct."""
    rng = np.random.default_rng(7600)
    key, iv = rng.integers(0, 256, 16, dtype=np.uint8).tobytes(), rng.integers(0, 256, 12, dtype=np.uint8).tobytes()
    eng = ra.Engine(key)
    for i in range(6):
        trecs, _, src, wsize = window(rng, [int(x) for x in rng.integers(1, 16385, 8)])
        w = (seal_resident if i % 2 else seal_stream)(eng, iv, trecs, src, wsize)
        for t in trecs:
            frag = src[int(t["src"]): int(t["src"]) + int(t["len"])].tobytes()
            want = oracle.tls_seal_record(key, iv, int(t["seq"]), int(t["type"]), frag)
            assert w[int(t["dst"]): int(t["dst"]) + len(want)].tobytes() == want
    eng.close()


def test_resident_lifetime_exit_under_load(gpu, monkeypatch):
    """A grid whose lifetime (1 s) runs out while jobs keep coming: it stops publishing, leaves once its jobs are
    complete, and the host starts the next instance for the jobs posted meanwhile -- every window correct."""
    rng = np.random.default_rng(7700)
    key, iv = rng.integers(0, 256, 16, dtype=np.uint8).tobytes(), rng.integers(0, 256, 12, dtype=np.uint8).tobytes()
    ra.resident_stop(0)
    monkeypatch.setenv("PTLS_MI355X_RESIDENT_LIFETIME_S", "1")
    try:
        eng = ra.Engine(key)
        trecs, _, src, wsize = window(rng, [4000] * 4)
        want = seal_stream(eng, iv, trecs, src, wsize).tobytes()
        t0, n = time.time(), 0
        while time.time() - t0 < 2.5:
            assert seal_resident(eng, iv, trecs, src, wsize).tobytes() == want
            n += 1
        assert ra.resident_launches(0) >= 2 and n > 100
        eng.close()
    finally:
        ra.resident_stop(0)  # (the next engine reads the restored environment)


def test_resident_copy_job_then_runs(gpu):
    """A copy job staging a window's input from pinned host memory into device memory (three ranges: whole, at an odd
    offset and length, and a few bytes), then the run job reading the copy -- the wire bytes of the stream kernels on
    the original; the copied bytes exact, nothing outside the ranges written."""
    import ctypes

    import torch
    rng = np.random.default_rng(7800)
    key, iv = rng.integers(0, 256, 16, dtype=np.uint8).tobytes(), rng.integers(0, 256, 12, dtype=np.uint8).tobytes()
    eng = ra.Engine(key)
    trecs, _, src, wsize = window(rng, [16384] * 6 + [777, 5000])
    host = torch.from_numpy(np.concatenate([src, rng.integers(0, 256, 9000, dtype=np.uint8)])).pin_memory()
    hip = ctypes.CDLL("libamdhip64.so")
    hp = ctypes.c_void_p()
    assert hip.hipHostGetDevicePointer(ctypes.byref(hp), ctypes.c_void_p(host.data_ptr()), 0) == 0
    d_in = torch.zeros(len(src) + 9000, dtype=torch.uint8, device="cuda")
    d_recs = dev(trecs.view(np.uint8))
    d_dst = torch.zeros(wsize, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    n = len(src)
    ranges = [(d_in.data_ptr(), hp.value, n), (d_in.data_ptr() + n + 3, hp.value + n + 3, 8191), (d_in.data_ptr() + n + 8200, hp.value + n + 8200, 5)]
    j1 = eng.resident_copy(ranges)
    j2 = eng.resident_tls_seal_records(iv, d_recs.data_ptr(), len(trecs), d_in.data_ptr(), d_dst.data_ptr())
    eng.resident_wait(j2)
    assert eng.resident_done(j1)
    got = d_in.cpu().numpy()
    h = host.numpy()
    assert got[:n].tobytes() == h[:n].tobytes()
    assert got[n: n + 3].tobytes() == b"\0" * 3 and got[n + 3: n + 3 + 8191].tobytes() == h[n + 3: n + 3 + 8191].tobytes()
    assert got[n + 3 + 8191: n + 8200].tobytes() == b"\0" * 6 and got[n + 8200: n + 8205].tobytes() == h[n + 8200: n + 8205].tobytes()
    assert not got[n + 8205:].any()
    assert d_dst.cpu().numpy().tobytes() == seal_stream(eng, iv, trecs, src, wsize).tobytes()
    eng.close()


def test_resident_many_relaunches(gpu):
    """A 300-us idle time and jobs arriving every 0-600 us: the grid leaves and starts again dozens of times (each new
    instance's workers read their starting job before its dispatcher publishes anything) -- every window correct."""
    rng = np.random.default_rng(7900)
    key, iv = rng.integers(0, 256, 16, dtype=np.uint8).tobytes(), rng.integers(0, 256, 12, dtype=np.uint8).tobytes()
    ra.resident_stop(0)
    prev_idle = ra.set_resident_idle_us(300)
    try:
        eng = ra.Engine(key)
        trecs, _, src, wsize = window(rng, [3000, 100])
        want = seal_stream(eng, iv, trecs, src, wsize).tobytes()
        import torch
        d_src, d_recs = dev(src), dev(trecs.view(np.uint8))
        d_dst = torch.zeros(wsize, dtype=torch.uint8, device="cuda")
        torch.cuda.synchronize()
        for i in range(150):
            d_dst.zero_()
            torch.cuda.synchronize()
            job = eng.resident_tls_seal_records(iv, d_recs.data_ptr(), len(trecs), d_src.data_ptr(), d_dst.data_ptr())
            eng.resident_wait(job)
            assert d_dst.cpu().numpy().tobytes() == want, i
            time.sleep(float(rng.uniform(0, 0.0006)))
        assert ra.resident_launches(0) > 10
        eng.close()
    finally:
        ra.resident_stop(0)
        ra.set_resident_idle_us(prev_idle)
