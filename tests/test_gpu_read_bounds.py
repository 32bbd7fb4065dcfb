"""Every kernel family against guard pages: records, AAD, descriptors and outputs flush against unmapped memory.

tests/cpp/guard_alloc.c maps the middle third of a reserved virtual range (HIP virtual memory) and leaves the two
outer thirds unmapped, so one byte read or written past a buffer's end (or before its start) is a GPU page fault,
reported by the device check after each case.  Round 4's intermittent illegal address needed an allocation that
happened to end at a page edge; here every case puts its record at both edges, for each kernel family of
conftest.FAMILIES, AEAD (section 3) and TLS-framed (section 4), sealing and opening, separate and in place (seal with
the fragment 5 bytes into its record slot, dst = src - 5; open over the wire record, dst = src + 5).  The CPU
counterpart, tests/test_read_bounds.py, checks the walk's every read against the record bounds in the host model."""
import ctypes as C

import numpy as np
import pytest

import oracle
import rapido_amd as ra
from conftest import FAMILIES, kernel_family
from rapido_amd.records import xorshift64star
from rapido_amd.hostmem import to_cpu, to_gpu

pytestmark = pytest.mark.gpu

LENS = [0, 1, 15, 16, 17, 100, 1399, 1400, 4097, 16383, 16384]
AADS = [0, 5, 13, 16, 17, 32]
REGION = 64 << 10  # rounded up to the allocation granularity


class Guard(C.Structure):
    _fields_ = [("reserved", C.c_void_p), ("reserved_len", C.c_size_t), ("data", C.c_void_p), ("len", C.c_size_t),
                ("handle", C.c_void_p)]


@pytest.fixture(scope="module")
def guards(gpu):
    from rapido_amd import build
    lib = C.CDLL(build.build_guard())
    lib.guard_alloc.argtypes = [C.c_size_t, C.POINTER(Guard)]
    lib.guard_free.argtypes = [C.POINTER(Guard)]
    for f in ("guard_h2d", "guard_d2h"):
        getattr(lib, f).argtypes = [C.c_void_p, C.c_void_p, C.c_size_t]
    lib.guard_memset.argtypes = [C.c_void_p, C.c_int, C.c_size_t]
    assert lib.guard_struct_size() == C.sizeof(Guard)
    gs = []
    for _ in range(3):  # inputs | descriptors, AAD, statuses | outputs
        g = Guard()
        rc = lib.guard_alloc(REGION, C.byref(g))
        if rc == -1:
            pytest.skip("device without HIP virtual memory management")
        assert rc == 0, f"guard_alloc: HIP error {rc}"
        gs.append(g)
    yield lib, gs
    for g in gs:
        assert lib.guard_free(C.byref(g)) == 0


class Region:
    """A guarded region: place(bytes, at="start"|"end") -> device address of bytes copied flush against that edge."""

    def __init__(self, lib, g):
        self.lib, self.base, self.len = lib, g.data, g.len

    def addr(self, nbytes, at):
        assert nbytes <= self.len
        return self.base if at == "start" else self.base + self.len - nbytes

    def put(self, data, at):
        data = np.ascontiguousarray(np.frombuffer(bytes(data), np.uint8))
        a = self.addr(len(data), at)
        assert self.lib.guard_h2d(a, data.ctypes.data, len(data)) == 0
        return a

    def get(self, a, n):
        out = np.zeros(max(n, 1), np.uint8)
        assert self.lib.guard_d2h(out.ctypes.data, a, n) == 0
        return out[:n].tobytes()

    def clear(self):
        assert self.lib.guard_memset(self.base, 0, self.len) == 0


def checked():
    ra.device_check()  # a page fault of the case just launched fails here, naming it


@pytest.mark.parametrize("family", FAMILIES)
@pytest.mark.parametrize("at", ["start", "end"])
def test_aead_records_at_guard_edges(guards, family, at):
    lib, gs = guards
    IN, AUX, OUT = (Region(lib, g) for g in gs)
    key, iv = bytes(range(16)), bytes(range(70, 82))
    eng = ra.Engine(key)
    other = "end" if at == "start" else "start"
    with kernel_family(family, framing=False):
        for i, ln in enumerate(LENS):
            alen = AADS[i % len(AADS)]
            pt = xorshift64star(900 + i, ln).tobytes()
            aad = xorshift64star(950 + i, alen).tobytes()
            for r in (IN, AUX, OUT):
                r.clear()
            # seal: input and AAD at the edge, descriptor at the other end, output (ciphertext || tag) at the edge
            src = IN.put(pt, at)
            d_aad = AUX.put(aad, at) if alen else AUX.base + AUX.len // 2
            dst = OUT.addr(ln + 16, at)
            rec = np.zeros(1, ra.RECORD_DTYPE)
            rec[0] = (0, 0, 0, 7 + i, ln, alen)
            d_rec = AUX.put(rec.view(np.uint8), other)  # (offsets 0: each arena base is the record itself)
            eng.seal_batch(iv, d_rec, 1, src, dst, d_aad)
            checked()
            ct = OUT.get(dst, ln + 16)
            assert ct == oracle.seal(key, oracle.build_iv(iv, 7 + i), aad, pt), (family, at, ln)
            # open: ciphertext || tag at the edge, plaintext at the edge, status at the other end
            for r in (IN, OUT):
                r.clear()
            src = IN.put(ct, at)
            dst = OUT.addr(max(ln, 1), at) if ln else OUT.base + OUT.len // 2
            st = AUX.base + AUX.len // 2 + 64
            eng.open_batch(iv, d_rec, 1, src, dst, d_aad, st)
            checked()
            assert np.frombuffer(AUX.get(st, 4), np.uint32)[0] == ln
            assert OUT.get(dst, ln) == pt, (family, at, ln)
    eng.close()
    checked()


@pytest.mark.parametrize("family", FAMILIES)
@pytest.mark.parametrize("at", ["start", "end"])
def test_tls_records_at_guard_edges(guards, family, at):
    lib, gs = guards
    IN, AUX, OUT = (Region(lib, g) for g in gs)
    key, iv = bytes(range(5, 21)), bytes(range(90, 102))
    eng = ra.Engine(key)
    other = "end" if at == "start" else "start"
    mid = AUX.base + AUX.len // 2
    with kernel_family(family, framing=True):
        for i, ln in enumerate(LENS):
            frag = xorshift64star(700 + i, ln).tobytes()
            want = oracle.tls_seal_record(key, iv, 40 + i, 23, frag)
            for r in (IN, AUX, OUT):
                r.clear()
            # seal, separate buffers: fragment and wire record flush against the edge
            src = IN.put(frag, at)
            dst = OUT.addr(ln + 22, at)
            t = np.zeros(1, ra.TLS_RECORD_DTYPE)
            t[0] = (0, 0, 40 + i, ln, 23)
            d_t = AUX.put(t.view(np.uint8), other)
            eng.tls_seal_records(iv, d_t, 1, src, dst)
            checked()
            assert OUT.get(dst, ln + 22) == want, (family, at, ln)
            # open, separate buffers: wire record and plaintext slot (fragment + type) flush against the edge
            src = IN.put(want, at)
            dst = OUT.addr(ln + 1, at)
            o = np.zeros(1, ra.TLS_RECORD_DTYPE)
            o[0] = (0, 0, 40 + i, ln + 17, 0)
            d_o = mid + 4096  # (the seal's descriptor stays at the edge for the in-place seal below)
            assert lib.guard_h2d(d_o, o.ctypes.data, o.nbytes) == 0
            eng.tls_open_records(iv, d_o, 1, src, dst, mid, mid + 64)
            checked()
            assert np.frombuffer(AUX.get(mid, 4), np.uint32)[0] == ln and AUX.get(mid + 64, 1) == b"\x17"
            assert OUT.get(dst, ln) == frag, (family, at, ln)
            # in place, as picotls's buffer: seal the fragment 5 bytes into its record slot (dst = src - 5) ...
            OUT.clear()
            slot = OUT.addr(ln + 22, at)
            fb = np.frombuffer(frag, np.uint8).copy()
            assert lib.guard_h2d(slot + 5, fb.ctypes.data, ln) == 0
            eng.tls_seal_records(iv, d_t, 1, slot + 5, slot)  # (descriptor offsets 0: src = slot + 5, dst = slot)
            checked()
            assert OUT.get(slot, ln + 22) == want, (family, at, "in place", ln)
            # ... and open it where it lies, plaintext over header + ciphertext (dst = src + 5)
            eng.tls_open_records(iv, d_o, 1, slot, slot + 5, mid, mid + 64)
            checked()
            assert np.frombuffer(AUX.get(mid, 4), np.uint32)[0] == ln
            assert OUT.get(slot + 5, ln) == frag, (family, at, "in place", ln)
    eng.close()
    checked()


@pytest.mark.parametrize("family", FAMILIES)
@pytest.mark.parametrize("at", ["start", "end"])
def test_tls_window_in_place_at_guard_edges(guards, family, at):
    """test_gpu_tls.py::test_in_place's exact launch -- six records of 0..16384 bytes, back to back in one buffer, sealed
    in ONE launch with each fragment 5 bytes into its slot (dst = src - 5), then opened in one launch where they lie
    (dst = src + 5) -- with the buffer flush against the guard at either end.  The cases above put one record per
    launch at the edges; this is the multi-record group (ten idle lanes, walks of 1 to 1026 steps) that preceded the
    illegal-address report of rounds 4 and 5."""
    lib, gs = guards
    _, AUX, OUT = (Region(lib, g) for g in gs)
    key, iv = bytes(range(16)), bytes(range(12))
    lens = [0, 1, 16, 100, 1400, 16384]
    slots = [ln + 22 for ln in lens]
    base = np.cumsum([0] + slots[:-1]).astype(np.uint64)
    total = int(sum(slots))
    eng = ra.Engine(key)
    with kernel_family(family, framing=True):
        OUT.clear()
        AUX.clear()
        buf = np.zeros(total, np.uint8)
        trecs = np.zeros(len(lens), ra.TLS_RECORD_DTYPE)
        frags = []
        for i, ln in enumerate(lens):
            f = xorshift64star(20 + i, ln).tobytes()
            frags.append(f)
            buf[int(base[i]) + 5: int(base[i]) + 5 + ln] = np.frombuffer(f, np.uint8)
            trecs[i] = (int(base[i]) + 5, int(base[i]), 50 + i, ln, 23)
        arena = OUT.put(buf, at)  # the window's buffer flush against the edge (its last tag ends on it, or its
        d_t = AUX.put(trecs.view(np.uint8), "end" if at == "start" else "start")  # first header starts on it)
        eng.tls_seal_records(iv, d_t, len(lens), arena, arena)
        checked()
        wire = OUT.get(arena, total)
        for i, ln in enumerate(lens):
            b = int(base[i])
            assert wire[b:b + ln + 22] == oracle.tls_seal_record(key, iv, 50 + i, 23, frags[i]), (family, at, ln)
        orecs = trecs.copy()
        orecs["src"], orecs["dst"], orecs["len"] = base, base + 5, np.array(lens) + 17
        mid = AUX.base + AUX.len // 2
        assert lib.guard_h2d(mid + 4096, orecs.ctypes.data, orecs.nbytes) == 0
        eng.tls_open_records(iv, mid + 4096, len(lens), arena, arena, mid, mid + 64)
        checked()
        assert list(np.frombuffer(AUX.get(mid, 4 * len(lens)), np.uint32)) == lens
        pt = OUT.get(arena, total)
        for i, ln in enumerate(lens):
            b = int(base[i]) + 5
            assert pt[b:b + ln] == frags[i], (family, at, ln)
    eng.close()
    checked()


@pytest.mark.parametrize("family", FAMILIES)
@pytest.mark.parametrize("at", ["start", "end"])
def test_status_and_types_at_guard_edges(guards, family, at):
    """The open's per-record outputs -- the status array and the TLS content types -- flush against a guard, and the
    length order (open_batch_ordered) flush against the other edge: the cases above keep them mid-region.  Six records
    (test_in_place's lengths) in one launch, one of them tampered, opened separately, in place, and with
    OPEN_STOP_AT_FAILURE (its later statuses written as TLS_NOT_PROCESSED); a write one element past either end of the
    arrays is a page fault here."""
    lib, gs = guards
    IN, AUX, OUT = (Region(lib, g) for g in gs)
    key, iv = bytes(range(40, 56)), bytes(range(12))
    lens = [0, 1, 16, 100, 1400, 16384]
    n, bad = len(lens), 3
    other = "end" if at == "start" else "start"
    mid_in, mid_aux, mid_out = IN.base + 4096, AUX.base + AUX.len // 2, OUT.base + 4096
    eng = ra.Engine(key)
    with kernel_family(family, framing=True):
        for r in (IN, AUX, OUT):
            r.clear()
        frags = [xorshift64star(60 + i, ln).tobytes() for i, ln in enumerate(lens)]
        wires = [bytearray(oracle.tls_seal_record(key, iv, 9 + i, 23 if i % 2 else 22, f)) for i, f in enumerate(frags)]
        wires[bad][-1] ^= 1
        woff = np.cumsum([0] + [len(w) for w in wires[:-1]]).astype(np.uint64)
        poff = np.cumsum([0] + [ln + 1 for ln in lens[:-1]]).astype(np.uint64)
        wire = b"".join(bytes(w) for w in wires)
        o = np.zeros(n, ra.TLS_RECORD_DTYPE)
        o["src"], o["dst"], o["seq"], o["len"] = woff, poff, 9 + np.arange(n), np.array(lens) + 17
        d_o = mid_aux
        assert lib.guard_h2d(d_o, o.ctypes.data, o.nbytes) == 0
        st, ty = AUX.addr(4 * n, at), OUT.addr(n, at)
        want_ty = [23 if i % 2 else 22 for i in range(n)]
        for flags in (0, ra.OPEN_STOP_AT_FAILURE):
            for inplace in (False, True):
                src = IN.put(wire, other) if inplace else mid_in
                if not inplace:
                    assert lib.guard_h2d(src, np.frombuffer(wire, np.uint8).ctypes.data, len(wire)) == 0
                recs = o.copy()
                if inplace:  # plaintext over each record's own header + ciphertext
                    recs["dst"] = woff + 5
                assert lib.guard_h2d(d_o, recs.ctypes.data, recs.nbytes) == 0
                eng.tls_open_records(iv, d_o, n, src, src if inplace else mid_out, st, ty, flags=flags)
                checked()
                got = list(np.frombuffer(AUX.get(st, 4 * n), np.uint32))
                want = [0xFFFFFFFF if i == bad else ra.TLS_NOT_PROCESSED if flags and i > bad else ln
                        for i, ln in enumerate(lens)]
                assert got == want, (family, at, flags, inplace)
                types = OUT.get(ty, n)
                for i in range(bad):
                    assert types[i] == want_ty[i], (family, at, flags, inplace, i)
                    d = int(recs["dst"][i])
                    pt = IN.get(src + d, lens[i]) if inplace else OUT.get(mid_out + d, lens[i])
                    assert pt == frags[i], (family, at, flags, inplace, i)
    with kernel_family(family, framing=False):
        for r in (IN, AUX, OUT):
            r.clear()
        pts = [xorshift64star(80 + i, ln).tobytes() for i, ln in enumerate(lens)]
        aad = xorshift64star(99, 13).tobytes()
        cts = [bytearray(oracle.seal(key, oracle.build_iv(iv, 5 + i), aad, p)) for i, p in enumerate(pts)]
        cts[bad][0 if lens[bad] == 0 else -1] ^= 1
        coff = np.cumsum([0] + [len(c) for c in cts[:-1]]).astype(np.uint64)
        poff = np.cumsum([0] + lens[:-1]).astype(np.uint64)
        recs = np.zeros(n, ra.RECORD_DTYPE)
        recs["src"], recs["dst"], recs["seq"], recs["len"], recs["aadlen"] = coff, poff, 5 + np.arange(n), lens, 13
        blob = b"".join(bytes(c) for c in cts)
        assert lib.guard_h2d(mid_in, np.frombuffer(blob, np.uint8).ctypes.data, len(blob)) == 0
        d_aad = mid_aux + 8192
        assert lib.guard_h2d(d_aad, np.frombuffer(aad, np.uint8).ctypes.data, 13) == 0
        assert lib.guard_h2d(mid_aux, recs.ctypes.data, recs.nbytes) == 0
        st = AUX.addr(4 * n, at)
        want = [0xFFFFFFFF if i == bad else ln for i, ln in enumerate(lens)]
        eng.open_batch(iv, mid_aux, n, mid_in, mid_out, d_aad, st)
        checked()
        assert list(np.frombuffer(AUX.get(st, 4 * n), np.uint32)) == want, (family, at)
        order = AUX.addr(4 * n, other)
        eng.order_by_length(mid_aux, n, order)
        checked()
        eng.open_batch_ordered(iv, mid_aux, order, n, mid_in, mid_out, d_aad, st)
        checked()
        assert list(np.frombuffer(AUX.get(st, 4 * n), np.uint32)) == want, (family, at, "ordered")
        for i in range(n):
            if i != bad:
                assert OUT.get(mid_out + int(poff[i]), lens[i]) == pts[i], (family, at, i)
    eng.close()
    checked()


@pytest.mark.parametrize("family", ["split", "window16", "batch"])
@pytest.mark.parametrize("at", ["start", "end"])
def test_multikey_records_at_guard_edges(guards, family, at):
    """The multi-key kernels (round 6) against the guards: eleven records of three sessions (LENS, interleaved keys),
    back to back with their inputs, outputs and the key-index array each flush against the edge, the descriptors and
    the statuses flush against the other; sealed, then opened separately and through a shared by-key order, every
    byte against the oracle under its own session's key."""
    import torch  # noqa: F401  (the device is torch's)
    lib, gs = guards
    IN, AUX, OUT = (Region(lib, g) for g in gs)
    keys = [bytes((b + 17 * k) & 0xFF for b in range(16)) for k in range(3)]
    ivs = [bytes((b + 5 * k) & 0xFF for b in range(12)) for k in range(3)]
    engines = [ra.Engine(k) for k in keys]
    mk = ra.MultiKey(engines, ivs)
    other = "end" if at == "start" else "start"
    n = len(LENS)
    kidx = np.array([(i * 2) % 3 for i in range(n)], np.uint32)
    pts = [xorshift64star(300 + i, ln).tobytes() for i, ln in enumerate(LENS)]
    aad = xorshift64star(333, 13).tobytes()
    soff = np.cumsum([0] + LENS[:-1]).astype(np.uint64)
    coff = np.cumsum([0] + [ln + 16 for ln in LENS[:-1]]).astype(np.uint64)
    ssize, csize = int(sum(LENS)), int(sum(LENS)) + 16 * n
    recs = np.zeros(n, ra.RECORD_DTYPE)
    recs["src"], recs["dst"], recs["aad"], recs["seq"], recs["len"], recs["aadlen"] = soff, coff, 0, 3 + np.arange(n), LENS, 13
    wants = [oracle.seal(keys[int(kidx[i])], oracle.build_iv(ivs[int(kidx[i])], 3 + i), aad, p) for i, p in enumerate(pts)]
    with kernel_family(family, framing=False):
        for r in (IN, AUX, OUT):
            r.clear()
        src = IN.put(b"".join(pts), at)
        dst = OUT.addr(csize, at)
        d_k = AUX.put(kidx.view(np.uint8), at)
        d_recs = AUX.put(recs.view(np.uint8), other)
        d_aad = AUX.base + AUX.len // 2
        assert lib.guard_h2d(d_aad, np.frombuffer(aad, np.uint8).ctypes.data, 13) == 0
        mk.seal_batch(d_recs, d_k, n, src, dst, d_aad)
        checked()
        ct = OUT.get(dst, csize)
        for i in range(n):
            c = int(coff[i])
            assert ct[c:c + LENS[i] + 16] == wants[i], (family, at, i)
        # open: ciphertexts at the edge, plaintexts at the edge, statuses at the other end (the descriptors move)
        IN.clear()
        OUT.clear()
        src = IN.put(ct, at)
        dst = OUT.addr(ssize, at)
        o = recs.copy()
        o["src"], o["dst"] = coff, soff
        d_o = AUX.base + AUX.len // 2 + 4096
        assert lib.guard_h2d(d_o, o.ctypes.data, o.nbytes) == 0
        st = AUX.addr(4 * n, other)
        mk.open_batch(d_o, d_k, n, src, dst, d_aad, st)
        checked()
        assert list(np.frombuffer(AUX.get(st, 4 * n), np.uint32)) == LENS, (family, at)
        assert OUT.get(dst, ssize) == b"".join(pts), (family, at)
        if family == "batch":  # the by-key order flush against an edge too (the inputs' other end), read by the open
            OUT.clear()
            order = IN.addr(4 * n, other)
            mk.order_by_key(d_k, n, order)
            checked()
            mk.open_batch_ordered(d_o, d_k, order, n, src, dst, d_aad, st)
            checked()
            assert list(np.frombuffer(AUX.get(st, 4 * n), np.uint32)) == LENS, (family, at, "ordered")
            assert OUT.get(dst, ssize) == b"".join(pts), (family, at, "ordered")
    for e in engines:
        e.close()
    checked()


@pytest.mark.parametrize("at", ["start", "end"])
def test_delivery_at_guard_edges(guards, at):
    """The delivery kernel (ptls_mi355x_tls_deliver_records, handle_input's receive loop on the device) writing each
    part's plaintexts back to back into an `out` flush against a guard, with a capacity of exactly what it should
    take: part A delivers all its records (one of 0 bytes, one of 16 KiB), part B stops before a tampered record and
    part C (any_type) takes one handshake record.  Its outputs, not only its inputs, meet the guard."""
    import torch
    lib, gs = guards
    IN, AUX, OUT = (Region(lib, g) for g in gs)
    key, iv = bytes(range(7, 23)), bytes(range(30, 42))
    lens = [100, 16384, 1, 777, 0, 300, 4096, 50, 60, 200]
    types = [23] * 9 + [22]
    bad = 7
    n = len(lens)
    eng = ra.Engine(key)
    for r in (IN, AUX, OUT):
        r.clear()
    frags = [xorshift64star(500 + i, ln).tobytes() for i, ln in enumerate(lens)]
    wires = [bytearray(oracle.tls_seal_record(key, iv, 3 + i, types[i], f)) for i, f in enumerate(frags)]
    wires[bad][-1] ^= 1
    woff = np.cumsum([0] + [len(w) for w in wires[:-1]]).astype(np.uint64)
    soff = np.cumsum([0] + [(ln + 1 + 15) // 16 * 16 for ln in lens[:-1]]).astype(np.uint64)  # 16-aligned slots
    wire = b"".join(bytes(w) for w in wires)
    d_wire = to_gpu(np.frombuffer(wire, np.uint8).copy())
    d_slots = torch.zeros(int(soff[-1]) + lens[-1] + 17, dtype=torch.uint8, device="cuda")
    o = np.zeros(n, ra.TLS_RECORD_DTYPE)
    o["src"], o["dst"], o["seq"], o["len"] = woff, soff, 3 + np.arange(n), np.array(lens) + 17
    mid = AUX.base + AUX.len // 2
    d_o, st, ty, d_parts = mid, mid - 4096, mid - 2048, mid + 4096
    assert lib.guard_h2d(d_o, o.ctypes.data, o.nbytes) == 0
    eng.tls_open_records(iv, d_o, n, d_wire.data_ptr(), d_slots.data_ptr(), st, ty)
    checked()
    assert list(np.frombuffer(AUX.get(st, 4 * n), np.uint32)) == [0xFFFFFFFF if i == bad else ln
                                                                    for i, ln in enumerate(lens)]
    want_a = b"".join(frags[0:5])
    want_b = b"".join(frags[5:bad])
    want_c = frags[9]
    other = "end" if at == "start" else "start"
    out_a, out_b = OUT.addr(len(want_a), at), OUT.addr(len(want_b), other)
    out_c = IN.addr(len(want_c), at)
    parts = np.zeros(3, ra.TLS_DELIVER_DTYPE)
    parts[0] = (d_slots.data_ptr(), out_a, len(want_a), 0, 5, 0, 0)
    parts[1] = (d_slots.data_ptr(), out_b, len(want_b), 5, 4, 0, 0)
    parts[2] = (d_slots.data_ptr(), out_c, len(want_c), 9, 1, 1, 0)
    assert lib.guard_h2d(d_parts, parts.ctypes.data, parts.nbytes) == 0
    assert ra.lib().ptls_mi355x_tls_deliver_records(eng.handle, d_o, st, ty, d_parts, 3, 5, None) == 0, ra.last_error()
    checked()
    assert OUT.get(out_a, len(want_a)) == want_a, at
    assert OUT.get(out_b, len(want_b)) == want_b, at
    assert IN.get(out_c, len(want_c)) == want_c, at
    eng.close()
    checked()
