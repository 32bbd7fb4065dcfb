"""No kernel family reads or writes outside a record (CPU, deterministic).

The walk's reads (gcm_core.h: walk_load, load_partial, the hoisted AAD block -- every one passes GCM_READ) are checked
by the host model against each record's own bytes: its input (plus the received tag for an open), its AAD, and the
descriptor array the idle loads point at; the walk's stores (every one passes GCM_WRITE) against each record's own
output.  Records sit 48 bytes apart, so a read that strays past either end of a
record -- which faults on the GPU wherever that end is the edge of a mapped page -- lands in a gap and is counted.
Every family the GPU suites route batches to (conftest.FAMILIES: the batch kernels at K = 1, 2, 4, 8, the window
kernels with 4 / 8 lanes and 64- / 32-position segments, the 16-lane and split kernels) is run seal and open, AEAD and
TLS-framed, on lengths around every block, segment and run edge.  tests/test_gpu_read_bounds.py runs the kernels
themselves against guard pages on the GPU."""
import ctypes as C

import numpy as np
import pytest

import oracle
from rapido_amd import RECORD_DTYPE, TLS_RECORD_DTYPE

GAP = 48
LENS = list(range(0, 34)) + [47, 48, 49, 63, 64, 65, 127, 128, 129, 255, 256, 257, 511, 512, 513, 1023, 1024, 1025,
                             1399, 1400, 1401, 4095, 4096, 4097, 8191, 8192, 8193, 16383, 16384, 16385]
AADS = [0, 1, 5, 13, 15, 16, 17, 31, 32, 33]


@pytest.fixture(scope="module")
def model():
    from rapido_amd import build
    lib = C.CDLL(build.build_model())
    vp = C.c_void_p
    lib.model_set_read_ranges.argtypes = [vp, C.c_size_t]
    lib.model_read_violations.argtypes = [vp]
    lib.model_read_violations.restype = C.c_uint64
    lib.model_set_write_ranges.argtypes = [vp, C.c_size_t]
    lib.model_write_violations.argtypes = [vp]
    lib.model_write_violations.restype = C.c_uint64
    lib.model_batch.argtypes = [C.c_int, C.c_int, vp, C.c_size_t, vp, vp, C.c_size_t, vp, vp, vp, vp]
    lib.model_batch_window.argtypes = [C.c_int, vp, C.c_size_t, vp, vp, C.c_size_t, vp, vp, vp, vp]
    lib.model_batch_win16.argtypes = [C.c_int, C.c_int, vp, C.c_size_t, vp, vp, C.c_size_t, vp, vp, vp, vp]
    lib.model_tls_batch.argtypes = [C.c_int, vp, C.c_size_t, vp, vp, C.c_size_t, vp, vp, vp, vp, vp]
    lib.model_tls_window.argtypes = [C.c_int, vp, C.c_size_t, vp, vp, C.c_size_t, vp, vp, vp, vp, vp]
    yield lib
    lib.model_set_read_ranges(None, 0)
    lib.model_set_write_ranges(None, 0)


class Checked:
    """Sets the allowed read (and, given, write) ranges for one model call and asserts no access fell outside them."""

    def __init__(self, lib, ranges, writes=None):
        self.lib, self.ranges = lib, np.array(ranges, dtype=np.uint64).reshape(-1, 2)
        self.writes = None if writes is None else np.array(writes, dtype=np.uint64).reshape(-1, 2)

    def __enter__(self):
        self.lib.model_set_read_ranges(self.ranges.ctypes.data, len(self.ranges))
        if self.writes is not None:
            self.lib.model_set_write_ranges(self.writes.ctypes.data, len(self.writes))

    def __exit__(self, *exc):
        first, wfirst = (C.c_uint64 * 2)(), (C.c_uint64 * 2)()
        bad = self.lib.model_read_violations(first)
        wbad = self.lib.model_write_violations(wfirst)
        self.lib.model_set_read_ranges(None, 0)
        self.lib.model_set_write_ranges(None, 0)
        if exc[0] is None:
            near = [(int(lo), int(hi)) for lo, hi in self.ranges if lo - 64 <= first[0] <= hi + 64]
            assert bad == 0, f"{bad} reads outside the records; first {first[1]} B at {first[0]:#x}, near {near}"
            if self.writes is not None:
                near = [(int(lo), int(hi)) for lo, hi in self.writes if lo - 64 <= wfirst[0] <= hi + 64]
                assert wbad == 0, f"{wbad} writes outside the records; first {wfirst[1]} B at {wfirst[0]:#x}, near {near}"


def aead_layout(lens, aads):
    """Records GAP bytes apart in src (and in aad); dst mirrors src (seal writes len + 16 there)."""
    n = len(lens)
    recs = np.zeros(n, RECORD_DTYPE)
    off = aoff = GAP
    for i, (ln, a) in enumerate(zip(lens, aads)):
        recs[i] = (off, off, aoff, 1000 + i, ln, a)
        off += ln + 16 + GAP
        aoff += a + GAP
    return recs, off, aoff


def aead_ranges(recs, src, aad, is_open):
    r = [(recs.ctypes.data, recs.ctypes.data + recs.nbytes)]
    for x in recs:
        s0 = src.ctypes.data + int(x["src"])
        r.append((s0, s0 + int(x["len"]) + (16 if is_open else 0)))
        a0 = aad.ctypes.data + int(x["aad"])
        r.append((a0, a0 + int(x["aadlen"])))
    return r


def out_ranges(base, offs, lens):
    """Each record's output bytes [base + off, base + off + len)"""
    return [(base.ctypes.data + int(o), base.ctypes.data + int(o) + int(n)) for o, n in zip(offs, lens)]


def call_aead(lib, fam, is_seal, key, iv, recs, src, dst, aad, st):
    args = (key, len(key), iv, recs.ctypes.data, len(recs), src.ctypes.data, dst.ctypes.data, aad.ctypes.data,
            st.ctypes.data)
    if fam in ("w16", "split"):
        return lib.model_batch_win16(int(is_seal), int(fam == "split"), *args)
    if isinstance(fam, str):
        lanes, _, seg = fam[1:].partition("s")
        lib.model_set_window_lanes(int(lanes))
        lib.model_set_window_seglen(int(seg or 64))
        return lib.model_batch_window(int(is_seal), *args)
    return lib.model_batch(int(is_seal), fam, *args)


@pytest.mark.parametrize("fam", [1, 2, 4, 8, "w4", "w8", "w8s32", "w16", "split"])
def test_aead_walk_reads_stay_inside_records(model, fam):
    lens = LENS if fam in (4, "w16", "split") else [x for x in LENS if x < 4096] + [16384]
    aads = [AADS[i % len(AADS)] for i in range(len(lens))]
    recs, nsrc, naad = aead_layout(lens, aads)
    rng = np.random.default_rng(5)
    src = rng.integers(0, 256, nsrc, dtype=np.uint8)
    aad = rng.integers(0, 256, naad, dtype=np.uint8)
    key, iv = bytes(range(16)), bytes(range(40, 52))
    ct = np.zeros_like(src)
    st = np.zeros(len(recs), np.uint32)
    with Checked(model, aead_ranges(recs, src, aad, False), out_ranges(ct, recs["dst"], recs["len"] + 16)):
        assert call_aead(model, fam, True, key, iv, recs, src, ct, aad, st) == 0
    want = np.zeros_like(src)
    oracle.batch(True, key, iv, recs, src, want, aad)
    for x in recs:  # (the walk checked is the walk that computes the right bytes)
        a, n = int(x["dst"]), int(x["len"])
        assert ct[a:a + n + 16].tobytes() == want[a:a + n + 16].tobytes(), n
    pt = np.zeros_like(src)
    with Checked(model, aead_ranges(recs, ct, aad, True), out_ranges(pt, recs["dst"], recs["len"])):
        assert call_aead(model, fam, False, key, iv, recs, ct, pt, aad, st) == 0
    assert (st == recs["len"]).all()


def tls_layout(lens, is_seal):
    """Seal: fragments GAP apart in src, wire records (len + 22) GAP apart in dst.  Open: wire records GAP apart."""
    n = len(lens)
    t = np.zeros(n, TLS_RECORD_DTYPE)
    off = doff = GAP
    for i, ln in enumerate(lens):
        if is_seal:
            t[i] = (off, doff, 77 + i, ln, [23, 22, 21][i % 3])
            off += ln + GAP
            doff += ln + 22 + GAP
        else:
            t[i] = (off, doff, 77 + i, ln + 17, 0)
            off += ln + 22 + GAP
            doff += ln + 1 + GAP
    return t, off, doff


@pytest.mark.parametrize("fam", ["batch", "w4", "w8", "w8s32"])
def test_tls_walk_reads_stay_inside_records(model, fam):
    lens = [x for x in LENS if x <= 16384]
    key, iv = bytes(range(3, 19)), bytes(range(60, 72))
    t, nsrc, ndst = tls_layout(lens, True)
    src = np.random.default_rng(6).integers(0, 256, nsrc, dtype=np.uint8)
    wire = np.zeros(ndst, np.uint8)
    st = np.zeros(len(t), np.uint32)
    ty = np.zeros(len(t), np.uint8)

    def call(is_seal, trecs, a, b):
        args = (key, len(key), iv, trecs.ctypes.data, len(trecs), a.ctypes.data, b.ctypes.data, st.ctypes.data,
                ty.ctypes.data, None)
        if fam == "batch":
            return model.model_tls_batch(int(is_seal), *args)
        lanes, _, seg = fam[1:].partition("s")
        model.model_set_window_lanes(int(lanes))
        model.model_set_window_seglen(int(seg or 64))
        return model.model_tls_window(int(is_seal), *args)

    ranges = [(t.ctypes.data, t.ctypes.data + t.nbytes)] + \
             [(src.ctypes.data + int(x["src"]), src.ctypes.data + int(x["src"]) + int(x["len"])) for x in t]
    with Checked(model, ranges, out_ranges(wire, t["dst"], t["len"].astype(np.int64) + 22)):
        assert call(True, t, src, wire) == 0
    for x in t:
        frag = src[int(x["src"]): int(x["src"]) + int(x["len"])].tobytes()
        want = oracle.tls_seal_record(key, iv, int(x["seq"]), int(x["type"]), frag)
        assert wire[int(x["dst"]): int(x["dst"]) + len(want)].tobytes() == want
    o = np.zeros(len(t), TLS_RECORD_DTYPE)
    o["src"], o["seq"], o["len"], o["type"] = t["dst"], t["seq"], t["len"] + 17, 0
    o["dst"] = np.cumsum([GAP] + [int(x) + 1 + GAP for x in t["len"][:-1]]).astype(np.uint64)
    pt = np.zeros(int(o["dst"][-1]) + int(t["len"][-1]) + 1 + GAP, np.uint8)
    ranges = [(o.ctypes.data, o.ctypes.data + o.nbytes)] + \
             [(wire.ctypes.data + int(x["src"]) + 5, wire.ctypes.data + int(x["src"]) + 5 + int(x["len"])) for x in o]
    with Checked(model, ranges, out_ranges(pt, o["dst"], o["len"].astype(np.int64) - 16)):
        assert call(False, o, wire, pt) == 0
    assert (st == t["len"]).all() and (ty == t["type"]).all()


def test_checker_catches_an_over_read(model):
    """The checker itself: a record declared 1 byte shorter than the walk reads is reported."""
    recs, nsrc, naad = aead_layout([100, 1400], [5, 13])
    src = np.zeros(nsrc, np.uint8)
    aad = np.zeros(naad, np.uint8)
    out = np.zeros_like(src)
    st = np.zeros(2, np.uint32)
    ranges = aead_ranges(recs, src, aad, False)
    ranges[2] = (ranges[2][0], ranges[2][1] - 1)  # record 0's input, one byte short
    with pytest.raises(AssertionError, match="reads outside the records"):
        with Checked(model, ranges):
            call_aead(model, 4, True, bytes(16), bytes(12), recs, src, out, aad, st)


def test_checker_catches_a_stray_write(model):
    """The write checker itself: an output range one byte short of what the walk stores is reported."""
    recs, nsrc, naad = aead_layout([100, 1400], [5, 13])
    src = np.zeros(nsrc, np.uint8)
    aad = np.zeros(naad, np.uint8)
    out = np.zeros_like(src)
    st = np.zeros(2, np.uint32)
    writes = out_ranges(out, recs["dst"], recs["len"])
    writes[1] = (writes[1][0], writes[1][1] - 1)  # record 1's ciphertext, one byte short
    with pytest.raises(AssertionError, match="writes outside the records"):
        with Checked(model, aead_ranges(recs, src, aad, False), writes):
            call_aead(model, 4, True, bytes(16), bytes(12), recs, src, out, aad, st)
