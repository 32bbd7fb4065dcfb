"""Multi-key batches on the GPU (include/ptls_mi355x.h "Multi-key batches"): the records of 2, 16 and
256 sessions -- each with its own traffic key and static IV, as a rapido server holds them (include/rapido.h:147,
lib/rapido.c:135-200) -- sealed and opened in ONE launch, every record bit-exact against the oracle under its own key,
on every kernel family a multi-key batch can take (split, 16-lane window, batch kernels), AES-128 and AES-256, AEAD and
TLS-framed.  Records of different keys are interleaved in the batch, so the launch's by-key sort is exercised."""
import numpy as np
import pytest

import oracle
import rapido_amd as ra
from conftest import kernel_family
from rapido_amd import records
from rapido_amd.hostmem import to_cpu, to_gpu

pytestmark = pytest.mark.gpu

MK_FAMILIES = ["split", "window16", "batch"]
EXPECT = {"split": "_wins_", "window16": "_win16_", "batch": "_k4_mk"}


def dev(a):
    import torch
    return to_gpu(np.ascontiguousarray(a))


def sessions(rng, nkeys, keylen):
    keys = [rng.integers(0, 256, keylen, dtype=np.uint8).tobytes() for _ in range(nkeys)]
    ivs = [rng.integers(0, 256, 12, dtype=np.uint8).tobytes() for _ in range(nkeys)]
    return keys, ivs


def aead_batch(rng, n, max_len):
    lens = rng.integers(0, max_len, n).astype(np.uint64)
    aadlens = rng.integers(0, 40, n).astype(np.uint64)
    for i, (ln, a) in enumerate([(0, 0), (1, 5), (15, 13), (16, 16), (17, 0), (1400, 5), (4096, 32)][:n]):
        lens[i], aadlens[i] = ln, a
    recs, src_bytes, aad_bytes = records.layout(lens, aadlens, align=16)
    recs["seq"] = rng.integers(0, 2 ** 62, n, dtype=np.uint64)
    src = rng.integers(0, 256, src_bytes + 16, dtype=np.uint8)
    aad = rng.integers(0, 256, max(aad_bytes, 1), dtype=np.uint8)
    return recs, src, aad


def oracle_seal(keys, ivs, kidx, recs, src, aad):
    want = np.zeros(len(src) + 16, np.uint8)
    for i, r in enumerate(recs):
        k = int(kidx[i])
        pt = bytes(src[int(r["src"]): int(r["src"]) + int(r["len"])])
        a = bytes(aad[int(r["aad"]): int(r["aad"]) + int(r["aadlen"])])
        ct = oracle.seal(keys[k], oracle.build_iv(ivs[k], int(r["seq"])), a, pt)
        want[int(r["dst"]): int(r["dst"]) + len(ct)] = np.frombuffer(ct, np.uint8)
    return want


@pytest.mark.parametrize("family", MK_FAMILIES)
@pytest.mark.parametrize("nkeys", [2, 16, 256])
@pytest.mark.parametrize("keylen", [16, 32])
def test_multikey_aead_vs_oracle(gpu, family, nkeys, keylen):
    import torch
    rng = np.random.default_rng(1000 + nkeys * 3 + keylen + len(family))
    n = {"split": 40, "window16": 200, "batch": 700}[family]
    keys, ivs = sessions(rng, nkeys, keylen)
    engines = [ra.Engine(k) for k in keys]
    mk = ra.MultiKey(engines, ivs)
    recs, src, aad = aead_batch(rng, n, 2500 if family != "batch" else 1800)
    kidx = rng.integers(0, nkeys, n).astype(np.uint32)  # interleaved sessions
    with kernel_family(family, framing=False):
        assert EXPECT[family] in ra.kernel_name_multikey(True, keylen, n, False)
        d_recs, d_src, d_aad, d_k = dev(recs.view(np.uint8)), dev(src), dev(aad), dev(kidx.view(np.int32))
        d_ct = torch.zeros(len(src) + 16, dtype=torch.uint8, device="cuda")
        mk.seal_batch(d_recs.data_ptr(), d_k.data_ptr(), n, d_src.data_ptr(), d_ct.data_ptr(), d_aad.data_ptr())
        torch.cuda.synchronize()
        got = to_cpu(d_ct)
        want = oracle_seal(keys, ivs, kidx, recs, src, aad)
        for i, r in enumerate(recs):
            a, b = int(r["dst"]), int(r["dst"]) + int(r["len"]) + 16
            assert bytes(got[a:b]) == bytes(want[a:b]), (i, int(kidx[i]), int(r["len"]))
        # open every record under its key; tamper three, and give one a key index out of range
        bad = got.copy()
        for i in (3, 7, 11):
            bad[int(recs[i]["dst"]) + int(recs[i]["len"]) + 2] ^= 0x20
        kbad = kidx.copy()
        kbad[20] = nkeys + 5
        d_bad, d_kb = dev(bad), dev(kbad.view(np.int32))
        d_pt = torch.full((len(src) + 16,), 0x5A, dtype=torch.uint8, device="cuda")
        d_st = torch.zeros(n, dtype=torch.int32, device="cuda")
        mk.open_batch(d_recs.data_ptr(), d_kb.data_ptr(), n, d_bad.data_ptr(), d_pt.data_ptr(), d_aad.data_ptr(),
                      d_st.data_ptr())
        torch.cuda.synchronize()
        st, pt = to_cpu(d_st).view(np.uint32), to_cpu(d_pt)
    for i, r in enumerate(recs):
        a, ln = int(r["dst"]), int(r["len"])
        if i in (3, 7, 11):
            assert st[i] == 0xFFFFFFFF and not pt[a:a + ln].any(), i
        elif i == 20:  # out-of-range key: refused, nothing written
            assert st[i] == 0xFFFFFFFF and (pt[a:a + ln] == 0x5A).all()
        else:
            assert st[i] == ln, (i, st[i])
            assert bytes(pt[a:a + ln]) == bytes(src[int(r["src"]): int(r["src"]) + ln]), i
    for e in engines:
        e.close()


def test_multikey_beyond_the_counting_sort(gpu):
    """More keys than the counting sort's LDS buckets (8191): the batch kernels' grouping falls back to hipCUB's radix
    sort.  9000 key slots over 64 contexts (a slot's key is context k % 64, its IV its own), 20 000 records with key
    indices over all slots and some out of range, sealed and opened against the oracle, ordered and unordered."""
    import torch
    rng = np.random.default_rng(9000)
    nslots, n = 9000, 20000
    keys, _ = sessions(rng, 64, 16)
    engines = [ra.Engine(k) for k in keys]
    ivs = [rng.integers(0, 256, 12, dtype=np.uint8).tobytes() for _ in range(nslots)]
    mk = ra.MultiKey([engines[k % 64] for k in range(nslots)], ivs)
    slot_keys = [keys[k % 64] for k in range(nslots)]
    recs, src, aad = aead_batch(rng, n, 600)
    kidx = rng.integers(0, nslots, n).astype(np.uint32)
    kidx[::997] = nslots + 3  # out of range: refused
    with kernel_family("batch", framing=False):
        assert "_k4_mk" in ra.kernel_name_multikey(True, 16, n, False)
        d_recs, d_src, d_aad, d_k = dev(recs.view(np.uint8)), dev(src), dev(aad), dev(kidx.view(np.int32))
        d_ct = torch.zeros(len(src) + 16, dtype=torch.uint8, device="cuda")
        mk.seal_batch(d_recs.data_ptr(), d_k.data_ptr(), n, d_src.data_ptr(), d_ct.data_ptr(), d_aad.data_ptr())
        torch.cuda.synchronize()
        got = to_cpu(d_ct)
        ok = kidx < nslots
        want = oracle_seal(slot_keys, ivs, np.where(ok, kidx, 0), recs, src, aad)
        for i in np.flatnonzero(ok)[::7]:  # a seventh of the records, every slot range
            r = recs[i]
            a, b = int(r["dst"]), int(r["dst"]) + int(r["len"]) + 16
            assert bytes(got[a:b]) == bytes(want[a:b]), (i, int(kidx[i]))
        for i in np.flatnonzero(~ok):
            r = recs[i]
            assert not got[int(r["dst"]): int(r["dst"]) + int(r["len"]) + 16].any(), i  # seal wrote nothing
        # open, through one by-key order shared by the launch (ptls_mi355x_order_by_key)
        d_order = torch.zeros(n, dtype=torch.int32, device="cuda")
        mk.order_by_key(d_k.data_ptr(), n, d_order.data_ptr())
        d_in = dev(got)
        d_pt = torch.zeros(len(src) + 16, dtype=torch.uint8, device="cuda")
        d_st = torch.zeros(n, dtype=torch.int32, device="cuda")
        mk.open_batch_ordered(d_recs.data_ptr(), d_k.data_ptr(), d_order.data_ptr(), n, d_in.data_ptr(),
                              d_pt.data_ptr(), d_aad.data_ptr(), d_st.data_ptr())
        torch.cuda.synchronize()
        st, pt = to_cpu(d_st).view(np.uint32), to_cpu(d_pt)
        order = to_cpu(d_order).view(np.uint32)
    ks = np.where(kidx[order] < nslots, kidx[order], nslots)
    assert (np.diff(ks.astype(np.int64)) >= 0).all() and sorted(order.tolist()) == list(range(n))
    for i, r in enumerate(recs):
        a, ln = int(r["dst"]), int(r["len"])
        if not ok[i]:
            assert st[i] == 0xFFFFFFFF, i
        else:
            assert st[i] == ln and bytes(pt[a:a + ln]) == bytes(src[int(r["src"]): int(r["src"]) + ln]), i
    for e in engines:
        e.close()


@pytest.mark.parametrize("family", MK_FAMILIES)
def test_multikey_seal_skips_out_of_range_keys(gpu, family):
    import torch
    rng = np.random.default_rng(77)
    keys, ivs = sessions(rng, 3, 16)
    engines = [ra.Engine(k) for k in keys]
    mk = ra.MultiKey(engines, ivs)
    n = 30
    recs, src, aad = aead_batch(rng, n, 600)
    kidx = (np.arange(n) % 3).astype(np.uint32)
    kidx[[4, 9]] = [3, 0xFFFFFFFF]
    with kernel_family(family, framing=False):
        d_recs, d_src, d_aad, d_k = dev(recs.view(np.uint8)), dev(src), dev(aad), dev(kidx.view(np.int32))
        d_ct = torch.full((len(src) + 16,), 0xA5, dtype=torch.uint8, device="cuda")
        mk.seal_batch(d_recs.data_ptr(), d_k.data_ptr(), n, d_src.data_ptr(), d_ct.data_ptr(), d_aad.data_ptr())
        torch.cuda.synchronize()
        got = to_cpu(d_ct)
    ok = kidx < 3
    want = oracle_seal(keys, ivs, np.where(ok, kidx, 0), recs, src, aad)
    for i, r in enumerate(recs):
        a, b = int(r["dst"]), int(r["dst"]) + int(r["len"]) + 16
        if ok[i]:
            assert bytes(got[a:b]) == bytes(want[a:b]), i
        else:
            assert (got[a:b] == 0xA5).all(), i  # no record under another session's key
    for e in engines:
        e.close()


def conn_iv(iv: bytes, conn_id: int) -> bytes:
    """rapido's derive_connection_aead_iv (lib/rapido.c:127-133): IV bytes 0..3 ^= BE32(connection_id)."""
    return (int.from_bytes(iv[:4], "big") ^ conn_id).to_bytes(4, "big") + iv[4:]


@pytest.mark.parametrize("family", MK_FAMILIES)
@pytest.mark.parametrize("nkeys", [2, 16, 256])
def test_multikey_tls_windows_vs_oracle(gpu, family, nkeys):
    """TLS 1.3 records of many sessions and connections in one framing launch each way: every wire record is the
    oracle's record layer under its session's key and its connection's IV; STOP_AT_FAILURE stops each (session,
    connection) at its own first failure."""
    import torch
    rng = np.random.default_rng(4000 + nkeys + len(family))
    keylen = 16 if nkeys != 16 else 32
    keys, ivs = sessions(rng, nkeys, keylen)
    engines = [ra.Engine(k) for k in keys]
    mk = ra.MultiKey(engines, ivs)
    n = {"split": 45, "window16": 240, "batch": 900}[family]
    lens = rng.integers(0, 16385 if family != "batch" else 3000, n)
    lens[:4] = [0, 1, 16384, 15]
    kidx = np.sort(rng.integers(0, nkeys, n)).astype(np.uint32)  # a server's windows: sessions one after another
    conn = rng.integers(0, 3, n).astype(np.uint32)
    conn.sort()
    order = np.lexsort((conn, kidx))
    kidx, conn = kidx[order], conn[order]
    trecs = np.zeros(n, ra.TLS_RECORD_DTYPE)
    off = woff = 0
    for i, ln in enumerate(lens):
        trecs[i] = (off, woff, 100 + i, int(ln), 23 if i % 4 else 22)
        off += int(ln)
        woff += int(ln) + 22
    src = np.frombuffer(rng.integers(0, 256, off + 16, dtype=np.uint8).tobytes(), np.uint8)
    with kernel_family(family, framing=True):
        assert EXPECT[family] in ra.kernel_name_multikey(True, keylen, n, True)
        d_src, d_recs, d_k, d_c = dev(src), dev(trecs.view(np.uint8)), dev(kidx.view(np.int32)), dev(conn.view(np.int32))
        d_wire = torch.zeros(woff + 16, dtype=torch.uint8, device="cuda")
        mk.tls_seal_records(d_recs.data_ptr(), d_k.data_ptr(), n, d_src.data_ptr(), d_wire.data_ptr(),
                            conn_ptr=d_c.data_ptr())
        torch.cuda.synchronize()
        wire = to_cpu(d_wire)
        for i, t in enumerate(trecs):
            frag = bytes(src[int(t["src"]): int(t["src"]) + int(t["len"])])
            want = oracle.tls_seal_record(keys[kidx[i]], conn_iv(ivs[kidx[i]], int(conn[i])), int(t["seq"]),
                                          int(t["type"]), frag)
            assert bytes(wire[int(t["dst"]): int(t["dst"]) + len(want)]) == want, (i, int(kidx[i]))
        orecs = trecs.copy()
        orecs["src"], orecs["len"] = trecs["dst"], trecs["len"] + 17
        orecs["dst"] = np.concatenate([[0], np.cumsum(trecs["len"].astype(np.int64) + 1)[:-1]]).astype(np.uint64)
        pt_size = int(orecs["dst"][-1]) + int(trecs["len"][-1]) + 1
        bad = wire.copy()
        tampered = [5, n // 2]
        for i in tampered:
            bad[int(orecs[i]["src"]) + 7] ^= 0x01
        for flags in (0, ra.OPEN_STOP_AT_FAILURE):
            d_w = dev(bad)
            d_pt = torch.zeros(pt_size, dtype=torch.uint8, device="cuda")
            d_st = torch.zeros(n, dtype=torch.int32, device="cuda")
            d_ty = torch.zeros(n, dtype=torch.uint8, device="cuda")
            mk.tls_open_records(dev(orecs.view(np.uint8)).data_ptr(), d_k.data_ptr(), n, d_w.data_ptr(), d_pt.data_ptr(),
                                d_st.data_ptr(), d_ty.data_ptr(), conn_ptr=d_c.data_ptr(), flags=flags)
            torch.cuda.synchronize()
            st, ty, pt = to_cpu(d_st).view(np.uint32), to_cpu(d_ty), to_cpu(d_pt)
            for i, t in enumerate(trecs):
                a, ln = int(orecs[i]["dst"]), int(t["len"])
                seg_bad = [b for b in tampered if kidx[b] == kidx[i] and conn[b] == conn[i] and b < i]
                if i in tampered:
                    assert st[i] == ra.TLS_BAD_RECORD_MAC, (flags, i)
                elif flags and seg_bad:  # behind its own (session, connection)'s first failure
                    assert st[i] == ra.TLS_NOT_PROCESSED, (flags, i, st[i])
                else:
                    assert st[i] == ln and ty[i] == t["type"], (flags, i, st[i])
                    assert bytes(pt[a:a + ln]) == bytes(src[int(t["src"]): int(t["src"]) + ln]), (flags, i)
    for e in engines:
        e.close()


def test_multikey_matches_single_key_launches(gpu):
    """The multi-key launch gives exactly the bytes of one single-key launch per key (the batch kernels, 64 keys)."""
    import torch
    rng = np.random.default_rng(9)
    nkeys, n = 64, 3000
    keys, ivs = sessions(rng, nkeys, 16)
    engines = [ra.Engine(k) for k in keys]
    mk = ra.MultiKey(engines, ivs)
    recs, src, aad = aead_batch(rng, n, 1500)
    kidx = rng.integers(0, nkeys, n).astype(np.uint32)
    d_recs, d_src, d_aad, d_k = dev(recs.view(np.uint8)), dev(src), dev(aad), dev(kidx.view(np.int32))
    d_mk = torch.zeros(len(src) + 16, dtype=torch.uint8, device="cuda")
    mk.seal_batch(d_recs.data_ptr(), d_k.data_ptr(), n, d_src.data_ptr(), d_mk.data_ptr(), d_aad.data_ptr())
    d_one = torch.zeros_like(d_mk)
    for k in range(nkeys):
        sub = recs[kidx == k]
        if len(sub):
            d_sub = dev(sub.view(np.uint8))
            engines[k].seal_batch(ivs[k], d_sub.data_ptr(), len(sub), d_src.data_ptr(), d_one.data_ptr(),
                                  d_aad.data_ptr())
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    assert torch.equal(d_mk, d_one)
    for e in engines:
        e.close()


def test_multikey_ordered_launches_share_one_sort(gpu):
    """ptls_mi355x_order_by_key once, then the _ordered seal and open over it: the bytes of the sorting launches, and an
    out-of-range key index sorted last and refused (batch kernels, 32 keys, AES-256)."""
    import torch
    rng = np.random.default_rng(31)
    nkeys, n = 32, 2500
    keys, ivs = sessions(rng, nkeys, 32)
    engines = [ra.Engine(k) for k in keys]
    mk = ra.MultiKey(engines, ivs)
    recs, src, aad = aead_batch(rng, n, 1500)
    kidx = rng.integers(0, nkeys, n).astype(np.uint32)
    kidx[77] = nkeys + 1
    d_recs, d_src, d_aad, d_k = dev(recs.view(np.uint8)), dev(src), dev(aad), dev(kidx.view(np.int32))
    d_order = torch.zeros(n, dtype=torch.int32, device="cuda")
    mk.order_by_key(d_k.data_ptr(), n, d_order.data_ptr())
    d_a = torch.zeros(len(src) + 16, dtype=torch.uint8, device="cuda")
    d_b = torch.zeros_like(d_a)
    mk.seal_batch_ordered(d_recs.data_ptr(), d_k.data_ptr(), d_order.data_ptr(), n, d_src.data_ptr(), d_a.data_ptr(),
                          d_aad.data_ptr())
    mk.seal_batch(d_recs.data_ptr(), d_k.data_ptr(), n, d_src.data_ptr(), d_b.data_ptr(), d_aad.data_ptr())
    torch.cuda.synchronize()
    assert torch.equal(d_a, d_b)
    order = to_cpu(d_order).view(np.uint32)
    assert sorted(order.tolist()) == list(range(n)) and order[-1] == 77  # a permutation, the stray key last
    sk = np.minimum(kidx[order], nkeys)
    assert (np.diff(sk.astype(np.int64)) >= 0).all()
    d_pt = torch.zeros_like(d_a)
    d_st = torch.zeros(n, dtype=torch.int32, device="cuda")
    mk.open_batch_ordered(d_recs.data_ptr(), d_k.data_ptr(), d_order.data_ptr(), n, d_a.data_ptr(), d_pt.data_ptr(),
                          d_aad.data_ptr(), d_st.data_ptr())
    torch.cuda.synchronize()
    st, pt = to_cpu(d_st).view(np.uint32), to_cpu(d_pt)
    for i, r in enumerate(recs):
        a, ln = int(r["dst"]), int(r["len"])
        if i == 77:
            assert st[i] == 0xFFFFFFFF
        else:
            assert st[i] == ln and bytes(pt[a:a + ln]) == bytes(src[int(r["src"]): int(r["src"]) + ln]), i
    for e in engines:
        e.close()


def test_multikey_argument_errors(gpu):
    import torch
    e16, e32 = ra.Engine(bytes(16)), ra.Engine(bytes(32))
    recs = np.zeros(1, ra.RECORD_DTYPE)
    d = dev(recs.view(np.uint8))
    k = torch.zeros(1, dtype=torch.int32, device="cuda")
    buf = torch.zeros(64, dtype=torch.uint8, device="cuda")
    with pytest.raises(RuntimeError, match="another key size"):
        ra.MultiKey([e16, e32], [bytes(12)] * 2).seal_batch(d.data_ptr(), k.data_ptr(), 1, buf.data_ptr(),
                                                            buf.data_ptr(), buf.data_ptr())
    with pytest.raises(RuntimeError, match="key indices are required"):
        ra.MultiKey([e16], [bytes(12)]).seal_batch(d.data_ptr(), 0, 1, buf.data_ptr(), buf.data_ptr(), buf.data_ptr())
    e16.close()
    e32.close()
