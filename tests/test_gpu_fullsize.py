"""GPU parity at BASELINE.json's full batch sizes, through size-independent properties.

- seal -> open round trip over the whole batch: every status equals the record length, and the
  opened plaintext equals the source byte-for-byte (compared on the device);
- a random sample of sealed records (SAMPLE = 1024 per config) is bit-exact against the CPU oracle (its multithreaded
  batch entry point over the sampled records, compacted);
- flipping one bit in a sample of records (ciphertext, tag) fails exactly those records, zeroes their
  output, and leaves every other record verified.

Configs (BASELINE.json configs[1..3] and the north-star shape): 1 M x 1400 B AES-128, 256 K x 16 KiB AES-128 (north
star), 256 K x 16 KiB AES-256, 256 K x 16385 B AES-128 (TLS-max inner plaintext), 1 M ragged U{64..16384} AES-128
(ordered launches).  Each case holds ~3 copies of its batch in HBM (<= 24 GB).
"""
import zlib

import numpy as np
import pytest

import oracle
import rapido_amd as ra
from rapido_amd import records
from rapido_amd.hostmem import to_cpu, to_gpu

pytestmark = pytest.mark.gpu

SAMPLE = 1024

CASES = [
    ("1400", 16, 1 << 20, 1400),
    ("16k-aes128", 16, 1 << 18, 16384),  # the north-star shape (BASELINE.json north_star)
    ("16k-aes256", 32, 1 << 18, 16384),
    ("16k-max-aes128", 16, 1 << 18, 16385),  # TLS-max inner plaintext: a 1-byte tail block per record
    ("ragged", 16, 1 << 20, None),
]


@pytest.mark.parametrize("name,keylen,n,length", CASES)
def test_full_size_round_trip(gpu, name, keylen, n, length):
    import torch
    rng = np.random.default_rng(zlib.crc32(name.encode()))
    lengths = rng.integers(64, 16385, n).astype(np.uint64) if length is None else np.full(n, length, np.uint64)
    recs, src_bytes, aad_bytes = records.layout(lengths, np.full(n, 5, dtype=np.uint64), align=256)
    recs["seq"] = rng.integers(0, 2 ** 48, n, dtype=np.uint64)
    aad = np.zeros(aad_bytes, dtype=np.uint8)
    aad[: 5 * n] = records.tls_aad(lengths)
    key = rng.integers(0, 256, keylen, dtype=np.uint8).tobytes()
    iv = rng.integers(0, 256, 12, dtype=np.uint8).tobytes()
    dev = gpu
    gen = torch.Generator(device=dev)
    gen.manual_seed(77)
    d_src = torch.randint(0, 256, (src_bytes,), dtype=torch.uint8, device=dev, generator=gen)
    d_ct = torch.zeros_like(d_src)
    d_recs = to_gpu(recs.view(np.uint8), dev)
    d_aad = to_gpu(aad, dev)
    d_st = torch.zeros(n, dtype=torch.int32, device=dev)
    d_order = torch.zeros(n, dtype=torch.int32, device=dev)
    eng = ra.Engine(key)
    ragged = length is None

    def seal(dst):
        if ragged:
            eng.order_by_length(d_recs.data_ptr(), n, d_order.data_ptr())
            eng.seal_batch_ordered(iv, d_recs.data_ptr(), d_order.data_ptr(), n, d_src.data_ptr(), dst.data_ptr(),
                                   d_aad.data_ptr())
        else:
            eng.seal_batch(iv, d_recs.data_ptr(), n, d_src.data_ptr(), dst.data_ptr(), d_aad.data_ptr())

    def open_(src, dst):
        d_st.zero_()
        if ragged:
            eng.open_batch_ordered(iv, d_recs.data_ptr(), d_order.data_ptr(), n, src.data_ptr(), dst.data_ptr(),
                                   d_aad.data_ptr(), d_st.data_ptr())
        else:
            eng.open_batch(iv, d_recs.data_ptr(), n, src.data_ptr(), dst.data_ptr(), d_aad.data_ptr(), d_st.data_ptr())
        torch.cuda.synchronize()
        return to_cpu(d_st).view(np.uint32)

    seal(d_ct)
    d_pt = torch.zeros_like(d_src)
    st = open_(d_ct, d_pt)
    assert (st == recs["len"]).all()
    # the payload bytes of every record round-trip (slot padding is not written by open)
    starts = to_gpu(recs["src"].astype(np.int64), dev)
    lens = to_gpu(recs["len"].astype(np.int64), dev)
    mark = torch.zeros(src_bytes + 1, dtype=torch.int32, device=dev)
    mark.index_add_(0, starts, torch.ones_like(starts, dtype=torch.int32))
    mark.index_add_(0, starts + lens, -torch.ones_like(starts, dtype=torch.int32))
    mask = torch.cumsum(mark, 0)[:src_bytes] > 0
    assert int(mask.sum(dtype=torch.int64).item()) == int(recs["len"].sum())
    assert not bool(((d_pt != d_src) & mask).any().item())  # elementwise: no >2^32-element boolean gather

    # a sample of SAMPLE records is bit-exact against the oracle: the sampled plaintexts compacted into a small batch
    # of their own (same keys, nonces and AADs), sealed by the oracle's multithreaded batch entry point
    sample = np.sort(rng.choice(n, size=SAMPLE, replace=False))
    sub = recs[sample].copy()
    ln_s = sub["len"].astype(np.int64)
    slot = (ln_s + 16 + 255) // 256 * 256
    offs = np.concatenate([[0], np.cumsum(slot)[:-1]]).astype(np.int64)
    sub_src = np.zeros(int(slot.sum()), np.uint8)
    got = np.zeros_like(sub_src)
    for k, i in enumerate(sample):
        a, ln, o = int(recs[i]["src"]), int(ln_s[k]), int(offs[k])
        sub_src[o: o + ln] = to_cpu(d_src[a: a + ln])
        got[o: o + ln + 16] = to_cpu(d_ct[a: a + ln + 16])
    sub_aad = np.concatenate([aad[int(r["aad"]): int(r["aad"]) + 5] for r in sub])
    sub["src"] = offs.astype(np.uint64)
    sub["dst"] = offs.astype(np.uint64)
    sub["aad"] = np.arange(SAMPLE, dtype=np.uint64) * 5
    want = np.zeros_like(sub_src)
    oracle.batch(True, key, iv, sub, sub_src, want, sub_aad)
    for k in range(SAMPLE):
        o, ln = int(offs[k]), int(ln_s[k])
        assert np.array_equal(got[o: o + ln + 16], want[o: o + ln + 16]), f"record {int(sample[k])}"

    # tamper: one ciphertext bit in some records, one tag bit in others
    bad_ct = rng.choice(n, size=8, replace=False)
    bad_tag = np.setdiff1d(rng.choice(n, size=16, replace=False), bad_ct)[:8]
    for i in bad_ct:
        p = int(recs[i]["src"]) + int(rng.integers(0, int(recs[i]["len"])))
        d_ct[p] ^= 1
    for i in bad_tag:
        p = int(recs[i]["src"]) + int(recs[i]["len"]) + int(rng.integers(0, 16))
        d_ct[p] ^= 0x80
    d_pt.fill_(0xA5)
    st = open_(d_ct, d_pt)
    bad = np.zeros(n, bool)
    bad[bad_ct] = True
    bad[bad_tag] = True
    assert (st[bad] == 0xFFFFFFFF).all()
    assert (st[~bad] == recs["len"][~bad]).all()
    for i in np.flatnonzero(bad):
        a, ln = int(recs[i]["src"]), int(recs[i]["len"])
        assert not d_pt[a: a + ln].any()
    eng.close()


def test_configs4_sharded_batch_equals_whole(gpu):
    """BASELINE.json configs[4] on one device: 8 M x 1400 B AES-128 records cut into the 8 per-GPU shards bench.py's
    ranks take (bench.rank_shard: 1 M each, no collective), each sealed by its own context on its own stream, give
    exactly the bytes of one launch over the whole batch; every shard then opens with every record verified."""
    import os
    import sys

    import torch
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from bench import rank_shard

    world, per = 8, 1 << 20
    n = world * per
    lengths = np.full(n, 1400, np.uint64)
    recs, src_bytes, aad_bytes = records.layout(lengths, np.full(n, 5, dtype=np.uint64), align=256)
    recs["seq"] = np.arange(n, dtype=np.uint64)  # rank r's first seq is its first global record (bench.measure)
    aad = np.zeros(aad_bytes, dtype=np.uint8)
    aad[: 5 * n] = records.tls_aad(lengths)
    key, iv = bytes(range(16)), bytes(range(0xA0, 0xAC))
    dev = gpu
    gen = torch.Generator(device=dev)
    gen.manual_seed(4)
    d_src = torch.randint(0, 256, (src_bytes,), dtype=torch.uint8, device=dev, generator=gen)
    d_whole = torch.zeros_like(d_src)
    d_shard = torch.zeros_like(d_src)
    d_recs = to_gpu(recs.view(np.uint8), dev)
    d_aad = to_gpu(aad, dev)
    dsize = recs.dtype.itemsize
    whole = ra.Engine(key)
    whole.seal_batch(iv, d_recs.data_ptr(), n, d_src.data_ptr(), d_whole.data_ptr(), d_aad.data_ptr())
    ranks = [(ra.Engine(key), torch.cuda.Stream(dev)) for _ in range(world)]
    torch.cuda.synchronize(dev)  # the buffers' fills on torch's stream precede the shard streams' launches
    for r, (eng, s) in enumerate(ranks):
        first, cnt = rank_shard(r, world, per)
        eng.seal_batch(iv, d_recs.data_ptr() + first * dsize, cnt, d_src.data_ptr(), d_shard.data_ptr(),
                       d_aad.data_ptr(), s.cuda_stream)
    torch.cuda.synchronize(dev)
    assert torch.equal(d_whole, d_shard)
    d_pt = torch.zeros_like(d_src)
    d_st = torch.zeros(n, dtype=torch.int32, device=dev)
    torch.cuda.synchronize(dev)
    for r, (eng, s) in enumerate(ranks):
        first, cnt = rank_shard(r, world, per)
        eng.open_batch(iv, d_recs.data_ptr() + first * dsize, cnt, d_shard.data_ptr(), d_pt.data_ptr(),
                       d_aad.data_ptr(), d_st.data_ptr() + 4 * first, s.cuda_stream)
    torch.cuda.synchronize(dev)
    assert (to_cpu(d_st).view(np.uint32) == 1400).all()
    # one sampled record of every shard is bit-exact against the oracle
    for r in range(world):
        i = r * per + int(np.random.default_rng(r).integers(0, per))
        a = int(recs[i]["src"])
        want = oracle.seal(key, oracle.build_iv(iv, i), aad[int(recs[i]["aad"]): int(recs[i]["aad"]) + 5].tobytes(),
                           to_cpu(d_src[a: a + 1400]).tobytes())
        assert to_cpu(d_shard[a: a + 1416]).tobytes() == want
    for eng, _ in ranks:
        eng.close()
    whole.close()
