"""Host-side batch layout helpers (rapido_amd/records.py)."""
import numpy as np
import pytest

from rapido_amd import RECORD_DTYPE, records


def test_layout_offsets_and_alignment():
    lens = np.array([0, 1, 1400, 16384, 17], dtype=np.uint64)
    recs, src_bytes, aad_bytes = records.layout(lens, np.full(5, 5, dtype=np.uint64), align=256)
    assert recs.dtype == RECORD_DTYPE
    assert (recs["src"] % 256 == 0).all() and (recs["dst"] == recs["src"]).all()
    ends = recs["src"] + recs["len"] + 16
    assert (ends[:-1] <= recs["src"][1:]).all() and ends[-1] <= src_bytes
    assert list(recs["aad"]) == [0, 5, 10, 15, 20] and aad_bytes >= 25


def test_tls_aad_matches_build_aad():
    # lib/picotls.c:621-628 with reclen = inlen + 16 (tag): 17 03 03 BE16(reclen)
    a = records.tls_aad(np.array([1400, 0, 16385], dtype=np.uint64)).reshape(3, 5)
    assert a[0].tolist() == [0x17, 3, 3, (1416 >> 8), 1416 & 0xFF]
    assert a[1].tolist() == [0x17, 3, 3, 0, 16]
    assert a[2].tolist() == [0x17, 3, 3, (16401 >> 8), 16401 & 0xFF]


def test_xorshift_deterministic():
    a = records.xorshift64star(5, 1000)
    assert (a == records.xorshift64star(5, 1000)).all()
    assert not (a == records.xorshift64star(6, 1000)).all()
    assert (records.xorshift64star(5, 100) == a[:100]).all()


def test_shard_by_bytes_balances_ragged_work():
    rng = np.random.default_rng(3)
    n = 100000
    lengths = rng.integers(64, 16385, n).astype(np.uint64)
    aadlens = np.full(n, 5, dtype=np.uint64)
    cost = (aadlens + 15) // 16 + (lengths + 15) // 16 + 1
    for world in (1, 2, 3, 8):
        shards = records.shard_by_bytes(lengths, aadlens, world)
        assert len(shards) == world
        # disjoint, in order, covering every record
        assert shards[0][0] == 0 and sum(c for _, c in shards) == n
        for (f0, c0), (f1, _) in zip(shards, shards[1:]):
            assert f0 + c0 == f1
        work = [int(cost[f:f + c].sum()) for f, c in shards]
        # balanced to within one record's cost (at most 1026 steps) of the ideal share
        ideal = int(cost.sum()) / world
        assert max(abs(w - ideal) for w in work) <= 1026


def test_shard_by_bytes_edges():
    assert records.shard_by_bytes([], [], 4) == [(0, 0)] * 4
    assert records.shard_by_bytes([100], [5], 3) in ([(0, 1), (1, 0), (1, 0)], [(0, 0), (0, 1), (1, 0)],
                                                      [(0, 0), (0, 0), (0, 1)])
    # one TLS-max record (1026 steps) then 1024 x 64 B (6 steps each): rank 0 takes it plus 426 small ones
    assert records.shard_by_bytes([16384] + [64] * 1024, [5] * 1025, 2) == [(0, 427), (427, 598)]
    with pytest.raises(ValueError):
        records.shard_by_bytes([1], [1], 0)
