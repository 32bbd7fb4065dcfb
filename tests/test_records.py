"""Host-side batch layout helpers (rapido_amd/records.py)."""
import numpy as np

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
