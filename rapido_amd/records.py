"""Record-batch layouts for the batch API (used by tests and bench.py).

A batch is three byte arenas (src, dst, aad) plus an array of ptls_mi355x_record_t
descriptors.  The synthetic workloads follow SURVEY.md sec. 8(d): records start on
256-byte boundaries, the AAD is the 5-byte TLS 1.3 record header built by picotls'
``build_aad`` (lib/picotls.c:621-628) for a sealed length of L + 16, seq = record index,
payload bytes from an xorshift64* stream.
"""
from __future__ import annotations

import numpy as np

from . import RECORD_DTYPE


def xorshift64star(seed: int, nbytes: int) -> np.ndarray:
    """Deterministic byte stream (xorshift64*), vectorised over 64 parallel lanes."""
    lanes = 64
    nwords = (nbytes + 8 * lanes - 1) // (8 * lanes)
    with np.errstate(over="ignore"):
        x = (np.arange(1, lanes + 1, dtype=np.uint64) * np.uint64(0x9E3779B97F4A7C15)) ^ np.uint64(seed | 1)
        out = np.empty((nwords, lanes), dtype=np.uint64)
        for i in range(nwords):
            x ^= x >> np.uint64(12)
            x ^= x << np.uint64(25)
            x ^= x >> np.uint64(27)
            out[i] = x * np.uint64(0x2545F4914F6CDD1D)
    return out.reshape(-1).view(np.uint8)[:nbytes].copy()


def tls_aad(lengths: np.ndarray) -> np.ndarray:
    """5-byte TLS 1.3 AAD per record: 17 03 03 BE16(len + 16) (lib/picotls.c:621-628, 636)."""
    n = len(lengths)
    a = np.empty((n, 5), dtype=np.uint8)
    sealed = lengths.astype(np.uint64) + 16
    a[:, 0], a[:, 1], a[:, 2] = 0x17, 0x03, 0x03
    a[:, 3] = (sealed >> 8) & 0xFF
    a[:, 4] = sealed & 0xFF
    return a.reshape(-1)


def layout(lengths, aadlens, align: int = 256, tag_room: bool = True):
    """Contiguous arena layout; returns (recs, src_bytes, aad_bytes).

    Each record's slot holds len + 16 bytes (room for the tag) rounded up to `align`;
    dst offsets equal src offsets (use a separate dst arena of the same size, or the same
    arena for in-place)."""
    lengths = np.asarray(lengths, dtype=np.uint64)
    aadlens = np.asarray(aadlens, dtype=np.uint64)
    n = len(lengths)
    room = lengths + (16 if tag_room else 0)
    slot = ((room + align - 1) // align) * align if align > 1 else room
    src_off = np.zeros(n, dtype=np.uint64)
    if n:
        src_off[1:] = np.cumsum(slot)[:-1]
    aad_off = np.zeros(n, dtype=np.uint64)
    if n:
        aad_off[1:] = np.cumsum(aadlens)[:-1]
    recs = np.zeros(n, dtype=RECORD_DTYPE)
    recs["src"] = src_off
    recs["dst"] = src_off
    recs["aad"] = aad_off
    recs["seq"] = np.arange(n, dtype=np.uint64)
    recs["len"] = lengths.astype(np.uint32)
    recs["aadlen"] = aadlens.astype(np.uint32)
    src_bytes = int(slot.sum()) + 16
    aad_bytes = int(aadlens.sum()) + 16
    return recs, src_bytes, aad_bytes


def tls_batch(lengths, seed: int, align: int = 256):
    """A TLS-framed synthetic batch: returns (recs, src, aad) as numpy arrays."""
    lengths = np.asarray(lengths, dtype=np.uint64)
    n = len(lengths)
    recs, src_bytes, aad_bytes = layout(lengths, np.full(n, 5, dtype=np.uint64), align)
    src = xorshift64star(seed, src_bytes)
    aad = np.zeros(aad_bytes, dtype=np.uint8)
    aad[: 5 * n] = tls_aad(lengths)
    return recs, src, aad


def shard_by_bytes(lengths, aadlens, world: int):
    """Contiguous shards of a global ragged batch, one per rank, balanced by GHASH work.

    A record's cost is its GHASH step count, ceil(aad/16) + ceil(len/16) + 1 (the length block),
    which is also what its AES-CTR work and HBM bytes scale with.  Rank r gets the records whose
    cumulative cost midpoint falls in [r/world, (r+1)/world) of the total, so shard boundaries sit at
    the prefix-sum quantiles.  Returns a list of (first, count) per rank; the shards are disjoint,
    cover the batch in order, and need no exchange (records are independent).
    """
    if world < 1:
        raise ValueError("world must be >= 1")
    lengths = np.asarray(lengths, dtype=np.uint64)
    aadlens = np.asarray(aadlens, dtype=np.uint64)
    if lengths.shape != aadlens.shape:
        raise ValueError("lengths and aadlens differ in shape")
    n = len(lengths)
    cost = (aadlens + 15) // 16 + (lengths + 15) // 16 + 1
    csum = np.cumsum(cost, dtype=np.uint64)
    total = int(csum[-1]) if n else 0
    mid = csum.astype(np.float64) - cost.astype(np.float64) / 2.0
    owner = np.minimum((mid * world / max(total, 1)).astype(np.int64), world - 1) if n else np.zeros(0, np.int64)
    bounds = np.searchsorted(owner, np.arange(world + 1), side="left")
    return [(int(bounds[r]), int(bounds[r + 1] - bounds[r])) for r in range(world)]
