"""TLS 1.3 record framing, CPU side: the oracle's restatement of the
picotls record layer pinned to the reference's own ptls_send / ptls_receive outputs
(tests/golden/tls_records.json), and the host-side planners of include/ptls_mi355x.h section 4
(ptls_mi355x_tls_plan_send / _parse_records) against the same wire bytes.  No GPU."""
import hashlib
import json
import os

import numpy as np
import pytest

import oracle
import rapido_amd as ra
from rapido_amd.records import xorshift64star

GOLDEN = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "tls_records.json")))
RC = {0: None, 20: oracle.TLS_BAD_MAC, 10: oracle.TLS_NO_TYPE}


def xs(seed, n):
    return xorshift64star(seed, n).tobytes()


def oracle_send(key, iv, seq0, data, content_type=23):
    """buffer_push_encrypted_records restated with the oracle (lib/picotls.c:664-684)."""
    wire, seq, off = b"", seq0, 0
    while off < len(data):
        frag = data[off: off + 16384]
        wire += oracle.tls_seal_record(key, iv, seq, content_type, frag)
        off += len(frag)
        seq += 1
    return wire, seq


@pytest.mark.parametrize("case", GOLDEN["send"], ids=lambda c: f"aes{c['keylen'] * 8}-{c['len']}")
def test_oracle_send_matches_reference(case):
    key, iv = xs(case["seed"] + 1, case["keylen"]), xs(case["seed"] + 2, 12)
    wire, seq = oracle_send(key, iv, case["seq0"], xs(case["seed"], case["len"]))
    assert len(wire) == case["wire_len"] and seq == case["seq_after"]
    assert hashlib.sha256(wire).hexdigest() == case["wire_sha256"]
    if "wire" in case:
        assert wire.hex() == case["wire"]


@pytest.mark.parametrize("i", range(len(GOLDEN["receive"])))
def test_oracle_receive_matches_reference(i):
    c = GOLDEN["receive"][i]
    key, iv, wire = bytes.fromhex(c["key"]), bytes.fromhex(c["iv"]), bytes.fromhex(c["wire"])
    got = oracle.tls_open_record(key, iv, c["seq"], wire)
    if c["rc"] == 0:
        assert got == (bytes.fromhex(c["plaintext"]), 23)
    else:
        assert got == RC[c["rc"]]


@pytest.mark.parametrize("case", GOLDEN["send"][:10], ids=lambda c: str(c["len"]))
def test_plan_send_matches_reference_layout(engine_lib, case):
    """The planner's record boundaries / seqs are the reference's (parse the reference wire back)."""
    key, iv = xs(case["seed"] + 1, case["keylen"]), xs(case["seed"] + 2, 12)
    data = xs(case["seed"], case["len"])
    wire, _ = oracle_send(key, iv, case["seq0"], data)
    recs, wire_len, seq = ra.tls_plan_send(case["len"], case["seq0"], 23, src_off=0, dst_off=0)
    assert wire_len == case["wire_len"] and seq == case["seq_after"]
    rc, parsed, used, seq2 = ra.tls_parse_records(wire, case["seq0"], src_off=0, dst_off=0)
    assert rc == 0 and used == len(wire) and seq2 == seq
    assert (parsed["src"] == recs["dst"]).all() and (parsed["seq"] == recs["seq"]).all()
    assert (parsed["len"] == recs["len"] + 17).all()
    assert (np.diff(parsed["dst"]) == (parsed["len"][:-1] - 16)).all()


def test_parse_records_edges(engine_lib):
    w1 = oracle.tls_seal_record(bytes(16), bytes(12), 0, 23, b"x" * 20)
    # incomplete record: stops before it, consumes nothing of it
    rc, recs, used, seq = ra.tls_parse_records(w1 + w1[:-1], 5)
    assert rc == 0 and len(recs) == 1 and used == len(w1) and seq == 6
    # a partial header
    rc, recs, used, _ = ra.tls_parse_records(w1 + b"\x17\x03", 0)
    assert (rc, len(recs), used) == (0, 1, len(w1))
    # non-application_data record: left to the slot path
    rc, recs, used, _ = ra.tls_parse_records(w1 + b"\x15\x03\x03\x00\x02\x02\x28" + w1, 0)
    assert (rc, len(recs), used) == (0, 1, len(w1))
    # length above PTLS_MAX_ENCRYPTED_RECORD_SIZE -> decode_error
    big = b"\x17\x03\x03" + (16384 + 257).to_bytes(2, "big")
    rc, recs, used, _ = ra.tls_parse_records(w1 + big + bytes(16384 + 257), 0)
    assert (rc, len(recs), used) == (50, 1, len(w1))
    # the maximum is accepted
    mx = b"\x17\x03\x03" + (16384 + 256).to_bytes(2, "big") + bytes(16384 + 256)
    rc, recs, used, _ = ra.tls_parse_records(mx, 0)
    assert (rc, len(recs), used) == (0, 1, len(mx))
    # max_records
    rc, recs, used, _ = ra.tls_parse_records(w1 * 5, 0, max_records=3)
    assert (rc, len(recs), used) == (0, 3, 3 * len(w1))


def test_plan_send_chunks(engine_lib):
    recs, wire, seq = ra.tls_plan_send(0, 9)
    assert len(recs) == 0 and wire == 0 and seq == 9
    recs, wire, seq = ra.tls_plan_send(3 * 16384 + 1, 9, 22, src_off=7, dst_off=100)
    assert list(recs["len"]) == [16384, 16384, 16384, 1] and list(recs["type"]) == [22] * 4
    assert list(recs["seq"]) == [9, 10, 11, 12] and seq == 13
    assert list(recs["src"]) == [7, 7 + 16384, 7 + 2 * 16384, 7 + 3 * 16384]
    assert list(recs["dst"]) == [100, 100 + 16406, 100 + 2 * 16406, 100 + 3 * 16406]
    assert wire == 3 * 16406 + 23
