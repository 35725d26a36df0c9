"""Pin the oracle before trusting it (CPU only).

* the generated table equals the reference's literal crcTable
  (enet-csharp/ENet/c/packet.cs:106-140, extracted into tests/golden/crc_table_ref.json);
* the pure-Python and C restatements of packet.cs:142-160 agree with every golden
  vector and with zlib (an independent CRC-32/ISO-HDLC implementation);
* the CRC-32/ISO-HDLC check value.
"""
import json
import os
import zlib

import numpy as np
import pytest

import oracle

GDIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _segments(vec, blob):
    return [bytes(blob[o:o + n]) for o, n in vec["segments"]]


def test_table_matches_reference_literal():
    ref = [int(x, 16) for x in json.load(open(os.path.join(GDIR, "crc_table_ref.json")))["table"]]
    assert len(ref) == 256
    assert ref == oracle.crc_table()


def test_c_oracle_table(oracle_lib):
    assert oracle_lib.table().tolist() == oracle.crc_table()


def test_check_value():
    # CRC-32/ISO-HDLC check = 0xCBF43926; enet_crc32 returns it byte-swapped on LE.
    assert oracle.enet_crc32_py([b"123456789"]) == 0x2639F4CB
    assert oracle.host_to_net_32(0xCBF43926) == 0x2639F4CB


def test_empty_is_zero():
    assert oracle.enet_crc32_py([]) == 0
    assert oracle.enet_crc32_py([b""]) == 0


def test_golden_python(golden):
    vecs, blob = golden
    for v in vecs:
        segs = _segments(v, blob)
        exp = int(v["crc"], 16)
        assert oracle.enet_crc32_py(segs) == exp
        assert oracle.host_to_net_32(zlib.crc32(b"".join(segs))) == exp


def test_golden_c(golden, oracle_lib):
    vecs, blob = golden
    for v in vecs:
        assert oracle_lib.crc32(b"".join(_segments(v, blob))) == int(v["crc"], 16)


def test_c_batch_and_mt(oracle_lib):
    rng = np.random.default_rng(7)
    lens = rng.integers(0, 3000, size=500).astype(np.uint32)
    off = np.zeros(500, dtype=np.uint64)
    np.cumsum(lens[:-1], out=off[1:])
    payload = rng.integers(0, 256, size=int(lens.sum()), dtype=np.uint8)
    a = oracle_lib.batch(payload, off, lens)
    b = oracle_lib.batch(payload, off, lens, threads=4)
    assert (a == b).all()
    for i in range(0, 500, 37):
        o, n = int(off[i]), int(lens[i])
        assert a[i] == oracle.host_to_net_32(zlib.crc32(payload[o:o + n].tobytes()))


def test_c_gather(golden, oracle_lib):
    vecs, blob = golden
    gv = [v for v in vecs if v["kind"] in ("gather", "kat")]
    seg_off, seg_len, first = [], [], [0]
    for v in gv:
        for o, n in v["segments"]:
            seg_off.append(o)
            seg_len.append(n)
        first.append(len(seg_off))
    out = oracle_lib.gather(blob, np.array(seg_off, np.uint64), np.array(seg_len, np.uint32),
                            np.array(first, np.uint32))
    assert out.tolist() == [int(v["crc"], 16) for v in gv]


def test_c_verify(golden, oracle_lib):
    vecs, blob = golden
    vv = [v for v in vecs if v["kind"] == "verify"]
    off = np.array([v["segments"][0][0] for v in vv], np.uint64)
    lens = np.array([v["segments"][0][1] for v in vv], np.uint32)
    slot = np.array([v["slot_off"] for v in vv], np.uint32)
    conn = np.array([int(v["connect_id"], 16) for v in vv], np.uint32)
    ok, _ = oracle_lib.verify(blob, off, lens, slot, conn)
    assert ok.astype(bool).tolist() == [v["expect_ok"] for v in vv]


@pytest.mark.parametrize("n", [0, 1, 3, 4, 5, 31, 32, 33, 1200])
def test_python_vs_zlib_lengths(n):
    data = bytes((i * 131 + 7) & 0xFF for i in range(n))
    assert oracle.enet_crc32_py([data]) == oracle.host_to_net_32(zlib.crc32(data))


def test_oracle_verify_has_no_length_limit(oracle_lib):
    """oracle_verify_batch follows protocol.cs:1052-1068 for any DGRAM length (no
    64 KiB cap): a 200 000-byte DGRAM stamped with its CRC verifies, one flipped
    bit drops it; a slot that does not fit the DGRAM drops (documented rule)."""
    rng = np.random.default_rng(3)
    L = 200_000
    buf = rng.integers(0, 256, size=L, dtype=np.uint8)
    conn = 0x1234ABCD
    buf[4:8] = np.frombuffer(np.uint32(conn).tobytes(), np.uint8)
    crc = oracle.host_to_net_32(zlib.crc32(buf.tobytes()))
    buf[4:8] = np.frombuffer(np.uint32(crc).tobytes(), np.uint8)
    off = np.array([0, 0, 0], np.uint64)
    lens = np.array([L, L, 6], np.uint32)
    slot = np.array([4, 4, 4], np.uint32)
    cid = np.array([conn, conn ^ 1, conn], np.uint32)
    ok, comp = oracle_lib.verify(buf, off, lens, slot, cid)
    assert ok.tolist() == [1, 0, 0] and int(comp[0]) == crc and int(comp[2]) == 0
