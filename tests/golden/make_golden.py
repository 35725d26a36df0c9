"""Generate the committed golden fixtures for the ENet CRC32 path.

Run from the repo root in the build container (it reads /root/reference, which
does not exist on the GPU box):  python tests/golden/make_golden.py

Outputs (all data, no code):
  crc_table_ref.json  -- the 256 literals of crcTable, parsed verbatim from
                         /root/reference/enet-csharp/ENet/c/packet.cs:106-140
  vectors.bin         -- concatenated input bytes of every vector
  vectors.json        -- per vector: kind, segment (offset,length) list into
                         vectors.bin, expected enet_crc32 value (wire-order uint,
                         exactly what packet.cs:159 returns), and for verify
                         vectors the slot offset / connectID / expected verdict.

Expected values come from oracle.enet_crc32_py (byte-serial restatement of
packet.cs:142-160 over the reference's own table) and are cross-checked against
an independent implementation, zlib.crc32 (CRC-32/ISO-HDLC), byte-swapped.
"""
from __future__ import annotations

import json
import os
import re
import sys
import zlib

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle  # noqa: E402

REF_PACKET_CS = "/root/reference/enet-csharp/ENet/c/packet.cs"


def parse_reference_table(path: str = REF_PACKET_CS) -> list[int]:
    lines = open(path, encoding="utf-8-sig").read().splitlines()
    body = "\n".join(lines[105:140])          # lines 106-140 (1-based)
    assert "crcTable" in lines[105], lines[105]
    vals = [int(x, 16) if x.lower().startswith("0x") else int(x)
            for x in re.findall(r"0x[0-9A-Fa-f]+|\b\d+\b", body.split("{", 1)[1])]
    assert len(vals) == 256, len(vals)
    return vals


def splitmix64(seed: int):
    s = seed & 0xFFFFFFFFFFFFFFFF
    while True:
        s = (s + 0x9E3779B97F4A7C15) & 0xFFFFFFFFFFFFFFFF
        z = s
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & 0xFFFFFFFFFFFFFFFF
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & 0xFFFFFFFFFFFFFFFF
        yield z ^ (z >> 31)


def rand_bytes(gen, n: int) -> bytes:
    out = bytearray()
    while len(out) < n:
        out += next(gen).to_bytes(8, "little")
    return bytes(out[:n])


def zlib_ref(data: bytes) -> int:
    return oracle.host_to_net_32(zlib.crc32(data) & 0xFFFFFFFF)


def main() -> None:
    table = parse_reference_table()
    assert table == oracle.crc_table(), "reference crcTable differs from the 0xEDB88320 table"
    with open(os.path.join(HERE, "crc_table_ref.json"), "w") as f:
        json.dump({"source": "enet-csharp/ENet/c/packet.cs:106-140",
                   "table": [f"0x{v:08X}" for v in table]}, f, indent=0)

    blob = bytearray()
    vecs = []
    gen = splitmix64(0x474F4C44)   # "GOLD"

    def add(kind: str, segments: list[bytes], **extra):
        segs = []
        for s in segments:
            segs.append([len(blob), len(s)])
            blob.extend(s)
        whole = b"".join(segments)
        exp = oracle.enet_crc32_py(segments)
        assert exp == zlib_ref(whole), (kind, len(whole))
        vecs.append({"kind": kind, "segments": segs, "crc": f"0x{exp:08X}", **extra})

    # Known-answer tests (CRC-32/ISO-HDLC check value and edge shapes).
    add("kat", [b"123456789"])
    add("kat", [b"123", b"456789"])
    add("kat", [b"12", b"", b"3456", b"789"])
    add("kat", [])
    add("kat", [b""])
    add("kat", [b"\x00"])
    add("kat", [b"\xff"])
    add("kat", [b"\x00" * 4096])
    add("kat", [b"\xff" * 4096])
    add("kat", [b"The quick brown fox jumps over the lazy dog"])
    # every length 0..64 (covers all tail / head alignments of 16- and 32-byte blocks)
    for n in range(0, 65):
        add("len_sweep", [rand_bytes(gen, n)])
    # random MTU-ish packets, incl. the configs' lengths
    for n in [96, 255, 256, 257, 511, 512, 733, 1023, 1024, 1025, 1199, 1200, 1201, 1360, 1392, 1400,
              2048, 4095, 4096]:
        add("random", [rand_bytes(gen, n)])
    for _ in range(40):
        n = 64 + next(gen) % 1337
        add("random", [rand_bytes(gen, n)])
    # gather lists, like the send path's host->buffers (protocol.cs:1546-1559, 1690-1698)
    for _ in range(24):
        k = 1 + next(gen) % 6
        segs = [rand_bytes(gen, int(next(gen) % 400)) for _ in range(k)]
        add("gather", segs)
    # cfg5-style fragment DGRAM: [4B header][4B slot][24B SendFragment][1360 payload]
    hdr = rand_bytes(gen, 4) + (0x1234ABCD).to_bytes(4, "little")
    add("gather", [hdr, rand_bytes(gen, 24), rand_bytes(gen, 1360)])
    add("gather", [hdr, rand_bytes(gen, 24), rand_bytes(gen, 256)])
    # 65-buffer gather list (ENET_BUFFER_MAXIMUM, include/enet.cs:417)
    add("gather", [rand_bytes(gen, int(next(gen) % 40)) for _ in range(65)])

    # receive-verify DGRAMs (protocol.cs:1052-1068): slot after a 2- or 4-byte header.
    for i in range(16):
        hs = 4 if i % 2 else 2
        connect = int(next(gen) & 0xFFFFFFFF) if i % 3 else 0
        body = rand_bytes(gen, int(12 + next(gen) % 1300))
        hdr_b = rand_bytes(gen, hs)
        stamped = oracle.enet_crc32_py([hdr_b + connect.to_bytes(4, "little") + body])
        corrupt = (i % 4 == 3)
        wire = bytearray(hdr_b + stamped.to_bytes(4, "little") + body)
        if corrupt:
            wire[-1 - (i % 7)] ^= 0x40
        add("verify", [bytes(wire)], slot_off=hs, connect_id=f"0x{connect:08X}",
            expect_ok=(not corrupt))

    with open(os.path.join(HERE, "vectors.bin"), "wb") as f:
        f.write(bytes(blob))
    with open(os.path.join(HERE, "vectors.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_golden.py",
                   "algorithm": "enet-csharp/ENet/c/packet.cs:142-160 (+ zlib cross-check)",
                   "vectors": vecs}, f, indent=1)
    print(f"{len(vecs)} vectors, {len(blob)} bytes")


if __name__ == "__main__":
    main()
