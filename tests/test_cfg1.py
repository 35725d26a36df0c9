"""BASELINE config 1: the CPU checksum callback driven as ENet's
protocol engine drives it in the loopback echo test (Test/TestWave.cs) with the
checksum on both hosts -- send stamp (c/protocol.cs:1690-1698) and receive verify
(c/protocol.cs:1052-1068) of every DGRAM of a reliable echo round trip
(tools/cfg1_loop.c).  libenethip's enet_hip_crc32 and the oracle's byte-serial
restatement of packet.cs:142-160 must agree on every CRC and every verify must
pass.  CPU only."""
import json
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "enet-csharp_amd", "libenethip.so")
ORACLE = os.path.join(ROOT, "oracle", "lib", "liboracle.so")


@pytest.fixture(scope="module")
def cfg1_bin(tmp_path_factory):
    if not os.path.exists(LIB) or not os.path.exists(ORACLE):
        pytest.skip("libenethip.so / liboracle.so not built (run __graft_entry__.build())")
    out = str(tmp_path_factory.mktemp("cfg1") / "cfg1_loop")
    subprocess.run(["gcc", "-O2", "-Wall", "-Wextra", "-Werror", "-o", out,
                    os.path.join(ROOT, "tools", "cfg1_loop.c"), "-ldl"], check=True)
    return out


@pytest.mark.parametrize("packets,payload", [(1024, 256), (37, 1), (5, 0), (64, 4082)])
def test_cfg1_round_trips_bit_exact(cfg1_bin, packets, payload):
    r = subprocess.run([cfg1_bin, LIB, ORACLE, str(packets), str(payload), "0.05"],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["mismatch"] == 0
    assert line["callback"]["verify_fail"] == 0 and line["reference_port"]["verify_fail"] == 0
    # 4 DGRAMs per round trip: 2 reliable (8 + 6 + payload) and 2 acks (8 + 8), each sent and received
    assert line["bytes_per_round_trip"] == pytest.approx(2 * (2 * (14 + payload) + 2 * 16))
