"""The UDP socket batching harness (include/enet_hip.h; csrc/host_io.cpp) over
loopback, on the CPU: DGRAMs built as an ENet host sends them, stamped by the
per-DGRAM callback engine (c/protocol.cs:1690-1698), sent with sendmmsg, received
with recvmmsg, put through ENet's header stage (c/protocol.cs:1001-1030) and
verified (c/protocol.cs:1052-1068).  The stamps and the keep / drop decisions are
checked against the oracle (oracle/enet_crc32_oracle.c) with the header stage
restated independently here.  The GPU pipelines of the same harness are checked in
tests/test_gpu_harness.py."""
import socket

import numpy as np
import pytest

import enethip
from enethip import workloads

LOOPBACK = 0x7F000001
STRIDE = 4096                       # ENet's receive buffer (c/protocol.cs:1219)


def sockets():
    rx = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    rx.setsockopt(socket.SOL_SOCKET, socket.SO_RCVBUF, 8 << 20)
    rx.bind(("127.0.0.1", 0))
    tx = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    tx.setsockopt(socket.SOL_SOCKET, socket.SO_SNDBUF, 8 << 20)
    tx.bind(("127.0.0.1", 0))
    return rx, tx, rx.getsockname()[1]


def oracle_stamps(oracle_lib, sb):
    """CRC of every DGRAM's gather list with the slot holding connectID (or 0)."""
    g = sb.gather
    return oracle_lib.gather(g.payload, g.seg_off, g.seg_len, g.seg_first)


def slots_of(sb):
    g = sb.gather
    pos = g.seg_off[g.seg_first[:-1]].astype(np.int64) + sb.slot_off.astype(np.int64)
    return g.payload[pos[:, None] + np.arange(4)].copy().view(np.uint32).ravel()


def expected_keep(oracle_lib, arena, stride, lens, peers):
    """protocol.cs:1001-1030 restated (peerID / flags / headerSize, drops before the
    checksum), then the oracle's verify (protocol.cs:1052-1068) of the rest."""
    n = len(lens)
    keep = np.zeros(n, np.uint8)
    idx, slot, conn = [], [], []
    for i in range(n):
        L = int(lens[i])
        if L == enethip.DGRAM_TRUNCATED or L < 2:
            continue
        d = arena[i * stride:i * stride + L]
        word = (int(d[0]) << 8) | int(d[1])
        flags, peer = word & 0xC000, word & ~0xF000 & 0xFFFF
        hs = 4 if flags & 0x8000 else 2
        if peer != 0xFFF and peer >= len(peers):
            continue
        if flags & 0x4000 or hs + 4 > L:
            continue
        idx.append(i)
        slot.append(hs)
        conn.append(0 if peer == 0xFFF else int(peers[peer]))
    if idx:
        off = np.array(idx, np.uint64) * np.uint64(stride)
        ok, _ = oracle_lib.verify(arena, off, lens[idx].astype(np.uint32), np.array(slot, np.uint32),
                                  np.array(conn, np.uint32))
        keep[idx] = ok
    return keep


def odd_dgrams(peers):
    """DGRAMs the header stage drops or that do not fit a receive slot."""
    out = [b"\x00",                                               # < 2 bytes
           (0x0123).to_bytes(2, "big") + b"\x00" * 30,            # peerID past the table
           (0x4000 | 1).to_bytes(2, "big") + b"\x11" * 40,        # compressed
           (0x8000 | 2).to_bytes(2, "big") + b"\x22" * 3,         # SENT_TIME, too short for the slot
           (0x0FFF).to_bytes(2, "big") + b"\x00" * (STRIDE + 10)]  # longer than the receive slot
    return out


def send_all(tx, port, sb, burst, rx_fn):
    """Send the batch in bursts (loopback keeps order; each burst drained before the
    next so the receive buffer cannot overflow); returns what rx_fn collected."""
    g = sb.gather
    got = []
    for a in range(0, sb.n, burst):
        b = min(sb.n, a + burst)
        sf = g.seg_first[a:b + 1]
        sent = enethip.udp_send(tx.fileno(), g.payload, g.seg_off, g.seg_len, sf, LOOPBACK, port)
        assert sent == b - a
        got.extend(rx_fn(b - a))
    return got


def test_callback_stamp_matches_oracle(oracle_lib):
    sb = workloads.send_batch(3000, seed=5)
    exp = oracle_stamps(oracle_lib, sb)
    g = sb.gather
    enethip.stamp_callback(g.payload, g.seg_off, g.seg_len, g.seg_first, sb.slot_off)
    assert (slots_of(sb) == exp).all()


@pytest.mark.parametrize("corrupt", [0, 97])
def test_loopback_stamp_send_receive_verify(oracle_lib, corrupt):
    """Send side and receive side end to end over a real socket: stamped DGRAMs keep,
    corrupted ones, unknown peers, compressed, short and oversized DGRAMs drop --
    each decision equal to the oracle's."""
    sb = workloads.send_batch(2000, seed=11 + corrupt)
    g = sb.gather
    exp_stamp = oracle_stamps(oracle_lib, sb)
    enethip.stamp_callback(g.payload, g.seg_off, g.seg_len, g.seg_first, sb.slot_off)
    assert (slots_of(sb) == exp_stamp).all()                       # (stamped against the oracle)
    rng = np.random.default_rng(corrupt)
    if corrupt:                                 # flip a bit of some DGRAMs after the stamp
        for d in rng.choice(sb.n, corrupt, replace=False):
            s = int(g.seg_first[d]) + int(rng.integers(0, 3))
            if g.seg_len[s]:
                g.payload[int(g.seg_off[s]) + int(rng.integers(0, int(g.seg_len[s])))] ^= np.uint8(8)
    rx, tx, port = sockets()
    try:
        arena = np.zeros(STRIDE * 300, np.uint8)
        rows, lens_all = [], []

        def rx_fn(k):
            n, lens, _, _ = enethip.udp_receive(rx.fileno(), arena, STRIDE, 300, timeout_ms=2000)
            assert n == k
            rows.append(arena[:n * STRIDE].copy())
            lens_all.append(lens.copy())
            return [n]

        send_all(tx, port, sb, 250, rx_fn)
        for dg in odd_dgrams(sb.peers):
            tx.sendto(dg, ("127.0.0.1", port))
            rx_fn(1)
        recv = np.concatenate(rows)
        lens = np.concatenate(lens_all)
        assert len(lens) == sb.n + 5
        assert lens[-1] == enethip.DGRAM_TRUNCATED and lens[0] == int(g.seg_len[0:3].sum())
        exp = expected_keep(oracle_lib, recv, STRIDE, lens, sb.peers)
        slot, conn, verdict = enethip.parse_headers(recv, STRIDE, lens, sb.peers)
        assert verdict[-5:].tolist() == [enethip.DROP_SHORT, enethip.DROP_PEER, enethip.DROP_COMPRESSED,
                                         enethip.DROP_SHORT, enethip.DROP_TRUNCATED]
        ok = enethip.verify_callback(recv, STRIDE, lens, slot, conn, verdict)
        assert (ok == exp).all(), np.nonzero(ok != exp)[0][:10]
        assert int(exp[:sb.n].sum()) == sb.n - corrupt
    finally:
        rx.close()
        tx.close()


def test_receive_timeout_and_arguments():
    rx, tx, port = sockets()
    try:
        arena = np.zeros(STRIDE * 4, np.uint8)
        n, _, _, _ = enethip.udp_receive(rx.fileno(), arena, STRIDE, 4, timeout_ms=10)   # nothing queued
        assert n == 0
        with pytest.raises(enethip.ENetHipError) as e:
            enethip.udp_receive(-1, arena, STRIDE, 4)
        assert e.value.code == -1
        lib = enethip.load()
        assert "Bad file descriptor" in enethip.error_string(-(enethip.ERRNO_BASE + 9))
        assert lib.enet_hip_udp_send(tx.fileno(), None, None, None, None, 1, 0, 0, None) == -1
    finally:
        rx.close()
        tx.close()
