#!/usr/bin/env python3
"""Socket-in-the-loop rates (BASELINE.json north_star: "packets arrive from and leave
via a UDP socket buffer"), over loopback on one host, for DESIGN.md.

Receive side: a sender thread streams pre-stamped ENet DGRAMs (workloads.send_batch,
~1.2 KB each) with enet_hip_udp_send (sendmmsg) as fast as it can; the receiver
drains the socket for SECONDS per mode:
  gpu      enet_hip_udp_receive_verify (recvmmsg -> header stage -> pitched H2D ->
           GPU verify -> keep mask);
  gpu2     the same in two halves over two arenas in turn
           (enet_hip_udp_receive_verify_submit / _complete): the GPU work of one batch
           overlaps the receive of the next;
  callback enet_hip_udp_receive + header stage + enet_hip_verify_callback (the
           per-DGRAM path ENet runs today: enet_hip_crc32 per DGRAM);
  port     the same with the oracle's byte-serial restatement of packet.cs:142-160
           (the reference's own loop, the CPU baseline);
  recv     enet_hip_udp_receive alone (the socket's own ceiling).
UDP_BENCH_CALLS=1: instead, the cost of one receive call (gpu, callback) on a socket
already holding k = 8, 32, 64 DGRAMs (UDP_BENCH_KS="8,...,256" for others; the streaming
rates above are bound by the sender thread: every mode but port keeps up with it).  UDP_BENCH_SEND_CALLS=1: the cost of one
stamp + send call (gpu, callback) over k = 8 ... 65536 DGRAMs of a pinned send batch.
Send side: stamp + send of the whole batch, GPU (enet_hip_udp_stamp_send) against the
callback stamp (enet_hip_stamp_callback + enet_hip_udp_send), a receiver thread
draining the socket.  One JSON line per mode; every kept / stamped DGRAM is checked
against the oracle before timing.
"""
import ctypes
import json
import os
import socket
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "enet-csharp_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]

import enethip  # noqa: E402
from enethip import workloads  # noqa: E402
import oracle  # noqa: E402

LOOPBACK = 0x7F000001
STRIDE = 4096
SECONDS = float(os.environ.get("UDP_BENCH_SECONDS", "3"))


def pinned(n):
    """Pinned host memory (enet_hip_host_alloc); plain memory where no GPU is visible
    (the CPU modes only: the GPU ones need a device anyway)."""
    lib = enethip.load()
    p = ctypes.c_void_p()
    if lib.enet_hip_host_alloc(n, ctypes.byref(p)) != 0:
        return np.zeros(n, np.uint8), None
    return np.frombuffer((ctypes.c_uint8 * n).from_address(p.value), dtype=np.uint8), p


def free(p):
    if p is not None:
        enethip.load().enet_hip_host_free(p)


def sockets():
    rx = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    rx.setsockopt(socket.SOL_SOCKET, socket.SO_RCVBUF, 256 << 20)
    rx.bind(("127.0.0.1", 0))
    tx = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    tx.setsockopt(socket.SOL_SOCKET, socket.SO_SNDBUF, 64 << 20)
    tx.bind(("127.0.0.1", 0))
    return rx, tx, rx.getsockname()[1]


def sockets_tx():
    tx = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    tx.setsockopt(socket.SOL_SOCKET, socket.SO_SNDBUF, 64 << 20)
    tx.bind(("127.0.0.1", 0))
    return tx


class Sender(threading.Thread):
    def __init__(self, tx, port, sb):
        super().__init__(daemon=True)
        self.tx, self.port, self.sb, self.stop, self.sent = tx, port, sb, False, 0

    def run(self):
        g = self.sb.gather
        while not self.stop:
            self.sent += enethip.udp_send(self.tx.fileno(), g.payload, g.seg_off, g.seg_len, g.seg_first,
                                          LOOPBACK, self.port)


def port_verify(ol, arena, lens, slot, conn, verdict):
    """The byte-serial port of packet.cs:142-160 on the DGRAMs the header stage passes."""
    ok = np.zeros(len(lens), np.uint8)
    idx = np.nonzero(verdict == 0)[0]
    if len(idx):
        o, _ = ol.verify(arena, idx.astype(np.uint64) * np.uint64(STRIDE), lens[idx], slot[idx], conn[idx])
        ok[idx] = o
    return ok


SENDERS = int(os.environ.get("UDP_BENCH_SENDERS", "1"))


def receive_mode(mode, ctx, sb, ol):
    rx, tx, port = sockets()
    arena, p = pinned(STRIDE * 8192)
    arena2, p2 = pinned(STRIDE * 8192) if mode == "gpu2" else (None, None)
    # UDP_BENCH_SENDERS > 1: more sender threads (each its own socket), so that the
    # receiver, not the sender, bounds the rate and the socket queue holds larger batches
    txs = [tx] + [sockets_tx() for _ in range(SENDERS - 1)]
    snds = [Sender(t, port, sb) for t in txs]
    for snd_i in snds:
        snd_i.start()
    snd = snds[0]
    got = kept = nbytes = calls = 0
    bad = 0
    pend = {}                                       # gpu2: slot -> (count, lengths, ok) in flight
    rs = 0                                          # gpu2: the slot to submit next
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < SECONDS or pend:
        if mode == "gpu2":
            if time.perf_counter() - t0 < SECONDS:
                if rs in pend:                      # (two in flight: the older one first)
                    n, lens, ok = pend.pop(rs)
                    ctx.udp_receive_verify_complete(rs)
                else:
                    n = 0
                n2, lens2, ok2 = ctx.udp_receive_verify_submit(rs, rx.fileno(), (arena, arena2)[rs], STRIDE,
                                                               8192, sb.peers, timeout_ms=100)
                if n2:
                    pend[rs] = (n2, lens2.copy(), ok2)
                rs ^= 1
                if n == 0:
                    continue
            else:                                   # time is up: the slots still in flight
                s0 = next(iter(pend))
                n, lens, ok = pend.pop(s0)
                ctx.udp_receive_verify_complete(s0)
        elif mode == "gpu":
            n, lens, ok = ctx.udp_receive_verify(rx.fileno(), arena, STRIDE, 8192, sb.peers, timeout_ms=100)
        else:
            n, lens, _, _ = enethip.udp_receive(rx.fileno(), arena, STRIDE, 8192, timeout_ms=100)
            if mode in ("callback", "port") and n:
                slot, conn, verdict = enethip.parse_headers(arena, STRIDE, lens, sb.peers)
                ok = (enethip.verify_callback(arena, STRIDE, lens, slot, conn, verdict) if mode == "callback"
                      else port_verify(ol, arena, lens, slot, conn, verdict))
            else:
                ok = np.ones(n, np.uint8)
        calls += 1
        got += n
        kept += int(ok.sum())
        bad += n - int(ok.sum())
        nbytes += int(lens[lens != enethip.DGRAM_TRUNCATED].astype(np.uint64).sum())
    dt = time.perf_counter() - t0
    for snd_i in snds:
        snd_i.stop = True
    for snd_i in snds:
        snd_i.join()
    rx.close()
    for t in txs:
        t.close()
    free(p)
    free(p2)
    assert bad == 0, f"{mode}: {bad} stamped DGRAMs dropped"
    return {"side": "receive", "mode": mode, "seconds": round(dt, 2), "dgrams": got, "kept": kept,
            "dgrams_per_s": round(got / dt), "GBps": round(nbytes / dt / 1e9, 3),
            "mean_batch": round(got / max(1, calls), 1), "senders": len(snds),
            "sender_dgrams_per_s": round(sum(x.sent for x in snds) / dt)}


class Drain(threading.Thread):
    def __init__(self, rx):
        super().__init__(daemon=True)
        self.rx, self.stop, self.got = rx, False, 0
        self.arena = np.zeros(STRIDE * 2048, np.uint8)

    def run(self):
        while not self.stop:
            n, _, _, _ = enethip.udp_receive(self.rx.fileno(), self.arena, STRIDE, 2048, timeout_ms=50)
            self.got += n


def send_mode(mode, ctx, sb, ol):
    rx, tx, port = sockets()
    dr = Drain(rx)
    dr.start()
    g = sb.gather
    base = g.payload.copy()                         # slots back to connectID before every pass
    arena, p = pinned(len(base))
    arena[:] = base
    exp = ol.gather(base, g.seg_off, g.seg_len, g.seg_first)
    pos = (g.seg_off[g.seg_first[:-1]] + sb.slot_off).astype(np.int64)
    passes = sent = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < SECONDS:
        arena[:] = base
        if mode == "gpu":
            sent += ctx.udp_stamp_send(tx.fileno(), arena, g.seg_off, g.seg_len, g.seg_first, sb.slot_off,
                                       LOOPBACK, port)
        else:
            enethip.stamp_callback(arena, g.seg_off, g.seg_len, g.seg_first, sb.slot_off)
            sent += enethip.udp_send(tx.fileno(), arena, g.seg_off, g.seg_len, g.seg_first, LOOPBACK, port)
        if passes == 0:
            slots = arena[pos[:, None] + np.arange(4)].copy().view(np.uint32).ravel()
            assert (slots == exp).all(), f"{mode} stamp differs from the oracle"
        passes += 1
    dt = time.perf_counter() - t0
    dr.stop = True
    dr.join()
    rx.close()
    tx.close()
    free(p)
    return {"side": "send", "mode": mode, "seconds": round(dt, 2), "passes": passes, "dgrams_sent": sent,
            "dgrams_per_s": round(sent / dt), "GBps": round(g.dgram_bytes * passes / dt / 1e9, 3),
            "received_by_drain": dr.got}


def call_latency(ctx, sb, mode, k, reps=300):
    """One receive call on a socket already holding k DGRAMs (sent just before, so the
    socket is not the limit): the per-batch cost of each receive form, recvmmsg
    included, median and 10th percentile over `reps` calls."""
    rx, tx, port = sockets()
    arena, p = pinned(STRIDE * 1024)
    g = sb.gather
    ts = []
    try:
        for r in range(reps + 10):
            a = (r * k) % (sb.n - k)
            sent = enethip.udp_send(tx.fileno(), g.payload, g.seg_off, g.seg_len, g.seg_first[a:a + k + 1],
                                    LOOPBACK, port)
            assert sent == k
            t0 = time.perf_counter()
            if mode == "gpu":
                n, lens, ok = ctx.udp_receive_verify(rx.fileno(), arena, STRIDE, k, sb.peers, timeout_ms=100)
            elif mode == "recv":                                 # (the socket call alone)
                n, lens, _, _ = enethip.udp_receive(rx.fileno(), arena, STRIDE, k, timeout_ms=100)
                ok = np.ones(n, np.uint8)
            else:
                n, lens, _, _ = enethip.udp_receive(rx.fileno(), arena, STRIDE, k, timeout_ms=100)
                slot, conn, verdict = enethip.parse_headers(arena, STRIDE, lens, sb.peers)
                ok = enethip.verify_callback(arena, STRIDE, lens, slot, conn, verdict)
            t1 = time.perf_counter()
            assert n == k and int(ok.sum()) == k, (mode, k, n, int(ok.sum()))
            if r >= 10:
                ts.append(t1 - t0)
    finally:
        rx.close()
        tx.close()
        free(p)
    ts = np.array(ts) * 1e6
    return {"side": "receive-call", "mode": mode, "dgrams_per_call": k, "calls": reps,
            "median_us": round(float(np.median(ts)), 1), "p10_us": round(float(np.percentile(ts, 10)), 1),
            "median_GBps": round(k * 1200 / float(np.median(ts)) / 1e3, 3)}


def send_call_latency(ctx, sb, mode, k, reps, ol):
    """One stamp + send call over the first k DGRAMs of a pinned send batch: the GPU
    stamp (enet_hip_udp_stamp_send) or the CPU callback stamp + enet_hip_udp_send;
    median and 10th percentile over `reps` calls (the slots restored between calls,
    outside the timing), a receiver thread draining the socket."""
    rx, tx, port = sockets()
    dr = Drain(rx)
    dr.start()
    g = sb.gather
    base = g.payload.copy()
    arena, p = pinned(len(base))
    arena[:] = base
    sf = g.seg_first[:k + 1]
    pos = (g.seg_off[g.seg_first[:k]] + sb.slot_off[:k]).astype(np.int64)
    ts = []
    try:
        for r in range(reps + 3):
            arena[pos[:, None] + np.arange(4)] = base[pos[:, None] + np.arange(4)]
            t0 = time.perf_counter()
            if mode == "gpu":
                sent = ctx.udp_stamp_send(tx.fileno(), arena, g.seg_off, g.seg_len, sf, sb.slot_off[:k], LOOPBACK, port)
            else:
                enethip.stamp_callback(arena, g.seg_off, g.seg_len, sf, sb.slot_off[:k])
                sent = enethip.udp_send(tx.fileno(), arena, g.seg_off, g.seg_len, sf, LOOPBACK, port)
            t1 = time.perf_counter()
            assert sent == k
            if r >= 3:
                ts.append(t1 - t0)
        slots = arena[pos[:, None] + np.arange(4)].copy().view(np.uint32).ravel()
        assert (slots == ol.gather(base, g.seg_off, g.seg_len, sf)).all(), f"{mode} stamp differs from the oracle"
    finally:
        dr.stop = True
        dr.join()
        rx.close()
        tx.close()
        free(p)
    ts = np.array(ts) * 1e6
    return {"side": "send-call", "mode": mode, "dgrams_per_call": k, "calls": reps,
            "median_us": round(float(np.median(ts)), 1), "p10_us": round(float(np.percentile(ts, 10)), 1)}


def main():
    sb = workloads.send_batch(int(os.environ.get("UDP_BENCH_DGRAMS", "65536")), body=(1188, 1188), seed=9)
    enethip.stamp_callback(sb.gather.payload, sb.gather.seg_off, sb.gather.seg_len, sb.gather.seg_first,
                           sb.slot_off)
    ol = oracle.OracleLib()
    ctx = enethip.Context(0)
    print(json.dumps({"cores": len(os.sched_getaffinity(0)), "dgrams_per_batch": sb.n,
                      "dgram_bytes": sb.gather.dgram_bytes}), flush=True)
    if os.environ.get("UDP_BENCH_SEND_CALLS"):       # per-call send costs only
        sb2 = workloads.send_batch(int(os.environ.get("UDP_BENCH_DGRAMS", "65536")), body=(1188, 1188), seed=10)
        for k, reps in ((8, 300), (64, 300), (512, 100), (4096, 30), (65536, 10)):
            for mode in ("gpu", "callback"):
                print(json.dumps(send_call_latency(ctx, sb2, mode, min(k, sb2.n), reps, ol)), flush=True)
        ctx.close()
        return
    if os.environ.get("UDP_BENCH_CALLS"):            # per-call costs only
        if os.environ.get("UDP_BENCH_PATH"):          # (a kernel path for the GPU verify: 13 = lean)
            ctx.set_kernel_path(int(os.environ["UDP_BENCH_PATH"]))
        ks = tuple(int(x) for x in os.environ.get("UDP_BENCH_KS", "8,32,64").split(","))
        for k in ks:
            for mode in os.environ.get("UDP_BENCH_CALL_MODES", "gpu,callback").split(","):
                print(json.dumps(call_latency(ctx, sb, mode, k)), flush=True)
        ctx.close()
        return
    modes = ("recv", "gpu", "gpu2", "callback", "port")
    if os.environ.get("UDP_BENCH_RECV_MODES"):       # (a subset of the receive modes, and no send side)
        modes = tuple(os.environ["UDP_BENCH_RECV_MODES"].split(","))
    for mode in modes:
        print(json.dumps(receive_mode(mode, ctx, sb, ol)), flush=True)
    if os.environ.get("UDP_BENCH_RECV_MODES"):
        ctx.close()
        return
    sb2 = workloads.send_batch(int(os.environ.get("UDP_BENCH_DGRAMS", "65536")), body=(1188, 1188), seed=10)
    for mode in ("gpu", "callback"):
        print(json.dumps(send_mode(mode, ctx, sb2, ol)), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
