"""GPU parity of the host-memory entry points and the socket pipelines
(csrc/host_pipeline.hip) against the oracle: the pipelined checksum of host
batches (cfg2 in full, many chunks, offsets out of order, multi-context shards),
the host gather lists at full cfg5 size (4096 x 64 KiB messages = 200 704
DGRAMs), and the GPU stamp / receive-verify over a loopback socket."""
import socket
import threading
import time

import numpy as np
import pytest

import enethip
from enethip import workloads
from test_gpu_parity import ctx  # noqa: F401  (fixture)
from test_udp_harness import (LOOPBACK, STRIDE, expected_keep, odd_dgrams, oracle_stamps, slots_of,  # noqa: F401
                              sockets)

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


def pinned(n):
    """Host memory from enet_hip_host_alloc (pinned), as a numpy view; (array, pointer)."""
    import ctypes
    lib = enethip.load()
    p = ctypes.c_void_p()
    assert lib.enet_hip_host_alloc(n, ctypes.byref(p)) == 0
    buf = (ctypes.c_uint8 * n).from_address(p.value)
    return np.frombuffer(buf, dtype=np.uint8), p


def free_pinned(p):
    enethip.load().enet_hip_host_free(p)


def test_batch_host_cfg2_pipelined(ctx, oracle_lib):  # noqa: F811
    """cfg2 (75 MiB: five 16-MiB chunks over two streams) from pinned host memory."""
    b = workloads.cfg2()
    exp = oracle_lib.batch(b.payload, b.off, b.lens, threads=16)
    arr, p = pinned(b.payload.nbytes)
    try:
        arr[:] = b.payload
        assert (ctx.crc32_batch_host(arr, b.off, b.lens) == exp).all()
    finally:
        free_pinned(p)


def test_batch_host_in_place(ctx, oracle_lib):  # noqa: F811
    """A pinned arena whose packets span at most 4 MiB, or cover under 4/5 of their span,
    is read in place over PCIe: packets at any alignment, overlapping,
    empty, ending on the arena's last byte; a sparse list over a 24-MiB span; the arena
    rewritten between calls -- against the oracle."""
    rng = np.random.default_rng(69)
    n = (24 << 20) + 7
    arr, p = pinned(n)
    try:
        for rep in range(2):
            arr[:] = rng.integers(0, 256, size=n, dtype=np.uint8)
            k = 3000
            lens = np.where(rng.integers(0, 8, size=k) == 0, 0, rng.integers(1, 1500, size=k)).astype(np.uint32)
            off = rng.integers(0, (3 << 20), size=k).astype(np.uint64)       # dense: a 3-MiB span
            off[:3] = n - lens[:3]                                        # (and three at the very end)
            exp = oracle_lib.batch(arr, off, lens)
            assert (ctx.crc32_batch_host(arr, off, lens) == exp).all(), rep
            off2 = rng.integers(0, n - 1500, size=k).astype(np.uint64)    # sparse over 24 MiB
            exp2 = oracle_lib.batch(arr, off2, lens)
            assert (ctx.crc32_batch_host(arr, off2, lens) == exp2).all(), rep
            assert (ctx.crc32_batch_host(arr, off2[5:6], lens[5:6]) == exp2[5:6]).all()
    finally:
        free_pinned(p)


def test_batch_host_chunks_and_orders(ctx, oracle_lib):  # noqa: F811
    """Many chunks (300 K mixed packets, pageable memory), packets in arbitrary order
    (the one-span fallback), a single packet and empty packets."""
    b = workloads.mixed(300_000, 0, 1400, seed=61, len_seed=62)
    exp = oracle_lib.batch(b.payload, b.off, b.lens, threads=16)
    assert (ctx.crc32_batch_host(b.payload, b.off, b.lens) == exp).all()
    perm = np.random.default_rng(63).permutation(b.n)
    assert (ctx.crc32_batch_host(b.payload, b.off[perm], b.lens[perm]) == exp[perm]).all()
    assert (ctx.crc32_batch_host(b.payload, b.off[7:8], b.lens[7:8]) == exp[7:8]).all()
    # packets alternating between two regions 24 MiB apart: every span
    # chunk would hold one packet; the plan takes the one-chunk form instead
    H, n2 = 24 << 20, 4000
    arena = np.frombuffer(np.random.default_rng(67).bytes(H + 64 * n2), dtype=np.uint8)
    off2 = np.array([(i // 2) * 64 + (H if i & 1 else 0) for i in range(n2)], np.uint64)
    len2 = np.full(n2, 64, np.uint32)
    assert (ctx.crc32_batch_host(arena, off2, len2) == oracle_lib.batch(arena, off2, len2)).all()
    with pytest.raises(enethip.ENetHipError):                # a packet past the arena: rejected
        ctx.crc32_batch_host(b.payload[:100], b.off[:2], np.array([50, 60], np.uint32) + 50)


def test_batch_multi_contexts(oracle_lib):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    b = workloads.mixed(400_001, 64, 1400, seed=64, len_seed=65)
    ctxs = [enethip.Context(i % max(1, enethip.device_count())) for i in range(3)]
    try:
        got = enethip.crc32_batch_multi(ctxs, b.payload, b.off, b.lens)
    finally:
        for c in ctxs:
            c.close()
    assert (got == oracle_lib.batch(b.payload, b.off, b.lens, threads=16)).all()


def test_gather_binned_host_full_cfg5(ctx, oracle_lib):  # noqa: F811
    """cfg5 at full size: 4096 messages x 64 KiB -> 200 704 three-buffer DGRAMs
    (274.9 MB) from pinned host memory, against the oracle's gather."""
    g = workloads.cfg5()
    assert g.n == 200_704
    exp = oracle_lib.gather(g.payload, g.seg_off, g.seg_len, g.seg_first)
    arr, p = pinned(g.payload.nbytes)
    try:
        arr[:] = g.payload
        got = ctx.gather_binned_host(arr, g.seg_off, g.seg_len, g.seg_first)
    finally:
        free_pinned(p)
    assert (got == exp).all(), np.nonzero(got != exp)[0][:10]
    # random gather lists (0-65 buffers, empty buffers and DGRAMs), pageable memory
    rng = np.random.default_rng(66)
    payload = rng.integers(0, 256, size=1 << 20, dtype=np.uint8)
    cnt = rng.integers(0, 66, size=500)
    sf = np.zeros(501, np.uint32)
    np.cumsum(cnt, out=sf[1:])
    ns = int(sf[-1])
    lens = np.where(rng.integers(0, 6, size=ns) == 0, 0, rng.integers(1, 1400, size=ns)).astype(np.uint32)
    offs = rng.integers(0, len(payload) - 1400, size=ns).astype(np.uint64)
    assert (ctx.gather_binned_host(payload, offs, lens, sf) == oracle_lib.gather(payload, offs, lens, sf)).all()
    with pytest.raises(enethip.ENetHipError):                # segFirst[n] > segCount: rejected
        ctx.gather_binned_host(payload, offs, lens, np.concatenate([sf[:-1], [ns + 1]]).astype(np.uint32))
    sl = sf[100:301]                                         # a slice of the list (segFirst[0] > 0)
    exp = oracle_lib.gather(payload, offs, lens, sf)
    assert (ctx.gather_binned_host(payload, offs, lens, sl) == exp[100:300]).all()


def test_gather_binned_host_in_place(ctx, oracle_lib):  # noqa: F811
    """A pinned arena whose used span is at most 4 MiB is read in place over PCIe (no
    copies): random gather lists (0-65 buffers, empty buffers and DGRAMs,
    segments ending at the arena's last byte), slices of the list, and the same arena
    rewritten between calls -- against the oracle's gather."""
    rng = np.random.default_rng(68)
    n = (1 << 20) + 5                                        # (not a multiple of 16)
    arr, p = pinned(n)
    try:
        for rep in range(3):
            arr[:] = rng.integers(0, 256, size=n, dtype=np.uint8)
            cnt = rng.integers(0, 66, size=400)
            sf = np.zeros(401, np.uint32)
            np.cumsum(cnt, out=sf[1:])
            ns = int(sf[-1])
            lens = np.where(rng.integers(0, 6, size=ns) == 0, 0, rng.integers(1, 1400, size=ns)).astype(np.uint32)
            offs = rng.integers(0, n - 1400, size=ns).astype(np.uint64)
            tail = rng.choice(ns, 5, replace=False)              # segments that end on the last byte
            offs[tail] = n - lens[tail]
            exp = oracle_lib.gather(arr, offs, lens, sf)
            got = ctx.gather_binned_host(arr, offs, lens, sf)
            assert (got == exp).all(), (rep, np.nonzero(got != exp)[0][:10])
            sl = sf[50 * rep:50 * rep + 201]
            assert (ctx.gather_binned_host(arr, offs, lens, sl) == exp[50 * rep:50 * rep + 200]).all()
    finally:
        free_pinned(p)


@pytest.mark.parametrize("corrupt,kind", [(0, "pinned"), (61, "pinned"), (61, "pageable")])
def test_gpu_stamp_send_and_receive_verify(ctx, oracle_lib, corrupt, kind):  # noqa: F811
    """The socket harness around the GPU: enet_hip_udp_stamp_send (GPU stamp,
    protocol.cs:1690-1698, then sendmmsg) and enet_hip_udp_receive_verify (recvmmsg,
    header stage, GPU verify, protocol.cs:1052-1068): stamps and keep mask equal to the
    oracle's, header-stage drops included.  A pinned arena is verified in place (the
    kernel reads it over PCIe, every batch reusing the same arena); a pageable one
    takes the pitched-H2D copy form."""
    sb = workloads.send_batch(3000, seed=70 + corrupt)
    g = sb.gather
    exp_stamp = oracle_stamps(oracle_lib, sb)
    rx, tx, port = sockets()
    arena, p = pinned(STRIDE * 512) if kind == "pinned" else (np.zeros(STRIDE * 512, np.uint8), None)
    try:
        rng = np.random.default_rng(corrupt)
        recv_rows, recv_lens, oks = [], [], []
        for a in range(0, sb.n, 400):
            b = min(sb.n, a + 400)
            sf = g.seg_first[a:b + 1]
            sent = ctx.udp_stamp_send(tx.fileno(), g.payload, g.seg_off, g.seg_len, sf, sb.slot_off[a:b],
                                      LOOPBACK, port)
            assert sent == b - a
            n, lens, ok = ctx.udp_receive_verify(rx.fileno(), arena, STRIDE, 512, sb.peers, timeout_ms=2000)
            assert n == b - a
            recv_rows.append(arena[:n * STRIDE].copy())
            recv_lens.append(lens.copy())
            oks.append(ok.copy())
        assert (slots_of(sb) == exp_stamp).all()
        ok = np.concatenate(oks)
        assert ok.sum() == sb.n                                   # every stamped DGRAM kept
        # corrupted re-sends and the odd DGRAMs: drops decided as the oracle decides
        if corrupt:
            for d in rng.choice(sb.n, corrupt, replace=False):
                s = int(g.seg_first[d]) + int(rng.integers(0, 3))
                if g.seg_len[s]:
                    g.payload[int(g.seg_off[s]) + int(rng.integers(0, int(g.seg_len[s])))] ^= np.uint8(2)
        sent = enethip.udp_send(tx.fileno(), g.payload, g.seg_off, g.seg_len, g.seg_first[:401], LOOPBACK, port)
        assert sent == 400
        for dg in odd_dgrams(sb.peers):
            tx.sendto(dg, ("127.0.0.1", port))
        got = 0
        rows, lens_l, oks2 = [], [], []
        while got < 405:
            n, lens, okb = ctx.udp_receive_verify(rx.fileno(), arena, STRIDE, 512, sb.peers, timeout_ms=2000)
            assert n > 0
            rows.append(arena[:n * STRIDE].copy())
            lens_l.append(lens.copy())
            oks2.append(okb.copy())
            got += n
        recv, lens, ok2 = np.concatenate(rows), np.concatenate(lens_l), np.concatenate(oks2)
        exp = expected_keep(oracle_lib, recv, STRIDE, lens, sb.peers)
        assert (ok2 == exp).all(), np.nonzero(ok2 != exp)[0][:10]
        assert exp[-5:].sum() == 0
    finally:
        if p is not None:
            free_pinned(p)
        rx.close()
        tx.close()


def compressible(sb, rng, frac=0.6):
    """Make the bodies of a fraction of the DGRAMs low-entropy (ENet command streams
    of repeated fields): those compress, the random ones do not (sent as they are)."""
    g = sb.gather
    for d in np.nonzero(rng.random(sb.n) < frac)[0]:
        s = int(g.seg_first[d]) + 2                          # the body segment
        o, L = int(g.seg_off[s]), int(g.seg_len[s])
        pat = rng.integers(0, 6, size=max(1, L // 16)).astype(np.uint8)
        g.payload[o:o + L] = np.resize(pat, L)


def expected_wire(oracle_lib, sb):
    """protocol.cs:1665-1705 restated: range-compress each DGRAM's commands (limit =
    their length), keep the compressed form only when shorter (header flag 0x4000),
    stamp the CRC over the UNCOMPRESSED gather list, wire = first buffer + (compressed
    or original commands).  Returns (wire DGRAMs, expected payload after the call)."""
    import oracle
    g = sb.gather
    pay = g.payload.copy()
    cmds, offs, lens = [], [], []
    pos = 0
    for d in range(sb.n):
        segs = range(int(g.seg_first[d]) + 1, int(g.seg_first[d + 1]))
        c = b"".join(bytes(pay[int(g.seg_off[s]):int(g.seg_off[s]) + int(g.seg_len[s])]) for s in segs)
        cmds.append(c)
        offs.append(pos)
        lens.append(len(c))
        pos += len(c)
    data = np.frombuffer(b"".join(cmds) + b"\0" * 16, np.uint8)
    out, oo, ol = oracle.range_coder_batch(oracle_lib, False, data, np.array(offs, np.uint64),
                                           np.array(lens, np.uint32), np.array(lens, np.uint32))
    keep = (ol > 0) & (ol < np.array(lens, np.uint32))
    for d in np.nonzero(keep)[0]:
        pay[int(g.seg_off[int(g.seg_first[d])])] |= 0x40
    crc = oracle_lib.gather(pay, g.seg_off, g.seg_len, g.seg_first)
    wire = []
    for d in range(sb.n):
        s0 = int(g.seg_first[d])
        o = int(g.seg_off[s0])
        so = o + int(sb.slot_off[d])
        pay[so:so + 4] = np.frombuffer(np.uint32(crc[d]).tobytes(), np.uint8)
        first = bytes(pay[o:o + int(g.seg_len[s0])])
        body = bytes(out[int(oo[d]):int(oo[d]) + int(ol[d])]) if keep[d] else cmds[d]
        wire.append(first + body)
    return wire, pay, keep


def expected_receive(oracle_lib, dgrams, peers):
    """protocol.cs:1001-1068 restated for range-coded hosts: header stage, the
    decompression of flagged DGRAMs (limit 4096 - headerSize, 0 = drop), then the
    checksum verify over the (decompressed) DGRAM.  -> (keep, DGRAM as kept)."""
    import oracle
    keep, outs = [], []
    for dg in dgrams:
        k, res = 0, dg
        if len(dg) >= 2:
            word = (dg[0] << 8) | dg[1]
            peer, hs = word & 0x0FFF, (4 if word & 0x8000 else 2)
            if peer == 0xFFF or peer < len(peers):
                ok_size = len(dg) >= hs + 4
                if ok_size and word & 0x4000:
                    body = np.frombuffer(dg[hs + 4:] + b"\0" * 16, np.uint8)
                    out, oo, ol = oracle.range_coder_batch(oracle_lib, True, body, np.array([0], np.uint64),
                                                           np.array([len(dg) - hs - 4], np.uint32),
                                                           np.array([4096 - hs - 4], np.uint32))
                    ok_size = ol[0] > 0
                    if ok_size:
                        res = dg[:hs + 4] + bytes(out[:int(ol[0])])
                if ok_size:
                    conn = 0 if peer == 0xFFF else int(peers[peer])
                    desired = int.from_bytes(res[hs:hs + 4], "little")
                    k = int(oracle_lib.crc32(res[:hs] + np.uint32(conn).tobytes() + res[hs + 4:]) == desired)
        keep.append(k)
        outs.append(res)
    return np.array(keep, np.uint8), outs


@pytest.mark.parametrize("corrupt", [0, 40])
def test_gpu_compress_stamp_send_and_decompress_verify(ctx, oracle_lib, corrupt):  # noqa: F811
    """the GPU pipelines with ENet's range coder beside the checksum.
    enet_hip_udp_compress_stamp_send puts on the wire exactly the DGRAMs the
    reference would (compress where shorter, flag, CRC over the uncompressed list);
    enet_hip_udp_receive_decompress_verify keeps exactly the DGRAMs the reference
    keeps and leaves them decompressed in their slots with their new lengths --
    corrupted compressed bodies (decoder failures or CRC mismatches) included."""
    rng = np.random.default_rng(90 + corrupt)
    sb = workloads.send_batch(1200, seed=91 + corrupt)
    compressible(sb, rng)
    g = sb.gather
    wire, exp_pay, keep = expected_wire(oracle_lib, sb)
    assert 0 < keep.sum() < sb.n                               # both forms on the wire
    rx, tx, port = sockets()
    arena, p = pinned(STRIDE * 512)
    try:
        got = []
        for a in range(0, sb.n, 300):
            b = min(sb.n, a + 300)
            sent = ctx.udp_compress_stamp_send(tx.fileno(), g.payload, g.seg_off, g.seg_len, g.seg_first[a:b + 1],
                                               sb.slot_off[a:b], LOOPBACK, port)
            assert sent == b - a
            while len(got) < b:
                n, lens, _, _ = enethip.udp_receive(rx.fileno(), arena, STRIDE, 512, timeout_ms=2000)
                assert n > 0
                got.extend(bytes(arena[i * STRIDE:i * STRIDE + int(lens[i])]) for i in range(n))
        assert (g.payload == exp_pay).all()                    # header flags and slots as the reference's
        assert got == wire
        # the wire form back through the GPU receive pipeline (some bodies corrupted)
        dgrams = list(wire)
        for d in rng.choice(sb.n, corrupt, replace=False) if corrupt else []:
            b = bytearray(dgrams[d])
            hs = 4 if b[0] & 0x80 else 2
            if len(b) > hs + 5:
                b[int(rng.integers(hs + 4, len(b)))] ^= 0x10
            dgrams[d] = bytes(b)
        exp_keep, exp_out = expected_receive(oracle_lib, dgrams, sb.peers)
        oks, outs, lens_all = [], [], []
        for a in range(0, sb.n, 300):
            b = min(sb.n, a + 300)
            for dg in dgrams[a:b]:
                tx.sendto(dg, ("127.0.0.1", port))
            k = 0
            while k < b - a:
                n, lens, ok = ctx.udp_receive_decompress_verify(rx.fileno(), arena, STRIDE, 512, sb.peers,
                                                                timeout_ms=2000)
                assert n > 0
                oks.append(ok.copy())
                lens_all.append(lens.copy())
                outs.extend(bytes(arena[i * STRIDE:i * STRIDE + int(lens[i])]) for i in range(n))
                k += n
        ok = np.concatenate(oks)
        assert (ok == exp_keep).all(), np.nonzero(ok != exp_keep)[0][:10]
        if corrupt:
            assert 0 < int((ok == 0).sum()) <= corrupt
        else:
            assert ok.all()
        for i in np.nonzero(exp_keep)[0]:
            assert outs[i] == exp_out[i], i                    # decompressed in place, new length
    finally:
        free_pinned(p)
        rx.close()
        tx.close()


def test_gpu_receive_verify_submit_complete_two_slots(ctx, oracle_lib):  # noqa: F811
    """enet_hip_udp_receive_verify_submit / _complete: batches received into two arenas
    in turn, each one's GPU verify in flight while the next is received; every keep
    mask equal to the oracle's (header stage restated: expected_keep), corrupted and odd
    DGRAMs among them.  While slot 0 is in flight the synchronous receive (which runs as
    slot 0) refuses and the slot cannot be submitted twice; the send and batch host
    entries, which have staging of their own (round 6), run and are exact."""
    sb = workloads.send_batch(2400, seed=95)
    g = sb.gather
    rng = np.random.default_rng(96)
    rx, tx, port = sockets()
    arenas = [pinned(STRIDE * 512), pinned(STRIDE * 512)]
    try:
        # stamp on the CPU (the oracle), corrupt 60 DGRAMs, then send in bursts of 300
        stamps = oracle_stamps(oracle_lib, sb)
        pos = g.seg_off[g.seg_first[:-1]].astype(np.int64) + sb.slot_off.astype(np.int64)
        for d in range(sb.n):
            g.payload[pos[d]:pos[d] + 4] = np.frombuffer(np.uint32(stamps[d]).tobytes(), np.uint8)
        for d in rng.choice(sb.n, 60, replace=False):
            s = int(g.seg_first[d]) + int(rng.integers(0, 3))
            if g.seg_len[s]:
                g.payload[int(g.seg_off[s]) + int(rng.integers(0, int(g.seg_len[s])))] ^= np.uint8(4)
        pending = {}
        got = 0
        kept = 0
        bursts = list(range(0, sb.n, 300))
        for k, a in enumerate(bursts):
            b = min(sb.n, a + 300)
            assert enethip.udp_send(tx.fileno(), g.payload, g.seg_off, g.seg_len, g.seg_first[a:b + 1],
                                    LOOPBACK, port) == b - a
            if k == len(bursts) - 1:
                for dg in odd_dgrams(sb.peers):
                    tx.sendto(dg, ("127.0.0.1", port))
            slot = k & 1
            arena = arenas[slot][0]
            rows = 0
            while rows < b - a:
                if slot in pending:                               # the slot's previous batch first
                    arena_p, n_p, lens_p, ok_p = pending.pop(slot)
                    ctx.udp_receive_verify_complete(slot)
                    assert (ok_p == expected_keep(oracle_lib, arena_p, STRIDE, lens_p, sb.peers)).all()
                    kept += int(ok_p.sum())
                n, lens, ok = ctx.udp_receive_verify_submit(slot, rx.fileno(), arena, STRIDE, 512, sb.peers,
                                                            timeout_ms=2000)
                assert n > 0
                if slot == 0 and k == 0:                          # in flight: the others refuse
                    with pytest.raises(enethip.ENetHipError):
                        ctx.udp_receive_verify_submit(slot, rx.fileno(), arenas[1][0], STRIDE, 512, sb.peers)
                    with pytest.raises(enethip.ENetHipError):
                        ctx.udp_receive_verify(rx.fileno(), arenas[1][0], STRIDE, 512, sb.peers)
                    # the host batch and gather entries run beside the slot in flight
                    hb = workloads.fixed(300, 700, seed=98)
                    assert (ctx.crc32_batch_host(hb.payload, hb.off, hb.lens) ==
                            oracle_lib.batch(hb.payload, hb.off, hb.lens)).all()
                    assert (ctx.gather_binned_host(g.payload, g.seg_off, g.seg_len, g.seg_first[:101]) ==
                            oracle_lib.gather(g.payload, g.seg_off, g.seg_len, g.seg_first[:101])).all()
                pending[slot] = (arena, n, lens.copy(), ok)
                got += n
                rows += n
                if rows < b - a:                                  # more of this burst: complete now
                    arena_p, n_p, lens_p, ok_p = pending.pop(slot)
                    ctx.udp_receive_verify_complete(slot)
                    assert (ok_p == expected_keep(oracle_lib, arena_p, STRIDE, lens_p, sb.peers)).all()
                    kept += int(ok_p.sum())
        for slot, (arena_p, n_p, lens_p, ok_p) in list(pending.items()):
            ctx.udp_receive_verify_complete(slot)
            assert (ok_p == expected_keep(oracle_lib, arena_p, STRIDE, lens_p, sb.peers)).all()
            kept += int(ok_p.sum())
        # the odd DGRAMs may still be queued: drain them through slot 0
        while got < sb.n + len(odd_dgrams(sb.peers)):
            n, lens, ok = ctx.udp_receive_verify_submit(0, rx.fileno(), arenas[0][0], STRIDE, 512, sb.peers,
                                                        timeout_ms=2000)
            assert n > 0
            ctx.udp_receive_verify_complete(0)
            assert (ok == expected_keep(oracle_lib, arenas[0][0], STRIDE, lens, sb.peers)).all()
            kept += int(ok.sum())
            got += n
        assert got == sb.n + len(odd_dgrams(sb.peers))
        assert sb.n - 60 <= kept < sb.n                           # the corrupted ones dropped
    finally:
        for _, p in arenas:
            free_pinned(p)
        rx.close()
        tx.close()


def test_send_runs_while_receive_waits(ctx, oracle_lib):  # noqa: F811
    """a receive's socket wait holds no lock of the context.  One
    thread blocks in enet_hip_udp_receive_verify on an idle socket (3 s timeout); on the
    same context another thread's enet_hip_udp_stamp_send and host batch call finish
    while it still waits, with stamps equal to the oracle's; the receive then times out
    with nothing received."""
    sb = workloads.send_batch(400, seed=97)
    g = sb.gather
    exp = oracle_stamps(oracle_lib, sb)
    rx1, tx1, port1 = sockets()
    rx2, tx2, port2 = sockets()
    arena, p = pinned(STRIDE * 64)
    res = {}

    def waiter():
        t0 = time.perf_counter()
        try:
            res["rx"] = ctx.udp_receive_verify(rx1.fileno(), arena, STRIDE, 64, sb.peers, timeout_ms=3000)
        except Exception as e:                                   # (reported by the main thread)
            res["err"] = e
        res["secs"] = time.perf_counter() - t0

    th = threading.Thread(target=waiter)
    try:
        th.start()
        time.sleep(0.3)                                          # the waiter is in its socket wait
        t0 = time.perf_counter()
        sent = ctx.udp_stamp_send(tx2.fileno(), g.payload, g.seg_off, g.seg_len, g.seg_first, sb.slot_off,
                                  LOOPBACK, port2)
        hb = workloads.fixed(200, 900, seed=99)
        crcs = ctx.crc32_batch_host(hb.payload, hb.off, hb.lens)
        dt = time.perf_counter() - t0
        assert th.is_alive(), "the receive returned before the sends ran"
        assert dt < 1.5, dt                                      # not held behind the 3-s wait
        assert sent == sb.n
        assert (slots_of(sb) == exp).all()
        assert (crcs == oracle_lib.batch(hb.payload, hb.off, hb.lens)).all()
        th.join(10)
        assert not th.is_alive()
        assert "err" not in res, res.get("err")
        assert res["rx"][0] == 0 and res["secs"] >= 2.5          # timed out, nothing received
    finally:
        th.join(10)
        free_pinned(p)
        for s_ in (rx1, tx1, rx2, tx2):
            s_.close()


def test_in_place_arenas_ending_on_a_page(ctx, oracle_lib):  # noqa: F811
    """the in-place paths on pinned arenas whose size is a whole number
    of pages, with packets and segments that end exactly on the arena's last byte (ragged
    and 16-byte-aligned ends, unaligned starts), so an over-read by a whole 16-B granule
    would leave the allocation instead of landing in the page's slack.  Batch and gather
    host entries against the oracle; the receive case is
    test_receive_verify_dgram_ending_on_the_arena."""
    rng = np.random.default_rng(100)
    for n in (1 << 20, 4 << 20):                                # (both at most the 4-MiB in-place span)
        arr, p = pinned(n)
        try:
            arr[:] = rng.integers(0, 256, size=n, dtype=np.uint8)
            tails = np.array([1, 2, 15, 16, 17, 31, 32, 33, 63, 64, 65, 255, 1199, 1200, 1399, 4096], np.uint32)
            k = 600
            lens = np.concatenate([tails, rng.integers(0, 1500, size=k).astype(np.uint32)])
            off = np.concatenate([n - tails.astype(np.uint64),
                                  rng.integers(0, n - 1500, size=k).astype(np.uint64)])
            assert (ctx.crc32_batch_host(arr, off, lens) == oracle_lib.batch(arr, off, lens)).all(), n
            # one packet alone, ending on the last byte (the smallest launch)
            for t in (3, 16, 1201):
                o1, l1 = np.array([n - t], np.uint64), np.array([t], np.uint32)
                assert (ctx.crc32_batch_host(arr, o1, l1) == oracle_lib.batch(arr, o1, l1)).all(), (n, t)
            # gather lists whose LAST segments end on the last byte
            cnt = rng.integers(1, 6, size=200)
            sf = np.zeros(201, np.uint32)
            np.cumsum(cnt, out=sf[1:])
            ns = int(sf[-1])
            sl = rng.integers(0, 1400, size=ns).astype(np.uint32)
            so = rng.integers(0, n - 1400, size=ns).astype(np.uint64)
            last = sf[1:] - 1
            sl[last[:16]] = tails
            so[last[:16]] = n - tails.astype(np.uint64)
            assert (ctx.gather_binned_host(arr, so, sl, sf) == oracle_lib.gather(arr, so, sl, sf)).all(), n
        finally:
            free_pinned(p)


def test_receive_verify_dgram_ending_on_the_arena(ctx, oracle_lib):  # noqa: F811
    """The in-place receive verify on a pinned arena of exactly 8 receive slots (32 KiB,
    page-multiple): the 8th DGRAM fills its 4096-B slot, so it ends on the arena's last
    byte; ragged lengths before it.  Keep mask against the oracle (expected_keep)."""
    rng = np.random.default_rng(101)
    rx, tx, port = sockets()
    arena, p = pinned(STRIDE * 8)
    try:
        lens = [17, 100, 1201, 1399, 33, 4095, 2049, STRIDE]
        for L in lens:
            body = bytearray(rng.integers(0, 256, size=L, dtype=np.uint8).tobytes())
            body[0:2] = (0x0FFF).to_bytes(2, "big")               # no peer: connectID 0 in the slot
            body[2:6] = b"\0\0\0\0"
            body[2:6] = int(oracle_lib.crc32(bytes(body))).to_bytes(4, "little")
            tx.sendto(bytes(body), ("127.0.0.1", port))
        # (loopback queues all 8 before the call: one recvmmsg takes them in order, the
        # full one into slot 7)
        n, ln, ok = ctx.udp_receive_verify(rx.fileno(), arena, STRIDE, 8, [], timeout_ms=2000)
        assert n == len(lens)
        assert list(ln) == lens
        assert (ok == expected_keep(oracle_lib, arena, STRIDE, ln, [])).all()
        assert ok.all()
    finally:
        free_pinned(p)
        rx.close()
        tx.close()


def _enet_dgram(oracle_lib, rng, L, peer, sent_time, conn):
    """An ENet DGRAM of L bytes as a host sends it: big-endian peer word (SENT_TIME flag:
    a 4-byte header), checksum slot after the header holding the CRC taken with the slot
    set to the peer's connectID (protocol.cs:1690-1698)."""
    hs = 4 if sent_time else 2
    b = bytearray(rng.integers(0, 256, size=L, dtype=np.uint8).tobytes())
    b[0:2] = ((peer & 0x0FFF) | (0x8000 if sent_time else 0)).to_bytes(2, "big")
    b[hs:hs + 4] = int(conn).to_bytes(4, "little")
    b[hs:hs + 4] = int(oracle_lib.crc32(bytes(b))).to_bytes(4, "little")
    return bytes(b)


def test_receive_verify_every_length(ctx, oracle_lib):  # noqa: F811
    """The receive verify of ENet-sized calls (at most 256 DGRAMs, read in place from a
    pinned arena) over every DGRAM length 6..4096, both header sizes (SENT_TIME or not),
    peers with connectIDs and peer 0xFFF, one DGRAM in nine corrupted in one byte: keep mask
    equal to the oracle's (expected_keep restates the header stage) in every call, and every
    intact DGRAM kept."""
    rng = np.random.default_rng(102)
    peers = rng.integers(1, 1 << 32, size=5, dtype=np.uint64).astype(np.uint32)
    dgrams, intact = [], []
    for L in range(6, STRIDE + 1):
        for sent_time in ((False, True) if L >= 8 else (False,)):
            if (L + sent_time) % 3:                              # (two thirds of the pairs: ~5400 DGRAMs)
                continue
            p = int(rng.integers(0, 6))
            peer = 0x0FFF if p == 5 else p
            dg = bytearray(_enet_dgram(oracle_lib, rng, L, peer, sent_time, 0 if peer == 0x0FFF else peers[peer]))
            bad = rng.random() < 1 / 9
            if bad:
                k = int(rng.integers(2, L))
                dg[k] ^= 1 << int(rng.integers(0, 8))
            dgrams.append(bytes(dg))
            intact.append(not bad)
    rx, tx, port = sockets()
    arena, p = pinned(STRIDE * 256)
    try:
        got, keep_all = 0, []
        for a in range(0, len(dgrams), 256):
            part = dgrams[a:a + 256]
            for dg in part:
                tx.sendto(dg, ("127.0.0.1", port))
            k = 0
            while k < len(part):
                n, lens, ok = ctx.udp_receive_verify(rx.fileno(), arena, STRIDE, 256, peers, timeout_ms=2000)
                assert n > 0
                exp = expected_keep(oracle_lib, arena, STRIDE, lens, peers)
                assert (ok == exp).all(), (a, k, np.nonzero(ok != exp)[0][:10], lens[np.nonzero(ok != exp)[0][:10]])
                keep_all.append(ok.copy())
                k += n
            got += k
        keep = np.concatenate(keep_all)
        assert got == len(dgrams)
        assert keep.sum() == sum(intact)                        # (corrupting a peer word may drop it too)
    finally:
        free_pinned(p)
        rx.close()
        tx.close()
