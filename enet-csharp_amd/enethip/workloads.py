"""Synthetic batches for the BASELINE.json configs.

Payload bytes are splitmix64 output, 8 little-endian bytes per draw; every
generator is deterministic in its seed.  These are inputs only -- expected CRCs
always come from the oracle (oracle/), never from here.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

GOLDEN = np.uint64(0x9E3779B97F4A7C15)
SEED_PAYLOAD = 0x454E6574   # "ENet"   
SEED_LENGTHS = 0x4C454E53   # "LENS"   
CONNECT_ID = 0x1234ABCD     # cfg5 slot value


def splitmix64(seed: int, count: int, start: int = 0) -> np.ndarray:
    """Draws start+1 .. start+count of splitmix64(seed) (vectorised, uint64 wraparound)."""
    with np.errstate(over="ignore"):
        i = np.arange(start + 1, start + count + 1, dtype=np.uint64)
        z = np.uint64(seed) + i * GOLDEN
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def payload_bytes(nbytes: int, seed: int = SEED_PAYLOAD) -> np.ndarray:
    words = splitmix64(seed, (nbytes + 7) // 8)
    return words.view(np.uint8)[:nbytes].copy()


@dataclass
class Batch:
    payload: np.ndarray   # uint8, packed
    off: np.ndarray       # uint64
    lens: np.ndarray      # uint32
    name: str

    @property
    def n(self) -> int:
        return len(self.off)

    @property
    def payload_bytes(self) -> int:
        return int(self.lens.astype(np.uint64).sum())


def fixed(n: int, length: int, seed: int = SEED_PAYLOAD, name: str = "") -> Batch:
    lens = np.full(n, length, dtype=np.uint32)
    off = np.arange(n, dtype=np.uint64) * np.uint64(length)
    return Batch(payload_bytes(n * length, seed), off, lens, name or f"{n}x{length}B")


def mixed(n: int, lo: int = 64, hi: int = 1400, seed: int = SEED_PAYLOAD, len_seed: int = SEED_LENGTHS,
          name: str = "") -> Batch:
    """Lengths uniform in [lo, hi], packed back to back (arbitrary byte alignment)."""
    lens = (np.uint64(lo) + splitmix64(len_seed, n) % np.uint64(hi - lo + 1)).astype(np.uint32)
    off = np.zeros(n, dtype=np.uint64)
    np.cumsum(lens[:-1], out=off[1:])
    return Batch(payload_bytes(int(lens.astype(np.uint64).sum()), seed), off, lens,
                 name or f"{n}x[{lo},{hi}]B")


def cfg2() -> Batch:
    """64 K packets x 1200 B (MTU-sized), packed: the headline config."""
    return fixed(65536, 1200, name="cfg2: 65536 x 1200 B")


def cfg3() -> Batch:
    """256 K packets, lengths uniform in [64, 1400]."""
    return mixed(262144, 64, 1400, name="cfg3: 262144 x U[64,1400] B")


def cfg4(shard: int = 0, shards: int = 1) -> Batch:
    """1 M packets x 1200 B; shard i of k = contiguous packet range."""
    n = 1 << 20
    lo, hi = n * shard // shards, n * (shard + 1) // shards
    length = 1200
    words_lo = lo * length // 8
    nbytes = (hi - lo) * length
    words = splitmix64(SEED_PAYLOAD, (nbytes + 7) // 8, start=words_lo)
    payload = words.view(np.uint8)[:nbytes].copy()
    lens = np.full(hi - lo, length, dtype=np.uint32)
    off = np.arange(hi - lo, dtype=np.uint64) * np.uint64(length)
    return Batch(payload, off, lens, f"cfg4: 1048576 x 1200 B shard {shard}/{shards}")


@dataclass
class GatherBatch:
    """DGRAMs as gather lists: [8 B header+slot][24 B SendFragment][payload chunk]."""
    payload: np.ndarray
    seg_off: np.ndarray    # uint64
    seg_len: np.ndarray    # uint32
    seg_first: np.ndarray  # uint32, n_dgrams + 1
    dgram_bytes: int
    name: str

    @property
    def n(self) -> int:
        return len(self.seg_first) - 1


def cfg5(messages: int = 4096, message_bytes: int = 65536, mtu: int = 1392) -> GatherBatch:
    """Fragmented reliable sends (c/peer.cs:130-132, 161-196): fragment = mtu - 4 - 24 - 4
    = 1360 B with checksums on; a 64 KiB message -> 48 x 1360 + 256.  Each DGRAM is a
    3-buffer gather list: [4 B header w/ sentTime][4 B slot = connectID][24 B cmd][chunk]."""
    frag = mtu - 4 - 24 - 4
    per_msg = (message_bytes + frag - 1) // frag
    n = messages * per_msg
    hdr_bytes = n * 8
    cmd_bytes = n * 24
    body_bytes = messages * message_bytes
    payload = payload_bytes(hdr_bytes + cmd_bytes + body_bytes)
    hdr = payload[:hdr_bytes].reshape(n, 8)
    hdr[:, 4:8] = np.frombuffer(np.uint32(CONNECT_ID).tobytes(), dtype=np.uint8)
    seg_off = np.zeros(3 * n, dtype=np.uint64)
    seg_len = np.zeros(3 * n, dtype=np.uint32)
    d = np.arange(n, dtype=np.uint64)
    msg = d // np.uint64(per_msg)
    k = d % np.uint64(per_msg)
    chunk_off = np.uint64(hdr_bytes + cmd_bytes) + msg * np.uint64(message_bytes) + k * np.uint64(frag)
    chunk_len = np.minimum(np.uint64(frag), np.uint64(message_bytes) - k * np.uint64(frag))
    seg_off[0::3] = d * np.uint64(8)
    seg_len[0::3] = 8
    seg_off[1::3] = np.uint64(hdr_bytes) + d * np.uint64(24)
    seg_len[1::3] = 24
    seg_off[2::3] = chunk_off
    seg_len[2::3] = chunk_len.astype(np.uint32)
    seg_first = (np.arange(n + 1, dtype=np.uint64) * np.uint64(3)).astype(np.uint32)
    total = int(seg_len.astype(np.uint64).sum())
    return GatherBatch(payload, seg_off, seg_len, seg_first, total,
                       f"cfg5: {messages} x {message_bytes} B -> {n} DGRAMs")


@dataclass
class FragmentBatch:
    """Received SEND_FRAGMENT DGRAMs ready for reassembly: DGRAM = [4 B header]
    [4 B checksum slot][24 B ENetProtocolSendFragment, network order][data].
    cmd_off[i] points at the command, cmd_avail[i] = data bytes after it, slots[i]
    = the message (reassembly slot) it belongs to.  msg_len / msg_count describe
    the slots; `messages` holds the original message bytes (the round-trip check)."""
    payload: np.ndarray
    cmd_off: np.ndarray     # uint64
    cmd_avail: np.ndarray   # uint32
    slots: np.ndarray       # int32
    msg_len: np.ndarray     # uint32
    msg_count: np.ndarray   # uint32
    messages: list
    data_bytes: int
    name: str

    @property
    def n(self) -> int:
        return len(self.cmd_off)


def send_fragment_cmd(count: int, number: int, total: int, offset: int, length: int, seq: int = 1) -> bytes:
    """include/protocol.cs:156-165 as c/peer.cs:183-193 fills it (network order)."""
    hdr = bytes([0x80 | 8, 0]) + (seq & 0xFFFF).to_bytes(2, "big")    # SEND_FRAGMENT | ACKNOWLEDGE, channel 0
    return (hdr + (seq & 0xFFFF).to_bytes(2, "big") + length.to_bytes(2, "big") + count.to_bytes(4, "big") +
            number.to_bytes(4, "big") + total.to_bytes(4, "big") + offset.to_bytes(4, "big"))


def fragments(message_lens, mtu: int = 1392, seed: int = SEED_PAYLOAD, shuffle: bool = True,
              duplicates: float = 0.0, name: str = "fragments") -> FragmentBatch:
    """Split messages as c/peer.cs:130-196 does (fragmentLength = mtu - 4 - 24 - 4 with
    checksums on, the last fragment shorter), one DGRAM per fragment, in shuffled
    arrival order, with a fraction of retransmitted duplicates."""
    frag = mtu - 4 - 24 - 4
    rng = np.random.default_rng(seed)
    lens = [int(x) for x in message_lens]
    total_data = sum(lens)
    body = payload_bytes(total_data, seed=seed)
    messages, pieces = [], []
    pos = 0
    for m, L in enumerate(lens):
        messages.append(body[pos:pos + L])
        cnt = (L + frag - 1) // frag
        for k in range(cnt):
            off = k * frag
            pieces.append((m, cnt, k, L, off, min(frag, L - off), pos + off))
        pos += L
    order = rng.permutation(len(pieces)) if shuffle else np.arange(len(pieces))
    order = list(order)
    ndup = int(duplicates * len(pieces))
    if ndup:
        dup = rng.choice(len(pieces), ndup, replace=True)
        for d in dup:
            order.insert(int(rng.integers(0, len(order) + 1)), int(d))
    n = len(order)
    sizes = np.array([32 + pieces[i][5] for i in order], dtype=np.uint64)
    starts = np.concatenate([[0], np.cumsum(sizes)[:-1]]).astype(np.uint64)
    arena = np.zeros(int(sizes.sum()) + 64, dtype=np.uint8)
    cmd_off = starts + np.uint64(8)
    cmd_avail = np.zeros(n, dtype=np.uint32)
    slots = np.zeros(n, dtype=np.int32)
    for i, pi in enumerate(order):
        m, cnt, k, L, off, ln, src = pieces[pi]
        a = int(starts[i])
        arena[a + 4:a + 8] = np.frombuffer(np.uint32(CONNECT_ID).tobytes(), dtype=np.uint8)
        arena[a + 8:a + 32] = np.frombuffer(send_fragment_cmd(cnt, k, L, off, ln), dtype=np.uint8)
        arena[a + 32:a + 32 + ln] = body[src:src + ln]
        cmd_avail[i] = ln
        slots[i] = m
    msg_count = np.array([(L + frag - 1) // frag for L in lens], dtype=np.uint32)
    return FragmentBatch(arena, cmd_off, cmd_avail, slots, np.array(lens, dtype=np.uint32), msg_count, messages,
                         total_data, name)


def cfg5_fragments(messages: int = 4096, message_bytes: int = 65536) -> FragmentBatch:
    """cfg5's 4096 x 64 KiB messages as received fragment DGRAMs (200 704 commands)."""
    return fragments([message_bytes] * messages, shuffle=True, name=f"cfg5 receive: {messages} x {message_bytes} B")


def overlapping_fragments(messages: int, seed: int = SEED_PAYLOAD, max_count: int = 12,
                          name: str = "overlapping fragments") -> FragmentBatch:
    """SEND_FRAGMENT commands a non-standard peer could send: per message, fragment
    numbers 0..count-1 (plus a few repeats) with arbitrary offsets and lengths, so
    byte ranges overlap in any order and every command carries different bytes.  The
    reference copies in arrival order (c/protocol.cs:619-630): where ranges overlap,
    the later command's bytes win."""
    rng = np.random.default_rng(seed)
    cmds = []                      # (slot, count, number, total, offset, length)
    lens, counts = [], []
    for m in range(messages):
        L = int(rng.integers(64, 6000))
        cnt = int(rng.integers(2, max_count + 1))
        lens.append(L)
        counts.append(cnt)
        numbers = list(range(cnt)) + [int(x) for x in rng.integers(0, cnt, int(rng.integers(0, 3)))]
        for k in numbers:
            off = int(rng.integers(0, L))
            ln = int(rng.integers(1, min(1360, L - off) + 1))
            cmds.append((m, cnt, k, L, off, ln))
    order = rng.permutation(len(cmds))
    n = len(cmds)
    sizes = np.array([32 + cmds[i][5] for i in order], dtype=np.uint64)
    starts = np.concatenate([[0], np.cumsum(sizes)[:-1]]).astype(np.uint64)
    arena = rng.integers(0, 256, int(sizes.sum()) + 64, dtype=np.uint8)
    cmd_off = starts + np.uint64(8)
    cmd_avail = np.zeros(n, dtype=np.uint32)
    slots = np.zeros(n, dtype=np.int32)
    for i, ci in enumerate(order):
        m, cnt, k, L, off, ln = cmds[ci]
        a = int(starts[i])
        arena[a + 8:a + 32] = np.frombuffer(send_fragment_cmd(cnt, k, L, off, ln), dtype=np.uint8)
        cmd_avail[i] = ln
        slots[i] = m
    return FragmentBatch(arena, cmd_off, cmd_avail, slots, np.array(lens, dtype=np.uint32),
                         np.array(counts, dtype=np.uint32), [], 0, name)


@dataclass
class SendBatch:
    """DGRAMs as an ENet host sends them with a checksum (c/protocol.cs:1640-1698): a
    gather list of [ENetProtocolHeader: peerID | flags | session (big endian), sentTime
    if SENT_TIME][4-B checksum slot = the peer's connectID, or 0 for peerID 0xFFF]
    [12-B command][body].  peers[p] = connectID of outgoing peer p (the receiver's
    table for incoming peer p); slot_off[d] = the slot's offset in DGRAM d's first
    buffer; seq[d] = a 4-byte sequence number at the start of the command."""
    gather: GatherBatch
    slot_off: np.ndarray   # uint32
    peer: np.ndarray       # uint32 (0xFFF = no peer)
    peers: np.ndarray      # uint32 connectIDs

    @property
    def n(self) -> int:
        return self.gather.n


def send_batch(n: int, n_peers: int = 7, body: tuple = (0, 1360), seed: int = SEED_PAYLOAD) -> SendBatch:
    rng = np.random.default_rng(seed)
    peers = rng.integers(1, 2**32, size=n_peers, dtype=np.uint64).astype(np.uint32)
    peer = rng.integers(0, n_peers + 1, size=n).astype(np.uint32)
    peer[peer == n_peers] = 0xFFF                           # connect requests: no peer yet
    sent_time = rng.integers(0, 2, size=n).astype(bool)
    hdr_len = np.where(sent_time, 8, 6).astype(np.uint32)   # header (2 or 4 B) + 4-B slot
    body_len = rng.integers(body[0], body[1] + 1, size=n).astype(np.uint32)
    hdr_off = np.zeros(n, np.uint64)
    np.cumsum(np.full(n, 8, np.uint64)[:-1], out=hdr_off[1:])
    cmd_base = np.uint64(8 * n)
    body_base = cmd_base + np.uint64(12 * n)
    body_off = body_base + np.concatenate([[0], np.cumsum(body_len.astype(np.uint64))[:-1]]).astype(np.uint64)
    payload = payload_bytes(int(body_base) + int(body_len.astype(np.uint64).sum()) + 16, seed)
    session = rng.integers(0, 4, size=n).astype(np.uint32)
    word = (peer | (sent_time.astype(np.uint32) << 15) | np.where(peer == 0xFFF, 0, session << 12)).astype(np.uint32)
    for d in range(n):
        o = int(hdr_off[d])
        payload[o:o + 2] = np.frombuffer(int(word[d]).to_bytes(2, "big"), np.uint8)
        s = o + int(hdr_len[d]) - 4
        cid = 0 if peer[d] == 0xFFF else int(peers[peer[d]])
        payload[s:s + 4] = np.frombuffer(np.uint32(cid).tobytes(), np.uint8)
        c = int(cmd_base) + 12 * d
        payload[c:c + 4] = np.frombuffer(np.uint32(d).tobytes(), np.uint8)   # sequence number
    seg_off = np.zeros(3 * n, np.uint64)
    seg_len = np.zeros(3 * n, np.uint32)
    seg_off[0::3], seg_len[0::3] = hdr_off, hdr_len
    seg_off[1::3], seg_len[1::3] = cmd_base + np.arange(n, dtype=np.uint64) * np.uint64(12), 12
    seg_off[2::3], seg_len[2::3] = body_off, body_len
    first = (np.arange(n + 1, dtype=np.uint64) * np.uint64(3)).astype(np.uint32)
    g = GatherBatch(payload, seg_off, seg_len, first, int(seg_len.astype(np.uint64).sum()),
                    f"send batch: {n} DGRAMs")
    return SendBatch(g, (hdr_len - 4).astype(np.uint32), peer, peers)
