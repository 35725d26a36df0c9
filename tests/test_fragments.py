"""Fragment reassembly oracle (c/protocol.cs:529-637) on CPU: the C restatement
against a pure-Python restatement of the same handler, the split/reassemble round
trip (c/peer.cs:130-196 then protocol.cs:566-634 recovers every message), the -1
paths and duplicates within and across batches.  No GPU."""
import numpy as np
import pytest

import oracle
from enethip import workloads

MAXP = 32 * 1024 * 1024          # ENET_HOST_DEFAULT_MAXIMUM_PACKET_SIZE (include/enet.cs)


def state(fb, words=None):
    words = words or int(max(1, (int(fb.msg_count.max()) + 31) // 32))
    msg_off = np.concatenate([[0], np.cumsum(fb.msg_len.astype(np.uint64))[:-1]]).astype(np.uint64)
    msg_bytes = np.zeros(int(fb.msg_len.astype(np.uint64).sum()) + 16, dtype=np.uint8)
    frags = np.zeros(len(fb.msg_len) * words, dtype=np.uint32)
    remaining = fb.msg_count.copy()
    return dict(msg_off=msg_off, msg_bytes=msg_bytes, fragments=frags, remaining=remaining, words=words)


def run_oracle(lib, fb, st, sel=None, payload=None):
    sel = np.arange(fb.n) if sel is None else sel
    return oracle.fragment_reassemble(lib, fb.payload if payload is None else payload, fb.cmd_off[sel],
                                      fb.cmd_avail[sel], fb.slots[sel], MAXP, st["msg_bytes"], st["msg_off"],
                                      fb.msg_len, fb.msg_count, st["fragments"], st["words"], st["remaining"])


def py_reassemble(payload, cmd_off, cmd_avail, slots, msg_len, msg_count, msg_off, msg_bytes, frags, words, remaining):
    """Pure-Python restatement of protocol.cs:546-552, 566-634 (small cases)."""
    status = []
    for i in range(len(cmd_off)):
        s = int(slots[i])
        if s < 0:
            status.append(0)
            continue
        c = bytes(payload[int(cmd_off[i]):int(cmd_off[i]) + 24])
        flen = int.from_bytes(c[6:8], "big")
        cnt, num, tot, off = (int.from_bytes(c[k:k + 4], "big") for k in (8, 12, 16, 20))
        if flen == 0 or flen > MAXP or flen > int(cmd_avail[i]):
            status.append(-1)
            continue
        if cnt > 1 << 20 or num >= cnt or tot > MAXP or tot < cnt or off >= tot or flen > tot - off:
            status.append(-1)
            continue
        if tot != int(msg_len[s]) or cnt != int(msg_count[s]) or cnt > 32 * words:
            status.append(-1)
            continue
        w = s * words + num // 32
        if frags[w] & (1 << (num % 32)):
            status.append(0)
            continue
        remaining[s] -= 1
        frags[w] |= 1 << (num % 32)
        flen = min(flen, int(msg_len[s]) - off)
        a = int(msg_off[s]) + off
        src = int(cmd_off[i]) + 24
        msg_bytes[a:a + flen] = payload[src:src + flen]
        status.append(1)
    return np.array(status, dtype=np.int8)


def test_round_trip_with_duplicates(oracle_lib):
    rng = np.random.default_rng(3)
    lens = rng.integers(1, 40000, 60)
    fb = workloads.fragments(lens, seed=11, duplicates=0.2)
    st = state(fb)
    status = run_oracle(oracle_lib, fb, st)
    assert (status >= 0).all()
    assert int((status == 1).sum()) == int(fb.msg_count.sum())            # each fragment copied once
    assert (st["remaining"] == 0).all()                                   # every message completed (632)
    for m, msg in enumerate(fb.messages):
        a = int(st["msg_off"][m])
        assert (st["msg_bytes"][a:a + len(msg)] == msg).all()


def test_c_oracle_matches_python_restatement(oracle_lib):
    rng = np.random.default_rng(5)
    fb = workloads.fragments(rng.integers(1, 9000, 25), seed=12, duplicates=0.3)
    # corrupt some commands into each -1 path, and skip some
    p = fb.payload.copy()
    bad = rng.choice(fb.n, 12, replace=False)
    for j, i in enumerate(bad):
        o = int(fb.cmd_off[i])
        kind = j % 6
        if kind == 0:
            p[o + 6:o + 8] = 0                                                   # dataLength 0
        elif kind == 1:
            p[o + 12:o + 16] = np.frombuffer((1 << 21).to_bytes(4, "big"), np.uint8)   # fragmentNumber >= count
        elif kind == 2:
            p[o + 20:o + 24] = np.frombuffer((10 ** 6).to_bytes(4, "big"), np.uint8)   # offset >= total
        elif kind == 3:
            p[o + 16:o + 20] = np.frombuffer((10 ** 5).to_bytes(4, "big"), np.uint8)   # total != slot's length
        elif kind == 4:
            p[o + 6:o + 8] = np.frombuffer((4000).to_bytes(2, "big"), np.uint8)       # longer than the DGRAM
        else:
            fb.slots[i] = -1                                                     # skipped by the caller
    st = state(fb)
    got = run_oracle(oracle_lib, fb, st, payload=p)
    st2 = state(fb)
    exp = py_reassemble(p, fb.cmd_off, fb.cmd_avail, fb.slots, fb.msg_len, fb.msg_count, st2["msg_off"],
                        st2["msg_bytes"], st2["fragments"], st2["words"], st2["remaining"])
    assert (got == exp).all()
    assert (got == -1).sum() >= 8
    for k in ("msg_bytes", "fragments", "remaining"):
        assert (st[k] == st2[k]).all(), k


def test_two_batches_equal_one(oracle_lib):
    fb = workloads.fragments([70000, 5, 1360, 1361, 2720], seed=13, duplicates=0.5)
    one = state(fb)
    s1 = run_oracle(oracle_lib, fb, one)
    two = state(fb)
    h = fb.n // 2
    s2 = np.concatenate([run_oracle(oracle_lib, fb, two, np.arange(h)), run_oracle(oracle_lib, fb, two, np.arange(h, fb.n))])
    assert (s1 == s2).all()
    for k in ("msg_bytes", "fragments", "remaining"):
        assert (one[k] == two[k]).all(), k


def test_split_sizes_follow_peer_cs():
    """c/peer.cs:130-136: 1360-byte fragments at mtu 1392 with checksums; a 64 KiB
    message -> 49 fragments, the last 256 bytes."""
    fb = workloads.fragments([65536], shuffle=False)
    assert fb.n == 49 and int(fb.msg_count[0]) == 49
    assert int(fb.cmd_avail[0]) == 1360 and int(fb.cmd_avail[-1]) == 256


def test_oracle_overlapping_fragments_match_python(oracle_lib):
    """The C oracle on overlapping fragment ranges equals the pure-Python handler:
    later commands' bytes win where ranges overlap (protocol.cs:619-630)."""
    fb = workloads.overlapping_fragments(40, seed=41)
    so, sp = state(fb), state(fb)
    st = run_oracle(oracle_lib, fb, so)
    sp_status = py_reassemble(fb.payload, fb.cmd_off, fb.cmd_avail, fb.slots, fb.msg_len, fb.msg_count,
                              sp["msg_off"], sp["msg_bytes"], sp["fragments"], sp["words"], sp["remaining"])
    assert list(st) == list(sp_status)
    assert (so["msg_bytes"] == sp["msg_bytes"]).all()
    assert (st == 1).sum() > 0
