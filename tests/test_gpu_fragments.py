"""GPU parity of enet_hip_fragment_reassemble_device (c/protocol.cs:529-637)
against the sequential oracle: status, reassembled bytes, bitmaps and
fragmentsRemaining bit-exact, with duplicates inside and across batches and every
-1 path; plus the cfg5-sized round trip (200 704 fragments)."""
import numpy as np
import pytest

import oracle
from enethip import workloads
from test_fragments import MAXP, run_oracle, state
from test_gpu_parity import ctx, dev  # noqa: F401  (fixture)

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


def dev_i32(a):
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.int32)).cuda()


def run_gpu(ctx, fb, st, sel=None, payload=None):  # noqa: F811
    sel = np.arange(fb.n) if sel is None else sel
    p = fb.payload if payload is None else payload
    d = dict(msg_bytes=dev(st["msg_bytes"]), fragments=dev(st["fragments"]), remaining=dev(st["remaining"]))
    status = torch.zeros(len(sel), dtype=torch.int8, device="cuda")
    ctx.fragment_reassemble_device(dev(p), dev(fb.cmd_off[sel]), dev(fb.cmd_avail[sel]), dev_i32(fb.slots[sel]),
                                   len(sel), MAXP, d["msg_bytes"], dev(st["msg_off"]), dev(fb.msg_len),
                                   dev(fb.msg_count), d["fragments"], st["words"], d["remaining"], len(fb.msg_len),
                                   status, stream=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    st["msg_bytes"] = d["msg_bytes"].cpu().numpy().view(np.uint8).copy()
    st["fragments"] = d["fragments"].cpu().numpy().view(np.uint32).copy()
    st["remaining"] = d["remaining"].cpu().numpy().view(np.uint32).copy()
    return status.cpu().numpy()


def corrupt(fb, rng, k=40):
    p = fb.payload.copy()
    for j, i in enumerate(rng.choice(fb.n, k, replace=False)):
        o = int(fb.cmd_off[i])
        kind = j % 6
        if kind == 0:
            p[o + 6:o + 8] = 0
        elif kind == 1:
            p[o + 12:o + 16] = np.frombuffer((1 << 21).to_bytes(4, "big"), np.uint8)
        elif kind == 2:
            p[o + 20:o + 24] = np.frombuffer((10 ** 6).to_bytes(4, "big"), np.uint8)
        elif kind == 3:
            p[o + 16:o + 20] = np.frombuffer((10 ** 5).to_bytes(4, "big"), np.uint8)
        elif kind == 4:
            p[o + 6:o + 8] = np.frombuffer((4000).to_bytes(2, "big"), np.uint8)
        else:
            fb.slots[i] = -1
    return p


@pytest.mark.parametrize("dups", [0.0, 0.5])
def test_fragments_match_oracle(ctx, oracle_lib, dups):  # noqa: F811
    rng = np.random.default_rng(21)
    fb = workloads.fragments(rng.integers(1, 80000, 300), seed=22, duplicates=dups)
    p = corrupt(fb, rng)
    so, sg = state(fb), state(fb)
    exp = run_oracle(oracle_lib, fb, so, payload=p)
    got = run_gpu(ctx, fb, sg, payload=p)
    assert (got == exp).all()
    for k in ("msg_bytes", "fragments", "remaining"):
        assert (so[k] == sg[k]).all(), k


def test_fragments_across_batches(ctx, oracle_lib):  # noqa: F811
    rng = np.random.default_rng(23)
    fb = workloads.fragments(rng.integers(1, 30000, 100), seed=24, duplicates=0.7)
    so, sg = state(fb), state(fb)
    cuts = [0, fb.n // 3, fb.n // 2, fb.n]
    for a, b in zip(cuts[:-1], cuts[1:]):
        sel = np.arange(a, b)
        assert (run_gpu(ctx, fb, sg, sel) == run_oracle(oracle_lib, fb, so, sel)).all()
    for k in ("msg_bytes", "fragments", "remaining"):
        assert (so[k] == sg[k]).all(), k
    assert (sg["remaining"] == 0).all()


def test_cfg5_round_trip(ctx):  # noqa: F811
    fb = workloads.cfg5_fragments(1024)            # 1024 x 64 KiB = 50 176 fragments
    st = state(fb)
    status = run_gpu(ctx, fb, st)
    assert (status == 1).all() and (st["remaining"] == 0).all()
    body = np.concatenate(fb.messages)
    assert (st["msg_bytes"][:len(body)] == body).all()


@pytest.mark.parametrize("words", [None, 64])
def test_fragments_both_decide_paths(ctx, oracle_lib, words):  # noqa: F811
    """Small batches against a large claim space (slots x bitmap bits > 8 n + 65536) take
    the atomic decide kernel; dense ones the slot-owned, atomic-free one.  Both must equal
    the sequential reference, duplicates and earlier batches included."""
    rng = np.random.default_rng(29)
    fb = workloads.fragments(rng.integers(1, 60000, 400), seed=30, duplicates=0.5)
    so, sg = state(fb, words), state(fb, words)
    order = rng.permutation(fb.n)
    for sel in (order[:300], order[300:900], order[900:]):    # 400 x 32 x words claim words
        assert (run_gpu(ctx, fb, sg, np.sort(sel)) == run_oracle(oracle_lib, fb, so, np.sort(sel))).all()
    for k in ("msg_bytes", "fragments", "remaining"):
        assert (so[k] == sg[k]).all(), k


@pytest.mark.parametrize("words", [None, 64])
def test_fragments_overlapping_ranges(ctx, oracle_lib, words):  # noqa: F811
    """Fragments of one slot whose byte ranges overlap (a non-standard peer): the
    reference copies in arrival order, so the later command's bytes win.  Overlapping
    slots are deferred to the serial pass; both decide paths (slot-owned and atomic)
    must equal the sequential oracle bit for bit, mixed with a standard batch."""
    ov = workloads.overlapping_fragments(300, seed=31)
    std = workloads.fragments(np.random.default_rng(32).integers(1, 20000, 60), seed=33, duplicates=0.3)
    for fb in (ov, std):
        so, sg = state(fb, words), state(fb, words)
        cuts = [0, fb.n // 2, fb.n]
        for a, b in zip(cuts[:-1], cuts[1:]):
            sel = np.arange(a, b)
            assert (run_gpu(ctx, fb, sg, sel) == run_oracle(oracle_lib, fb, so, sel)).all()
        for k in ("msg_bytes", "fragments", "remaining"):
            assert (so[k] == sg[k]).all(), k


def slots_path(claim_space, n):
    """fragment_kernels.hpp frag_slots_path: the slot-owned decide kernel and the
    claim-space copy descriptors when the claim space is at most 8 n + 65536 words."""
    return claim_space <= 8 * n + 65536


def test_fragments_slots_threshold_and_scratch_regrowth(ctx, oracle_lib):  # noqa: F811
    """the claim-space descriptor path at its edges.  3000 slots x 1
    bitmap word = 96 000 claim words, so a batch of n = 3808 sits exactly on 8 n + 65536
    (slots path, q_src/q_dst/q_len sized by the claim space) and n = 3807 one step past
    it (atomic path).  Before them a small layout; after them the same slots with 2
    words (192 000 claim words: the claim words and the descriptor scratch both regrow
    on a slots-path call).  Every call against the sequential oracle."""
    rng = np.random.default_rng(61)
    small = workloads.fragments(rng.integers(1, 3000, 200), seed=62, duplicates=0.2)
    so, sg = state(small, 1), state(small, 1)
    assert slots_path(200 * 32, small.n)
    assert (run_gpu(ctx, small, sg) == run_oracle(oracle_lib, small, so)).all()
    for k in ("msg_bytes", "fragments", "remaining"):
        assert (so[k] == sg[k]).all(), k

    big = workloads.fragments(rng.integers(1000, 9000, 3000), seed=63, duplicates=0.5)
    assert int(big.msg_count.max()) <= 32 and big.n > 3808 + 3807
    for words in (1, 2):
        so, sg = state(big, words), state(big, words)
        claims = 3000 * 32 * words
        cuts = [0, 3808, 3808 + 3807, big.n] if words == 1 else [0, big.n]
        for a, b in zip(cuts[:-1], cuts[1:]):
            if words == 1 and b - a == 3808:
                assert slots_path(claims, b - a) and claims == 8 * (b - a) + 65536
            if words == 1 and b - a == 3807:
                assert not slots_path(claims, b - a)
            if words == 2:
                assert slots_path(claims, b - a), "the regrowth call must take the slots path"
            sel = np.arange(a, b)
            assert (run_gpu(ctx, big, sg, sel) == run_oracle(oracle_lib, big, so, sel)).all(), (words, a, b)
        for k in ("msg_bytes", "fragments", "remaining"):
            assert (so[k] == sg[k]).all(), (words, k)


def test_fragments_scratch_layout_changes(ctx, oracle_lib):  # noqa: F811
    """The context's claim scratch (claim words, then per-slot winner counts and the
    deferred flag) across calls whose (slots, bitmap words) layouts differ -- more
    slots with the same claim-word count, fewer, then more again -- each a small
    batch of overlapping fragments against a large claim space (the atomic decide
    path, where winner counts defer overlapping slots)."""
    for i, (slots, words) in enumerate(((4000, 1), (2500, 2), (5000, 1), (2500, 2), (4000, 1), (1000, 2))):
        fb = workloads.overlapping_fragments(slots, seed=50 + i)
        so, sg = state(fb, words), state(fb, words)
        sel = np.arange(min(fb.n, 2000))                  # 8 n + 65536 < slots x 32 x words: atomic
        assert (run_gpu(ctx, fb, sg, sel) == run_oracle(oracle_lib, fb, so, sel)).all(), (slots, words)
        for k in ("msg_bytes", "fragments", "remaining"):
            assert (so[k] == sg[k]).all(), (slots, words, k)


def test_fragments_atomic_path_many_fragment_messages(ctx, oracle_lib):  # noqa: F811
    """Round 6: the atomic decide path checks each slot's winners for overlap
    (frag_clash_kernel) instead of deferring every slot with two or more winners to the
    serial pass.  Messages of 1563 fragments (mtu 96) against 64 bitmap words per slot
    (60 slots x 2048 claim words > 8 n + 65536): a slot with a few of its fragments in a
    batch is not walked (its winners stay serial), one with hundreds is walked, small
    messages beside them, duplicates across batches -- every batch against the oracle."""
    rng = np.random.default_rng(71)
    lens = [100_000] * 4 + [int(x) for x in rng.integers(1, 5000, 56)]
    fb = workloads.fragments(lens, mtu=96, seed=72, duplicates=0.1)
    assert int(fb.msg_count.max()) == 1563
    words = 64
    so, sg = state(fb, words), state(fb, words)
    slot = fb.slots
    big = [np.flatnonzero(slot == m) for m in range(4)]
    small = np.flatnonzero(slot >= 4)
    batches = [
        np.concatenate([big[0][:4], big[1][:800], small[:700]]),     # sparse slot 0, walked slot 1
        np.concatenate([big[0][4:10], big[2][:3], small[700:]]),     # sparse slots 0 and 2
        np.concatenate([big[1][800:], big[3], big[2][3:1500]]),      # walked 1, 2 and 3
        np.concatenate([big[0][10:], big[2][1500:]]),
    ]
    for sel in batches:
        sel = np.sort(sel)
        assert not slots_path(len(lens) * 32 * words, len(sel)), len(sel)
        assert (run_gpu(ctx, fb, sg, sel) == run_oracle(oracle_lib, fb, so, sel)).all()
    for k in ("msg_bytes", "fragments", "remaining"):
        assert (so[k] == sg[k]).all(), k
