"""GPU parity of the linear-stream kernel (crc32_lin.hip, kernel paths 22 / 23)
against the oracle, through the C-ABI: the full cfg2 / cfg3 / cfg4-shard batches,
batch lists, and the shapes the unit logic branches on -- packed and gapped units,
starts and ends on and off 16- / 32- / 128-byte and tile boundaries, empty and
tiny packets, packets inside one super-block, packets spanning many tiles,
unsorted and overlapping units (the per-lane direct fold), every base alignment
mod 128.  Bit-exact."""
import numpy as np
import pytest

import enethip
from enethip import workloads

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

LIN, LIN_PLAIN = 22, 23


@pytest.fixture(scope="module")
def lctx():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    torch.cuda.init()
    c = enethip.Context(0, diag=True)         # (a diagnostics-library path)
    c.set_kernel_path(LIN)
    yield c
    c.close()


def dev(a: np.ndarray):
    a = np.ascontiguousarray(a)
    view = {np.dtype(np.uint64): np.int64, np.dtype(np.uint32): np.int32, np.dtype(np.uint8): np.uint8}[a.dtype]
    return torch.from_numpy(a.view(view)).cuda()


def run(ctx, payload, off, lens, shift=0):
    """One enet_hip_crc32_batch_device call; `shift` moves the arena's device start
    (the kernel aligns tiles to absolute 128-byte lines)."""
    buf = np.zeros(len(payload) + shift + 256, np.uint8)
    buf[shift:shift + len(payload)] = payload
    d = dev(buf)
    d_o = dev(np.asarray(off, np.uint64) + np.uint64(shift))
    d_l = dev(np.asarray(lens, np.uint32))
    out = torch.full((len(off),), -1, dtype=torch.int32, device="cuda")
    ctx.crc32_batch_device(d, d_o, d_l, len(off), out, stream=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    return out.cpu().numpy().view(np.uint32)


def packed(rng, n, lens=None, gaps=None, lo=0, hi=3000):
    lens = np.asarray(lens if lens is not None else rng.integers(lo, hi + 1, n), np.uint32)
    gaps = np.zeros(n, np.int64) if gaps is None else np.asarray(gaps, np.int64)
    off = np.zeros(n, np.uint64)
    pos = int(rng.integers(0, 300))
    for i in range(n):
        pos += int(gaps[i])
        off[i] = pos
        pos += int(lens[i])
    payload = np.frombuffer(rng.bytes(pos + 512), dtype=np.uint8).copy()
    return payload, off, lens


@pytest.mark.parametrize("path", [LIN, LIN_PLAIN])
def test_lin_cfg2_full(lctx, oracle_lib, path):
    lctx.set_kernel_path(path)
    try:
        b = workloads.fixed(65536, 1200, seed=0x454E6574, name="cfg2")
        got = run(lctx, b.payload, b.off, b.lens)
        assert (got == oracle_lib.batch(b.payload, b.off, b.lens, threads=16)).all()
    finally:
        lctx.set_kernel_path(LIN)


def test_lin_cfg3_full(lctx, oracle_lib):
    b = workloads.mixed(262144, 64, 1400, seed=0x4C454E53, name="cfg3")
    got = run(lctx, b.payload, b.off, b.lens)
    exp = oracle_lib.batch(b.payload, b.off, b.lens, threads=16)
    bad = np.nonzero(got != exp)[0]
    assert bad.size == 0, (bad[:8], b.lens[bad[:8]], b.off[bad[:8]] % 128)


def test_lin_cfg4_shard(lctx, oracle_lib):
    b = workloads.cfg4(3, 8)
    assert (run(lctx, b.payload, b.off, b.lens) == oracle_lib.batch(b.payload, b.off, b.lens, threads=16)).all()


@pytest.mark.parametrize("shift", [0, 1, 15, 16, 17, 31, 32, 64, 100, 127])
def test_lin_alignments_and_lengths(lctx, oracle_lib, shift):
    """Every length class the boundary logic distinguishes, at every base shift."""
    rng = np.random.default_rng(100 + shift)
    choices = [0, 1, 2, 3, 4, 5, 15, 16, 17, 31, 32, 33, 63, 64, 65, 95, 96, 97, 127, 128, 129, 255, 256, 257,
               1200, 1360, 1392, 4096, 8191, 8192, 8193]
    lens = rng.choice(choices, 3000).astype(np.uint32)
    payload, off, lens = packed(rng, 3000, lens=lens)
    assert (run(lctx, payload, off, lens, shift) == oracle_lib.batch(payload, off, lens)).all()


def test_lin_gaps(lctx, oracle_lib):
    """Sorted units with gaps between packets (ends that are not the next start)."""
    rng = np.random.default_rng(7)
    for trial in range(4):
        n = 2000
        gaps = np.where(rng.random(n) < 0.3, rng.integers(0, 400, n), 0)
        payload, off, lens = packed(rng, n, gaps=gaps, lo=0, hi=1500)
        assert (run(lctx, payload, off, lens, trial * 37) == oracle_lib.batch(payload, off, lens)).all()


def test_lin_tiny_and_empty(lctx, oracle_lib):
    rng = np.random.default_rng(8)
    payload, off, lens = packed(rng, 20000, lo=0, hi=40)
    assert (run(lctx, payload, off, lens) == oracle_lib.batch(payload, off, lens)).all()
    z = np.zeros(1000, np.uint32)                                # all empty
    payload2, off2, _ = packed(rng, 1000, lens=z)
    assert (run(lctx, payload2, off2, z) == 0).all()


def test_lin_long_packets(lctx, oracle_lib):
    """Packets spanning many 8 KiB tiles (Horner through whole tiles)."""
    rng = np.random.default_rng(9)
    lens = rng.choice([65536, 65535, 100000, 17, 30000, 1200], 300).astype(np.uint32)
    payload, off, lens = packed(rng, 300, lens=lens)
    assert (run(lctx, payload, off, lens, 5) == oracle_lib.batch(payload, off, lens)).all()


def test_lin_unsorted_and_overlapping(lctx, oracle_lib):
    """Units that are not sorted or overlap take the per-lane direct fold."""
    rng = np.random.default_rng(10)
    payload, off, lens = packed(rng, 5000, lo=0, hi=2000)
    perm = rng.permutation(5000)
    assert (run(lctx, payload, off[perm], lens[perm]) == oracle_lib.batch(payload, off[perm], lens[perm])).all()
    off2 = off.copy()
    off2[::7] = off2[::7] // 2                                    # overlaps
    assert (run(lctx, payload, off2, lens) == oracle_lib.batch(payload, off2, lens)).all()
    # one huge gap (span far longer than the bytes)
    off3 = off.copy()
    off3[2500:] += np.uint64(1 << 26)
    big = np.zeros(len(payload) + (1 << 26), np.uint8)
    big[:len(payload)] = payload
    big[1 << 26:] = payload
    assert (run(lctx, big, off3, lens) == oracle_lib.batch(big, off3, lens)).all()


def test_lin_batch_lists(lctx, oracle_lib):
    """Several batches per launch (unit numbering across batches), empty ones among them."""
    rng = np.random.default_rng(11)
    descs, exps, keep = [], [], []
    for n in (0, 1, 61, 62, 63, 124, 125, 7000, 0, 20000, 3):
        payload, off, lens = packed(rng, n, lo=0, hi=2500) if n else (np.zeros(16, np.uint8), np.zeros(0, np.uint64),
                                                                      np.zeros(0, np.uint32))
        d = dev(payload if len(payload) else np.zeros(16, np.uint8))
        out = torch.full((max(n, 1),), -1, dtype=torch.int32, device="cuda")
        descs.append((d, dev(off), dev(lens), n, out))
        exps.append(oracle_lib.batch(payload, off, lens) if n else np.zeros(0, np.uint32))
        keep.append(out)
    lctx.crc32_batch_list_device(descs, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    for (d, o, l, n, out), exp in zip(descs, exps):
        assert (out[:n].cpu().numpy().view(np.uint32) == exp).all(), n


def test_lin_repeat_deterministic(lctx, oracle_lib):
    """Back-to-back launches on one stream give the same CRCs (no state kept)."""
    b = workloads.fixed(30000, 1200, seed=3, name="t")
    exp = oracle_lib.batch(b.payload, b.off, b.lens)
    for s in (0, 3, 64):
        assert (run(lctx, b.payload, b.off, b.lens, s) == exp).all()
