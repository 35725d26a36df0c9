"""GPU parity: the HIP path (through the C-ABI of libenethip.so) against the oracle.

Bit-exact everywhere (integer/byte work).  Sizes run from the golden vectors up
to BASELINE.json's full configs; the oracle (C, multithreaded) finishes those in
about a second, so the full sizes are checked element for element, plus
size-independent properties (linearity, tuning invariance, determinism)."""
import numpy as np
import pytest

import enethip
from enethip import workloads

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def ctx():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    torch.cuda.init()
    c = enethip.Context(0)
    yield c
    c.close()


@pytest.fixture(scope="module")
def dctx():
    """The diagnostics library (libenethip_diag.so): the sweep-only kernel paths."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    torch.cuda.init()
    c = enethip.Context(0, diag=True)
    yield c
    c.close()


PRODUCT_PATHS = (0, 13, 17)   # built in libenethip.so; every other path: libenethip_diag.so only
PRODUCT_LANES = (0, 4, 8)     # lanes per packet libenethip.so takes; 1, 2, 16, 32, 64: diagnostics only


def on(ctx, dctx, path, lanes=0):
    """The context whose library builds kernel path `path` at `lanes` lanes per packet."""
    return ctx if path in PRODUCT_PATHS and lanes in PRODUCT_LANES else dctx


WGS = (0, 1, 2)    # workgroups per CU of the vring kernel: the default (2), one, two


def dev(a: np.ndarray):
    a = np.ascontiguousarray(a)
    view = {np.dtype(np.uint64): np.int64, np.dtype(np.uint32): np.int32, np.dtype(np.uint8): np.uint8}[a.dtype]
    return torch.from_numpy(a.view(view)).cuda()


def run_batch(ctx, payload, off, lens, lanes=0, wgs=0):
    ctx.set_tuning(lanes, wgs)
    d_p, d_o, d_l = dev(payload if len(payload) else np.zeros(16, np.uint8)), dev(off), dev(lens)
    out = torch.zeros(len(off), dtype=torch.int32, device="cuda")
    ctx.crc32_batch_device(d_p, d_o, d_l, len(off), out, stream=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    return out.cpu().numpy().view(np.uint32)


def golden_batch(golden):
    vecs, blob = golden
    off, lens, exp = [], [], []
    parts = []
    pos = 0
    for v in vecs:
        data = b"".join(bytes(blob[o:o + n]) for o, n in v["segments"])
        parts.append(data)
        off.append(pos)
        lens.append(len(data))
        exp.append(int(v["crc"], 16))
        pos += len(data)
    payload = np.frombuffer(b"".join(parts), dtype=np.uint8).copy()
    return payload, np.array(off, np.uint64), np.array(lens, np.uint32), np.array(exp, np.uint32)


@pytest.mark.parametrize("lanes", [1, 2, 4, 8, 16, 64])
def test_golden_vectors(ctx, dctx, golden, lanes):
    payload, off, lens, exp = golden_batch(golden)
    got = run_batch(on(ctx, dctx, 0, lanes), payload, off, lens, lanes)
    bad = np.nonzero(got != exp)[0]
    assert len(bad) == 0, [(int(i), int(lens[i]), hex(got[i]), hex(exp[i])) for i in bad[:10]]


@pytest.mark.parametrize("lanes", [1, 4, 32])
def test_random_unaligned_sparse(ctx, dctx, oracle_lib, lanes):
    rng = np.random.default_rng(100 + lanes)
    n = 5000
    lens = rng.integers(0, 5000, size=n).astype(np.uint32)
    lens[:40] = np.arange(40)                       # every tiny length
    gaps = rng.integers(0, 37, size=n).astype(np.uint64)
    off = np.zeros(n, dtype=np.uint64)
    off[1:] = np.cumsum(lens[:-1].astype(np.uint64) + gaps[:-1])
    off += np.uint64(3)
    perm = rng.permutation(n)                       # packets in arbitrary order
    off, lens = off[perm], lens[perm]
    payload = rng.integers(0, 256, size=int((off + lens).max()) + 5, dtype=np.uint8)
    got = run_batch(on(ctx, dctx, 0, lanes), payload, off, lens, lanes)
    exp = oracle_lib.batch(payload, off, lens, threads=8)
    assert (got == exp).all(), np.nonzero(got != exp)[0][:10]


def test_cfg2_full(ctx, dctx, oracle_lib):
    b = workloads.cfg2()
    exp = oracle_lib.batch(b.payload, b.off, b.lens, threads=16)
    for lanes in (1, 4, 8):
        assert (run_batch(on(ctx, dctx, 0, lanes), b.payload, b.off, b.lens, lanes) == exp).all(), lanes


def test_cfg3_full(ctx, dctx, oracle_lib):
    b = workloads.cfg3()
    exp = oracle_lib.batch(b.payload, b.off, b.lens, threads=16)
    for lanes in (2, 4):
        assert (run_batch(on(ctx, dctx, 0, lanes), b.payload, b.off, b.lens, lanes) == exp).all(), lanes


def run_binned(ctx, payload, off, lens, lanes=0, path=0, wgs=0):
    ctx.set_tuning(lanes, wgs)
    ctx.set_kernel_path(path)
    try:
        n = len(off)
        d_p, d_o, d_l = dev(payload if len(payload) else np.zeros(16, np.uint8)), dev(off), dev(lens)
        out = torch.zeros(n, dtype=torch.int32, device="cuda")
        ws_bytes = ctx.binned_workspace_size(n)
        ws = torch.zeros(ws_bytes, dtype=torch.uint8, device="cuda")
        ctx.crc32_batch_device_binned(d_p, d_o, d_l, n, out, ws, ws_bytes,
                                      stream=torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        return out.cpu().numpy().view(np.uint32)
    finally:
        ctx.set_kernel_path(0)
        ctx.set_tuning(0, 0)


BINNED_PATHS = (0, 17)        # 0: the default (the vring kernel's records instance), 17: the vring path itself


def test_binned_cfg3_full(ctx, oracle_lib):
    """Length-binned entry (records reordered on the GPU): same CRCs, caller order,
    on the lean (default) and vring record paths."""
    b = workloads.cfg3()
    exp = oracle_lib.batch(b.payload, b.off, b.lens, threads=16)
    for path in BINNED_PATHS:
        for lanes in (4, 8):
            assert (run_binned(ctx, b.payload, b.off, b.lens, lanes, path) == exp).all(), (path, lanes)


def test_binned_vring_many_groups(ctx, oracle_lib):
    """Binned records on the vring kernel: 1.2 M tiny packets (one-stage groups, a
    record load per group) and 40 K long ones (many stages per group)."""
    tiny = workloads.mixed(1_200_000, 0, 40, seed=277, len_seed=278)
    exp_t = oracle_lib.batch(tiny.payload, tiny.off, tiny.lens, threads=16)
    big = workloads.mixed(40_000, 2000, 9000, seed=279, len_seed=280)
    exp_b = oracle_lib.batch(big.payload, big.off, big.lens, threads=16)
    for lanes in (4, 8):
        assert (run_binned(ctx, tiny.payload, tiny.off, tiny.lens, lanes, 17) == exp_t).all(), ("tiny", lanes)
        assert (run_binned(ctx, big.payload, big.off, big.lens, lanes, 17) == exp_b).all(), ("big", lanes)


@pytest.mark.parametrize("lanes", [1, 4, 8])
@pytest.mark.parametrize("path", BINNED_PATHS)
def test_binned_golden_and_edges(ctx, dctx, golden, oracle_lib, lanes, path):
    payload, off, lens, exp = golden_batch(golden)
    assert (run_binned(on(ctx, dctx, path, lanes), payload, off, lens, lanes, path) == exp).all()
    # lengths over every bin incl. the clamped last one (>= 8160 B), empties, one-packet batches
    rng = np.random.default_rng(7 + lanes)
    n = 20000
    lens = rng.integers(0, 9000, size=n).astype(np.uint32)
    lens[:64] = 0
    lens[64:128] = np.arange(64) * 32
    off = rng.integers(0, 1 << 20, size=n).astype(np.uint64)
    payload = rng.integers(0, 256, size=(1 << 20) + 9000, dtype=np.uint8)
    exp = oracle_lib.batch(payload, off, lens, threads=8)
    assert (run_binned(on(ctx, dctx, path, lanes), payload, off, lens, lanes, path) == exp).all()
    assert (run_binned(on(ctx, dctx, path, lanes), payload, off[:1], lens[:1], lanes, path) == exp[:1]).all()


@pytest.mark.parametrize("wgs", [1, 2])
def test_binned_records_instance_per_workgroup_count(ctx, golden, oracle_lib, wgs):
    """The records instance at one workgroup per CU (its x^(-8 c) tables in LDS) and at
    two (the compact instance: tz mod 8 by unsteps): cfg3 in full, the golden vectors,
    every bin with empties and ragged ends, tiny one-stage and long many-stage groups."""
    b = workloads.cfg3()
    exp = oracle_lib.batch(b.payload, b.off, b.lens, threads=16)
    payload, off, lens, exp_g = golden_batch(golden)
    rng = np.random.default_rng(31 + wgs)
    n = 20000
    e_lens = rng.integers(0, 9000, size=n).astype(np.uint32)
    e_lens[:64] = 0
    e_lens[64:128] = np.arange(64) * 32 + 31
    e_off = rng.integers(0, 1 << 20, size=n).astype(np.uint64)
    e_pay = rng.integers(0, 256, size=(1 << 20) + 9000, dtype=np.uint8)
    exp_e = oracle_lib.batch(e_pay, e_off, e_lens, threads=8)
    tiny = workloads.mixed(300_000, 0, 40, seed=281, len_seed=282)
    exp_t = oracle_lib.batch(tiny.payload, tiny.off, tiny.lens, threads=16)
    for lanes in (4, 8):
        assert (run_binned(ctx, b.payload, b.off, b.lens, lanes, 0, wgs) == exp).all(), ("cfg3", lanes)
        assert (run_binned(ctx, payload, off, lens, lanes, 0, wgs) == exp_g).all(), ("golden", lanes)
        assert (run_binned(ctx, e_pay, e_off, e_lens, lanes, 0, wgs) == exp_e).all(), ("edges", lanes)
        assert (run_binned(ctx, e_pay, e_off[:1], e_lens[:1], lanes, 0, wgs) == exp_e[:1]).all(), ("one", lanes)
        assert (run_binned(ctx, tiny.payload, tiny.off, tiny.lens, lanes, 0, wgs) == exp_t).all(), ("tiny", lanes)


def test_binned_records_are_a_length_ordered_permutation(ctx, oracle_lib):
    """The two-launch form's records (kernel path 17, and the default past the local
    tiles' limit; documented layout: n x {len, off_lo, off_hi, index} first) are a
    permutation of the batch: each 1024-packet tile ordered by non-increasing 32-byte bin
    of the window length (offset mod 64 + length), full tiles interleaved group by group;
    600 K packets, ragged last tile."""
    rng = np.random.default_rng(11)
    n = 600_000
    lens = rng.integers(0, 1500, size=n).astype(np.uint32)
    lens[rng.integers(0, n, size=50)] = rng.integers(8160, 20000, size=50).astype(np.uint32)   # clamped bin
    off = rng.integers(0, 1 << 22, size=n).astype(np.uint64)
    payload = rng.integers(0, 256, size=(1 << 22) + 20000, dtype=np.uint8)
    ctx.set_tuning(8, 0)
    ctx.set_kernel_path(17)
    try:
        d_p, d_o, d_l = dev(payload), dev(off), dev(lens)
        out = torch.zeros(n, dtype=torch.int32, device="cuda")
        ws_bytes = ctx.binned_workspace_size(n)
        ws = torch.zeros(ws_bytes, dtype=torch.uint8, device="cuda")
        ctx.crc32_batch_device_binned(d_p, d_o, d_l, n, out, ws, ws_bytes, stream=torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
    finally:
        ctx.set_kernel_path(0)
        ctx.set_tuning(0, 0)
    rec = ws[:16 * n].cpu().numpy().view(np.uint32).reshape(n, 4)
    idx = rec[:, 3].astype(np.int64)
    assert (np.sort(idx) == np.arange(n)).all()
    assert (rec[:, 0] == lens[idx]).all()
    assert ((rec[:, 1].astype(np.uint64) | (rec[:, 2].astype(np.uint64) << np.uint64(32))) == off[idx]).all()
    # full tiles: sorted group q of tile t sits at global group q * T + t (8 records at 8 lanes);
    # the ragged last tile stays in place
    T, kpk = n // 1024, 8
    pos = np.arange(n)
    t_of = idx // 1024
    full = pos < T * 1024
    grp = pos[full] // kpk
    assert (t_of[full] == grp % T).all()
    assert (t_of[~full] == T).all()
    bins = np.minimum((rec[:, 0] + (rec[:, 1] & 63)) >> 5, 255).astype(np.int64)   # window lz + L
    order = np.lexsort((pos, t_of))                           # each tile's records in position order
    same = np.diff(t_of[order]) == 0
    assert (np.diff(bins[order])[same] <= 0).all()            # longest bin first inside a tile
    exp = oracle_lib.batch(payload, off, lens, threads=16)
    assert (out.cpu().numpy().view(np.uint32) == exp).all()


@pytest.mark.parametrize("wgs", [1, 2])
@pytest.mark.parametrize("lanes", [4, 8])
def test_binned_local_tiles_layout_and_limit(ctx, oracle_lib, wgs, lanes):
    """The one-launch binned checksum (default path, vring_launch_local): workgroup k
    orders its own tile of T packets, so the workspace's records [k T, (k + 1) T) are a
    permutation of packets [k T, (k + 1) T) in non-increasing 32-byte bins of the window
    length (offset mod 64 + length).  T = the batch over the grid (CUs x workgroups per
    CU) in whole groups, at least one group per wave, at most 2048 (two per thread).
    Checked at several sizes, up to the one-tile-per-workgroup limit, and one packet past
    it (the bin kernel and the records instance)."""
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    G = cus * wgs
    limit = 2048 * G
    kpk = 64 // lanes
    rng = np.random.default_rng(97 + wgs + lanes)
    payload = rng.integers(0, 256, size=(1 << 21) + 4096, dtype=np.uint8)
    for n in (1, 17, 255, 16 * kpk + 3, 5000, G * 16 * kpk + 1, 1024 * G + 1, limit - 7, limit, limit + 1):
        lens = rng.integers(0, 300, size=n).astype(np.uint32)
        lens[rng.integers(0, n, size=max(1, n // 500))] = rng.integers(4000, 4096, size=max(1, n // 500)).astype(np.uint32)
        lens[: min(n, 5)] = 0
        off = rng.integers(0, 1 << 21, size=n).astype(np.uint64)
        ctx.set_tuning(lanes, wgs)
        try:
            d_p, d_o, d_l = dev(payload), dev(off), dev(lens)
            out = torch.zeros(n, dtype=torch.int32, device="cuda")
            ws_bytes = ctx.binned_workspace_size(n)
            ws = torch.zeros(ws_bytes, dtype=torch.uint8, device="cuda")
            ctx.crc32_batch_device_binned(d_p, d_o, d_l, n, out, ws, ws_bytes,
                                          stream=torch.cuda.current_stream().cuda_stream)
            torch.cuda.synchronize()
        finally:
            ctx.set_tuning(0, 0)
        exp = oracle_lib.batch(payload, off, lens, threads=16)
        assert (out.cpu().numpy().view(np.uint32) == exp).all(), n
        if n > limit:
            continue
        per_wg = -(-n // G)                                     # ceil(n / G), then whole groups
        T = min(max(-(-per_wg // kpk) * kpk, kpk * 16), 2048)
        rec = ws[:16 * n].cpu().numpy().view(np.uint32).reshape(n, 4)
        idx = rec[:, 3].astype(np.int64)
        pos = np.arange(n)
        assert (idx // T == pos // T).all(), n                  # each record stays in its workgroup's tile
        assert (np.sort(idx) == pos).all(), n
        assert (rec[:, 0] == lens[idx]).all(), n
        assert ((rec[:, 1].astype(np.uint64) | (rec[:, 2].astype(np.uint64) << np.uint64(32))) == off[idx]).all(), n
        bins = np.minimum((rec[:, 0] + (rec[:, 1] & 63)) >> 5, 255).astype(np.int64)
        same = np.diff(pos // T) == 0
        assert (np.diff(bins)[same] <= 0).all(), n              # longest bin first inside a tile


def test_binned_rejects_small_workspace(ctx):
    d = torch.zeros(64, dtype=torch.uint8, device="cuda")
    o = torch.zeros(4, dtype=torch.int64, device="cuda")
    ln = torch.zeros(4, dtype=torch.int32, device="cuda")
    out = torch.zeros(4, dtype=torch.int32, device="cuda")
    need = ctx.binned_workspace_size(4)
    ws = torch.zeros(need, dtype=torch.uint8, device="cuda")
    with pytest.raises(enethip.ENetHipError):
        ctx.crc32_batch_device_binned(d, o, ln, 4, out, ws, need - 1)


def test_cfg4_shard_full(ctx, oracle_lib):
    b = workloads.cfg4(1, 8)
    exp = oracle_lib.batch(b.payload, b.off, b.lens, threads=16)
    assert (run_batch(ctx, b.payload, b.off, b.lens) == exp).all()


def test_linearity_and_determinism(ctx):
    # For equal-length packets CRC is affine over GF(2): crc(a^b^c) = crc(a)^crc(b)^crc(c).
    rng = np.random.default_rng(5)
    n, L = 3000, 1200
    a, b_, c = (rng.integers(0, 256, size=n * L, dtype=np.uint8) for _ in range(3))
    off = np.arange(n, dtype=np.uint64) * np.uint64(L)
    lens = np.full(n, L, np.uint32)
    ca, cb, cc = (run_batch(ctx, x, off, lens) for x in (a, b_, c))
    cx = run_batch(ctx, a ^ b_ ^ c, off, lens)
    assert (cx == (ca ^ cb ^ cc)).all()
    assert (run_batch(ctx, a, off, lens, 4, 1) == ca).all()


N_STREAM_GEOMS = 13          # 6 LDS-ring + 5 register-stream geometries + 2 lean-kernel geometries
LEAN_PATHS = (13, 14)        # crc32_lean.hip geometries (path 0 runs the first for 4 and 8 lanes)


@pytest.mark.parametrize("geom", range(N_STREAM_GEOMS))
def test_stream_geometries(ctx, dctx, golden, oracle_lib, geom):
    """Every stream-kernel geometry (path 2 + k) x 4/8/16 lanes: golden vectors,
    unaligned mixed sizes (empty packets included) and many groups per wave."""
    payload, off, lens, exp = golden_batch(golden)
    b = workloads.mixed(30000, 0, 3000, seed=40 + geom, len_seed=41 + geom)
    exp_b = oracle_lib.batch(b.payload, b.off, b.lens, threads=16)
    small = workloads.mixed(200000, 1, 100, seed=7, len_seed=8)
    exp_s = oracle_lib.batch(small.payload, small.off, small.lens, threads=16)
    try:
        for lanes in (4, 8, 16):
            c = on(ctx, dctx, 2 + geom, lanes)
            c.set_kernel_path(2 + geom)
            assert (run_batch(c, payload, off, lens, lanes) == exp).all(), ("golden", lanes)
            assert (run_batch(c, b.payload, b.off, b.lens, lanes) == exp_b).all(), ("mixed", lanes)
        c = on(ctx, dctx, 2 + geom, 4)
        c.set_kernel_path(2 + geom)
        assert (run_batch(c, small.payload, small.off, small.lens, 4) == exp_s).all()
    finally:
        for c in (ctx, dctx):
            c.set_kernel_path(0)
            c.set_tuning(0, 0)


def _verify_expect(oracle_lib, payload, off, lens, slot, conn):
    return oracle_lib.verify(payload, off, lens, slot, conn)


@pytest.mark.parametrize("path", LEAN_PATHS)
def test_lean_many_chunks(ctx, dctx, oracle_lib, path):
    """Many metadata chunks per wave (tiny packets: one-stage groups, so the
    producer runs into chunks the consumer has not prefetched yet) and long
    packets (many stages per group), crc and verify, 4 and 8 lanes."""
    tiny = workloads.mixed(1_200_000, 0, 40, seed=77, len_seed=78)
    exp_t = oracle_lib.batch(tiny.payload, tiny.off, tiny.lens, threads=16)
    big = workloads.mixed(40_000, 2000, 9000, seed=79, len_seed=80)
    exp_b = oracle_lib.batch(big.payload, big.off, big.lens, threads=16)
    rng = np.random.default_rng(81)
    vp, vo, vl, vs, vc = _verify_inputs(rng, 300_000)
    exp_ok, exp_comp = oracle_lib.verify(vp, vo, vl, vs, vc)
    ctx = on(ctx, dctx, path)
    try:
        ctx.set_kernel_path(path)
        for lanes in (4, 8):
            assert (run_batch(ctx, tiny.payload, tiny.off, tiny.lens, lanes) == exp_t).all(), ("tiny", lanes)
            assert (run_batch(ctx, big.payload, big.off, big.lens, lanes) == exp_b).all(), ("big", lanes)
            ctx.set_tuning(lanes, 0)
            d_ok = torch.zeros(len(vo), dtype=torch.uint8, device="cuda")
            d_comp = torch.zeros(len(vo), dtype=torch.int32, device="cuda")
            ctx.verify_batch_device(dev(vp), dev(vo), dev(vl), dev(vs), dev(vc), len(vo), d_ok, d_comp,
                                    stream=torch.cuda.current_stream().cuda_stream)
            torch.cuda.synchronize()
            assert (d_ok.cpu().numpy() == exp_ok).all(), ("verify ok", lanes)
            assert (d_comp.cpu().numpy().view(np.uint32) == exp_comp).all(), ("verify crc", lanes)
    finally:
        ctx.set_kernel_path(0)
        ctx.set_tuning(0, 0)


def test_host_entry_point(ctx, oracle_lib):
    b = workloads.mixed(20000, 1, 4096, seed=9, len_seed=10)
    ctx.set_tuning(0, 0)
    got = ctx.crc32_batch_host(b.payload, b.off, b.lens)
    assert (got == oracle_lib.batch(b.payload, b.off, b.lens, threads=8)).all()


def test_multi_context_shards(oracle_lib):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    b = workloads.mixed(30001, 64, 1400, seed=3, len_seed=4)
    ctxs = [enethip.Context(i % max(1, enethip.device_count())) for i in range(3)]
    try:
        got = enethip.crc32_batch_multi(ctxs, b.payload, b.off, b.lens)
    finally:
        for c in ctxs:
            c.close()
    assert (got == oracle_lib.batch(b.payload, b.off, b.lens, threads=8)).all()


def _verify_inputs(rng, n):
    """DGRAMs as ENet puts them on the wire: [2 or 4 B header][4 B slot][commands]."""
    lens = rng.integers(6, 1400, size=n).astype(np.uint32)
    slot = np.where(rng.integers(0, 2, size=n) == 1, 4, 2).astype(np.uint32)
    lens = np.maximum(lens, slot + 4)
    conn = rng.integers(0, 2**32, size=n, dtype=np.uint64).astype(np.uint32)
    conn[::5] = 0                                   # "no peer" DGRAMs
    off = np.zeros(n, dtype=np.uint64)
    off[1:] = np.cumsum(lens[:-1].astype(np.uint64))
    payload = rng.integers(0, 256, size=int(lens.sum()), dtype=np.uint8)
    for i in range(n):                              # stamp like protocol.cs:1690-1698
        o, s = int(off[i]), int(slot[i])
        payload[o + s:o + s + 4] = np.frombuffer(np.uint32(conn[i]).tobytes(), np.uint8)
    return payload, off, lens, slot, conn


def test_verify_batch(ctx, dctx, oracle_lib):
    rng = np.random.default_rng(21)
    n = 4000
    payload, off, lens, slot, conn = _verify_inputs(rng, n)
    # stamp the true checksum (computed over the DGRAM with slot = connectID)
    stamped = oracle_lib.batch(payload, off, lens, threads=8)
    for i in range(n):
        o, s = int(off[i]), int(slot[i])
        payload[o + s:o + s + 4] = np.frombuffer(np.uint32(stamped[i]).tobytes(), np.uint8)
    bad = rng.choice(n, size=300, replace=False)
    for i in bad:                                   # corrupt a byte (or the slot) of some DGRAMs
        j = int(off[i]) + int(rng.integers(0, int(lens[i])))
        payload[j] ^= np.uint8(1 << int(rng.integers(0, 8)))
    exp_ok, exp_comp = oracle_lib.verify(payload, off, lens, slot, conn)
    assert exp_ok.sum() == n - 300
    for lanes in (1, 4, 8, 16):
        c = on(ctx, dctx, 0, lanes)
        c.set_tuning(lanes, 0)
        d_ok = torch.zeros(n, dtype=torch.uint8, device="cuda")
        d_comp = torch.zeros(n, dtype=torch.int32, device="cuda")
        c.verify_batch_device(dev(payload), dev(off), dev(lens), dev(slot), dev(conn), n, d_ok, d_comp,
                              stream=torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        assert (d_ok.cpu().numpy() == exp_ok).all()
        assert (d_comp.cpu().numpy().view(np.uint32) == exp_comp).all()
        c.set_tuning(0, 0)


def _verify_list_batch(oracle_lib, rng, n):
    """One receive batch for the list tests: half the DGRAMs stamped with their true
    CRC (vectorised stamp), a tenth of all corrupted; the oracle's ok / computed."""
    payload, off, lens, slot, conn = _verify_inputs(rng, n)
    if n:
        stamped = oracle_lib.batch(payload, off, lens, threads=8)
        good = np.nonzero(rng.integers(0, 2, size=n) == 1)[0]
        pos = (off[good] + slot[good]).astype(np.int64)[:, None] + np.arange(4)
        payload[pos] = stamped[good].view(np.uint8).reshape(-1, 4)
        bad = rng.choice(n, size=max(1, n // 10), replace=False)
        payload[off[bad].astype(np.int64) + rng.integers(0, lens[bad].astype(np.int64))] ^= np.uint8(0x20)
    exp_ok, exp_comp = oracle_lib.verify(payload, off, lens, slot, conn)
    return payload, off, lens, slot, conn, exp_ok, exp_comp


def _run_verify_list(ctx, batches, with_computed=True):
    keep, descs, outs = [], [], []
    for payload, off, lens, slot, conn, _, _ in batches:
        n = len(off)
        d = [dev(payload if len(payload) else np.zeros(16, np.uint8))] + \
            [dev(x) if n else dev(np.zeros(1, x.dtype)) for x in (off, lens, slot, conn)]
        ok = torch.full((max(1, n),), 7, dtype=torch.uint8, device="cuda")
        comp = torch.full((max(1, n),), -1, dtype=torch.int32, device="cuda") if with_computed else None
        keep.append(d)
        outs.append((ok, comp))
        descs.append((d[0], d[1], d[2], d[3], d[4], n, ok, comp))
    ctx.verify_batch_list_device(descs, stream=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    return [(ok.cpu().numpy()[:len(b[1])], None if comp is None else comp.cpu().numpy().view(np.uint32)[:len(b[1])])
            for (ok, comp), b in zip(outs, batches)]


def test_verify_batch_list(ctx, dctx, oracle_lib):
    """enet_hip_verify_batch_list_device: receive batches of every shape (empty,
    one DGRAM, odd sizes, 20 000 mixed DGRAMs) in one launch, at the default, 4,
    8 and 16 lanes (16: one launch per batch), with and without computed[]; and 70
    batches (three launches of at most 32), each against the oracle's verify."""
    rng = np.random.default_rng(91)
    batches = [_verify_list_batch(oracle_lib, rng, n) for n in (0, 1, 3, 700, 20_000, 0, 5000, 33)]
    try:
        for lanes in (0, 4, 8, 16):
            c = on(ctx, dctx, 0, lanes)
            c.set_tuning(lanes, 0)
            for wc in (True, False):
                for i, ((ok, comp), b) in enumerate(zip(_run_verify_list(c, batches, wc), batches)):
                    assert (ok == b[5]).all(), (lanes, wc, i)
                    if wc:
                        assert (comp == b[6]).all(), (lanes, i)
            c.set_tuning(0, 0)
        many = [_verify_list_batch(oracle_lib, rng, int(rng.integers(0, 900))) for _ in range(70)]
        for i, ((ok, comp), b) in enumerate(zip(_run_verify_list(ctx, many), many)):
            assert (ok == b[5]).all() and (comp == b[6]).all(), i
        assert sum(int(b[5].sum()) for b in batches) > 0
    finally:
        ctx.set_tuning(0, 0)


@pytest.mark.parametrize("n", [1, 3000, 70_000])
def test_verify_binned(ctx, dctx, oracle_lib, n):
    """Binned receive verify: mixed-length DGRAMs (6..1400 B, 2- and 4-byte headers),
    half correctly stamped, the rest corrupted or unstamped; ok/computed in caller order."""
    rng = np.random.default_rng(31 + n)
    payload, off, lens, slot, conn = _verify_inputs(rng, n)
    stamped = oracle_lib.batch(payload, off, lens, threads=8)
    good = rng.integers(0, 2, size=n) == 1
    for i in np.nonzero(good)[0]:
        o, s = int(off[i]), int(slot[i])
        payload[o + s:o + s + 4] = np.frombuffer(np.uint32(stamped[i]).tobytes(), np.uint8)
    exp_ok, exp_comp = oracle_lib.verify(payload, off, lens, slot, conn)
    for lanes in (1, 4, 8):
        c = on(ctx, dctx, 0, lanes)
        c.set_tuning(lanes, 0)
        d_ok = torch.zeros(n, dtype=torch.uint8, device="cuda")
        d_comp = torch.zeros(n, dtype=torch.int32, device="cuda")
        wsb = c.verify_binned_workspace_size(n)
        ws = torch.zeros(wsb, dtype=torch.uint8, device="cuda")
        c.verify_batch_device_binned(dev(payload), dev(off), dev(lens), dev(slot), dev(conn), n, d_ok, ws, wsb,
                                     d_comp, stream=torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        assert (d_ok.cpu().numpy() == exp_ok).all(), lanes
        assert (d_comp.cpu().numpy().view(np.uint32) == exp_comp).all(), lanes
        c.set_tuning(0, 0)
    if n > 1:
        assert 0 < exp_ok.sum() < n


def test_verify_golden(ctx, golden):
    vecs, blob = golden
    vv = [v for v in vecs if v["kind"] == "verify"]
    off = np.array([v["segments"][0][0] for v in vv], np.uint64)
    lens = np.array([v["segments"][0][1] for v in vv], np.uint32)
    slot = np.array([v["slot_off"] for v in vv], np.uint32)
    conn = np.array([int(v["connect_id"], 16) for v in vv], np.uint32)
    d_ok = torch.zeros(len(vv), dtype=torch.uint8, device="cuda")
    ctx.set_tuning(0, 0)
    ctx.verify_batch_device(dev(blob), dev(off), dev(lens), dev(slot), dev(conn), len(vv), d_ok)
    ctx.synchronize()
    assert d_ok.cpu().numpy().astype(bool).tolist() == [v["expect_ok"] for v in vv]


def test_gather_golden_and_cfg5(ctx, golden, oracle_lib):
    vecs, blob = golden
    seg_off, seg_len, first, exp = [], [], [0], []
    for v in vecs:
        for o, n in v["segments"]:
            seg_off.append(o)
            seg_len.append(n)
        first.append(len(seg_off))
        exp.append(int(v["crc"], 16))
    out = torch.zeros(len(exp), dtype=torch.int32, device="cuda")
    ctx.gather_device(dev(blob), dev(np.array(seg_off, np.uint64)), dev(np.array(seg_len, np.uint32)),
                      dev(np.array(first, np.uint32)), len(exp), out)
    ctx.synchronize()
    assert out.cpu().numpy().view(np.uint32).tolist() == exp
    g = workloads.cfg5(messages=256)
    out = torch.zeros(g.n, dtype=torch.int32, device="cuda")
    ctx.gather_device(dev(g.payload), dev(g.seg_off), dev(g.seg_len), dev(g.seg_first), g.n, out)
    ctx.synchronize()
    assert (out.cpu().numpy().view(np.uint32) == oracle_lib.gather(g.payload, g.seg_off, g.seg_len,
                                                                   g.seg_first)).all()


def _run_gather_binned(ctx, payload, seg_off, seg_len, seg_first):
    n, ns = len(seg_first) - 1, int(seg_first[-1])
    out = torch.full((max(1, n),), -1, dtype=torch.int32, device="cuda")
    wsb = ctx.gather_binned_workspace_size(ns)
    ws = torch.zeros(max(16, wsb), dtype=torch.uint8, device="cuda")
    ctx.gather_binned_device(dev(payload if len(payload) else np.zeros(16, np.uint8)),
                             dev(seg_off) if ns else None, dev(seg_len) if ns else None, ns,
                             dev(seg_first), n, out, ws, wsb, stream=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    return out.cpu().numpy().view(np.uint32)[:n]


def _gather_cases(golden, oracle_lib):
    """test_gather_binned's gather lists: (payload, seg_off, seg_len, seg_first, expected)."""
    vecs, blob = golden
    seg_off, seg_len, first, exp = [], [], [0], []
    for v in vecs:
        for o, n in v["segments"]:
            seg_off.append(o)
            seg_len.append(n)
        first.append(len(seg_off))
        exp.append(int(v["crc"], 16))
    cases = [(blob, np.array(seg_off, np.uint64), np.array(seg_len, np.uint32), np.array(first, np.uint32),
              np.array(exp, np.uint32))]
    g = workloads.cfg5(messages=256)
    cases.append((g.payload, g.seg_off, g.seg_len, g.seg_first,
                  oracle_lib.gather(g.payload, g.seg_off, g.seg_len, g.seg_first)))
    rng = np.random.default_rng(77)
    payload = rng.integers(0, 256, size=3 << 20, dtype=np.uint8)
    cnt = rng.integers(0, 66, size=3000)
    cnt[::50] = 0
    ns = int(cnt.sum())
    lens = np.where(rng.integers(0, 8, size=ns) == 0, 0, rng.integers(1, 1500, size=ns)).astype(np.uint32)
    offs = rng.integers(0, len(payload) - 1500, size=ns).astype(np.uint64)
    sf = np.zeros(len(cnt) + 1, np.uint32)
    np.cumsum(cnt, out=sf[1:])
    cases.append((payload, offs, lens, sf, oracle_lib.gather(payload, offs, lens, sf)))
    empty_first = np.zeros(7, np.uint32)
    cases.append((payload[:64], np.zeros(0, np.uint64), np.zeros(0, np.uint32), empty_first, np.zeros(6, np.uint32)))
    # only segments the join folds itself (<= 48 B: the checksum pass gets no record at
    # all), and lengths around that split (47 / 48 / 49 B)
    for lo, hi in ((1, 49), (47, 50)):
        sl = rng.integers(lo, hi, size=4000).astype(np.uint32)
        so = rng.integers(0, len(payload) - 100, size=4000).astype(np.uint64)
        f = np.arange(0, 4001, 4, dtype=np.uint32)
        cases.append((payload, so, sl, f, oracle_lib.gather(payload, so, sl, f)))
    # an average of exactly 3 segments per DGRAM that only every other DGRAM has (2, 4, 2,
    # 4, ...): the join's guess of DGRAM d's first segment (3 d) is wrong half the time
    cnt2 = np.tile(np.array([2, 4], np.uint32), 1500)
    sf2 = np.zeros(len(cnt2) + 1, np.uint32)
    np.cumsum(cnt2, out=sf2[1:])
    ns2 = int(sf2[-1])
    sl2 = rng.integers(1, 1500, size=ns2).astype(np.uint32)
    so2 = rng.integers(0, len(payload) - 1500, size=ns2).astype(np.uint64)
    cases.append((payload, so2, sl2, sf2, oracle_lib.gather(payload, so2, sl2, sf2)))
    return cases


def test_gather_binned(ctx, golden, oracle_lib):
    """enet_hip_crc32_gather_binned_device (send-side gather lists, protocol.cs:1690-1698):
    the golden multi-buffer vectors, cfg5's 3-segment DGRAMs, random gather lists of 0-65
    segments (empty segments and empty DGRAMs among them, arbitrary byte alignment,
    segments shared between DGRAMs), a list of only empty DGRAMs, lists of only short
    segments (folded by the join) and of lengths around the join's 48-byte split, each
    against the oracle's gather, at the default, 4 and 8 lanes and 1 / 2 workgroups per CU."""
    cases = _gather_cases(golden, oracle_lib)
    try:
        for lanes, wgs in ((0, 0), (4, 0), (8, 0), (0, 1), (0, 2)):
            ctx.set_tuning(lanes, wgs)
            for i, (p, so, sl, f, e) in enumerate(cases):
                got = _run_gather_binned(ctx, p, so, sl, f)
                assert (got == e).all(), (lanes, i, np.nonzero(got != e)[0][:5])
    finally:
        ctx.set_tuning(0, 0)


def test_gather_split_join_diagnostics(dctx, golden, oracle_lib):
    """The split join (diagnostics 4194304, gather_join.hpp: the short segments folded
    beside the binning tiles, each long segment's CRC XORed in afterwards with
    x^(8 bytes after it)) -- measured slower than the one-pass join and kept out of the
    product -- on every test_gather_binned list at 4 and 8 lanes, against the oracle."""
    cases = _gather_cases(golden, oracle_lib)
    try:
        dctx.diag_ablation(4194304)
        for lanes in (0, 4):
            dctx.set_tuning(lanes, 0)
            for i, (p, so, sl, f, e) in enumerate(cases):
                got = _run_gather_binned(dctx, p, so, sl, f)
                assert (got == e).all(), (lanes, i, np.nonzero(got != e)[0][:5])
    finally:
        dctx.diag_ablation(0)
        dctx.set_tuning(0, 0)


def test_gather_binned_back_to_back_and_graph(ctx, oracle_lib):
    """The binned gather's three passes (bin, records checksum, join) over workspaces that
    calls reuse: 12 calls back to back on one non-default stream without a sync, three
    batches with their own output / workspace pairs in turn (one of them with more empty
    DGRAMs than segments), then the same calls captured in a CUDA graph and replayed
    twice.  Every output against the oracle."""
    g1, g2 = workloads.cfg5(messages=64), workloads.cfg5(messages=48, message_bytes=20000)
    rng = np.random.default_rng(5)
    sf3 = np.zeros(41, np.uint32)                             # 40 DGRAMs, 6 segments: dgramCount > segCount + 2
    sf3[35:] = np.arange(1, 7, dtype=np.uint32)
    so3 = rng.integers(0, 4000, size=6).astype(np.uint64)
    sl3 = np.array([1360, 24, 0, 8, 300, 49], np.uint32)
    p3 = rng.integers(0, 256, size=8192, dtype=np.uint8)
    batches = []
    for p, so, sl, sf in ((g1.payload, g1.seg_off, g1.seg_len, g1.seg_first),
                          (g2.payload, g2.seg_off, g2.seg_len, g2.seg_first), (p3, so3, sl3, sf3)):
        n, ns = len(sf) - 1, int(sf[-1])
        wsb = ctx.gather_binned_workspace_size(ns)
        batches.append(dict(p=dev(p), so=dev(so), sl=dev(sl), sf=dev(sf), n=n, ns=ns, wsb=wsb,
                            ws=torch.zeros(wsb, dtype=torch.uint8, device="cuda"),
                            out=torch.full((n,), -1, dtype=torch.int32, device="cuda"),
                            exp=oracle_lib.gather(p, so, sl, sf)))
    st = torch.cuda.Stream()

    def call(b):
        ctx.gather_binned_device(b["p"], b["so"], b["sl"], b["ns"], b["sf"], b["n"], b["out"], b["ws"], b["wsb"],
                                 stream=st.cuda_stream)

    def check():
        for b in batches:
            got = b["out"].cpu().numpy().view(np.uint32)
            assert (got == b["exp"]).all(), np.nonzero(got != b["exp"])[0][:5]
            b["out"].fill_(-1)
        torch.cuda.synchronize()

    torch.cuda.synchronize()
    for i in range(12):
        call(batches[i % 3])
    st.synchronize()
    check()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph, stream=st):
        for i in range(6):
            call(batches[i % 3])
    for _ in range(2):
        graph.replay()
        torch.cuda.synchronize()
        check()


def test_bad_tuning_raises(ctx):
    with pytest.raises(enethip.ENetHipError):
        ctx.set_tuning(3, 0)


@pytest.mark.parametrize("wgs", WGS)
@pytest.mark.parametrize("path", (0, 17, 18, 19, 20, 21))
def test_vring_many_groups(ctx, dctx, oracle_lib, path, wgs):
    """The default VGPR-ring kernel (4 and 8 lanes, one or two workgroups per CU):
    tiny packets (one-stage groups, the producer switching group every stage, empty
    packets among them), long ones (many stages per group, the tail-first order's
    last stage far from the rest) and cfg2-shaped packed MTU packets, each against
    the oracle.  18: nontemporal stage loads; 19, 20: walks; 21: the tail-first stage order."""
    tiny = workloads.mixed(1_200_000, 0, 40, seed=177, len_seed=178)
    exp_t = oracle_lib.batch(tiny.payload, tiny.off, tiny.lens, threads=16)
    big = workloads.mixed(40_000, 2000, 9000, seed=179, len_seed=180)
    exp_b = oracle_lib.batch(big.payload, big.off, big.lens, threads=16)
    mtu = workloads.mixed(100_000, 1200, 1200, seed=181, len_seed=182)
    exp_m = oracle_lib.batch(mtu.payload, mtu.off, mtu.lens, threads=16)
    ctx = on(ctx, dctx, path)
    try:
        ctx.set_kernel_path(path)
        for lanes in (4, 8):
            assert (run_batch(ctx, tiny.payload, tiny.off, tiny.lens, lanes, wgs) == exp_t).all(), ("tiny", lanes)
            assert (run_batch(ctx, big.payload, big.off, big.lens, lanes, wgs) == exp_b).all(), ("big", lanes)
            assert (run_batch(ctx, mtu.payload, mtu.off, mtu.lens, lanes, wgs) == exp_m).all(), ("mtu", lanes)
    finally:
        ctx.set_kernel_path(0)
        ctx.set_tuning(0, 0)


def test_product_library_rejects_sweep_paths(ctx):
    """libenethip.so builds no sweep path and no lane count but 4 and 8 (the direct
    and LDS-stream kernels, paths 1 / 2 and 1, 2, 16, 32, 64 lanes, exist in
    libenethip_diag.so only since round 5)."""
    for path in (1, 2, 3, 8, 14, 18, 19, 20, 21, 22, 23):
        with pytest.raises(enethip.ENetHipError):
            ctx.set_kernel_path(path)
    ctx.set_kernel_path(0)
    for lanes in (1, 2, 16, 32, 64):
        with pytest.raises(enethip.ENetHipError):
            ctx.set_tuning(lanes, 0)
    for lanes in (0, 4, 8):
        ctx.set_tuning(lanes, 0)
    ctx.set_tuning(0, 0)


def _batch_list_cases(oracle_lib):
    """(payload, off, lens, expected) per batch: empty, single packets, golden-like
    small lengths, cfg2-shaped MTU packets, long packets, tiny packets."""
    specs = [(0, 0, 0, 1), (1, 0, 0, 2), (1, 1, 1, 3), (17, 0, 64, 4), (65_536, 1200, 1200, 5),
             (3000, 2000, 9000, 6), (250_000, 0, 40, 7), (5, 31, 33, 8), (70_000, 1, 1400, 9)]
    out = []
    for n, lo, hi, seed in specs:
        b = workloads.mixed(n, lo, hi, seed=300 + seed, len_seed=400 + seed) if n else None
        if b is None:
            out.append((np.zeros(16, np.uint8), np.zeros(0, np.uint64), np.zeros(0, np.uint32),
                        np.zeros(0, np.uint32)))
        else:
            out.append((b.payload, b.off, b.lens, oracle_lib.batch(b.payload, b.off, b.lens, threads=16)))
    return out


def _run_list(ctx, cases):
    keep, descs, outs = [], [], []
    for payload, off, lens, _ in cases:
        d = (dev(payload if len(payload) else np.zeros(16, np.uint8)),
             dev(off) if len(off) else dev(np.zeros(1, np.uint64)),
             dev(lens) if len(lens) else dev(np.zeros(1, np.uint32)))
        o = torch.full((max(1, len(off)),), -1, dtype=torch.int32, device="cuda")
        keep.append(d)
        outs.append(o)
        descs.append((d[0], d[1], d[2], len(off), o))
    ctx.crc32_batch_list_device(descs, stream=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    return [o.cpu().numpy().view(np.uint32)[:len(c[1])] for o, c in zip(outs, cases)]


LIST_PATHS = (0, 13, 19, 20, 21)  # 0: the vring kernel (default), 13: the lean kernel's list instance,
                                  # 19 / 20: vring with workgroups walking contiguous ranges, 21: tail first


@pytest.mark.parametrize("wgs", WGS)
@pytest.mark.parametrize("path", LIST_PATHS)
def test_batch_list(ctx, dctx, oracle_lib, path, wgs):
    """enet_hip_crc32_batch_list_device: batches of every shape in one launch,
    each against the oracle; vring (path 0) or lean (13) lists at the default, 4 and
    8 lanes, one or two workgroups per CU; 16 lanes (one launch per batch on the
    stream kernel)."""
    cases = _batch_list_cases(oracle_lib)
    try:
        for lanes in (0, 4, 8, 16):
            c = on(ctx, dctx, path, lanes)
            c.set_kernel_path(path)
            c.set_tuning(lanes, wgs)
            for i, (got, cs) in enumerate(zip(_run_list(c, cases), cases)):
                assert (got == cs[3]).all(), (path, lanes, i, np.nonzero(got != cs[3])[0][:5])
    finally:
        for c in (ctx, dctx):
            c.set_kernel_path(0)
            c.set_tuning(0, 0)


@pytest.mark.parametrize("wgs", WGS)
@pytest.mark.parametrize("path", LIST_PATHS)
def test_batch_list_many_launches(ctx, dctx, oracle_lib, path, wgs):
    """More batches than one launch takes (48): 110 small batches of varied sizes,
    plus the reverse order (the grid is sized by the largest batch)."""
    rng = np.random.default_rng(55)
    cases = []
    for i in range(110):
        n = int(rng.integers(0, 3000))
        b = workloads.mixed(n, 0, 1500, seed=500 + i, len_seed=600 + i) if n else None
        if b is None:
            cases.append((np.zeros(16, np.uint8), np.zeros(0, np.uint64), np.zeros(0, np.uint32),
                          np.zeros(0, np.uint32)))
        else:
            cases.append((b.payload, b.off, b.lens, oracle_lib.batch(b.payload, b.off, b.lens, threads=16)))
    ctx = on(ctx, dctx, path)
    try:
        ctx.set_kernel_path(path)
        ctx.set_tuning(0, wgs)
        for order in (cases, cases[::-1]):
            for i, (got, c) in enumerate(zip(_run_list(ctx, order), order)):
                assert (got == c[3]).all(), (path, i, len(c[1]))
    finally:
        ctx.set_kernel_path(0)
        ctx.set_tuning(0, 0)


def test_vring_trace_instance(dctx, oracle_lib):
    """The diagnostics (trace) instance of the vring kernel computes the same CRCs
    and fills one 8 x u64 record per wave."""
    ctx = dctx
    b = workloads.mixed(100_000, 0, 3000, seed=91, len_seed=92)
    exp = oracle_lib.batch(b.payload, b.off, b.lens, threads=16)
    # 8 x u64 per wave: up to 2 workgroups per CU (the default) x 16 waves
    props = torch.cuda.get_device_properties(0)
    tr = torch.zeros(2 * props.multi_processor_count * 16 * 8, dtype=torch.int64, device="cuda")
    ctx.diag_trace(tr)
    try:
        for lanes in (4, 8):
            tr.zero_()
            assert (run_batch(ctx, b.payload, b.off, b.lens, lanes) == exp).all(), lanes
            t = tr.cpu().numpy().view(np.uint64).reshape(-1, 8)
            live = t[t[:, 0] > 0]
            assert len(live) > 0 and (live[:, 5] >= live[:, 0]).all()
            assert int(live[:, 7].sum()) == (len(b.off) + (64 // lanes) - 1) // (64 // lanes)
    finally:
        ctx.diag_trace(None)
        ctx.set_tuning(0, 0)


@pytest.mark.parametrize("wgs", WGS)
def test_all_empty_groups_every_path(ctx, dctx, oracle_lib, wgs):
    """Groups whose packets are all empty (a stage count of zero before the
    clamp): a lone empty packet, a batch of empty packets, and runs of empty
    packets amid others -- every lane count, the default and direct paths, and
    every stream geometry."""
    rng = np.random.default_rng(66)
    lens = rng.integers(0, 300, size=4000).astype(np.uint32)
    lens[100:300] = 0                          # empty runs longer than any group
    lens[1000:1064] = 0
    lens[-70:] = 0                             # the batch ends in empty groups
    off = np.zeros(len(lens), np.uint64)
    np.cumsum(lens[:-1].astype(np.uint64), out=off[1:])
    payload = rng.integers(0, 256, size=int(lens.astype(np.uint64).sum()) + 16, dtype=np.uint8)
    exp = oracle_lib.batch(payload, off, lens, threads=8)
    cases = [(np.zeros(16, np.uint8), np.zeros(1, np.uint64), np.zeros(1, np.uint32), np.zeros(1, np.uint32)),
             (np.zeros(16, np.uint8), np.zeros(64, np.uint64), np.zeros(64, np.uint32), np.zeros(64, np.uint32)),
             (payload, off, lens, exp)]
    paths = [0, 1, 17] if wgs else [0, 1] + [2 + g for g in range(N_STREAM_GEOMS)] + [17, 18, 21]
    for path in paths:
        try:
            for lanes in (1, 2, 4, 8, 16, 32, 64):
                c = on(ctx, dctx, path, lanes)
                c.set_kernel_path(path)
                for i, (p, o, l, e) in enumerate(cases):
                    got = run_batch(c, p, o, l, lanes, wgs)
                    assert (got == e).all(), (path, lanes, i, np.nonzero(got != e)[0][:5])
        finally:
            for c in (ctx, dctx):
                c.set_kernel_path(0)
                c.set_tuning(0, 0)


def test_verify_dgrams_over_64k(ctx, oracle_lib):
    """Receive verify has no length limit of its own (protocol.cs:1052-1068 CRCs
    receivedDataLength bytes): DGRAMs of 64 KiB - 1 .. 200 000 B, stamped and
    corrupted, through the single-batch, list and binned entries, against the
    oracle's verify (which holds no 64 KiB limit either)."""
    rng = np.random.default_rng(65)
    lens = np.array([65535, 65536, 65537, 70000, 131072, 200000, 100, 65540], np.uint32)
    n = len(lens)
    slot = np.array([4, 2, 4, 4, 2, 4, 4, 2], np.uint32)
    conn = rng.integers(0, 2**32, size=n, dtype=np.uint64).astype(np.uint32)
    off = np.zeros(n, np.uint64)
    np.cumsum(lens[:-1].astype(np.uint64) + np.uint64(3), out=off[1:])
    payload = rng.integers(0, 256, size=int(off[-1] + lens[-1]) + 16, dtype=np.uint8)
    for i in range(n):
        o, s = int(off[i]), int(slot[i])
        payload[o + s:o + s + 4] = np.frombuffer(np.uint32(conn[i]).tobytes(), np.uint8)
    stamped = oracle_lib.batch(payload, off, lens, threads=8)
    for i in range(n):
        o, s = int(off[i]), int(slot[i])
        payload[o + s:o + s + 4] = np.frombuffer(np.uint32(stamped[i]).tobytes(), np.uint8)
    payload[int(off[3]) + 66000] ^= np.uint8(4)              # corrupt one long DGRAM
    exp_ok, exp_comp = oracle_lib.verify(payload, off, lens, slot, conn)
    assert exp_ok.tolist() == [1, 1, 1, 0, 1, 1, 1, 1]
    for lanes in (0, 4, 8):
        ctx.set_tuning(lanes, 0)
        d_ok = torch.zeros(n, dtype=torch.uint8, device="cuda")
        d_comp = torch.zeros(n, dtype=torch.int32, device="cuda")
        ctx.verify_batch_device(dev(payload), dev(off), dev(lens), dev(slot), dev(conn), n, d_ok, d_comp,
                                stream=torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        assert (d_ok.cpu().numpy() == exp_ok).all(), lanes
        assert (d_comp.cpu().numpy().view(np.uint32) == exp_comp).all(), lanes
        (ok_l, comp_l), = _run_verify_list(ctx, [(payload, off, lens, slot, conn, exp_ok, exp_comp)])
        assert (ok_l == exp_ok).all() and (comp_l == exp_comp).all(), ("list", lanes)
        wsb = ctx.verify_binned_workspace_size(n)
        ws = torch.zeros(wsb, dtype=torch.uint8, device="cuda")
        d_ok.zero_()
        ctx.verify_batch_device_binned(dev(payload), dev(off), dev(lens), dev(slot), dev(conn), n, d_ok, ws, wsb,
                                       d_comp, stream=torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        assert (d_ok.cpu().numpy() == exp_ok).all(), ("binned", lanes)
    ctx.set_tuning(0, 0)


# ---- dynamic rounds (crc32_vring.hip: rounds >= 2 claimed from a per-launch counter)

def test_dynamic_rounds_claim_lines_reused_across_streams(dctx, oracle_lib):
    """More launches than the context's 256 claim lines, spread over three streams at
    once, batch sizes from one group to several rounds per workgroup and lanes 4 / 8:
    every launch's CRCs are exact (a claim line left non-zero, or shared by two
    running launches, would skip or repeat chunks)."""
    rng = np.random.default_rng(0xD1)
    sizes = [1, 7, 9, 300, 4096, 20000, 65536]
    batches = []
    for i, n in enumerate(sizes):
        lens = rng.integers(0, 1500, n).astype(np.uint32)
        off = np.zeros(n, np.uint64)
        off[1:] = np.cumsum(lens[:-1].astype(np.uint64))
        payload = np.frombuffer(rng.bytes(int(lens.sum()) + 64), np.uint8).copy()
        batches.append((dev(payload), dev(off), dev(lens), n, oracle_lib.batch(payload, off, lens, threads=16)))
    streams = [torch.cuda.Stream() for _ in range(3)]
    ctx = dctx
    try:
        for mode in (524288, 8388608):                # the chip-wide and the pair rounds
            ctx.diag_ablation(mode)
            for lanes in (8, 4):
                ctx.set_tuning(lanes, 0)
                outs = []
                for k in range(300):
                    d_p, d_o, d_l, n, exp = batches[k % len(batches)]
                    st = streams[k % 3]
                    out = torch.full((n,), -1, dtype=torch.int32, device="cuda")
                    st.wait_stream(torch.cuda.current_stream())      # (the fill first: the side streams do not wait)
                    with torch.cuda.stream(st):
                        ctx.crc32_batch_device(d_p, d_o, d_l, n, out, stream=st.cuda_stream)
                    outs.append((out, exp, k))
                torch.cuda.synchronize()
                for out, exp, k in outs:
                    assert (out.cpu().numpy().view(np.uint32) == exp).all(), (mode, lanes, k)
    finally:
        ctx.diag_ablation(0)
        ctx.set_tuning(0, 0)


def test_dynamic_rounds_graph_capture_replays(dctx, oracle_lib):
    """a dynamic-rounds launch captured in a graph would replay its
    one {claim line, generation} and skip chunks on the second replay.  Under capture
    the entry takes the static deal (crc32_kernels.hip with_claim): the captured
    launches, replayed three times, stay exact in both dynamic modes and lane counts."""
    rng = np.random.default_rng(0xD2)
    n = 20000
    lens = rng.integers(0, 1500, n).astype(np.uint32)
    off = np.zeros(n, np.uint64)
    off[1:] = np.cumsum(lens[:-1].astype(np.uint64))
    payload = np.frombuffer(rng.bytes(int(lens.sum()) + 64), np.uint8).copy()
    exp = oracle_lib.batch(payload, off, lens, threads=16)
    d_p, d_o, d_l = dev(payload), dev(off), dev(lens)
    st = torch.cuda.Stream()
    try:
        for mode in (524288, 8388608):
            dctx.diag_ablation(mode)
            for lanes in (8, 4):
                dctx.set_tuning(lanes, 0)
                out = torch.full((n,), -1, dtype=torch.int32, device="cuda")
                torch.cuda.synchronize()
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, stream=st):
                    dctx.crc32_batch_device(d_p, d_o, d_l, n, out, stream=st.cuda_stream)
                for rep in range(3):
                    out.fill_(-1)
                    g.replay()
                    torch.cuda.synchronize()
                    assert (out.cpu().numpy().view(np.uint32) == exp).all(), (mode, lanes, rep)
                del g
    finally:
        dctx.diag_ablation(0)
        dctx.set_tuning(0, 0)


def test_dynamic_rounds_match_static_deal(dctx, oracle_lib):
    """The dynamic rounds (diagnostics ablation 524288: CRCs still exact) and the static
    deal give the same CRCs on cfg3's mixed lengths, single batches and lists."""
    b = workloads.mixed(262144, 64, 1400, seed=0x44594E, name="cfg3")
    exp = oracle_lib.batch(b.payload, b.off, b.lens, threads=16)
    try:
        for mode in (0, 524288, 8388608):         # static, chip-wide rounds, pair rounds
            dctx.diag_ablation(mode)
            dctx.set_kernel_path(0)
            got = run_batch(dctx, b.payload, b.off, b.lens)
            assert (got == exp).all(), mode
    finally:
        dctx.diag_ablation(0)
        dctx.set_tuning(0, 0)



def test_gather_binned_short_segment_bounds(dctx, golden, oracle_lib):
    """The binned gather with other short-segment bounds (diagnostics A/B: segments of
    at most b bytes folded by the join, the rest binned), b = 0, 8, 24 and the default,
    on test_gather_binned's lists: the split moves, the CRCs do not."""
    cases = _gather_cases(golden, oracle_lib)
    try:
        for b in (0, 8, 24, 48):
            dctx.diag_ablation(16777216 * (1 + b) if b < 48 else 0)
            for i, (p, so, sl, f, e) in enumerate(cases):
                got = _run_gather_binned(dctx, p, so, sl, f)
                assert (got == e).all(), (b, i, np.nonzero(got != e)[0][:5])
    finally:
        dctx.diag_ablation(0)


def test_binned_memory_order_diagnostic(dctx, golden, oracle_lib):
    """The binned entry with its records left in memory order (diagnostics 2^30, the
    A/B that prices the length sort): the records instance still writes every CRC to
    its caller index -- cfg3, the golden vectors and every bin with empties."""
    b = workloads.cfg3()
    exp = oracle_lib.batch(b.payload, b.off, b.lens, threads=16)
    payload, off, lens, exp_g = golden_batch(golden)
    rng = np.random.default_rng(41)
    n = 20000
    e_lens = rng.integers(0, 9000, size=n).astype(np.uint32)
    e_lens[:64] = 0
    e_off = rng.integers(0, 1 << 20, size=n).astype(np.uint64)
    e_pay = rng.integers(0, 256, size=(1 << 20) + 9000, dtype=np.uint8)
    exp_e = oracle_lib.batch(e_pay, e_off, e_lens, threads=8)
    try:
        dctx.diag_ablation(1 << 30)
        for lanes in (4, 8):
            assert (run_binned(dctx, b.payload, b.off, b.lens, lanes) == exp).all(), ("cfg3", lanes)
            assert (run_binned(dctx, payload, off, lens, lanes) == exp_g).all(), ("golden", lanes)
            assert (run_binned(dctx, e_pay, e_off, e_lens, lanes) == exp_e).all(), ("edges", lanes)
    finally:
        dctx.diag_ablation(0)
