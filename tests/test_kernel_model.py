"""CPU checks of the kernel's algebra and LDS schedule (see tests/kernel_model.py).

These run without a GPU: they prove the lane schedule is conflict-free by
construction and that the windowing / INIT / carry-combine arithmetic reproduces
the oracle bit for bit.  The -m gpu tests then check the hardware does the same.
"""
import random

import pytest

import kernel_model as km
import oracle


def test_slicing_tables_and_image():
    # T_t[j] is byte j followed by t zero bytes
    for t in (0, 1, 7, 31):
        for j in (0, 1, 0x80, 0xFF):
            reg = 0
            reg = (reg >> 8) ^ km.T0[(reg ^ j) & 0xFF]
            for _ in range(t):
                reg = (reg >> 8) ^ km.T0[reg & 0xFF]
            assert km.TS[t][j] == reg
    img = km.image(1)
    assert img[64 * 5 + km.col_byte(9) // 4] == km.TS[9][5]
    assert img[64 * 5 + km.col_byte(20) // 4] == km.TS[20][5]
    # advancing tables: T'_t = T_{t + 32(P-1)}
    img4 = km.image(4)
    ref = km.TS[3][7]
    for _ in range(96):
        ref = km.zstep(ref)
    assert img4[64 * 7 + km.col_byte(3) // 4] == ref


def test_free_columns_disjoint_from_tables():
    used = {km.col_byte(t) for t in range(32)}
    free = {km.free_col(c) for c in range(32)}
    assert not (used & free) and len(used | free) == 64
    img = km.image(8)
    for r in range(32):
        assert img[km.init_addr(r) // 4] == km.INIT[r]
    for i in (0, 1, 31, 200, 255, 256, 511):
        assert img[km.cinv_addr(i) // 4] == km.CINV[i]
    rng = random.Random(9)
    for k in range(1, 8):
        for _ in range(10):
            v = rng.getrandbits(32)
            got = 0
            for b in range(4):
                got ^= img[km.corr_addr(k, b, (v >> (8 * b)) & 0xFF) // 4]
            assert got == km.mulmod(v, km.CINV[32 * k])


def test_cinv_inverts_x8n():
    for n in (0, 1, 2, 31, 32, 100, 511):
        assert km.mulmod(km.CINV[n], km.x8n(n)) == km.ONE


def test_lds_bank_conflict_free():
    """Every lookup instruction: the 32 lanes of each half-wave hit 32 distinct banks
    (ds_read_b32: bank = (addr/4) mod 32, lane groups 0-31 and 32-63)."""
    rng = random.Random(1)
    for _ in range(20):
        words = [rng.getrandbits(32) for _ in range(8)]
        per_lane = [km.lookup_addresses(l, words) for l in range(64)]
        for i in range(32):
            for g in (range(0, 32), range(32, 64)):
                banks = {(per_lane[l][i] // 4) % 32 for l in g}
                assert len(banks) == 32, (i, sorted(banks))


def test_each_lane_reads_every_byte_once():
    rng = random.Random(2)
    block = bytes(rng.getrandbits(8) for _ in range(32))
    words = [int.from_bytes(block[4 * q:4 * q + 4], "little") for q in range(8)]
    inv = {km.col_byte(t): t for t in range(32)}
    for lane in range(64):
        addrs = km.lookup_addresses(lane, words)
        used = set()
        for a in addrs:
            row, t = a // 256, inv[a % 256]
            m = t ^ 31
            assert block[m] == row      # looked-up row is byte m of the block
            used.add(m)
        assert used == set(range(32))


def test_fold_block_equals_sarwate():
    rng = random.Random(3)
    for lane in (0, 5, 17, 33, 63):
        for _ in range(5):
            block = bytes(rng.getrandbits(8) for _ in range(32))
            reg = rng.getrandbits(32)
            ref = reg
            for b in block:
                ref = (ref >> 8) ^ km.T0[(ref ^ b) & 0xFF]
            assert km.fold_block(reg, block, lane) == ref


def test_init_states():
    for r in range(32):
        reg = km.INIT[r]
        for _ in range(r):
            reg = (reg >> 8) ^ km.T0[reg & 0xFF]
        assert reg == 0xFFFFFFFF


def test_mulmod_is_zero_advance():
    rng = random.Random(4)
    for n in (0, 1, 3, 32, 100, 1200):
        for _ in range(3):
            r = rng.getrandbits(32)
            ref = r
            for _ in range(n):
                ref = (ref >> 8) ^ km.T0[ref & 0xFF]
            assert km.mulmod(r, km.x8n(n)) == ref


@pytest.mark.parametrize("lanes", [1, 2, 4, 8, 64])
def test_direct_packet_model_matches_oracle(lanes):
    rng = random.Random(10 + lanes)
    for L in [0, 1, 3, 4, 15, 16, 17, 31, 32, 33, 63, 64, 65, 100, 257, 1200, 1201]:
        pkt = bytes(rng.getrandbits(8) for _ in range(L))
        for addr in (0, 16, 1200 * 7, 4093):
            assert km.crc_packet(pkt, lanes, addr=addr) == oracle.enet_crc32_py([pkt]), (L, lanes, addr)


@pytest.mark.parametrize("P", [1, 4, 8, 16])
def test_stream_packet_model_matches_oracle(P):
    rng = random.Random(100 + P)
    for L in [0, 1, 3, 4, 15, 16, 17, 31, 32, 33, 63, 64, 65, 100, 257, 511, 512, 1200, 1201]:
        pkt = bytes(rng.getrandbits(8) for _ in range(L))
        for addr in (0, 1, 15, 16, 1200 * 7, 4093):
            assert km.stream_crc(pkt, P, addr) == oracle.enet_crc32_py([pkt]), (L, P, addr)


def test_segment_cuts_are_line_aligned():
    for addr in range(0, 4096, 48):
        for L in (1200, 1392, 300, 4096):
            for lanes in (2, 4, 8):
                cuts = km.segment_cuts(addr, L, lanes)
                assert cuts == sorted(cuts) and cuts[0] == 0 and cuts[-1] == L
                for c in cuts[1:-1]:
                    assert c in (0, L) or (addr + c) % 128 == 0


def test_verify_model(golden):
    vecs, blob = golden
    n = 0
    for v in vecs:
        if v["kind"] != "verify":
            continue
        o, ln = v["segments"][0]
        pkt = bytes(blob[o:o + ln])
        for P in (4, 8):
            for addr in (0, 5):
                ok, _ = km.stream_verify(pkt, v["slot_off"], int(v["connect_id"], 16), P, addr)
                assert ok == v["expect_ok"]
        n += 1
    assert n > 0


@pytest.mark.parametrize("P", [4, 8])
def test_lean_group_model_matches_oracle(P):
    """crc32_lean.hip's data path (coalesced chunk DMA, own-packet producer,
    permuted conflict-free dword reads, lean lane schedule) equals the reference
    CRC for aligned, unaligned and empty packets and every rotation."""
    import random
    import zlib
    rnd = random.Random(1000 + P)
    npk = 64 // P
    for trial in range(6):
        lens = [rnd.choice([0, 1, 15, 16, 31, 32, 33, 100, 255, 256, 1200, rnd.randint(0, 700)]) for _ in range(npk)]
        offs, pos = [], 48 + rnd.randint(0, 40)
        for L in lens:
            offs.append(pos)
            pos += L + rnd.choice([0, 0, 1, 7, 16])
        arena = bytes(rnd.getrandbits(8) for _ in range(pos + 64))
        got = km.lean_group(arena, offs, lens, P)
        for j in range(npk):
            pkt = arena[offs[j]:offs[j] + lens[j]]
            exp = int.from_bytes((zlib.crc32(pkt) & 0xFFFFFFFF).to_bytes(4, "little"), "big")
            assert got[j] == exp, (trial, j, lens[j], offs[j])


@pytest.mark.parametrize("P", [4, 8])
def test_image_from_basis(P):
    """The lean kernel rebuilds its LDS image from a 9-row basis: equal to the
    host image at every dword it can read (all but INIT/CINV rows >= 32 and CINV
    n >= 256)."""
    img, rb = km.image(P), km.rebuilt_image(P)
    for j in range(256):
        for d in range(64):
            if d == km.KCINV_DWORD + 2 or (d in (km.KINIT_DWORD, km.KCINV_DWORD) and j >= 32):
                continue
            assert rb[64 * j + d] == img[64 * j + d], (j, d)


def test_binned_order_is_a_permutation_and_balances_groups():
    """bin_tile_kernel's placement (crc32_lean.hip): a permutation that keeps each tile's
    records ordered by length, and on cfg3-like lengths cuts the lean kernel's work
    (sum of group maxima, in stages) well below the unbinned batch's."""
    rng = random.Random(5)
    n = 4 * 1024 + 300                                     # 4 full tiles + a ragged one
    lens = [rng.randint(64, 1400) for _ in range(n)]
    for lanes in (4, 8):
        kpk = 64 // lanes
        order = km.binned_order(lens, kpk)
        assert sorted(order) == list(range(n))
        full = n // 1024
        for t in range(full):                              # tile t's records in position order
            mine = [i for i in order if i // 1024 == t]
            bins = [km.bin_of(lens[i]) for i in mine]
            assert bins == sorted(bins)
            assert all(order.index(i) // kpk % full == t for i in mine[:64])
        plain = km.group_stage_cost(lens, list(range(n)), kpk, lanes)
        binned = km.group_stage_cost(lens, order, kpk, lanes)
        assert binned < 0.7 * plain, (lanes, binned, plain)


@pytest.mark.parametrize("P", [4, 8])
def test_vring_image_from_basis(P):
    """crc32_vring.hip rebuilds its LDS image from the 10-row basis2: equal to the
    host image wherever that kernel reads (INIT / CINV rows < 64, CINV n < 256)."""
    img, rb = km.image(P), km.vring_image(P)
    for j in range(256):
        for d in range(64):
            if d == km.KCINV_DWORD + 2 or (d in (km.KINIT_DWORD, km.KCINV_DWORD) and j >= 64):
                continue
            assert rb[64 * j + d] == img[64 * j + d], (j, d)


@pytest.mark.parametrize("P", [4, 8])
def test_vring_model_matches_oracle(P):
    """The vring kernel's arithmetic (64-byte-aligned window starts, zero-line
    pieces, edge masks, strided advancing folds, lane overshoot corrections
    x^(-256 o), tz correction) equals packet.cs:142-160 for every start alignment
    mod 64 and lengths across block / stage boundaries, empty packets included."""
    rng = random.Random(0x5652 + P)
    arena = bytes(rng.getrandbits(8) for _ in range(16384))
    ol = oracle.OracleLib()
    cases = [(a, L) for a in range(0, 64, 5) for L in (0, 1, 15, 16, 17, 31, 32, 33, 63, 64, 65)]
    cases += [(rng.randrange(0, 2048), rng.randrange(0, 1500)) for _ in range(40)]
    cases += [(1200 * i, 1200) for i in range(8)]          # cfg2 shapes
    for a, L in cases:
        lane_base = P * rng.randrange(0, 64 // P)
        got = km.vring_packet(arena, 128 + a, L, P, lane_base)
        exp = ol.crc32(arena[128 + a:128 + a + L])
        assert got == exp, (a, L, P, hex(got), hex(exp))


@pytest.mark.parametrize("P", [4, 8])
def test_vring_end_aligned_model_matches_oracle(P):
    """The records instance's end-aligned windows (the last block ends on the packet's
    last byte: no trailing zero bytes to undo, no tail edge; lz = 32 nb - L leading zero
    bytes, the partly covered head piece masked): equal to packet.cs:142-160 for every
    start and end alignment, lengths across block and stage boundaries, empty packets,
    and packets shorter than their group."""
    rng = random.Random(0x4541 + P)
    arena = bytes(rng.getrandbits(8) for _ in range(16384))
    ol = oracle.OracleLib()
    cases = [(a, L, 0) for a in range(0, 64, 3) for L in (0, 1, 15, 16, 17, 31, 32, 33, 63, 64, 65, 255, 257)]
    cases += [(rng.randrange(0, 2048), rng.randrange(0, 3000), rng.randrange(0, 14)) for _ in range(60)]
    for a, L, gs in cases:
        ws, lz, e, nb = km.vring_window(128 + a, L, True)
        assert e == 32 * nb and 0 <= lz < 32 and ws + lz == 128 + a
        lane_base = P * rng.randrange(0, 64 // P)
        got = km.vring_packet(arena, 128 + a, L, P, lane_base, group_stages=gs, end_aligned=True)
        exp = ol.crc32(arena[128 + a:128 + a + L])
        assert got == exp, (a, L, P, gs, hex(got), hex(exp))


@pytest.mark.parametrize("P", [4, 8])
def test_vring_tail_first_model_matches_oracle(P):
    """The vring kernel's tail-first stage order (the group's last stage folded
    first, from a zero register into rt; the others in order; then rt ^ adv(reg),
    adv = four lookups in T'_31 .. T'_28): equal to packet.cs:142-160 for every
    start alignment, lengths across stage boundaries, empty packets, and packets
    shorter than their group (whose own last stage is not the group's)."""
    rng = random.Random(0x5254 + P)
    arena = bytes(rng.getrandbits(8) for _ in range(16384))
    ol = oracle.OracleLib()
    cases = [(a, L, 0) for a in range(0, 64, 7) for L in (0, 1, 17, 32, 33, 255, 256, 257, 511, 1200, 1400)]
    cases += [(rng.randrange(0, 2048), rng.randrange(0, 3000), rng.randrange(0, 14)) for _ in range(40)]
    cases += [(1200 * i, 1200, 0) for i in range(8)]        # cfg2 shapes
    assert km.vring_stage_order(5, True) == [4, 0, 1, 2, 3] and km.vring_stage_order(1, True) == [0]
    for a, L, gs in cases:
        lane_base = P * rng.randrange(0, 64 // P)
        got = km.vring_packet(arena, 128 + a, L, P, lane_base, rotate=True, group_stages=gs)
        exp = ol.crc32(arena[128 + a:128 + a + L])
        assert got == exp, (a, L, P, gs, hex(got), hex(exp))


@pytest.mark.parametrize("snake", [False, True])
@pytest.mark.parametrize("batch_groups,grid", [([4096] * 5, 512), ([1], 1), ([0, 3, 0, 17], 2),
                                               ([5000, 1, 70, 2, 800], 300), ([33] * 48, 7), ([16384], 256),
                                               ([16383], 256), ([1000], 17)])
def test_vring_dynamic_slots_cover_every_group_once(batch_groups, grid, snake):
    """The vring kernel's dynamic slots (crc32_vring.hip slot_group / take / locate):
    whatever order a workgroup's waves take slots in, every group of every batch is
    processed exactly once, in its own batch, and each wave's groups ascend -- with the
    records instance's reversed odd rounds (snake) too, partial last rounds included."""
    import random
    from kernel_model import vring_dynamic_deal
    rng = random.Random(sum(batch_groups) + grid)
    nonempty = [n for n in batch_groups if n]                 # (the host drops empty batches)
    grid = max(1, min(grid, (sum(nonempty) + 15) // 16))      # (the host's grid rule)
    seen, per_wave, total = vring_dynamic_deal(nonempty, grid, rng, snake=snake)
    assert sorted(seen) == list(range(total))
    g0 = [sum(nonempty[:b]) for b in range(len(nonempty))]
    for gg, (b, local) in seen.items():
        assert 0 <= local < nonempty[b] and g0[b] + local == gg
    assert sum(per_wave) == total


@pytest.mark.parametrize("batch_groups,grid", [([512] * 5, 16), ([1], 1), ([0, 3, 0, 17], 2),
                                               ([900, 1, 70, 2, 300], 9), ([33] * 48, 7), ([4000], 3)])
def test_vring_dynamic_rounds_cover_every_group_once(batch_groups, grid):
    """The vring kernel's dynamic rounds (DYN 1, and the pair rounds of DYN 2): whatever the interleaving of all
    workgroups' waves and the completion order of their round claims, every group is
    processed exactly once in its own batch, a wave's groups ascend, no wave waits
    forever and no round-table entry is rewritten while it is still to be read."""
    import random
    from kernel_model import vring_dynamic_rounds_deal
    nonempty = [n for n in batch_groups if n]
    grid = max(1, min(grid, (sum(nonempty) + 15) // 16))
    for seed in range(3):
        rng = random.Random(seed * 7919 + sum(batch_groups) + grid)
        for pairs in (False, True):
            g = grid
            if pairs:                              # (the host: an even grid of at least 2)
                if g < 2:
                    continue
                g &= ~1
            seen, per_wave, total = vring_dynamic_rounds_deal(nonempty, g, rng, pairs=pairs)
            assert sorted(seen) == list(range(total))
            g0 = [sum(nonempty[:b]) for b in range(len(nonempty))]
            for gg, (b, local) in seen.items():
                assert 0 <= local < nonempty[b] and g0[b] + local == gg
            assert sum(per_wave) == total


def test_gather_join_matches_oracle(oracle_lib):
    """The binned gather's join (crc32_gather_join_kernel, restated as
    km.gather_join) turns per-segment CRCs into the DGRAM's enet_crc32 over the
    concatenated buffers (packet.cs:142-160 walking the gather list), for lists of
    0-6 segments with empty ones among them, against the oracle."""
    rng = random.Random(2024)
    for _ in range(300):
        segs = [bytes(rng.getrandbits(8) for _ in range(rng.choice([0, 0, 1, 3, 8, 24, 57, 200])))
                for _ in range(rng.randint(0, 6))]
        crcs = [oracle_lib.crc32(s) for s in segs]
        assert km.gather_join(crcs, [len(s) for s in segs]) == oracle_lib.crc32(b"".join(segs))



def test_gather_split_join_matches_oracle(oracle_lib):
    """The split join of the binned gather (gather_join.hpp: pre-join with the long
    segments' registers taken as 0 and x^(8 after) recorded, post-join XOR of each long
    segment's CRC times it) over lists of 0-9 segments mixing short (<= 48 B, folded)
    and long ones in any order, empty ones among them, at every offset mod 4, against
    the oracle's CRC of the concatenation."""
    rng = random.Random(99)
    arena = bytes(rng.getrandbits(8) for _ in range(8192))
    for _ in range(300):
        segs = [(rng.randrange(0, 6000), rng.choice([0, 1, 3, 8, 24, 47, 48, 49, 60, 200, 1360]))
                for _ in range(rng.randint(0, 9))]
        exp = oracle_lib.crc32(b"".join(arena[a:a + L] for a, L in segs))
        assert km.gather_split_join(arena, segs) == exp, segs

def test_unstep_column_is_cinv():
    """The vring kernel's tz correction: tz unsteps through the U column equal the multiply
    by CINV[tz] = x^(-8 tz) for every tz < 32 (random registers), U is a permutation-derived
    table that is GF(2)-linear in its row (so the image basis rebuilds it), and it undoes a
    zero-byte Sarwate step exactly."""
    U = km.unstep_table()
    assert all(U[a ^ b] == U[a] ^ U[b] for a in range(256) for b in (1, 2, 4, 8, 16, 32, 64, 128))
    cinv = km.cinv_table(32)
    rng = random.Random(7)
    for _ in range(300):
        r, tz = rng.getrandbits(32), rng.randrange(32)
        assert km.unstep(r, tz, U) == km.mulmod(r, cinv[tz])
        assert km.unstep(km.zstep(r), 1, U) == r


def test_tz_tables_equal_unsteps():
    """The vring kernel's tz correction: four lookups in the x^(-128) / x^(-64)
    multiplier tables plus < 8 unsteps equals tz zero-byte unsteps (= CINV[tz])."""
    rng = random.Random(0x545A)
    tabs = km.tz_tables()
    for _ in range(300):
        reg = rng.getrandbits(32)
        tz = rng.randrange(32)
        slow = reg
        for _ in range(tz):
            slow = km.unstep_zero(slow)
        assert km.vr_unstep_tz(reg, tz, tabs) == slow == km.mulmod(reg, km.CINV[tz]), (hex(reg), tz)


def test_tz_small_tables_equal_unsteps():
    """The records instance's tz correction: the 16 / 8 tables, then four lookups in the
    x^(-8 c) table of c = tz mod 8 (vr_tz7_mul), equal tz zero-byte unsteps (= CINV[tz])."""
    rng = random.Random(0x545B)
    tabs, small = km.tz_tables(), km.tz_small_tables()
    for tz in range(32):
        for _ in range(12):
            reg = rng.getrandbits(32)
            assert km.vr_unstep_tz(reg, tz, tabs, small) == km.mulmod(reg, km.CINV[tz]), (hex(reg), tz)


def _edge_mask_slot(regs, hs16, lo, hi):
    """crc32_vring.hip vr_edge_mask_slot on one lane: register R of (A, B) holds block
    bytes [oR, oR + 16), oA = hs16, oB = 16 - hs16; per dword i and bound b,
    s = clamp(4 (b - oR) - 16 i, 0, 16), m = (~0 << s) << s; v &= m (low bound),
    v &= ~m (high bound)."""
    out = []
    for r, o in zip(regs, (hs16, 16 - hs16)):
        vals = []
        for i, v in enumerate(r):
            s = min(max(4 * (lo - o) - 16 * i, 0), 16)
            v &= ((0xFFFFFFFF << s) << s) & 0xFFFFFFFF
            t = min(max(4 * (hi - o) - 16 * i, 0), 16)
            v &= ~((0xFFFFFFFF << t) << t) & 0xFFFFFFFF
            vals.append(v)
        out.append(vals)
    return out


def test_vring_edge_mask_slot_keeps_exactly_the_window():
    import numpy as np
    """The in-place edge mask keeps exactly the block bytes in [lo, hi), for both
    half-swap orders and bounds inside and outside the 32-byte block."""
    rng = np.random.default_rng(5)
    block = rng.integers(1, 256, 32, dtype=np.uint8)          # no zero bytes: a kept byte stays nonzero
    for hs16 in (0, 16):
        a = block[hs16:hs16 + 16].view("<u4").tolist()           # register A: bytes [hs16, hs16 + 16)
        b = block[16 - hs16:32 - hs16].view("<u4").tolist()
        for lo in range(-6, 40):
            for hi in range(lo, 42):
                ma, mb = _edge_mask_slot([a, b], hs16, lo, hi)
                got = np.zeros(32, np.uint8)
                got[hs16:hs16 + 16] = np.array(ma, "<u4").view(np.uint8)
                got[16 - hs16:32 - hs16] = np.array(mb, "<u4").view(np.uint8)
                keep = (np.arange(32) >= lo) & (np.arange(32) < hi)
                assert (got == np.where(keep, block, 0)).all(), (hs16, lo, hi)


def test_gather_join_fold_small_matches_oracle(oracle_lib):
    """The join's short-segment fold (fold_small: preloaded aligned dwords, v_alignbyte,
    slicing-by-4, Sarwate tail), chained over 1-4 short segments at every offset mod 4,
    equals the oracle's CRC of their concatenation."""
    rng = random.Random(7)
    arena = bytes(rng.getrandbits(8) for _ in range(4096))
    for _ in range(400):
        segs = [(rng.randrange(0, 4000), rng.randint(1, 64)) for _ in range(rng.randint(1, 4))]
        reg = 0xFFFFFFFF
        for a, L in segs:
            reg = km.fold_small(reg, arena, a, L)
        assert km.finalize(reg) == oracle_lib.crc32(b"".join(arena[a:a + L] for a, L in segs))


def test_snake_deal_balances_binned_ranks():
    """Why the records instance reverses odd rounds: cfg3's rank-interleaved records (256
    tiles, 16-record groups, rank q of 64 ~ longest first) give workgroup k about rank
    16 r + k / 16 in round r.  The plain deal hands workgroup 0 the longest rank of every
    round (1.5 x the last workgroup's bytes); reversed odd rounds even the sums out."""
    from kernel_model import vring_slot_group
    G, W, T, ranks = 256, 16, 256, 64
    wt = G * W
    length = lambda q: 1400 - q * (1336 / (ranks - 1))           # rank q's typical length
    def work(snake):
        per = []
        for k in range(G):
            tot = 0.0
            for sl in range(ranks * T // G):                      # every slot of the workgroup
                g = vring_slot_group(k, sl, wt, W, G, snake)
                tot += length(g // T)
            per.append(tot)
        return max(per) / min(per)
    assert work(False) > 1.4
    assert work(True) < 1.02


@pytest.mark.parametrize("ng", list(range(0, 70)) + [128, 129, 200])
def test_local_tile_slots_cover_every_group_once(ng):
    """The local-tile records instance (crc32_vring.hip BIN 3): whatever order its waves
    take slots in, each of the tile's groups is taken exactly once, a wave's groups
    ascend (so its stop at the first dead slot loses nothing), and the round-1 reversal
    (full rounds only) keeps the live slots a prefix of every round."""
    import random
    from kernel_model import vring_local_deal
    for seed in range(3):
        groups, per_wave = vring_local_deal(ng, random.Random(seed * 1000 + ng))
        assert sorted(groups) == list(range(ng))
        for w, gs in per_wave.items():
            assert gs == sorted(gs), (w, gs)


@pytest.mark.parametrize("ng", list(range(0, 70)))
def test_local_sort_places_each_waves_first_two_groups(ng):
    """The sort's LDS placement agrees with the deal: wave w's metadata area holds its
    first group (slot w) and its staging area its second (slot 16 + w), reversed round 1
    included; no area receives two groups."""
    from kernel_model import vring_local_meta_area, vring_local_slot_group
    W = 16
    placed = {}
    for g in range(ng):
        a = vring_local_meta_area(g, ng, W)
        if a is not None:
            assert a not in placed, (a, g, placed[a])
            placed[a] = g
    for w in range(W):
        for area, sl in (("M", w), ("X", W + w)):
            g = vring_local_slot_group(sl, ng, W)
            if g < ng:
                assert placed.get((area, w)) == g, (area, w, g)
            else:
                assert (area, w) not in placed


def test_local_round_one_reversal_balances_the_static_groups():
    """Why round 1 is reversed: in a length-sorted tile, group g's packets get shorter
    with g, so wave w's two static groups w and 16 + w are both long for w = 0; w and
    31 - w sum to about the same for every wave."""
    from kernel_model import vring_local_slot_group
    W, ng = 16, 32
    length = lambda g: 1400 - g * (1336 / (ng - 1))
    plain = [length(w) + length(W + w) for w in range(W)]
    rev = [length(vring_local_slot_group(w, ng)) + length(vring_local_slot_group(W + w, ng)) for w in range(W)]
    assert max(plain) / min(plain) > 1.3
    assert max(rev) / min(rev) < 1.001


@pytest.mark.parametrize("kpk", [8, 16])
@pytest.mark.parametrize("max_wgs", [256, 512])
def test_local_tile_rule(kpk, max_wgs):
    """vring_launch_local's tile: whole groups, at least a group per wave, at most 2048
    packets (two per thread), a grid within max_wgs whose tiles cover the batch; the
    default path falls back to the two-launch form exactly past 2048 x max_wgs."""
    from kernel_model import vring_local_tile
    for n in [1, 15, 16, 255, 256, 257, 5000, 65536, 262144, 602112, 2048 * max_wgs - 1, 2048 * max_wgs,
              2048 * max_wgs + 1]:
        r = vring_local_tile(n, max_wgs, kpk)
        if n > 2048 * max_wgs:
            assert r is None
            continue
        T, grid = r
        assert T % kpk == 0 and kpk * 16 <= T <= 2048
        assert grid <= max_wgs and (grid - 1) * T < n <= grid * T
