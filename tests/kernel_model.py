"""Host-side model of the gfx950 kernels' arithmetic (test infrastructure).

Restates, in Python integers, what crc32_kernels.hip does per lane -- the 64 KiB
LDS image (slicing tables + INIT/CINV in the free columns), the per-lane v_perm
selectors and column bytes, the dword swaps, slicing-by-32 folding, and the two
ways a packet is spread over P lanes:

  * stream kernel (crc32_stream_kernel): STRIDED blocks.  The packet's window
    is END-aligned (packet end 16-byte aligned) or starts at the 16-byte granule
    holding its first byte; lane k folds every P-th window block with the advancing
    tables T'_t = T_{t+32(P-1)}, so
    after each block its register has also skipped the P-1 blocks the other
    lanes own.  Head (lz) and tail (tz) bytes are zeroed; the assignment is
    rotated so that lane k ends exactly 32k + tz bytes past the data end, undone
    by one GF(2) multiply by x^(-8n) (CINV table) before the XOR over the lanes.
  * direct kernel (crc32_direct_kernel / gather): CONTIGUOUS segments cut at
    128-byte-aligned addresses, END-aligned windows started at INIT[rp], and the
    classic carry-combine reg(A||B) = reg(A) * x^(8|B|) ^ reg(B).

It models the arithmetic, not the hardware: parity on the device is established
by the -m gpu tests.
"""
from __future__ import annotations

POLY = 0xEDB88320
ONE = 0x80000000          # the polynomial "1" in the reflected representation


def t0(n: int) -> int:
    c = n
    for _ in range(8):
        c = (c >> 1) ^ POLY if c & 1 else c >> 1
    return c


T0 = [t0(n) for n in range(256)]


def zstep(reg: int) -> int:
    """One zero byte through the Sarwate register."""
    return (reg >> 8) ^ T0[reg & 0xFF]


def slicing_tables(k: int = 32, skip: int = 0) -> list[list[int]]:
    """T_t[j] = byte j followed by t + skip zero bytes, t < k."""
    first = []
    for j in range(256):
        r = T0[j]
        for _ in range(skip):
            r = zstep(r)
        first.append(r)
    T = [first]
    for _ in range(1, k):
        T.append([zstep(v) for v in T[-1]])
    return T


TS = slicing_tables(32)


# ---------------------------------------------------------------- GF(2) helpers
def mulmod(a: int, b: int) -> int:
    p = 0
    for j in range(32):
        if (a >> (31 - j)) & 1:
            p ^= b
        b = (b >> 1) ^ (POLY if b & 1 else 0)
    return p


def x8n(n: int) -> int:
    r = ONE
    for _ in range(n):
        r = zstep(r)
    return r


def x_inverse() -> int:
    """x^-1 mod p = (p(x) + 1) / x, reflected (bit 31-i <-> x^i)."""
    # p(x) + 1 = x^32 + sum of POLY's terms without the constant; divide by x
    # POLY reflected: bit (31-i) set <-> x^i in p (i < 32); x^0 is bit 31.
    v = 0
    for i in range(1, 32):                      # term x^i of p, i >= 1 -> x^(i-1)
        if (POLY >> (31 - i)) & 1:
            v |= 1 << (31 - (i - 1))
    v |= 1 << (31 - 31)                         # x^32 / x = x^31
    return v


XINV = x_inverse()
assert mulmod(XINV, x8n(0) >> 1) == ONE       # x^-1 * x = 1  (x = ONE >> 1)


def cinv_table(n: int = 512) -> list[int]:
    """CINV[i] = x^(-8i) mod p."""
    xinv8 = ONE
    for _ in range(8):
        xinv8 = mulmod(xinv8, XINV)
    out = [ONE]
    for _ in range(1, n):
        out.append(mulmod(out[-1], xinv8))
    return out


CINV = cinv_table()


def unstep_zero(reg_next: int) -> int:
    top = reg_next >> 24
    n = next(k for k in range(256) if (T0[k] >> 24) == top)
    return (((reg_next ^ T0[n]) << 8) & 0xFFFFFFFF) | n


INIT = [0xFFFFFFFF]
for _ in range(63):                                 # INIT[r], r < 64 (vring windows: lz < 64)
    INIT.append(unstep_zero(INIT[-1]))


# ---------------------------------------------------------------- 64 KiB LDS image
def col_byte(t: int) -> int:
    """Byte offset of table t inside a 256-byte row: dword 2t + (t >> 4)."""
    return 8 * t + 4 * (t >> 4)


def free_col(c: int) -> int:
    """Byte offset of free column c (c < 32): the dwords no slicing table uses."""
    return 4 * (2 * c + 1 if c < 16 else 2 * c)


# Free columns are 256-entry tables indexed by the row (a byte value), so a
# lookup is one v_perm (byte -> address byte 1, column -> byte 0) + ds_read.
KCORR_COL = 0             # columns 4(k-1) + b, k = 1..7: byte b of a register times x^(-256k)
KINIT_COL = 29            # INIT[r], r < 32 (rows 0..31)
KCINV_COL = 30            # CINV[n], n < 512: rows n & 255 of columns 30 + (n >> 8)


def init_addr(r: int) -> int:
    return 256 * r + free_col(KINIT_COL)


def cinv_addr(n: int) -> int:
    return 256 * (n & 255) + free_col(KCINV_COL + (n >> 8))


def corr_addr(k: int, b: int, v: int) -> int:
    return 256 * v + free_col(KCORR_COL + 4 * (k - 1) + b)


def lds_image(P: int = 1) -> list[int]:
    """dword 64*j + 2t + (t>>4) = T'_t[j] = T_{t + 32(P-1)}[j]; free columns hold
    the per-lane correction tables (k < min(P, 8)), INIT and CINV."""
    T = slicing_tables(32, 32 * (P - 1))
    img = [0] * (256 * 64)
    for j in range(256):
        for t in range(32):
            img[64 * j + col_byte(t) // 4] = T[t][j]
    for k in range(1, min(P, 8)):                  # lane k's overshoot of 32k bytes, undone
        for b in range(4):                         # by four byte-indexed lookups
            for v in range(256):
                img[corr_addr(k, b, v) // 4] = mulmod(v << (8 * b), CINV[32 * k])
    for r in range(64):
        img[init_addr(r) // 4] = INIT[r]
    for n in range(512):
        img[cinv_addr(n) // 4] = CINV[n]
    return img


_IMG_CACHE: dict[int, list[int]] = {}


def image(P: int = 1) -> list[int]:
    if P not in _IMG_CACHE:
        _IMG_CACHE[P] = lds_image(P)
    return _IMG_CACHE[P]


KBASIS_ROWS = 9
KINIT_DWORD = free_col(KINIT_COL) // 4      # 58
KCINV_DWORD = free_col(KCINV_COL) // 4      # 60 (CINV n < 256)


def table_basis(P: int) -> list[int]:
    """The lean kernel's 9 x 64-dword table basis (HostTables::basis,
    csrc/crc32_kernels.hip): row b < 8 = image row 2^b with the INIT / CINV dwords
    zeroed (every other column is GF(2)-linear in the row index), row 8 =
    INIT[0..31] | CINV[0..31]."""
    img = image(P)
    skip = (KINIT_DWORD, KCINV_DWORD, KCINV_DWORD + 2)
    B = [0 if d in skip else img[64 * (1 << b) + d] for b in range(8) for d in range(64)]
    return B + INIT[:32] + CINV[:32]


def image_from_basis(B: list[int]) -> list[int]:
    """crc32_lean.hip's in-LDS rebuild: row j = XOR of basis rows b with bit b of j
    set; INIT / CINV rows < 32 from basis row 8 (rows >= 32 of those columns, and
    CINV n >= 256, are never read by that kernel)."""
    img = [0] * (256 * 64)
    for j in range(256):
        row = [0] * 64
        for b in range(8):
            if (j >> b) & 1:
                row = [x ^ y for x, y in zip(row, B[64 * b:64 * b + 64])]
        if j < 32:
            row[KINIT_DWORD] = B[512 + j]
            row[KCINV_DWORD] = B[544 + j]
        img[64 * j:64 * j + 64] = row
    return img


_RB_CACHE: dict[int, list[int]] = {}


def rebuilt_image(P: int) -> list[int]:
    if P not in _RB_CACHE:
        _RB_CACHE[P] = image_from_basis(table_basis(P))
    return _RB_CACHE[P]


def v_perm(s0: int, s1: int, sel: int) -> int:
    """V_PERM_B32: byte_permute({S0, S1}, sel); S1 = bytes 0-3, S0 = bytes 4-7."""
    data = (s1 & 0xFFFFFFFF) | ((s0 & 0xFFFFFFFF) << 32)
    out = 0
    for k in range(4):
        sb = (sel >> (8 * k)) & 0xFF
        if sb < 8:
            b = (data >> (8 * sb)) & 0xFF
        elif sb == 12:
            b = 0x00
        elif sb >= 13:
            b = 0xFF
        else:  # 8..11: sign replication (unused by the kernel)
            src = (data >> (8 * (2 * (sb - 8) + 1) + 7)) & 1
            b = 0xFF if src else 0
        out |= b << (8 * k)
    return out


def make_sched(lane: int):
    l5 = lane & 31
    col = []
    for g in range(8):
        r = 0
        for h in range(4):
            i = 4 * g + h
            t = (i ^ l5) ^ 31
            r |= col_byte(t) << (8 * h)
        col.append(r)
    # byte 0 of the address = column byte h of col (S1), byte 1 = data byte (S0)
    sel = [h | ((4 + (h ^ (l5 & 3))) << 8) | 0x0C0C0000 for h in range(4)]
    return col, sel, bool((l5 >> 2) & 1), bool((l5 >> 3) & 1), bool((l5 >> 4) & 1)


def lookup_addresses(lane: int, words: list[int]) -> list[int]:
    """LDS byte address of each of the 32 lookups of fold_block (words in original
    order, state already XORed): halves put in lane order, two dword-swap rounds,
    then one v_perm per lookup (no shift)."""
    col, sel, sw1, sw2, hs = make_sched(lane)
    w = (words[4:8] + words[0:4]) if hs else list(words)
    x = [w[q ^ 1] if sw1 else w[q] for q in range(8)]
    d = [x[q ^ 2] if sw2 else x[q] for q in range(8)]
    return [v_perm(d[i >> 2], col[i >> 2], sel[i & 3]) for i in range(32)]


def fold_block(reg: int, block: bytes, lane: int, P: int = 1) -> int:
    img = image(P)
    w = [int.from_bytes(block[4 * q:4 * q + 4], "little") for q in range(8)]
    w[0] ^= reg
    acc = 0
    for addr in lookup_addresses(lane, w):
        assert addr % 4 == 0 and addr < 65536
        acc ^= img[addr // 4]
    return acc


def finalize(reg: int) -> int:
    return int.from_bytes((~reg & 0xFFFFFFFF).to_bytes(4, "little"), "big")


# ---------------------------------------------------------------- stream kernel
def stream_window(addr: int, L: int):
    """(lz, NB, tz): the window ENDS at the 16-byte granule boundary at or after
    the packet end (tz = that distance < 16, zeroed) and spans NB whole 32-byte
    blocks, lz < 32 of them in front of the packet (zeroed; a 16-byte piece wholly
    in front is read from a zero buffer).  Every byte read lies in a granule that
    holds packet bytes or is replaced by zeros."""
    if L == 0:
        return 0, 0, 0
    tz = (-(addr + L)) % 16
    nb = (L + tz + 31) // 32
    return 32 * nb - tz - L, nb, tz


def stream_lane_blocks(k: int, P: int, nb: int) -> list[int]:
    """Rotated assignment: lane k folds window blocks w with (w + r) % P == k,
    r = (-nb) % P, so that lane k ends exactly 32k bytes past the window end."""
    r = (-nb) % P
    return list(range((k - r) % P, nb, P))


def stream_packet(pkt: bytes, P: int, addr: int = 0, lane_base: int = 0,
                  slot: tuple[int, int] | None = None) -> tuple[int, int]:
    """What crc32_stream_kernel's P lanes compute for one packet at byte address
    `addr`.  slot = (slot_offset, connect_id) models the verify mode: the 4 slot
    bytes are replaced by connect_id inside the lane that folds them and the
    original bytes are returned as `desired`.  Returns (register, desired)."""
    L = len(pkt)
    lz, nb, tz = stream_window(addr, L)
    win = bytes(lz) + pkt + bytes(tz)          # head/tail bytes zeroed by the kernel
    img = image(P)
    r = (-nb) % P
    desired = 0
    regs = []
    for k in range(P):
        lane = lane_base + k
        reg = INIT[lz] if k == r else 0
        blocks = stream_lane_blocks(k, P, nb)
        for w in blocks:
            blk = bytearray(win[32 * w:32 * w + 32])
            if slot is not None:
                so, cid = slot
                for q in range(4):
                    pos = lz + so + q - 32 * w
                    if 0 <= pos < 32:
                        desired |= blk[pos] << (8 * q)
                        blk[pos] = (cid >> (8 * q)) & 0xFF
            reg = fold_block(reg, bytes(blk), lane, P)
        if blocks:
            assert blocks[-1] + P - nb == k        # overshoot is exactly k blocks
        regs.append(reg)
    total = 0
    for k in range(P):                             # lane k sits 32k + tz bytes past the data end
        reg = regs[k]
        if k and k < 8:                            # x^(-256k): four byte-indexed table lookups
            reg = (img[corr_addr(k, 0, reg & 0xFF) // 4] ^ img[corr_addr(k, 1, (reg >> 8) & 0xFF) // 4] ^
                   img[corr_addr(k, 2, (reg >> 16) & 0xFF) // 4] ^ img[corr_addr(k, 3, reg >> 24) // 4])
        elif k:
            reg = mulmod(reg, img[cinv_addr(32 * k) // 4])
        total ^= reg
    if tz:
        total = mulmod(total, img[cinv_addr(tz) // 4])
    return total, desired


def stream_crc(pkt: bytes, P: int, addr: int = 0, lane_base: int = 0) -> int:
    return finalize(stream_packet(pkt, P, addr, lane_base)[0])


def stream_verify(pkt: bytes, slot_off: int, connect: int, P: int, addr: int = 0) -> tuple[bool, int]:
    if slot_off + 4 > len(pkt):
        return False, 0
    reg, desired = stream_packet(pkt, P, addr, 0, (slot_off, connect))
    comp = finalize(reg)
    return comp == desired, comp


# ---------------------------------------------------------------- direct kernel
def fold_window(reg: int, seg: bytes, lane: int) -> int:
    L = len(seg)
    nb = (L + 31) // 32
    win = bytes(32 * nb - L) + seg
    for j in range(nb):
        reg = fold_block(reg, win[32 * j:32 * j + 32], lane)
    return reg


def segment_cuts(addr: int, L: int, lanes: int) -> list[int]:
    """Direct kernel's cut points: packet [addr, addr+L) split at 128-byte-aligned
    absolute addresses nearest to the even split (offsets relative to addr)."""
    cuts = [0]
    for k in range(1, lanes):
        r = (addr + (L * k) // lanes + 64) & ~127
        cuts.append(min(max(r, addr), addr + L) - addr)
    cuts.append(L)
    return cuts


def crc_packet(pkt: bytes, lanes: int = 1, lane_base: int = 0, addr: int = 0) -> int:
    L = len(pkt)
    cuts = segment_cuts(addr, L, lanes)
    total = 0
    for k in range(lanes):
        seg = pkt[cuts[k]:cuts[k + 1]]
        nb = (len(seg) + 31) // 32
        rp = 32 * nb - len(seg)
        reg = INIT[rp] if k == 0 else 0
        reg = fold_window(reg, seg, lane_base + k)
        after = L - cuts[k + 1]
        if after:
            reg = mulmod(reg, x8n(after))
        total ^= reg
    return finalize(total)


# ---------------------------------------------------------------- lean kernel
def lean_sched(lane: int, P: int):
    """crc32_lean.hip's LeanSched: pi(l) = 4 D(l) + b(l); D = l3 | l4 << 1 | s << 2
    with s = l2 (P = 8) or l1 (P = 4); b = l0 | o << 1 with o the other bit."""
    l5 = lane & 31
    sb, ob = (2, 1) if P == 8 else (1, 2)
    D = ((l5 >> 3) & 3) | (((l5 >> sb) & 1) << 2)
    b = (l5 & 1) | (((l5 >> ob) & 1) << 1)
    pi = 4 * D + b
    col = []
    for g in range(8):
        r = 0
        for h in range(4):
            r |= col_byte(31 - ((4 * g + h) ^ pi)) << (8 * h)
        col.append(r)
    sel = [h | ((4 + (h ^ b)) << 8) | 0x0C0C0000 for h in range(4)]
    dq = [4 * (r ^ D) for r in range(8)]
    return D, col, sel, dq


def lean_block_address(lane: int, P: int, w0: int) -> int:
    """LDS byte offset (ring slot 0) of lane (j, k)'s 32-byte block: pieces 2w0,
    2w0+1 of the packet's chunk, DMA'd by lanes (j, 2w0 mod P), (j, 2w0 mod P + 1)
    of instruction 2w0 // P."""
    j = lane // P
    return 1024 * ((2 * w0) // P) + 16 * (j * P + (2 * w0) % P)


def lean_group(arena: bytes, offs: list[int], lens: list[int], P: int, check_banks: bool = True) -> list[int]:
    """One group (64/P packets, 64 lanes) through the lean kernel's data path:
    producer DMA of pieces k and P + k per lane per stage into the 2 KiB ring slot,
    consumer permuted dword reads (bank-checked), fold with the lean schedule,
    lane corrections, lane XOR, tz correction.  Returns the finalized CRCs."""
    npk = 64 // P
    assert len(offs) == npk
    img = rebuilt_image(P)                         # the image as the kernel rebuilds it in LDS
    wins = [stream_window(offs[j], lens[j]) for j in range(npk)]   # (lz, nb, tz)
    stages = max(1, max(((nb + P - 1) // P) for _, nb, _ in wins))
    regs = [0] * 64
    rot = [(-nb) % P for _, nb, _ in wins]
    for lane in range(64):
        j, k = divmod(lane, P)
        lz, nb, tz = wins[j]
        if k == rot[j]:
            regs[lane] = img[init_addr(lz) // 4]
    for s in range(stages):
        slot = bytearray(2048)
        for lane in range(64):                     # producer: own packet, pieces k and P + k
            j, k = divmod(lane, P)
            lz, nb, tz = wins[j]
            ws = offs[j] + lens[j] + tz - 32 * nb
            for i, q in enumerate((k, P + k)):
                piece = 2 * P * s + q              # window piece index
                ok = piece < 2 * nb and not (s == 0 and q == 0 and lz >= 16)
                a = ws + 16 * piece
                data = arena[a:a + 16] if ok else bytes(16)
                slot[1024 * i + 16 * lane:1024 * i + 16 * lane + 16] = data
        banks = [[None] * 64 for _ in range(8)]
        for lane in range(64):                     # consumer
            j, k = divmod(lane, P)
            lz, nb, tz = wins[j]
            w0 = (k - rot[j]) % P
            cnt = (nb - 1 - w0) // P + 1 if w0 < nb else 0
            D, col, sel, dq = lean_sched(lane, P)
            rb = lean_block_address(lane, P, w0)
            x = []
            for r in range(8):
                a = rb + dq[r]
                banks[r][lane] = (a // 4) % 32
                x.append(int.from_bytes(slot[a:a + 4], "little"))
            if s >= cnt:
                continue
            w = w0 + P * s                         # window block folded now
            blk = bytearray(b"".join(v.to_bytes(4, "little") for v in [x[r ^ D] for r in range(8)]))
            for t in range(32):                    # edge_fix: head / tail bytes outside the packet
                if (w == 0 and t < lz) or (w == nb - 1 and t >= 32 - tz):
                    blk[t] = 0
            xs = [int.from_bytes(blk[4 * (r ^ D):4 * (r ^ D) + 4], "little") for r in range(8)]
            d = [xs[r] ^ (regs[lane] if r == D else 0) for r in range(8)]
            acc = 0
            for i in range(32):
                addr = v_perm(d[i >> 2], col[i >> 2], sel[i & 3])
                acc ^= img[addr // 4]
            regs[lane] = acc
        if check_banks:
            for r in range(8):
                for h in (0, 32):
                    assert len(set(banks[r][h:h + 32])) == 32, ("bank conflict", r, h)
    out = []
    for j in range(npk):
        lz, nb, tz = wins[j]
        total = 0
        for k in range(P):
            reg = regs[j * P + k]
            if k:
                reg = (img[corr_addr(k, 0, reg & 0xFF) // 4] ^ img[corr_addr(k, 1, (reg >> 8) & 0xFF) // 4] ^
                       img[corr_addr(k, 2, (reg >> 16) & 0xFF) // 4] ^ img[corr_addr(k, 3, reg >> 24) // 4])
            total ^= reg
        if tz:
            total = mulmod(total, img[cinv_addr(tz) // 4])
        out.append(finalize(total))
    return out


# ---------------------------------------------------------------- length bins
# bin_tile_kernel (crc32_lean.hip): placement of the ordered records.

BIN_TILE = 1024


def bin_of(length: int, off: int = 0) -> int:
    """32-byte bins of the vring window length lz + L (lz = off mod 64), longest first
    (bin 0 holds windows >= 8160 B)."""
    return 255 - min((length + (off & 63)) >> 5, 255)


def binned_order(lens, kpk: int, offs=None):
    """Caller index held by each record position: every 1024-packet tile sorted by
    bin (ties in index order here; on the GPU the order inside a bin is free), sorted
    group q of full tile t placed as global group q * T + t, a ragged last tile in place."""
    n = len(lens)
    full = n // BIN_TILE
    order = [0] * n
    for t in range((n + BIN_TILE - 1) // BIN_TILE):
        ids = range(t * BIN_TILE, min(n, (t + 1) * BIN_TILE))
        srt = sorted(ids, key=lambda i: (bin_of(int(lens[i]), 0 if offs is None else int(offs[i])), i))
        for s, i in enumerate(srt):
            dst = ((s // kpk) * full + t) * kpk + s % kpk if t < full else t * BIN_TILE + s
            order[dst] = i
    return order


def group_stage_cost(lens, order, kpk: int, lanes: int) -> int:
    """Sum over groups of the group's stage count (its longest packet, P*32-byte stages):
    the lean kernel's work in stages, whatever the packets' own lengths."""
    total = 0
    for g in range(0, len(order), kpk):
        total += max((int(lens[i]) + 31) // 32 // lanes + 1 for i in order[g:g + kpk])
    return total


# ---------------------------------------------------------------- vring kernel
# crc32_vring.hip: 64-byte-aligned window starts, lane k folds blocks k, k+P, ...
# loaded straight into registers (halves swapped by the load address when the
# lane's hs bit is set), lane k ends o = (k - nb) mod P blocks past the window end.
VR_BASIS_ROWS = 10


def vring_basis(P: int) -> list[int]:
    """HostTables::basis2: rows 0..7 as the lean basis, row 8 = INIT[0..63],
    row 9 = CINV[0..63]."""
    return table_basis(P)[:512] + INIT[:64] + CINV[:64]


def vring_image_from_basis(B: list[int]) -> list[int]:
    """crc32_vring.hip's in-LDS rebuild (INIT / CINV rows < 64 from rows 8, 9)."""
    img = [0] * (256 * 64)
    for j in range(256):
        row = [0] * 64
        for b in range(8):
            if (j >> b) & 1:
                row = [x ^ y for x, y in zip(row, B[64 * b:64 * b + 64])]
        if j < 64:
            row[KINIT_DWORD] = B[512 + j]
            row[KCINV_DWORD] = B[576 + j]
        img[64 * j:64 * j + 64] = row
    return img


_VR_CACHE: dict[int, list[int]] = {}


def vring_image(P: int) -> list[int]:
    if P not in _VR_CACHE:
        _VR_CACHE[P] = vring_image_from_basis(vring_basis(P))
    return _VR_CACHE[P]


def vring_window(addr: int, L: int, end_aligned: bool = False):
    """(ws, lz, e, nb): window start (64-byte aligned), packet bytes [lz, e) of it.
    end_aligned (the records instance's EA windows, for packets whose end is 16-byte
    aligned): the window of nb = ceil(L / 32) blocks ends on the packet's last byte, so
    e = 32 nb (no trailing zero bytes: tz = 0) and lz = 32 nb - L < 32.  (The model
    takes any end alignment.)"""
    if end_aligned:
        nb = (L + 31) // 32
        return addr + L - 32 * nb, 32 * nb - L, 32 * nb, nb
    lz = addr & 63
    e = lz + L
    nb = (e + 31) // 32 if L else 0
    return addr - lz, lz, e, nb


def vring_stage_order(S: int, rotate: bool):
    """crc32_vring.hip's stage order of a group of S stages: in order, or (rotate,
    the tail-first schedule) the last stage first, then 0 .. S-2."""
    if not rotate or S <= 1:
        return list(range(S))
    return [S - 1] + list(range(S - 1))


def vring_adv(img, reg: int) -> int:
    """reg * x^(256 P): the fold of a block holding reg in its first 4 bytes and
    zeros elsewhere, four lookups in the advancing tables T'_31 .. T'_28."""
    acc = 0
    for m in range(4):
        acc ^= img[(((reg >> (8 * m)) & 0xFF) * 256 + col_byte(31 - m)) // 4]
    return acc


def vring_packet(arena: bytes, addr: int, L: int, P: int, lane_base: int = 0, rotate: bool = False,
                 group_stages: int = 0, end_aligned: bool = False) -> int:
    """What crc32_vring_kernel's P lanes (lanes lane_base .. lane_base+P-1) compute
    for the packet arena[addr:addr+L]; returns the wire CRC.  rotate: the
    tail-first stage order (the group's last stage first, folded from a zero
    register into rt; rt ^ adv(reg) joins it at the end); group_stages: the
    group's stage count (>= this packet's own); end_aligned: vring_window's EA windows."""
    img = vring_image(P)
    ws, lz, e, nb = vring_window(addr, L, end_aligned)
    stages = max((nb + P - 1) // P, group_stages)
    order = vring_stage_order(stages, rotate)
    total = 0
    for k in range(P):
        lane = lane_base + k
        col, sel, sw1, sw2, hs = make_sched(lane)
        reg = (img[init_addr(lz) // 4] if nb else 0xFFFFFFFF) if k == 0 else 0
        rt = 0
        cnt = (nb - 1 - k) // P + 1 if nb > k else 0
        for step, st in enumerate(order):
            tail_first = rotate and stages > 1 and step == 0
            q0 = 32 * (k + P * st)
            pieces = []
            for po in ((q0 + 16, q0) if hs else (q0, q0 + 16)):   # lane order A, B
                valid = po < e and po + 16 > lz
                pieces.append(arena[ws + po:ws + po + 16] if valid else bytes(16))
            A = [int.from_bytes(pieces[0][4 * i:4 * i + 4], "little") for i in range(4)]
            B = [int.from_bytes(pieces[1][4 * i:4 * i + 4], "little") for i in range(4)]
            orig = (B + A) if hs else (A + B)
            blk = bytearray(b"".join(v.to_bytes(4, "little") for v in orig))
            for t in range(32):                    # edge mask: keep [lz, e) only
                if not (lz <= q0 + t < e):
                    blk[t] = 0
            if st >= cnt:
                continue
            w = [int.from_bytes(blk[4 * q:4 * q + 4], "little") for q in range(8)]
            w[0] ^= 0 if tail_first else reg
            acc = 0
            for a in lookup_addresses(lane, w):
                acc ^= img[a // 4]
            if tail_first:
                rt = acc
            else:
                reg = acc
        if rotate and stages > 1 and stages - 1 < cnt:
            reg = rt ^ vring_adv(img, reg)
        o = (k - nb) % P
        if o:
            reg = (img[corr_addr(o, 0, reg & 0xFF) // 4] ^ img[corr_addr(o, 1, (reg >> 8) & 0xFF) // 4] ^
                   img[corr_addr(o, 2, (reg >> 16) & 0xFF) // 4] ^ img[corr_addr(o, 3, reg >> 24) // 4])
        total ^= reg
    tz = 32 * nb - e if nb else 0
    if tz:
        total = mulmod(total, img[cinv_addr(tz) // 4])
    return finalize(total)


# ---------------------------------------------------------------- vring slots
def vring_slot_group(blk: int, sl: int, wt: int, W: int = 16, grid: int = 0, snake: bool = False) -> int:
    """crc32_vring.hip slot_group: workgroup blk's slot sl is global group
    16 blk + sl % 16 + (sl / 16) wt (wt = the launch's waves); snake (the records
    instance, round 6): odd rounds deal the workgroups in reverse, blk -> grid - 1 - blk."""
    r = sl // W
    k = grid - 1 - blk if (snake and r & 1) else blk
    return W * k + (sl % W) + r * wt


def vring_local_tile(n: int, max_wgs: int, kpk: int, W: int = 16, cap: int = 2048):
    """crc32_vring.hip vring_launch_local: packets per workgroup T (the batch over max_wgs
    workgroups, in whole groups, at least a group per wave, at most cap) and the grid
    ceil(n / T); None when the batch does not fit one tile per workgroup."""
    T = -(-n // max_wgs)
    T = max(-(-T // kpk) * kpk, kpk * W)
    T = min(T, cap)
    grid = -(-n // T)
    return (T, grid) if grid <= max_wgs else None


def vring_local_slot_group(sl: int, ng: int, W: int = 16) -> int:
    """The local-tile instance's slot_group: the workgroup's own groups in slot order,
    round 1 reversed when it is full (ng >= 2 W)."""
    return 3 * W - 1 - sl if (sl // W == 1 and ng >= 2 * W) else sl


def vring_local_meta_area(g: int, ng: int, W: int = 16):
    """Where the local sort puts group g's metadata: ("M", w) = wave w's metadata area
    (round 0), ("X", w) = wave w's staging of its second group (round 1), None = read
    later by a metadata DMA."""
    if g < W:
        return ("M", g)
    if g < 2 * W:
        return ("X", 2 * W - 1 - g if ng >= 2 * W else g - W)
    return None


def vring_local_deal(ng: int, rng, W: int = 16):
    """Simulate one workgroup of the local-tile instance: every wave takes slots wave
    and 16 + wave, then slots from the workgroup's counter (from 32), in a random
    interleaving, until a slot maps past the tile's last group.  Returns the groups in
    the order taken and each wave's groups."""
    ctr = 2 * W
    taken = {w: 0 for w in range(W)}
    alive = set(range(W))
    groups, per_wave = [], {w: [] for w in range(W)}
    while alive:
        w = rng.choice(sorted(alive))
        if taken[w] < 2:
            sl = w + W * taken[w]
        else:
            sl = ctr
            ctr += 1
        taken[w] += 1
        g = vring_local_slot_group(sl, ng, W)
        if g >= ng:
            alive.discard(w)
            continue
        groups.append(g)
        per_wave[w].append(g)
    return groups, per_wave


def vring_dynamic_deal(batch_groups, grid: int, rng, W: int = 16, snake: bool = False):
    """Simulate one launch of the vring kernel's dynamic slots: every wave takes
    slots wave and 16 + wave, then slots from its workgroup's counter (starting at
    32) in a random interleaving of the workgroup's waves, until a slot maps past
    the last group.  Returns {global group: (batch, local group)} as the waves
    processed them, and the groups per wave."""
    g0, total = [], 0
    for n in batch_groups:
        g0.append(total)
        total += n
    wt = grid * W
    seen, per_wave = {}, []

    def locate(b, gg):
        while b + 1 < len(g0) and gg >= g0[b + 1]:
            b += 1
        return b

    for blk in range(grid):
        ctr = 2 * W
        cur = {w: [0, 0, True] for w in range(W)}           # cursor batch, taken, alive
        count = [0] * W
        order = []
        while any(c[2] for c in cur.values()):
            w = rng.choice([x for x, c in cur.items() if c[2]])
            c = cur[w]
            if c[1] < 2:
                sl = w + W * c[1]
            else:
                sl = ctr
                ctr += 1
            c[1] += 1
            gg = vring_slot_group(blk, sl, wt, W, grid, snake)
            if gg >= total:
                c[2] = False
                continue
            b = locate(c[0], gg)
            assert b >= c[0], "a wave's groups ascend, so its batch cursor only moves forward"
            c[0] = b
            assert gg not in seen, f"group {gg} taken twice"
            seen[gg] = (b, gg - g0[b])
            count[w] += 1
            order.append(w)
        per_wave.extend(count)
    return seen, per_wave, total


def vring_dynamic_rounds_deal(batch_groups, grid: int, rng, W: int = 16, K: int = 64, S: int = 3,
                              pairs: bool = False):
    """Simulate one launch of the vring kernel's dynamic rounds (crc32_vring.hip DYN:
    take / vr_claim_next / vr_round_publish / vr_round_chunk), all workgroups' waves
    interleaved at random: rounds r < S (S = 3 static takes) of workgroup k are chunks
    k + r G; the wave taking slot 16 r (r >= S - 1) waits for round r's entry (r >= S),
    claims a chunk S G + c from the launch's counter -- the atomic completing at a
    random later step, the wave blocked meanwhile -- and publishes it as round r + 1; a
    wave taking a slot of round r >= S waits for round r's entry.  A slot maps to group 16 chunk + slot % 16
    and a wave stops at its first group past the end.  Checks that no wave waits
    forever and that no round entry (K of them, r % K) is rewritten while a wave that
    took a slot of its round has not read it yet; returns {global group: (batch, local
    group)}, the groups per wave and the launch's groups.  pairs (DYN 2): workgroups k
    and k + H (H = G / 2, G even) claim from the pair's own counter, chunk p + (2 S + c) H
    (p = k mod H) -- their static rounds k + r G are the pair's chunks p + (2 r + k / H) H."""
    g0, total = [], 0
    for n in batch_groups:
        g0.append(total)
        total += n
    G = grid
    H = G // 2
    if pairs:
        assert G % 2 == 0 and G >= 2
    counter = 0
    pair_ctr = [0] * max(H, 1)
    seen, per_wave = {}, []
    wgs = [dict(ctr=S * W, pub={}, unread={}) for _ in range(G)]
    # per wave: wg, wave, slots taken, batch cursor, state, slot, groups
    waves = [dict(k=k, w=w, taken=0, b=0, st="take", sl=0, n=0) for k in range(G) for w in range(W)]
    alive = set(range(len(waves)))

    def ready(v):
        wg, r = wgs[v["k"]], v["sl"] // W
        if v["st"] in ("take", "claiming"):
            return True                                     # (claiming: the atomic may complete)
        if v["st"] == "claim_src":                          # the claimer waits for round r's entry
            return r < S or r in wg["pub"]
        if v["st"] == "read":
            return r < S or r in wg["pub"]
        raise AssertionError(v["st"])

    steps = 0
    while alive:
        steps += 1
        assert steps < 100 * (total + G * W) + 10000, "no progress"
        enabled = [i for i in alive if ready(waves[i])]
        assert enabled, "deadlock: every live wave waits"
        v = waves[rng.choice(enabled)]
        wg = wgs[v["k"]]
        if v["st"] == "take":
            if v["taken"] < S:
                v["sl"] = v["w"] + W * v["taken"]
            else:
                v["sl"] = wg["ctr"]
                wg["ctr"] += 1
            v["taken"] += 1
            r = v["sl"] // W
            if r >= S:
                wg["unread"][r] = wg["unread"].get(r, 0) + 1
            v["st"] = "claim_src" if (r >= S - 1 and v["sl"] % W == 0) else "read"
        elif v["st"] == "claim_src":
            v["st"] = "claiming"
        elif v["st"] == "claiming":                         # the atomic returns: publish round r + 1
            r1 = v["sl"] // W + 1
            assert not wg["unread"].get(r1 - K), "round entry rewritten while still to be read"
            wg["pub"].pop(r1 - K, None)
            if pairs:
                p = v["k"] % H
                wg["pub"][r1] = p + (2 * S + pair_ctr[p]) * H
                pair_ctr[p] += 1
            else:
                wg["pub"][r1] = S * G + counter
                counter += 1
            v["st"] = "read"
        else:                                               # read: the slot's group
            r = v["sl"] // W
            chunk = v["k"] + r * G if r < S else wg["pub"][r]
            if r >= S:
                wg["unread"][r] -= 1
            gg = W * chunk + v["sl"] % W
            if gg >= total:
                alive.discard(id_ := waves.index(v))
                per_wave.append(v["n"])
                continue
            b = v["b"]
            while b + 1 < len(g0) and gg >= g0[b + 1]:
                b += 1
            assert not seen or v["n"] == 0 or gg > v.get("last", -1), "a wave's groups ascend"
            v["b"], v["last"] = b, gg
            assert gg not in seen, f"group {gg} taken twice"
            seen[gg] = (b, gg - g0[b])
            v["n"] += 1
            v["st"] = "take"
    return seen, per_wave, total


# ---------------------------------------------------------------- gather join
def gather_join(seg_crcs, seg_lens) -> int:
    """crc32_gather_join_kernel (enet_hip_crc32_gather_binned_device): a DGRAM's CRC from
    its segments' finalized CRCs (each = finalize(reg(0xFFFFFFFF, segment))).
    reg' = (reg ^ ~0) x^(8 len) ^ reg(~0, segment), from reg = ~0; empty segments skipped."""
    reg, first = 0xFFFFFFFF, True
    for c, L in zip(seg_crcs, seg_lens):
        if L == 0:
            continue
        r = ~int.from_bytes(c.to_bytes(4, "little"), "big") & 0xFFFFFFFF     # ~bswap32(crc)
        reg = (0 if first else mulmod(reg ^ 0xFFFFFFFF, x8n(L))) ^ r
        first = False
    return finalize(reg)



def gather_split_join(arena: bytes, segs, small: int = 48) -> int:
    """The split join (gather_join.hpp): the pre-join walks the DGRAM with every long
    segment's own register R_q taken as 0 -- short segments folded (fold_small), long
    ones reg' = (reg ^ ~0) x^(8 L) -- and records x^(8 after_q) for each long q; the
    post-join XORs bswap(R_q x^(8 after_q)) into finalize(A) (~crc_q when after_q = 0).
    segs = [(offset, length)] into arena."""
    total = sum(L for _, L in segs)
    reg, pos, pend = 0xFFFFFFFF, 0, []
    for a, L in segs:
        if L == 0:
            continue
        pos += L
        if L <= small:
            reg = fold_small(reg, arena, a, L)
        else:
            reg = 0 if reg == 0xFFFFFFFF else mulmod(reg ^ 0xFFFFFFFF, x8n(L))
            after = total - pos
            pend.append((a, L, x8n(after) if after else ONE))
    out = finalize(reg)
    for a, L, m in pend:                                     # the post-join, one segment each
        r = 0xFFFFFFFF
        for b in arena[a:a + L]:
            r = t0((r ^ b) & 0xFF) ^ (r >> 8)
        c = finalize(r)                                      # the records pass's seg_crc
        r = ~int.from_bytes(c.to_bytes(4, "little"), "big") & 0xFFFFFFFF
        add = (~c & 0xFFFFFFFF) if m == ONE else int.from_bytes(mulmod(r, m).to_bytes(4, "little"), "big")
        out ^= add
    return out

def fold_small(reg: int, arena: bytes, a: int, L: int) -> int:
    """crc32_kernels.hip fold_small (the join's short segments, <= 64 B): the aligned
    dwords covering [a, a + L) loaded first, each 4 bytes one slicing-by-4 step on the
    dword v_alignbyte cuts at a mod 4 (T_3 for the first byte .. T_0 for the last),
    the last L mod 4 bytes Sarwate steps."""
    sh, base = a & 3, a & ~3
    nd = (sh + L + 3) >> 2
    d = [int.from_bytes(arena[base + 4 * k:base + 4 * k + 4], "little") if k < nd else 0 for k in range(18)]

    def alignbyte(hi, lo, s):
        return ((hi << 32 | lo) >> (8 * s)) & 0xFFFFFFFF

    nf = L >> 2
    for i in range(nf):
        x = reg ^ alignbyte(d[i + 1], d[i], sh)
        reg = TS[3][x & 0xFF] ^ TS[2][(x >> 8) & 0xFF] ^ TS[1][(x >> 16) & 0xFF] ^ TS[0][x >> 24]
    tail = alignbyte(d[nf + 1], d[nf], sh)
    for j in range(L & 3):
        reg = TS[0][(reg ^ (tail >> (8 * j))) & 0xFF] ^ (reg >> 8)
    return reg


# ---------------------------------------------------------------- unstep column
def unstep_table() -> list[int]:
    """Free column 28 of every image (kUnstepCol): U[t0(b) >> 24] = (t0(b) << 8) | b, so one
    zero byte is undone as reg x^(-8) = (reg << 8) ^ U[reg >> 24].  The vring kernel applies
    CINV[tz] = x^(-8 tz) as tz such unsteps (vr_unstep)."""
    U = [0] * 256
    for b in range(256):
        t = t0(b)
        U[t >> 24] = ((t << 8) & 0xFFFFFFFF) | b
    return U


def unstep(reg: int, n: int, U=None) -> int:
    U = U or unstep_table()
    for _ in range(n):
        reg = ((reg << 8) & 0xFFFFFFFF) ^ U[reg >> 24]
    return reg


# ---------------------------------------------------------------- tz multipliers
def tz_tables() -> list[list[list[int]]]:
    """crc32_vring.hip's zero-byte multiplier tables (HostTables::tz, tz_addr):
    table k (0: 16 zero bytes, 1: 8), byte b, entry v = (v << 8b) x^(-8 (16 or 8))."""
    return [[[mulmod(v << (8 * b), CINV[16 if k == 0 else 8]) for v in range(256)] for b in range(4)]
            for k in range(2)]


def tz_small_tables() -> list[list[list[int]]]:
    """The records instance's small tables (HostTables::tz after the two above,
    tz_small_addr): table c (1..7) byte b, entry v = (v << 8b) x^(-8 c)."""
    return [[[mulmod(v << (8 * b), CINV[c]) for v in range(256)] for b in range(4)] for c in range(1, 8)]


def vr_unstep_tz(reg: int, tz: int, tabs=None, small=None) -> int:
    """vr_unstep_tz: reg x^(-8 tz), tz < 32 -- the 16- and 8-byte parts as four
    table lookups each, the rest as zero-byte unsteps."""
    tabs = tabs or tz_tables()
    for k, z in ((0, 16), (1, 8)):
        if tz & z:
            reg = tabs[k][0][reg & 0xFF] ^ tabs[k][1][(reg >> 8) & 0xFF] ^ tabs[k][2][(reg >> 16) & 0xFF] ^ \
                tabs[k][3][reg >> 24]
    if small is not None and tz & 7:                    # (the records instance: vr_tz7_mul)
        t = small[(tz & 7) - 1]
        return t[0][reg & 0xFF] ^ t[1][(reg >> 8) & 0xFF] ^ t[2][(reg >> 16) & 0xFF] ^ t[3][reg >> 24]
    for _ in range(tz & 7):
        reg = unstep_zero(reg)
    return reg
