"""Host-side model of the gfx950 kernel's arithmetic (test infrastructure).

Restates, in Python integers, exactly what crc32_kernels.hip does per lane --
LDS image layout, per-lane v_perm selectors and column bytes, the dword swaps,
slicing-by-32 folding, END-aligned windows with INIT[r'], splitting a packet over
P lanes and the GF(2) carry-combine -- so the algebra and the bank mapping can be
checked on CPU against the oracle before any GPU run.  It models the arithmetic,
not the hardware: parity on the device is established by the -m gpu tests.
"""
from __future__ import annotations

POLY = 0xEDB88320


def t0(n: int) -> int:
    c = n
    for _ in range(8):
        c = (c >> 1) ^ POLY if c & 1 else c >> 1
    return c


T0 = [t0(n) for n in range(256)]


def slicing_tables(k: int = 32) -> list[list[int]]:
    T = [T0[:]]
    for _ in range(1, k):
        prev = T[-1]
        T.append([(prev[j] >> 8) ^ T0[prev[j] & 0xFF] for j in range(256)])
    return T


TS = slicing_tables(32)


def lds_image() -> list[int]:
    """dword j*64 + 2t + c = T_t[j]  (256 rows x 64 dwords = 64 KiB)."""
    img = [0] * (256 * 64)
    for j in range(256):
        for t in range(32):
            for c in range(2):
                img[j * 64 + 2 * t + c] = TS[t][j]
    return img


IMG = lds_image()


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
        else:  # 8..11: sign replication of bytes 1,3,5,7 (unused by the kernel)
            src = (data >> (8 * (2 * (sb - 8) + 1) + 7)) & 1
            b = 0xFF if src else 0
        out |= b << (8 * k)
    return out


def make_sched(lane: int):
    v, c = lane & 15, (lane >> 4) & 1
    col = []
    for g in range(8):
        r = 0
        for h in range(4):
            i = 4 * g + h
            t = (i ^ v) ^ 31
            r |= (8 * t + 4 * c) << (8 * h)
        col.append(r)
    sel = [h | ((4 + (h ^ (v & 3))) << 8) | 0x0C0C0000 for h in range(4)]
    return col, sel, bool((v >> 2) & 1), bool((v >> 3) & 1)


def lookup_addresses(lane: int, words: list[int]) -> list[int]:
    """LDS byte address of each of the 32 lookups of fold_block (state already XORed)."""
    col, sel, sw1, sw2 = make_sched(lane)
    x = [words[q ^ 1] if sw1 else words[q] for q in range(8)]
    d = [x[q ^ 2] if sw2 else x[q] for q in range(8)]
    return [v_perm(d[i >> 2], col[i >> 2], sel[i & 3]) for i in range(32)]


def fold_block(reg: int, block: bytes, lane: int) -> int:
    w = [int.from_bytes(block[4 * q:4 * q + 4], "little") for q in range(8)]
    w[0] ^= reg
    acc = 0
    for addr in lookup_addresses(lane, w):
        assert addr % 4 == 0 and addr < 65536
        acc ^= IMG[addr // 4]
    return acc


def mulmod(a: int, b: int) -> int:
    p = 0
    for j in range(32):
        if (a >> (31 - j)) & 1:
            p ^= b
        b = (b >> 1) ^ (POLY if b & 1 else 0)
    return p


def x8n(n: int) -> int:
    r = 0x80000000
    for _ in range(n):
        r = (r >> 8) ^ T0[r & 0xFF]
    return r


def unstep_zero(reg_next: int) -> int:
    top = reg_next >> 24
    n = next(k for k in range(256) if (T0[k] >> 24) == top)
    return (((reg_next ^ T0[n]) << 8) & 0xFFFFFFFF) | n


INIT = [0xFFFFFFFF]
for _ in range(31):
    INIT.append(unstep_zero(INIT[-1]))


def fold_window(reg: int, pkt: bytes, j0: int, j1: int, lane: int) -> int:
    L = len(pkt)
    nb = (L + 31) // 32
    rp = 32 * nb - L
    win = bytes(rp) + pkt          # bytes in front of the packet read as zero
    for j in range(j0, j1):
        reg = fold_block(reg, win[32 * j:32 * j + 32], lane)
    return reg


def crc_packet(pkt: bytes, lanes: int = 1, lane_base: int = 0) -> int:
    """What one packet's P lanes compute (packets start at lane_base, a multiple of P)."""
    L = len(pkt)
    nb = (L + 31) // 32
    rp = 32 * nb - L
    per, rem = nb // lanes, nb % lanes
    total = 0
    for k in range(lanes):
        j0 = k * per + min(k, rem)
        j1 = j0 + per + (1 if k < rem else 0)
        reg = INIT[rp] if k == 0 else 0
        reg = fold_window(reg, pkt, j0, j1, lane_base + k)
        after = nb - j1
        if after:
            reg = mulmod(reg, x8n(32 * after))
        total ^= reg
    return int.from_bytes((~total & 0xFFFFFFFF).to_bytes(4, "little"), "big")


def verify_packet(pkt: bytes, slot_off: int, connect: int, lanes: int = 1) -> tuple[bool, int]:
    L = len(pkt)
    if slot_off + 4 > L:
        return False, 0
    nb = (L + 31) // 32
    rp = 32 * nb - L
    per, rem = nb // lanes, nb % lanes
    total = 0
    for k in range(lanes):
        j0 = k * per + min(k, rem)
        j1 = j0 + per + (1 if k < rem else 0)
        reg = fold_window(INIT[rp] if k == 0 else 0, pkt, j0, j1, k)
        if nb - j1:
            reg = mulmod(reg, x8n(32 * (nb - j1)))
        total ^= reg
    desired = int.from_bytes(pkt[slot_off:slot_off + 4], "little")
    total ^= mulmod(desired ^ connect, x8n(L - slot_off))
    comp = int.from_bytes((~total & 0xFFFFFFFF).to_bytes(4, "little"), "big")
    return comp == desired, comp
