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
    """dword j*32 + t = T_t[j]  (256 rows x 32 dwords = 32 KiB, crc32_device.hpp)."""
    img = [0] * (256 * 32)
    for j in range(256):
        for t in range(32):
            img[j * 32 + t] = TS[t][j]
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
    l5 = lane & 31
    col = []
    for g in range(8):
        r = 0
        for h in range(4):
            i = 4 * g + h
            t = (i ^ l5) ^ 31
            r |= (8 * t) << (8 * h)
        col.append(r)
    sel = [h | ((4 + (h ^ (l5 & 3))) << 8) | 0x0C0C0000 for h in range(4)]
    return col, sel, bool((l5 >> 2) & 1), bool((l5 >> 3) & 1), bool((l5 >> 4) & 1)


def lookup_addresses(lane: int, words: list[int]) -> list[int]:
    """LDS byte address of each of the 32 lookups of fold_block (words in original
    order, state already XORed): halves put in lane order, two dword-swap rounds,
    then v_perm(...) >> 1."""
    col, sel, sw1, sw2, hs = make_sched(lane)
    w = (words[4:8] + words[0:4]) if hs else list(words)
    x = [w[q ^ 1] if sw1 else w[q] for q in range(8)]
    d = [x[q ^ 2] if sw2 else x[q] for q in range(8)]
    return [v_perm(d[i >> 2], col[i >> 2], sel[i & 3]) >> 1 for i in range(32)]


def fold_block(reg: int, block: bytes, lane: int) -> int:
    w = [int.from_bytes(block[4 * q:4 * q + 4], "little") for q in range(8)]
    w[0] ^= reg
    acc = 0
    for addr in lookup_addresses(lane, w):
        assert addr % 4 == 0 and addr < 32768
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


def segment_cuts(addr: int, L: int, lanes: int) -> list[int]:
    """make_task's cut points: packet [addr, addr+L) split at 128-byte-aligned
    absolute addresses nearest to the even split (offsets relative to addr)."""
    cuts = [0]
    for k in range(1, lanes):
        r = (addr + (L * k) // lanes + 64) & ~127
        cuts.append(min(max(r, addr), addr + L) - addr)
    cuts.append(L)
    return cuts


def crc_packet(pkt: bytes, lanes: int = 1, lane_base: int = 0, addr: int = 0) -> int:
    """What one packet's P lanes compute: lane k folds segment [cut_k, cut_k+1) as
    its own end-aligned window (zero-init except lane 0, which starts at
    INIT[rp]), then the partial registers are advanced and XORed."""
    L = len(pkt)
    cuts = segment_cuts(addr, L, lanes)
    total = 0
    for k in range(lanes):
        seg = pkt[cuts[k]:cuts[k + 1]]
        nb = (len(seg) + 31) // 32
        rp = 32 * nb - len(seg)
        reg = INIT[rp] if k == 0 else 0
        reg = fold_window(reg, seg, 0, nb, lane_base + k)
        after = L - cuts[k + 1]
        if after:
            reg = mulmod(reg, x8n(after))
        total ^= reg
    return int.from_bytes((~total & 0xFFFFFFFF).to_bytes(4, "little"), "big")


def verify_packet(pkt: bytes, slot_off: int, connect: int, lanes: int = 1) -> tuple[bool, int]:
    L = len(pkt)
    if slot_off + 4 > L:
        return False, 0
    cuts = segment_cuts(0, L, lanes)
    total = 0
    for k in range(lanes):
        seg = pkt[cuts[k]:cuts[k + 1]]
        nb = (len(seg) + 31) // 32
        rp = 32 * nb - len(seg)
        reg = fold_window(INIT[rp] if k == 0 else 0, seg, 0, nb, k)
        if L - cuts[k + 1]:
            reg = mulmod(reg, x8n(L - cuts[k + 1]))
        total ^= reg
    desired = int.from_bytes(pkt[slot_off:slot_off + 4], "little")
    total ^= mulmod(desired ^ connect, x8n(L - slot_off))
    comp = int.from_bytes((~total & 0xFFFFFFFF).to_bytes(4, "little"), "big")
    return comp == desired, comp
