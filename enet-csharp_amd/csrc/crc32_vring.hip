// crc32_vring.hip -- the VGPR-ring CRC32 kernel for gfx950 (MI355X): the default
// batched checksum path of libenethip.  Path replaced: ENet.enet_crc32
// (/root/reference/enet-csharp/ENet/c/packet.cs:142-160) over a whole batch of
// DGRAMs, one CRC per packet, in wire order (packet.cs:159).
//
// Arithmetic (tests/kernel_model.py): P = 2^LG lanes per packet
// fold its 32-byte window blocks strided -- lane k folds blocks k, k+P, k+2P, ...
// -- with the advancing slicing-by-32 tables T'_t = T_{t+32(P-1)} of the P image
// in LDS, so every fold also skips the P-1 blocks the other lanes own.
//   * Window: starts at the 64-byte boundary at or before the packet's first
//     byte (lz < 64 leading bytes) and spans nb = ceil((lz + L)/32) blocks, so
//     tz = 32 nb - lz - L < 32 trailing bytes.  Block 0's lane starts at INIT[lz]
//     (the register that lz zero bytes carry to 0xFFFFFFFF, packet.cs:144).
//   * Lane k ends o = (k - nb) mod P blocks past the window end: one multiply by
//     x^(-256 o) (four byte-indexed lookups in the image's correction columns),
//     a DPP XOR of the P lanes, then x^(-8 tz) (CINV[tz]) on the packet's lane 0.
//   * Data goes straight into VGPRs: stage s of a packet = its window bytes
//     [256 s, 256 s + 256) at P = 8, lane k loading its own block k + P s as two
//     16-byte loads, a two-slot register ring (one stage in flight while one is
//     folded).  A 16-byte piece wholly outside [lz, lz + L) is read from a zero
//     line instead; a partly covered piece (a packet start or end off a 16-byte
//     boundary) is masked on the fold side in a wave-uniform edge branch.
//   * LDS holds the 64 KiB table image (rebuilt per workgroup from a 2.5 KiB
//     GF(2) basis while the first stage is in flight) and each wave's 768-B
//     metadata area (79.5 KiB), so two 16-wave workgroups share a CU (32 waves;
//     64 VGPRs, of which v48-v63 are the ring).
//   * One launch may cover a list of batches (enet_hip_crc32_batch_list_device):
//     each batch's groups dealt over all waves, the launch's start and drain paid
//     once for the list.
// Measured design choices (tools/pipebench.hip, profiles/r02_*): 64-byte window
// starts beat the end-aligned 16-byte windows of the lean kernel (every DMA run
// then covers whole 64-byte sectors), and the register ring at 32 waves per CU
// beats the LDS-DMA ring at 16.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "crc32_vring.hpp"

namespace enethip {

constexpr int kVrW = 16;                                        // waves per workgroup
constexpr uint32_t kVrStaging = kLdsTableBytes;                 // basis rows land after the image
// per wave, the metadata of the next group: ONE LDS-DMA instruction whose 64 lanes
// load the group's fields, field f of packet p (of the group's kPk) at +4 (f kPk + p):
// f = 0 the length, 1 / 2 the offset's low / high dword (BIN: the record's dwords
// {len, off_lo, off_hi, index}, f = 3 the index).  3 x 8 fields at 8 lanes per
// packet, 3 x 16 or 4 x 16 at 4; the remaining lanes repeat field 0.  (Round 2 used
// one instruction per field, each lane loading its own packet's copy: 3 or 4 VMEM
// instructions and 768 / 1024 B of LDS per wave, against 1 and 256 B here.)
constexpr uint32_t kVrMeta = kVrStaging + kVrBasisRows * 256;
constexpr uint32_t kVrMetaWave = 256;
constexpr uint32_t kVrCtr = kVrMeta + kVrW * kVrMetaWave;       // the workgroup's slot counter (16 B)
// the zero-byte multiplier tables (tz_addr, KernelTables::tz), DMA'd once per workgroup
constexpr uint32_t kVrTz = kVrCtr + 16;
// the workgroup's round table (dynamic rounds, VrBatches::claim): entry r % 64 =
// {tag r, chunk of round r}, 8 B each.  An entry is rewritten 64 rounds (1024
// slot takes of the workgroup) after it was published; its readers read it right
// after their own take of a slot of its round
constexpr uint32_t kVrRound = kVrTz + kTzTableDwords * 4;
constexpr int kVrRounds = 64;
// ... and the launch's claim words (VrBatches::claim), kept here, not in SGPRs
constexpr uint32_t kVrClaimPtr = kVrRound + kVrRounds * 8;
constexpr int kVrLds = kVrClaimPtr + 16;                         // 79 KiB: two workgroups per CU
static_assert(2 * kVrLds <= 160 * 1024, "two workgroups per CU");
// length-binned records (BIN): the same area and layout, plus the x^(-8 c) tables for
// c < 8 (tz_small_addr) -- 106.5 KiB: one workgroup per CU, the records entries' default
constexpr uint32_t kVrMetaWaveBin = kVrMetaWave;
constexpr uint32_t kVrCtrBin = kVrCtr;
constexpr uint32_t kVrTz7 = kVrLds;
// ... and the workgroup's 16 partial maxima of the binned gather's tile counts
constexpr uint32_t kVrTileMax = kVrTz7 + kTzSmallDwords * 4;
constexpr int kVrLdsBin = kVrTileMax + kVrW * 4;
static_assert(kVrLdsBin <= 160 * 1024, "records instance LDS");
// the compact records instance (BIN = 2): no x^(-8 c) tables (tz mod 8 by unsteps), the
// tile maxima right after the plain layout -- 79 KiB, two workgroups per CU
constexpr uint32_t kVrTileMaxC = kVrLds;
constexpr int kVrLdsBinC = kVrTileMaxC + kVrW * 4;
static_assert(2 * kVrLdsBinC <= 160 * 1024, "compact records instance: two workgroups per CU");
template <int BIN>
constexpr uint32_t vr_tile_max() { return BIN >= 2 ? kVrTileMaxC : kVrTileMax; }
// the local-tile records instance (BIN = 3): its prologue's counting sort -- 256 bins and
// the 4 scan waves' totals -- in the image area, which is free until barrier A
constexpr uint32_t kVrLocalBins = 256;
constexpr uint32_t kVrLocalHist = 0;
// ... and the staging of the metadata of each wave's second group (round 1), 256 B a wave
constexpr uint32_t kVrLocalNext = 2048;
static_assert(4u * (kVrLocalBins + kVrLocalBins / 64u) <= kVrLocalNext, "local sort's bins");
static_assert(kVrLocalNext + 256u * kVrW <= kLdsTableBytes, "local sort in the image area");
constexpr uint32_t kVrLocalItems = kVrLocalTile / (64u * kVrW);           // packets per thread
static_assert(kVrLocalItems * 64u * kVrW == kVrLocalTile, "whole packets per thread");
// an LDS add returning the old value (inline asm: no vmcnt wait put in front of it)
__device__ __forceinline__ uint32_t lds_add_rtn(uint32_t addr, uint32_t v) {
    uint32_t r;
    asm volatile("ds_add_rtn_u32 %0, %1, %2\n\ts_waitcnt lgkmcnt(0)" : "=v"(r) : "v"(addr), "v"(v) : "memory");
    return r;
}
// BIN's index stash (two slots of kPk dwords per wave) fits the basis staging area
static_assert(kVrW * 2 * 16 * 4 <= kVrBasisRows * 256, "index stash over the basis staging area");

// Global loads as inline asm, waited for by explicit counted vmcnt.  The
// compiler's own wait insertion loses count across the loop's group-switch
// branches and falls back to vmcnt(0) right after the next stage is issued,
// which empties the ring; and a loaded value the compiler can see is one it may
// copy while the load is still in flight.  So the stage loads write fixed
// registers -- ring slot 0 = v[48:55], slot 1 = v[56:63] -- that the compiler never
// allocates (amdgpu_num_vgpr on the kernel) and knows only as clobbered by the
// loads; the fold reads them in place after the wait (vr_shuffle_slot).  The
// metadata goes to LDS by LDS-DMA (no registers) and is read after its wait.  The
// build checks on the generated ISA that no compiler instruction touches a
// register while a load into it may be in flight (tools/isa_inflight_check.py,
// run by the Makefile).
// NT = 1: the loads carry the nontemporal cache policy (streamed once, not kept)
#define VR_LOAD2(LO, HI, POL)                                                                  \
    "global_load_dwordx4 v[" #LO "], %0, off" POL "\n\tglobal_load_dwordx4 v[" #HI "], %1, off" POL
template <int SLOT, int NT>
__device__ __forceinline__ void vr_issue_stage(uint64_t a0, uint64_t a1) {
    // NT: 0 = default policy, 1 = nt, 2 = sc1, 3 = sc0 sc1 (2, 3: tuning sweeps only)
#define VR_ISSUE(LO, HI, POL, ...)                                                              \
    asm volatile(VR_LOAD2(LO, HI, POL) :: "v"(a0), "v"(a1) : __VA_ARGS__)
#define VR_SLOT0 "v48", "v49", "v50", "v51", "v52", "v53", "v54", "v55"
#define VR_SLOT1 "v56", "v57", "v58", "v59", "v60", "v61", "v62", "v63"
    if constexpr (SLOT == 0) {
        if constexpr (NT == 0) VR_ISSUE(48:51, 52:55, "", VR_SLOT0);
        else if constexpr (NT == 1) VR_ISSUE(48:51, 52:55, " nt", VR_SLOT0);
        else if constexpr (NT == 2) VR_ISSUE(48:51, 52:55, " sc1", VR_SLOT0);
        else VR_ISSUE(48:51, 52:55, " sc0 sc1", VR_SLOT0);
    } else {
        if constexpr (NT == 0) VR_ISSUE(56:59, 60:63, "", VR_SLOT1);
        else if constexpr (NT == 1) VR_ISSUE(56:59, 60:63, " nt", VR_SLOT1);
        else if constexpr (NT == 2) VR_ISSUE(56:59, 60:63, " sc1", VR_SLOT1);
        else VR_ISSUE(56:59, 60:63, " sc0 sc1", VR_SLOT1);
    }
#undef VR_SLOT0
#undef VR_SLOT1
#undef VR_ISSUE
}
// the stage of SLOT has landed once at most N younger loads are in flight (no
// outputs: the fold reads the slot registers in place, vr_shuffle_slot)
template <int N>
__device__ __forceinline__ void vr_wait_stage() {
    asm volatile("s_waitcnt vmcnt(%0)" :: "n"(N) : "memory");
}
// a landed slot as values (the edge path, which masks them first)
template <int SLOT>
__device__ __forceinline__ void vr_read_stage(u32x4& a, u32x4& b) {
    if constexpr (SLOT == 0)
        asm volatile("" : "={v[48:51]}"(a), "={v[52:55]}"(b));
    else
        asm volatile("" : "={v[56:59]}"(a), "={v[60:63]}"(b));
}
// the group's metadata into the wave's LDS area at `base`: one M0-relative LDS-DMA
// (lane l's dword at base + 4 l, from the lane's own address); the LDS reads of the
// previous group's metadata are complete first (lgkmcnt(0)), so the DMA cannot
// overtake them
__device__ __forceinline__ void vr_issue_meta(uint64_t addr, uint32_t base) {
    asm volatile("s_waitcnt lgkmcnt(0)\n\t"
                 "s_mov_b32 m0, %1\n\t"
                 "global_load_lds_dword %0, off"
                 :: "v"(addr), "s"(base) : "m0", "memory");
}
// the metadata of the lane's packet p (of kPk) once at most N younger loads are in
// flight (BIN: and the record's caller index; VF: the slot offset and connectID)
template <int BIN, int VF, uint32_t kPk>
__device__ __forceinline__ void vr_read_meta(uint32_t base, uint32_t p, uint32_t& L, uint64_t& off, uint32_t& idx,
                                             uint32_t& so, uint32_t& conn) {
    L = lds_load(base + 4u * p);
    off = static_cast<uint64_t>(lds_load(base + 4u * (kPk + p))) |
          (static_cast<uint64_t>(lds_load(base + 4u * (2u * kPk + p))) << 32);
    if constexpr (BIN) idx = lds_load(base + 4u * (3u * kPk + p));
    if constexpr (VF) {
        so = lds_load(base + 4u * (3u * kPk + p));
        conn = lds_load(base + 4u * (4u * kPk + p));
    }
}
template <int N, int BIN, int VF, uint32_t kPk>
__device__ __forceinline__ void vr_wait_meta(uint32_t base, uint32_t p, uint32_t& L, uint64_t& off, uint32_t& idx,
                                             uint32_t& so, uint32_t& conn) {
    asm volatile("s_waitcnt vmcnt(%0)" :: "n"(N) : "memory");
    vr_read_meta<BIN, VF, kPk>(base, p, L, off, idx, so, conn);
}

// Receive verify (protocol.cs:1052-1068) in the lane folding the slot: the slot's
// bytes [rel, rel + 4) of this block (block byte offsets, may lie partly outside)
// are collected into `desired` (at their byte positions of the slot) and replaced
// by connectID's.  A, B in lane order (swapped when hs: A holds block bytes [16, 32)).
__device__ __forceinline__ void vr_slot_fix(u32x4& A, u32x4& B, uint32_t hs, int32_t rel, uint32_t conn,
                                            uint32_t& desired) {
    const bool sw = hs != 0;
    const u32x4 h0 = sw ? B : A, h1 = sw ? A : B;
    uint32_t v[8] = {h0.x, h0.y, h0.z, h0.w, h1.x, h1.y, h1.z, h1.w};
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        const int d = rel - 4 * q;                       // the slot's start relative to dword q
        if (d > -4 && d < 4) {
            uint32_t M, C;
            if (d >= 0) {
                M = 0xFFFFFFFFu << (8 * d);
                C = conn << (8 * d);
                desired |= v[q] >> (8 * d);
            } else {
                M = 0xFFFFFFFFu >> (-8 * d);
                C = conn >> (-8 * d);
                desired |= (v[q] & M) << (-8 * d);
            }
            v[q] = (v[q] & ~M) | (C & M);
        }
    }
    const u32x4 n0 = {v[0], v[1], v[2], v[3]}, n1 = {v[4], v[5], v[6], v[7]};
    A = sw ? n1 : n0;
    B = sw ? n0 : n1;
}
// every load retired (the wave's exit: no load may land after it has ended)
__device__ __forceinline__ void vr_drain() {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// false: the lane id and its derived constants are computed once and may be kept
// live across the ring loop (the kernel has VGPRs to spare below the ring)
constexpr bool kVrLaneRecompute = false;

// the lane id, not hoistable (see the kernel)
__device__ __forceinline__ uint32_t vr_lane() {
    uint32_t l;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
    return l;
}

// Zero the bytes of a block that lie outside the packet, [lo, hi) kept (block byte
// offsets, may lie outside [0, 32)), in place on the landed slot registers (the edge
// path then folds them like any stage, vr_shuffle_slot): register R of the slot's
// pair (A, B) holds block bytes [oR, oR + 16), oR = 0 or 16 by the lane's half swap
// (hs16 = lane & 16: A holds [16, 32) when set).  Dword i of R keeps bytes j with
// lo <= oR + 4i + j < hi.  Per dword and bound: s = clamp(4 (bound - oR) - 16 i, 0,
// 16) and m = (~0 << s) << s (0 .. 32 bits without the 5-bit shift wrap), kept =
// v & m (low bound) or v & ~m (high bound): four or five VALU.  Each bound is applied
// only where some lane of the wave needs it (wave-uniform branches).
#define VR_MASK_DWORD(REG, X, OFF, APPLY)                                                   \
    "v_subrev_u32 %[t], " OFF ", " X "\n\t"                                                \
    "v_med3_i32 %[t], %[t], 0, 16\n\t"                                                     \
    "v_lshlrev_b32 %[m], %[t], -1\n\t"                                                     \
    "v_lshlrev_b32 %[m], %[t], %[m]\n\t" APPLY(REG)
#define VR_KEEP_LO(REG) "v_and_b32 " REG ", " REG ", %[m]\n\t"
#define VR_DROP_HI(REG) "v_bfi_b32 " REG ", %[m], 0, " REG "\n\t"
#define VR_MASK_REG(R0, R1, R2, R3, X, APPLY)                                                 \
    "v_med3_i32 %[t], " X ", 0, 16\n\t"                                                        \
    "v_lshlrev_b32 %[m], %[t], -1\n\t"                                                         \
    "v_lshlrev_b32 %[m], %[t], %[m]\n\t" APPLY(R0)                                            \
    VR_MASK_DWORD(R1, X, "16", APPLY) VR_MASK_DWORD(R2, X, "32", APPLY) VR_MASK_DWORD(R3, X, "48", APPLY)
template <int SLOT>
__device__ __forceinline__ void vr_edge_mask_slot(uint32_t hs16, int32_t lo, int32_t hi) {
    const int32_t oa = static_cast<int32_t>(hs16), ob = 16 - oa;
    uint32_t t, m;
    if (__builtin_amdgcn_ballot_w64(lo > 0)) {
        const int32_t xa = 4 * (lo - oa), xb = 4 * (lo - ob);
        if constexpr (SLOT == 0)
            asm volatile(VR_MASK_REG("v48", "v49", "v50", "v51", "%[xa]", VR_KEEP_LO)
                         VR_MASK_REG("v52", "v53", "v54", "v55", "%[xb]", VR_KEEP_LO)
                         : [t] "=&v"(t), [m] "=&v"(m) : [xa] "v"(xa), [xb] "v"(xb));
        else
            asm volatile(VR_MASK_REG("v56", "v57", "v58", "v59", "%[xa]", VR_KEEP_LO)
                         VR_MASK_REG("v60", "v61", "v62", "v63", "%[xb]", VR_KEEP_LO)
                         : [t] "=&v"(t), [m] "=&v"(m) : [xa] "v"(xa), [xb] "v"(xb));
    }
    if (__builtin_amdgcn_ballot_w64(hi < 32)) {
        const int32_t ya = 4 * (hi - oa), yb = 4 * (hi - ob);
        if constexpr (SLOT == 0)
            asm volatile(VR_MASK_REG("v48", "v49", "v50", "v51", "%[ya]", VR_DROP_HI)
                         VR_MASK_REG("v52", "v53", "v54", "v55", "%[yb]", VR_DROP_HI)
                         : [t] "=&v"(t), [m] "=&v"(m) : [ya] "v"(ya), [yb] "v"(yb));
        else
            asm volatile(VR_MASK_REG("v56", "v57", "v58", "v59", "%[ya]", VR_DROP_HI)
                         VR_MASK_REG("v60", "v61", "v62", "v63", "%[yb]", VR_DROP_HI)
                         : [t] "=&v"(t), [m] "=&v"(m) : [ya] "v"(ya), [yb] "v"(yb));
    }
}

// Lane constants of the fold (make_sched's, compressed).  The column byte of
// table t is col_byte(t) = t << 3 | (t >> 4) << 2, GF(2)-linear in t, so the
// column of step i = 4g + h for lane l, col_byte(31 ^ i ^ l5), is the
// compile-time bytes of col_byte(31 ^ i) XOR one per-lane byte col_byte(l5):
// one register instead of eight, one XOR per 4 lookups.
// The four v_perm selectors of make_sched differ by constants: sel[h] =
// sel0 ^ (h * 0x101), one register instead of four.
struct VrSched {
    uint32_t cl;        // col_byte(l & 31) in all four bytes
    uint32_t sel0;      // make_sched's sel[0]
    uint32_t hs;
};

__device__ __forceinline__ VrSched make_vr_sched(uint32_t lane) {
    const LaneSched a = make_sched(lane);
    VrSched s;
    s.cl = __builtin_amdgcn_perm(0u, col_byte(lane & 31u), 0u);   // the byte in all four (no multiply)
    s.sel0 = a.sel[0];
    s.hs = a.hs;
    return s;
}

// reg x^(-8 z) for z = 16 (K = 0) or 8 (K = 1): four lookups in the zero-byte
// multiplier tables at kVrTz (tz_addr), addresses by shift-and-add (asm: hipcc
// would hoist the 4 table bases into VGPRs)
template <int K>
__device__ __forceinline__ uint32_t vr_tz_mul(uint32_t reg, uint32_t tzbase) {
    uint32_t a0, a1, a2, a3;
    const uint32_t b = tzbase + 4096u * K;
    asm volatile("v_and_b32 %[a0], 0xff, %[r]\n\t"
                 "v_bfe_u32 %[a1], %[r], 8, 8\n\t"
                 "v_bfe_u32 %[a2], %[r], 16, 8\n\t"
                 "v_lshrrev_b32 %[a3], 24, %[r]\n\t"
                 "v_lshl_add_u32 %[a0], %[a0], 2, %[b0]\n\t"
                 "v_lshl_add_u32 %[a1], %[a1], 2, %[b1]\n\t"
                 "v_lshl_add_u32 %[a2], %[a2], 2, %[b2]\n\t"
                 "v_lshl_add_u32 %[a3], %[a3], 2, %[b3]\n\t"
                 "ds_read_b32 %[a0], %[a0]\n\t"
                 "ds_read_b32 %[a1], %[a1]\n\t"
                 "ds_read_b32 %[a2], %[a2]\n\t"
                 "ds_read_b32 %[a3], %[a3]\n\t"
                 "s_waitcnt lgkmcnt(0)\n\t"
                 "v_bitop3_b32 %[r], %[a0], %[a1], %[a2] bitop3:0x96\n\t"
                 "v_xor_b32 %[r], %[r], %[a3]"
                 : [r] "+v"(reg), [a0] "=&v"(a0), [a1] "=&v"(a1), [a2] "=&v"(a2), [a3] "=&v"(a3)
                 : [b0] "s"(b), [b1] "s"(b + 1024u), [b2] "s"(b + 2048u), [b3] "s"(b + 3072u)
                 : "memory");
    return reg;
}

// reg x^(-8 c), 0 < c < 8: four lookups in the records instance's small tables
// (kVrTz7, tz_small_addr); the unsteps they replace were one U-column lookup each,
// every active lane on one bank (up to seven 16-way conflicts per group at 4 lanes)
__device__ __forceinline__ uint32_t vr_tz7_mul(uint32_t reg, uint32_t c) {
    const uint32_t base = kVrTz7 + 4096u * (c - 1u);
    const uint32_t x0 = lds_load(base + 4u * (reg & 0xFFu));
    const uint32_t x1 = lds_load(base + 1024u + 4u * ((reg >> 8) & 0xFFu));
    const uint32_t x2 = lds_load(base + 2048u + 4u * ((reg >> 16) & 0xFFu));
    const uint32_t x3 = lds_load(base + 3072u + 4u * (reg >> 24));
    return xor3(x0, x1, x2) ^ x3;
}

// reg x^(-8 tz), tz < 32: the 16- and 8-byte parts by the tables, the rest by unsteps
// (SMALL, the records instance: by the small tables)
template <bool SMALL = false>
__device__ __forceinline__ uint32_t vr_unstep_tz(uint32_t reg, uint32_t tz, uint32_t tzbase) {
    if (tz & 16u) reg = vr_tz_mul<0>(reg, tzbase);
    if (tz & 15u) {                                          // (one test for the smaller steps: cfg2's tz is 0 or 16)
        if (tz & 8u) reg = vr_tz_mul<1>(reg, tzbase);
        if constexpr (SMALL) {
            if (tz & 7u) reg = vr_tz7_mul(reg, tz & 7u);
        } else {
            if (tz & 4u) {
#pragma unroll
                for (int j = 0; j < 4; ++j) reg = unstep_byte(reg);
            }
            if (tz & 2u) {
                reg = unstep_byte(reg);
                reg = unstep_byte(reg);
            }
            if (tz & 1u) reg = unstep_byte(reg);
        }
    }
    return reg;
}

template <int G>
__device__ __forceinline__ constexpr uint32_t vr_col_const() {
    uint32_t r = 0;
    for (int h = 0; h < 4; ++h) r |= col_byte(31u ^ static_cast<uint32_t>(4 * G + h)) << (8 * h);
    return r;
}

// The fold's data preparation (fold_block_lane's first half, crc32_device.hpp):
// the register XORed into the block's first dword (A.x, or B.x when the lane
// takes the halves swapped: hs), then the two dword-swap rounds -- d[q] =
// w[q ^ ((lane >> 2) & 3)] -- as bitwise selects by the lane's masks m1, m2.  One
// asm block, so the 8 source dwords are read where they are (the slot registers
// of vr_issue_stage, or any registers for the edge path's masked copy) and the
// only live values are the 8 results and 2 temporaries.
#define VR_SHUFFLE_ASM(S0, S1, S2, S3, S4, S5, S6, S7)                                            \
    "v_bfe_i32 %[t0], %[lane], 4, 1\n\t"                      /* hs */                                \
    "v_bitop3_b32 %[d0], " S0 ", %[reg], %[t0] bitop3:0xb4\n\t" /* w0 = A.x ^ (reg & ~hs) */        \
    "v_bitop3_b32 %[d4], " S4 ", %[reg], %[t0] bitop3:0x78\n\t" /* w4 = B.x ^ (reg & hs) */         \
    "v_bfe_i32 %[t0], %[lane], 2, 1\n\t"                      /* m1 */                                \
    "v_bitop3_b32 %[d1], " S1 ", %[d0], %[t0] bitop3:0xd8\n\t" /* x1 = m1 ? w0 : w1 */              \
    "v_bitop3_b32 %[d0], %[d0], " S1 ", %[t0] bitop3:0xd8\n\t" /* x0 = m1 ? w1 : w0 */              \
    "v_bitop3_b32 %[d2], " S2 ", " S3 ", %[t0] bitop3:0xd8\n\t"                                       \
    "v_bitop3_b32 %[d3], " S3 ", " S2 ", %[t0] bitop3:0xd8\n\t"                                       \
    "v_bitop3_b32 %[d5], " S5 ", %[d4], %[t0] bitop3:0xd8\n\t"                                        \
    "v_bitop3_b32 %[d4], %[d4], " S5 ", %[t0] bitop3:0xd8\n\t"                                        \
    "v_bitop3_b32 %[d6], " S6 ", " S7 ", %[t0] bitop3:0xd8\n\t"                                       \
    "v_bitop3_b32 %[d7], " S7 ", " S6 ", %[t0] bitop3:0xd8\n\t"                                       \
    "v_bfe_i32 %[t0], %[lane], 3, 1\n\t"                      /* m2: d[q] = m2 ? x[q^2] : x[q] */    \
    "v_bitop3_b32 %[t1], %[d0], %[d2], %[t0] bitop3:0xd8\n\t"                                         \
    "v_bitop3_b32 %[d2], %[d2], %[d0], %[t0] bitop3:0xd8\n\t"                                         \
    "v_mov_b32 %[d0], %[t1]\n\t"                                                                       \
    "v_bitop3_b32 %[t1], %[d1], %[d3], %[t0] bitop3:0xd8\n\t"                                         \
    "v_bitop3_b32 %[d3], %[d3], %[d1], %[t0] bitop3:0xd8\n\t"                                         \
    "v_mov_b32 %[d1], %[t1]\n\t"                                                                       \
    "v_bitop3_b32 %[t1], %[d4], %[d6], %[t0] bitop3:0xd8\n\t"                                         \
    "v_bitop3_b32 %[d6], %[d6], %[d4], %[t0] bitop3:0xd8\n\t"                                         \
    "v_mov_b32 %[d4], %[t1]\n\t"                                                                       \
    "v_bitop3_b32 %[t1], %[d5], %[d7], %[t0] bitop3:0xd8\n\t"                                         \
    "v_bitop3_b32 %[d7], %[d7], %[d5], %[t0] bitop3:0xd8\n\t"                                         \
    "v_mov_b32 %[d5], %[t1]"
#define VR_SHUFFLE_OUTS(d)                                                                        \
    [d0] "=&v"(d[0]), [d1] "=&v"(d[1]), [d2] "=&v"(d[2]), [d3] "=&v"(d[3]), [d4] "=&v"(d[4]),    \
        [d5] "=&v"(d[5]), [d6] "=&v"(d[6]), [d7] "=&v"(d[7]), [t0] "=&v"(t0), [t1] "=&v"(t1)

// The same preparation IN PLACE on a landed slot (round 5): the register XORed into
// the slot's dword 0 or 4 (hs), then the two swap rounds as v_swap_b32 under EXEC
// masks -- lanes with bit 2 of l5 swap dwords q <-> q ^ 1, lanes with bit 3 swap
// q <-> q ^ 2 -- so the fold reads the slot registers themselves (vr_slot_values):
// 1 + 2 VALU + 8 swaps against vr_shuffle_slot's 25 VALU with 8 result copies.  The
// masks are the lane patterns of those bits (0xF0 and 0xFF00 repeated); EXEC is
// restored before the block ends (the fold runs on whole waves).  Only a landed slot
// may be written (tools/isa_inflight_check.py checks every path).
#define VR_ROTATE_ASM(S0, S1, S2, S3, S4, S5, S6, S7)                                             \
    "v_bfe_i32 %[t0], %[lane], 4, 1\n\t"                      /* hs */                                \
    "v_bitop3_b32 " S0 ", " S0 ", %[reg], %[t0] bitop3:0xb4\n\t" /* A.x ^= reg & ~hs */             \
    "v_bitop3_b32 " S4 ", " S4 ", %[reg], %[t0] bitop3:0x78\n\t" /* B.x ^= reg & hs */              \
    "s_mov_b64 %[sv], exec\n\t"                                                                        \
    "s_and_b32 exec_lo, exec_lo, 0xf0f0f0f0\n\t"              /* m1 lanes */                          \
    "s_and_b32 exec_hi, exec_hi, 0xf0f0f0f0\n\t"                                                       \
    "v_swap_b32 " S0 ", " S1 "\n\t"                                                                    \
    "v_swap_b32 " S2 ", " S3 "\n\t"                                                                    \
    "v_swap_b32 " S4 ", " S5 "\n\t"                                                                    \
    "v_swap_b32 " S6 ", " S7 "\n\t"                                                                    \
    "s_mov_b64 exec, %[sv]\n\t"                                                                        \
    "s_and_b32 exec_lo, exec_lo, 0xff00ff00\n\t"              /* m2 lanes */                          \
    "s_and_b32 exec_hi, exec_hi, 0xff00ff00\n\t"                                                       \
    "v_swap_b32 " S0 ", " S2 "\n\t"                                                                    \
    "v_swap_b32 " S1 ", " S3 "\n\t"                                                                    \
    "v_swap_b32 " S4 ", " S6 "\n\t"                                                                    \
    "v_swap_b32 " S5 ", " S7 "\n\t"                                                                    \
    "s_mov_b64 exec, %[sv]"
template <int SLOT>
__device__ __forceinline__ void vr_rotate_slot(uint32_t reg, uint32_t lane, uint32_t (&d)[8]) {
    uint32_t t0;
    uint64_t sv;
    if constexpr (SLOT == 0) {
        asm volatile(VR_ROTATE_ASM("v48", "v49", "v50", "v51", "v52", "v53", "v54", "v55")
                     : [t0] "=&v"(t0), [sv] "=&s"(sv) : [reg] "v"(reg), [lane] "v"(lane)
                     : "v48", "v49", "v50", "v51", "v52", "v53", "v54", "v55", "memory");
        asm volatile("" : "={v48}"(d[0]), "={v49}"(d[1]), "={v50}"(d[2]), "={v51}"(d[3]), "={v52}"(d[4]),
                          "={v53}"(d[5]), "={v54}"(d[6]), "={v55}"(d[7]));
    } else {
        asm volatile(VR_ROTATE_ASM("v56", "v57", "v58", "v59", "v60", "v61", "v62", "v63")
                     : [t0] "=&v"(t0), [sv] "=&s"(sv) : [reg] "v"(reg), [lane] "v"(lane)
                     : "v56", "v57", "v58", "v59", "v60", "v61", "v62", "v63", "memory");
        asm volatile("" : "={v56}"(d[0]), "={v57}"(d[1]), "={v58}"(d[2]), "={v59}"(d[3]), "={v60}"(d[4]),
                          "={v61}"(d[5]), "={v62}"(d[6]), "={v63}"(d[7]));
    }
}

template <int SLOT>
__device__ __forceinline__ void vr_shuffle_slot(uint32_t reg, uint32_t lane, uint32_t (&d)[8]);
// true: the fold reads the slot registers rotated in place (vr_rotate_slot); false: the
// round-2 copies (vr_shuffle_slot)
constexpr bool kVrRotateInPlace = true;
// (IP = false: the records instance's record-order diagnostics (ABL 64), which spill
// 8 bytes with the in-place form)
template <int SLOT, bool IP = true>
__device__ __forceinline__ void vr_prepare(uint32_t reg, uint32_t lane, uint32_t (&d)[8]) {
    if constexpr (kVrRotateInPlace && IP) vr_rotate_slot<SLOT>(reg, lane, d);
    else vr_shuffle_slot<SLOT>(reg, lane, d);
}

template <int SLOT>
__device__ __forceinline__ void vr_shuffle_slot(uint32_t reg, uint32_t lane, uint32_t (&d)[8]) {
    uint32_t t0, t1;
    if constexpr (SLOT == 0)
        asm volatile(VR_SHUFFLE_ASM("v48", "v49", "v50", "v51", "v52", "v53", "v54", "v55")
                     : VR_SHUFFLE_OUTS(d) : [reg] "v"(reg), [lane] "v"(lane));
    else
        asm volatile(VR_SHUFFLE_ASM("v56", "v57", "v58", "v59", "v60", "v61", "v62", "v63")
                     : VR_SHUFFLE_OUTS(d) : [reg] "v"(reg), [lane] "v"(lane));
}
__device__ __forceinline__ void vr_shuffle(uint32_t reg, uint32_t lane, const u32x4& A, const u32x4& B,
                                           uint32_t (&d)[8]) {
    uint32_t t0, t1;
    asm volatile(VR_SHUFFLE_ASM("%[a0]", "%[a1]", "%[a2]", "%[a3]", "%[b0]", "%[b1]", "%[b2]", "%[b3]")
                 : VR_SHUFFLE_OUTS(d)
                 : [reg] "v"(reg), [lane] "v"(lane), [a0] "v"(A.x), [a1] "v"(A.y), [a2] "v"(A.z), [a3] "v"(A.w),
                   [b0] "v"(B.x), [b1] "v"(B.y), [b2] "v"(B.z), [b3] "v"(B.w));
}

// fold_block_lane's lookups (crc32_device.hpp) on the prepared dwords, at most 8
// table lookups in flight: groups of 4, group g+1 issued before group g is
// XOR-reduced (32 waves per CU hide the LDS latency instead of ILP).
__device__ __forceinline__ uint32_t vr_lookups(const uint32_t (&d)[8], const VrSched& s) {
    uint32_t v[2][4];
    uint32_t acc = 0;
    auto issue = [&](auto gc) __attribute__((always_inline)) {
        constexpr int g = decltype(gc)::value;
        const uint32_t col = vr_col_const<g>() ^ s.cl;
#pragma unroll
        for (int i = 0; i < 4; ++i)
            v[g & 1][i] = lds_load(__builtin_amdgcn_perm(d[g], col, s.sel0 ^ (0x101u * static_cast<uint32_t>(i))));
    };
    auto reduce = [&](int g) __attribute__((always_inline)) {
        const uint32_t(&u)[4] = v[g & 1];
        acc = xor3(xor3(acc, u[0], u[1]), u[2], u[3]);        // two 3-input XORs per 4 lookups
        // (pinned here: sunk into the caller's "block in the window" branch, the
        // XORs would keep all 32 lookups live at once)
        asm volatile("" : "+v"(acc));
    };
    issue(std::integral_constant<int, 0>{});
    static_for<1, 8>([&](auto gc) __attribute__((always_inline)) {
        __builtin_amdgcn_sched_barrier(0);
        issue(gc);
        reduce(decltype(gc)::value - 1);
    });
    __builtin_amdgcn_sched_barrier(0);
    reduce(7);
    return acc;
}

// The fused fold of a landed slot (round 5, the product instances): vr_rotate_slot's
// in-place preparation, then vr_lookups' 32 lookups reading the slot registers
// themselves, in ONE asm block -- with the fold in C++ the compiler copied the 8
// rotated slot registers out first (its operands must be registers it allocates).
// Same schedule as vr_lookups: group g's four lookups issued, then group g-1's four
// reduced after a counted lgkmcnt(4) (LDS returns in order), at most 8 in flight.
#define VR_LK(S, C, T0, T1, T2, T3)                                                               \
    "v_perm_b32 " T0 ", " S ", " C ", %[s0]\n\t"                                                  \
    "v_perm_b32 " T1 ", " S ", " C ", %[s1]\n\t"                                                  \
    "v_perm_b32 " T2 ", " S ", " C ", %[s2]\n\t"                                                  \
    "v_perm_b32 " T3 ", " S ", " C ", %[s3]\n\t"                                                  \
    "ds_read_b32 " T0 ", " T0 "\n\t"                                                             \
    "ds_read_b32 " T1 ", " T1 "\n\t"                                                             \
    "ds_read_b32 " T2 ", " T2 "\n\t"                                                             \
    "ds_read_b32 " T3 ", " T3 "\n\t"
#define VR_RED(T0, T1, T2, T3)                                                                    \
    "v_bitop3_b32 %[acc], %[acc], " T0 ", " T1 " bitop3:0x96\n\t"                                 \
    "v_bitop3_b32 %[acc], %[acc], " T2 ", " T3 " bitop3:0x96\n\t"
#define VR_LKX(...) VR_LK(__VA_ARGS__)
#define VR_REDX(...) VR_RED(__VA_ARGS__)
#define VR_TA "%[a0]", "%[a1]", "%[a2]", "%[a3]"
#define VR_TB "%[b0]", "%[b1]", "%[b2]", "%[b3]"
#define VR_FOLD_ASM(S0, S1, S2, S3, S4, S5, S6, S7)                                               \
    VR_ROTATE_ASM(S0, S1, S2, S3, S4, S5, S6, S7) "\n\t"                                          \
    VR_LKX(S0, "%[c0]", VR_TA)                                                                      \
    VR_LKX(S1, "%[c1]", VR_TB)                                                                      \
    "s_waitcnt lgkmcnt(4)\n\t"                                                                     \
    "v_bitop3_b32 %[acc], %[a0], %[a1], %[a2] bitop3:0x96\n\t"                                     \
    "v_xor_b32 %[acc], %[acc], %[a3]\n\t"                                                          \
    VR_LKX(S2, "%[c2]", VR_TA) "s_waitcnt lgkmcnt(4)\n\t" VR_REDX(VR_TB)                             \
    VR_LKX(S3, "%[c3]", VR_TB) "s_waitcnt lgkmcnt(4)\n\t" VR_REDX(VR_TA)                             \
    VR_LKX(S4, "%[c4]", VR_TA) "s_waitcnt lgkmcnt(4)\n\t" VR_REDX(VR_TB)                             \
    VR_LKX(S5, "%[c5]", VR_TB) "s_waitcnt lgkmcnt(4)\n\t" VR_REDX(VR_TA)                             \
    VR_LKX(S6, "%[c6]", VR_TA) "s_waitcnt lgkmcnt(4)\n\t" VR_REDX(VR_TB)                             \
    VR_LKX(S7, "%[c7]", VR_TB) "s_waitcnt lgkmcnt(4)\n\t" VR_REDX(VR_TA)                             \
    "s_waitcnt lgkmcnt(0)\n\t" VR_REDX(VR_TB)
template <int SLOT>
__device__ __forceinline__ uint32_t vr_fold_slot(uint32_t reg, uint32_t lane, const VrSched& s) {
    uint32_t acc, t0, a0, a1, a2, a3, b0, b1, b2, b3;
    uint64_t sv;
    const uint32_t c0 = vr_col_const<0>() ^ s.cl, c1 = vr_col_const<1>() ^ s.cl, c2 = vr_col_const<2>() ^ s.cl,
                   c3 = vr_col_const<3>() ^ s.cl, c4 = vr_col_const<4>() ^ s.cl, c5 = vr_col_const<5>() ^ s.cl,
                   c6 = vr_col_const<6>() ^ s.cl, c7 = vr_col_const<7>() ^ s.cl;
    const uint32_t s0 = s.sel0, s1 = s.sel0 ^ 0x101u, s2 = s.sel0 ^ 0x202u, s3 = s.sel0 ^ 0x303u;
#define VR_FOLD_OPERANDS                                                                                 \
    : [acc] "=&v"(acc), [t0] "=&v"(t0), [sv] "=&s"(sv), [a0] "=&v"(a0), [a1] "=&v"(a1), [a2] "=&v"(a2),   \
      [a3] "=&v"(a3), [b0] "=&v"(b0), [b1] "=&v"(b1), [b2] "=&v"(b2), [b3] "=&v"(b3)                     \
    : [reg] "v"(reg), [lane] "v"(lane), [c0] "v"(c0), [c1] "v"(c1), [c2] "v"(c2), [c3] "v"(c3),           \
      [c4] "v"(c4), [c5] "v"(c5), [c6] "v"(c6), [c7] "v"(c7), [s0] "v"(s0), [s1] "v"(s1), [s2] "v"(s2),   \
      [s3] "v"(s3)
    if constexpr (SLOT == 0)
        asm volatile(VR_FOLD_ASM("v48", "v49", "v50", "v51", "v52", "v53", "v54", "v55") VR_FOLD_OPERANDS
                     : "v48", "v49", "v50", "v51", "v52", "v53", "v54", "v55", "memory");
    else
        asm volatile(VR_FOLD_ASM("v56", "v57", "v58", "v59", "v60", "v61", "v62", "v63") VR_FOLD_OPERANDS
                     : "v56", "v57", "v58", "v59", "v60", "v61", "v62", "v63", "memory");
#undef VR_FOLD_OPERANDS
    return acc;
}

// Batches of one launch: their groups in one concatenated space (batch b's from
// VrBatch::g0), dealt in slots.  Workgroup k's slot s is global group
// 16 k + s % 16 + (s / 16) * wt (wt = the launch's waves): rounds of 16 consecutive
// groups, one round per workgroup every wt groups, so every batch is spread over
// the whole chip and the start (metadata, table image) and the drain are paid once
// per launch.  A wave takes its first two slots statically (wave, 16 + wave) and
// every later one from its workgroup's LDS counter, so the waves a SIMD favours
// take more groups and the workgroup's waves end together: with a static deal the
// waves of a 20-batch launch ended between 40 % and 100 % of its span
// (tools/list_timeline.py, profiles/r02d_list_timeline_*).
// Dynamic rounds (DYN, VrBatches::claim set): a round is a chunk of 16 groups,
// workgroup k's rounds 0, 1 and 2 are chunks k, G + k and 2 G + k (G workgroups; all
// taken statically, so no claim is made in the prologue), and each later round is
// claimed from the launch's claim word (chunk 3 G + c), so the workgroups the chip
// favours take more chunks and the launch's workgroups end together too.  The wave
// taking the first slot of round r >= 2 claims round r + 1 (after round r's claim is
// published when r >= 3: a workgroup's chunks ascend) and publishes it in the LDS
// round table; a wave taking a slot of round r >= 3 reads round r's entry (polled:
// published at least 16 slots earlier).  Live slots stay a prefix of
// the slot sequence (chunks ascend, a chunk's dead groups are its last ones), so the
// waves stop at the first dead slot as before and no claimed live chunk is left.
// Dynamic rounds.  The helpers take wave-uniform (SGPR) operands and build their
// VGPR operands inside the asm: constants the compiler could see (LDS addresses, the
// atomic's 1) were hoisted out of the ring loop into VGPRs held across it.
// vr_claim_next: lane 0 takes the next chunk number of the launch from its claim
// word {generation, count} (address and generation at kVrClaimPtr): a returning
// 64-bit device-scope add, waited for (which retires the wave's ring loads too, once
// per round of 16 groups per workgroup).  A word still tagged with an older
// generation (a launch before this one used the line) is moved to {gen, 0} by a
// 64-bit max, and the add repeated: no reset between launches, so no end-of-launch
// atomics.  (Round 4's first form counted the waves ending on one word to reset it:
// 8192 returning atomics on one address at the launch's end, serialised at the
// chip's ~88 per us, added 40-90 us.)  A newer generation (not possible while the
// host hands out the lines in turn) gives ~0: chunks past the end.  dyn = the
// launch's dynamic chunks: none (a launch the static rounds cover) gives ~0 with no
// atomic.  (A plain agent-scope load of the word first, to skip the claims past the
// last chunk, made cfg2 lists 1.6x slower.)
__device__ __forceinline__ uint32_t vr_claim_next(uint32_t dyn) {
    if (dyn == 0u) return ~0u;
    uint32_t c = 0;
    if ((threadIdx.x & 63u) == 0u) {
        uint32_t t;
        uint64_t p, old;
        asm volatile("v_mov_b32 %0, %2\n\t"
                     "ds_read_b64 %1, %0\n\t"
                     "s_waitcnt lgkmcnt(0)"
                     : "=&v"(t), "=&v"(p) : "i"(kVrClaimPtr) : "memory");
        uint32_t gen;
        asm volatile("v_mov_b32 %0, %1\n\t"
                     "ds_read_b32 %0, %0 offset:8\n\t"
                     "s_waitcnt lgkmcnt(0)"
                     : "=&v"(gen) : "i"(kVrClaimPtr) : "memory");
        for (;;) {
            uint32_t one32;                                  // (made here, not a constant hoisted out of the ring loop)
            asm volatile("v_mov_b32 %0, 1" : "=v"(one32));
            const uint64_t one = one32;
            asm volatile("global_atomic_add_x2 %0, %1, %2, off sc0\n\t"
                         "s_waitcnt vmcnt(0)"
                         : "=&v"(old) : "v"(p), "v"(one) : "memory");
            const uint32_t g = static_cast<uint32_t>(old >> 32);
            if (g == gen) {
                c = static_cast<uint32_t>(old);
                break;
            }
            if (g > gen) {
                c = ~0u;
                break;
            }
            const uint64_t tag = static_cast<uint64_t>(gen) << 32;
            asm volatile("global_atomic_umax_x2 %0, %1, %2, off sc0\n\t"
                         "s_waitcnt vmcnt(0)"
                         : "=&v"(old) : "v"(p), "v"(tag) : "memory");
        }
    }
    return __builtin_amdgcn_readfirstlane(c);
}
// the round table entry of round r: its chunk once published (tag == r), polled.  One
// 8-byte read takes {tag, chunk}: the chunk was written before the tag
__device__ __forceinline__ uint32_t vr_round_chunk(uint32_t r) {
    const uint32_t e = kVrRound + 8u * (r & (kVrRounds - 1u));
    for (;;) {
        uint64_t tc;
        uint32_t a;
        asm volatile("v_mov_b32 %1, %2\n\t"
                     "ds_read_b64 %0, %1\n\t"
                     "s_waitcnt lgkmcnt(0)"
                     : "=&v"(tc), "=&v"(a) : "s"(e) : "memory");
        const uint32_t tag = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(tc));
        if (tag == r) return __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(tc >> 32));
        // a tag past r means round r's entry was overwritten (64 rounds later) before
        // this wave read it: the interleaving the host-side model excludes.  Fail loudly
        // instead of polling forever (~0u = the unpublished sentinel)
        if (tag != ~0u && tag - r - 1u < 0x7FFFFFFFu) __builtin_trap();
        __builtin_amdgcn_s_sleep(1);
    }
}
// publish round r's chunk: the chunk first, then (after it is written) the tag
__device__ __forceinline__ void vr_round_publish(uint32_t r, uint32_t chunk) {
    const uint32_t e = kVrRound + 8u * (r & (kVrRounds - 1u));
    if ((threadIdx.x & 63u) == 0u) {
        uint32_t a, v;
        asm volatile("v_mov_b32 %0, %2\n\t"
                     "v_mov_b32 %1, %3\n\t"
                     "ds_write_b32 %0, %1 offset:4\n\t"
                     "s_waitcnt lgkmcnt(0)\n\t"
                     "v_mov_b32 %1, %4\n\t"
                     "ds_write_b32 %0, %1\n\t"
                     "s_waitcnt lgkmcnt(0)"
                     : "=&v"(a), "=&v"(v) : "s"(e), "s"(chunk), "s"(r) : "memory");
    }
}

struct VrIt {
    uint32_t b;         // batch
    uint64_t g;         // global group
};

// 64 VGPRs (8 waves per SIMD: two 16-wave workgroups per CU), of which the compiler
// may allocate v0-v47 only: amdgpu_num_vgpr(N) limits it to 2N VGPRs on gfx950
// (the unified VGPR/AGPR file doubles the request), so the ring registers
// v48-v63 are reserved -- never allocated, still counted in the kernel's VGPRs.
// TR = 1: the diagnostics instance that writes the per-wave trace; TR = 2: only its
// end record (slots taken, last slot, end time, HW_ID, groups), the product's code
// path otherwise (diagnostics library, ablation 128).
// ABL (diagnostics): bit 0 = no edge masking, bit 1 = no table lookups (the fold
// XORs the prepared dwords) -- both wrong CRCs by design; bit 2 = each stage's
// wait also retires the stage just issued (no load in flight during a fold); bit 3
// = 128-byte window starts and line-shaped stage loads (wrong CRCs by design);
// bit 4 = no end-of-packet corrections (wrong CRCs by design); bit 5 (8 lanes) = each
// produce runs at s_setprio 3, the rest of the turn at 0 (correct CRCs; round 6 probe)
// BIN = 1: the batch's metadata are length-binned records (VrBatch::off points at
// them, 4 dwords per packet), read in record order; packet r's CRC goes to
// out[record r's index] (enet_hip_crc32_batch_device_binned).  One workgroup per CU;
// BIN = 2, the compact records instance: the same without the x^(-8 c) tables (tz mod 8
// by unsteps), two workgroups per CU.
// BIN = 3, the local-tile records instance (vring_launch_local): as BIN = 2, but each
// workgroup orders its own tile of packets in its prologue (no bin kernel, no second
// launch) and checksums that tile's groups, longest first.
// ROT = 1: the tail-first stage order (below; diagnostics library); 0 = stages in
// window order (the product).
// VF = 1: receive verify (protocol.cs:1052-1068) over a VrVBatches list, 8 lanes per
// packet: the slot's lane substitutes connectID in registers (vr_slot_fix), and the
// packet's lane 0 writes ok[] and computed[].
// DYN = 1: dynamic rounds (above); built for the product-shaped instances (TR != 1,
// no ablation, nt, walks or tail-first order).  DYN = 2 (diagnostics): pair rounds --
// workgroups k and k + H (H = G / 2, G even) share the chunks p + j H (p = k mod H):
// the same static rounds (k + r G = p + (2 r + k / H) H), then j = 2 kStatic + c from the
// pair's own claim word, so the two balance against each other with no word shared
// by more than two workgroups.
template <int LG, int TR = 0, int NT = 0, int ABL = 0, int BIN = 0, int WK = 0, int ROT = 0, int VF = 0, int DYN = 0>
__global__ void __launch_bounds__(64 * kVrW) __attribute__((amdgpu_waves_per_eu(8, 8), amdgpu_num_vgpr(24)))
crc32_vring_kernel(std::conditional_t<VF != 0, VrVBatches, VrBatches> bl, KernelTables tb, const uint32_t* basis,
                   uint64_t* trace) {
    constexpr uint32_t P = 1u << LG, kPk = 64u >> LG;
    // verify metadata: 5 fields x 8 packets in one 64-lane DMA
    static_assert(!VF || (LG == 3 && !BIN), "receive verify: 8 lanes per packet, plain metadata");
    // Tail-first stage order.  A group of S > 1 stages runs its last stage first,
    // then stages 0 .. S-2.  Packed packets share a 128-byte line at every packet
    // boundary: packet j's last stage reads it, packet j+1's first stage too.  In
    // order, those two reads are S-1 stages apart, long enough for the XCD's L2 to
    // evict the line (FETCH_SIZE 1.105 x the payload on cfg2); tail first, they are
    // adjacent steps.  Lane k folds its last-stage block from a zero register into
    // rt, the other stages as before into reg; fold(b ^ r) = fold(b) ^ adv(r), so
    // the packet's lane register is rt ^ adv(reg), adv(r) = r x^(256 P) = four
    // lookups in the advancing tables T'_31 .. T'_28 (tests/kernel_model.py,
    // vring_packet(rotate=True)).  Binned records are not neighbours in memory: no
    // gain there, so the records instance keeps the plain order.
    constexpr bool kRot = ROT && !BIN && !(ABL & 8);
    // the window stage of step j of a group of S stages
    auto stage_of = [](uint32_t j, uint32_t S) __attribute__((always_inline)) -> uint32_t {
        if constexpr (!kRot) return j;
        return S > 1u ? (j == 0u ? S - 1u : j - 1u) : 0u;
    };
    // ... and its inverse (~0u stays ~0u)
    auto step_of = [](uint32_t a, uint32_t S) __attribute__((always_inline)) -> uint32_t {
        if constexpr (!kRot) return a;
        return (S <= 1u || a == ~0u) ? a : (a == S - 1u ? 0u : a + 1u);
    };
    // The lane id and everything derived from it (k, p, the fold's lane constants):
    // kept live across the ring loop in the in-order instances; the tail-first and
    // records instances recompute the lane id every iteration from a fresh v_mbcnt
    // (asm volatile, so not hoisted) -- their rt / record register needs the VGPR
    // room, and held across the loop those values made hipcc spill.
    uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t wv = static_cast<uint64_t>(blockIdx.x) * kVrW + wave;
    const uint64_t wt = static_cast<uint64_t>(gridDim.x) * kVrW;
    constexpr bool kDyn = DYN != 0 && !WK && BIN != 3;
    // slots taken statically per wave: rounds 0 .. kStatic - 1 are chunks k + r G
    constexpr uint32_t kStatic = kDyn ? 3u : 2u;
    if constexpr (kDyn) {                                    // wave 0, before its takes: no round published
        if (threadIdx.x < static_cast<uint32_t>(kVrRounds)) lds_store(kVrRound + 8u * threadIdx.x, ~0u);
        // the claim word's address and generation (read where used: held across the
        // ring loop they cost SGPRs)
        // (DYN 2: the pair's word)
        const uint64_t* word = bl.claim + (DYN == 2 ? blockIdx.x % (gridDim.x >> 1) : 0u);
        if (threadIdx.x < 3u)
            lds_store(kVrClaimPtr + 4u * threadIdx.x,
                      threadIdx.x < 2u ? static_cast<uint32_t>(reinterpret_cast<uint64_t>(word) >> (32u * threadIdx.x))
                                       : bl.claim_gen);
    }
    auto lane_k = [&]() __attribute__((always_inline)) { return lane & (P - 1u); };   // block lane
    auto lane_p = [&]() __attribute__((always_inline)) { return lane >> LG; };         // packet of the group
    const uint64_t zero = reinterpret_cast<uint64_t>(tb.zero);
    // batch b's packets and the launch's groups; BIN with tile counts (the binned
    // gather): the ranks up to the fullest tile's, R = ceil(max_t count_t / kPk), i.e.
    // R x tiles groups, every record of them valid (kept or empty padding).  The
    // workgroup reduces the counts once: wave w takes tiles w, w + 16, ... (from L2),
    // its maximum goes to LDS, one raw barrier, every wave reads the 16 maxima (no
    // global atomic; a launch over tens of millions of segments reads each count
    // once per workgroup, not once per wave).
    // BIN = 3 (the local-tile records instance, vring_launch_local): workgroup k orders
    // its own packets [k T, (k + 1) T) here, two per thread, those of at least
    // local_keep_min bytes (lcnt of them) -- a counting sort by window length (bin_of's
    // 32-byte bins, longest first) in LDS: each packet's place in its bin (an LDS add), an
    // exclusive scan of the bins (wave scans by DPP shifts, then the four waves'
    // totals), then its record {len, off_lo, off_hi, index} to local_rec[k T + rank].  The first two rounds' metadata also go straight to LDS
    // (vr_read_meta's layout: field f of packet p at +4 (f kPk + p)): round 0's group g to
    // wave g's metadata area, round 1's to a staging area of the wave whose slot 16 + w
    // takes it, copied over once the wave has read round 0's.  So the first two groups
    // need no metadata DMA, and the record stores -- read by the DMAs from the third
    // group on, by this CU's waves -- are waited for only before barrier A, with the
    // first stage's loads in flight.  One
    // tile per workgroup streams as fast as the bin kernel's rank-interleaved order
    // (tools/dealprobe.hip: 42.2 against 41.9 us for cfg3, profiles/r06_local/).
    // basis row `wave` (waves < 10) and, waves 0..7, one KiB each of the zero-byte
    // multiplier tables: LDS-DMAs, outside the image area
    auto issue_tables = [&]() __attribute__((always_inline)) {
        if (wave < static_cast<uint32_t>(kVrBasisRows))
            dma4(basis + static_cast<size_t>(LG == 2 ? 1 : 2) * kVrBasisDwords + 64u * wave + lane,
                 kVrStaging + 256u * wave);
        if (wave < static_cast<uint32_t>(kTzTableDwords / 256)) dma16(tb.tz + 256u * wave + 4u * lane, kVrTz + 1024u * wave);
    };
    uint64_t lrec = 0, lcnt = 0;                             // BIN 3: records, and the tile's kept packets
    if constexpr (BIN == 3) {
        if (TR == 1 && (threadIdx.x & 63u) == 0u) trace[8u * wv] = __builtin_amdgcn_s_memrealtime();   // (start)
        issue_tables();                                      // (they land while the tile is sorted)
        const uint64_t first = static_cast<uint64_t>(blockIdx.x) * bl.tile_local, nb = bl.b[0].n;
        const uint64_t tn = first < nb ? umin64(nb - first, bl.tile_local) : 0u;   // the tile's packets
        lrec = reinterpret_cast<uint64_t>(bl.local_rec) + 16u * first;
        const uint32_t t = threadIdx.x;
        // item i of thread t = the tile's packet t + 1024 i; kept: live and at least
        // local_keep_min bytes (the binned gather leaves its short segments to the join)
        uint32_t L[kVrLocalItems], bin[kVrLocalItems], slot[kVrLocalItems];
        uint64_t o[kVrLocalItems];
        bool kept[kVrLocalItems];
#pragma unroll
        for (uint32_t i = 0; i < kVrLocalItems; ++i) {
            const uint32_t j = t + 64u * kVrW * i;
            L[i] = j < tn ? bl.b[0].len[first + j] : 0u;
            o[i] = j < tn ? bl.b[0].off[first + j] : 0u;
        }
        if (t < kVrLocalBins) lds_store(kVrLocalHist + 4u * t, 0u);
        static_assert(kVrMetaWaveBin * kVrW == 4u * 64u * kVrW, "one metadata dword per thread");
        lds_store(kVrMeta + 4u * t, 0u);                     // (a partial group's missing packets: zeros)
        lds_store(kVrLocalNext + 4u * t, 0u);
        __syncthreads();
#pragma unroll
        for (uint32_t i = 0; i < kVrLocalItems; ++i) {
            kept[i] = t + 64u * kVrW * i < tn && L[i] >= bl.local_keep_min;
            bin[i] = kVrLocalBins - 1u - min((L[i] + (static_cast<uint32_t>(o[i]) & 63u)) >> 5, kVrLocalBins - 1u);
            slot[i] = kept[i] ? lds_add_rtn(kVrLocalHist + 4u * bin[i], 1u) : 0u;
        }
        __syncthreads();
        uint32_t mine = 0, incl = 0;
        if (t < kVrLocalBins) {
            mine = lds_load(kVrLocalHist + 4u * t);
            incl = mine;
#pragma unroll
            for (uint32_t sh = 1; sh < 64u; sh <<= 1) {
                const uint32_t u = static_cast<uint32_t>(__shfl_up(static_cast<int>(incl), sh));
                incl += (t & 63u) >= sh ? u : 0u;
            }
            if ((t & 63u) == 63u) lds_store(kVrLocalHist + 4u * (kVrLocalBins + (t >> 6)), incl);
        }
        __syncthreads();
        uint32_t pre = 0, total = 0;                         // (total: the tile's kept packets)
#pragma unroll
        for (uint32_t w = 0; w < kVrLocalBins / 64u; ++w) {
            const uint32_t ws = lds_load(kVrLocalHist + 4u * (kVrLocalBins + w));
            pre += w < (t >> 6) ? ws : 0u;
            total += ws;
        }
        if (t < kVrLocalBins) lds_store(kVrLocalHist + 4u * t, pre + incl - mine);   // the bin's first rank
        lcnt = total;
        const uint32_t ng = (total + kPk - 1u) / kPk;
        __syncthreads();
#pragma unroll
        for (uint32_t i = 0; i < kVrLocalItems; ++i) {
            if (!kept[i]) continue;
            const uint32_t rank = lds_load(kVrLocalHist + 4u * bin[i]) + slot[i];
            const uint32_t olo = static_cast<uint32_t>(o[i]), ohi = static_cast<uint32_t>(o[i] >> 32);
            const uint32_t idx = static_cast<uint32_t>(first + t + 64u * kVrW * i);
            reinterpret_cast<uint4*>(lrec)[rank] = make_uint4(L[i], olo, ohi, idx);
            const uint32_t g = rank / kPk, p = rank % kPk;
            const uint32_t dst = g < kVrW ? kVrMeta + kVrMetaWaveBin * g
                               : g < 2u * kVrW ? kVrLocalNext + 256u * (ng >= 2u * kVrW ? 2u * kVrW - 1u - g : g - kVrW)
                                               : ~0u;
            if (dst != ~0u) {
                lds_store(dst + 4u * p, L[i]);
                lds_store(dst + 4u * (kPk + p), olo);
                lds_store(dst + 4u * (2u * kPk + p), ohi);
                lds_store(dst + 4u * (3u * kPk + p), idx);
            }
        }
        __syncthreads();                                     // (LDS only: the record stores stay in flight)
    }
    uint64_t n0 = BIN == 3 ? lcnt : bl.b[0].n, ngroups_all = BIN == 3 ? (lcnt + kPk - 1u) / kPk : bl.groups;
    if constexpr (BIN == 1 || BIN == 2) {
        if (bl.tile_counts) {
            uint32_t m = 0;
            for (uint32_t t = wave * 64u + (threadIdx.x & 63u); t < bl.tiles; t += 64u * kVrW)
                m = max(m, bl.tile_counts[t]);
            m = wave_max_u(m);
            if ((threadIdx.x & 63u) == 0u) *reinterpret_cast<__attribute__((address_space(3))) uint32_t*>(
                static_cast<uintptr_t>(vr_tile_max<BIN>() + 4u * wave)) = m;
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the store is in LDS
            __builtin_amdgcn_s_barrier();
            uint32_t mm = 0;
#pragma unroll
            for (uint32_t w = 0; w < kVrW; ++w) mm = max(mm, lds_load(vr_tile_max<BIN>() + 4u * w));
            const uint32_t r = __builtin_amdgcn_readfirstlane((mm + kPk - 1u) / kPk);   // (uniform: SGPRs)
            ngroups_all = static_cast<uint64_t>(r) * bl.tiles;
            n0 = ngroups_all * kPk;
        }
    }
    auto batch_n = [&](uint32_t b) __attribute__((always_inline)) -> uint64_t { return BIN ? n0 : bl.b[b].n; };

    // ---- the wave's group sequence: slots of the workgroup (wave-uniform)
    // WK = 1 (walks): workgroup k owns the contiguous groups [k gw, (k + 1) gw) of the
    // concatenated space and takes them in order, so its waves walk one region of
    // the arena front to back (the access shape of tools/streamprobe.hip's chunk
    // and sub-stream probes) instead of a round of 16 groups every wt groups
    const uint64_t gw = WK ? (ngroups_all + gridDim.x - 1u) / gridDim.x : 0u;
    // Length-binned records (BIN) are rank-interleaved (length_bin_tiles: group q T + t =
    // rank q of tile t, longest first), so round r's 16 groups of workgroup k are about one
    // rank, 16 r + k / 16 at cfg3's 256 tiles: in the plain deal workgroup 0 took the
    // longest rank of every round and the last workgroup the shortest, 1.5 x less work,
    // and the records kernel's span ended 9 us after its median wave (tools/bin_timeline.py,
    // profiles/r06_cfg3/).  Odd rounds therefore deal the workgroups in reverse order
    // (k -> G - 1 - k): still a permutation of the round's groups, and every workgroup's
    // rounds sum to about the same bytes (boustrophedon).
    constexpr bool kSnake = BIN == 1 || BIN == 2;
    auto slot_group = [&](uint32_t sl) __attribute__((always_inline)) -> uint64_t {
        if constexpr (WK) return sl < gw ? static_cast<uint64_t>(blockIdx.x) * gw + sl : ~0ull;
        // BIN = 3: the workgroup's own groups in slot order, round 1 reversed when it is
        // full, so each wave's two static groups (w and 31 - w) sum to about the same
        // bytes; later rounds are taken as the waves free up (a partial round stays in
        // order: live slots a prefix)
        if constexpr (BIN == 3)
            return (sl / kVrW == 1u && ngroups_all >= 2u * kVrW) ? 3u * kVrW - 1u - sl : sl;
        if (kDyn && sl >= kStatic * kVrW) return static_cast<uint64_t>(vr_round_chunk(sl / kVrW)) * kVrW + (sl & (kVrW - 1u));
        const uint32_t r = sl / kVrW;
        const uint64_t k = (kSnake && (r & 1u)) ? gridDim.x - 1u - blockIdx.x : blockIdx.x;
        return k * kVrW + (sl & (kVrW - 1u)) + static_cast<uint64_t>(r) * wt;
    };
    // `it` moved to global group gg (its batch found from it.b on: a wave's groups
    // ascend -- with dynamic rounds too); false past the launch's last group
    auto locate = [&](VrIt& it, uint64_t gg) __attribute__((always_inline)) -> bool {
        if (gg >= ngroups_all) return false;
        if constexpr (!BIN)                                  // (BIN: one batch, vring_launch_list)
            while (it.b + 1u < bl.count && gg >= bl.b[it.b + 1u].g0) ++it.b;
        it.g = gg;
        return true;
    };
    uint32_t taken = 0;                                      // slots this wave has taken
    // the next slot: the first kStatic static, later ones from the workgroup's counter
    uint32_t last_slot = 0;                                  // (TR 2: the last slot taken)
    auto take = [&]() __attribute__((always_inline)) -> uint32_t {
        uint32_t sl = 0;
        if (taken < kStatic) {
            sl = wave + kVrW * taken;
        } else {
            // ds_add_rtn as inline asm: as a C++ atomic, hipcc put an s_waitcnt vmcnt(0)
            // in front of it (an LDS atomic that may alias an LDS-DMA in flight), which
            // drained the ring at every group switch.  The counter is no DMA's target.
            if ((threadIdx.x & 63u) == 0u)
                asm volatile("v_mov_b32 %0, 1\n\t"
                             "ds_add_rtn_u32 %0, %1, %0\n\t"
                             "s_waitcnt lgkmcnt(0)"
                             : "=&v"(sl) : "v"(BIN ? kVrCtrBin : kVrCtr) : "memory");
            sl = __builtin_amdgcn_readfirstlane(sl);
            if constexpr (TR == 2) last_slot = sl;
        }
        ++taken;
        // the first slot of round r >= kStatic - 1: claim round r + 1, after round r's
        // claim is published if r is dynamic (a workgroup's chunks ascend)
        if (kDyn && sl >= (kStatic - 1u) * kVrW && (sl & (kVrW - 1u)) == 0u) {
            const uint32_t r = sl / kVrW;
            if (r >= kStatic) (void)vr_round_chunk(r);
            const uint64_t chunks = (ngroups_all + kVrW - 1u) >> 4, G = wt >> 4;
            if constexpr (DYN == 2) {
                // the pair's dynamic chunks: p + j H for j >= 2 kStatic, below the launch's chunks
                const uint64_t H = G >> 1, pp = blockIdx.x % H;
                const uint64_t jn = chunks > pp ? (chunks - pp + H - 1u) / H : 0u;
                const uint32_t c = vr_claim_next(jn > 2u * kStatic ? static_cast<uint32_t>(umin64(jn - 2u * kStatic, ~0u - 1u)) : 0u);
                vr_round_publish(r + 1u, c == ~0u ? c : static_cast<uint32_t>(umin64(pp + (2u * kStatic + c) * H, ~0u - 1u)));
            } else {
                // (the launch's dynamic chunks: its chunks past the kStatic G static ones)
                const uint64_t stat = G * kStatic;
                const uint32_t c = vr_claim_next(chunks > stat ? static_cast<uint32_t>(umin64(chunks - stat, ~0u - 1u)) : 0u);
                vr_round_publish(r + 1u, c == ~0u ? c : static_cast<uint32_t>(G) * kStatic + c);   // kStatic G + c
            }
        }
        return sl;
    };
    auto advance = [&](VrIt& it) __attribute__((always_inline)) -> bool { return locate(it, slot_group(take())); };
    auto group_base = [&](const VrIt& it) __attribute__((always_inline)) -> uint64_t {   // its first packet
        return (it.g - bl.b[it.b].g0) * kPk;
    };
    VrIt pit{0u, 0u};                                        // the producer's group
    const bool any = advance(pit);
    VrIt qit = pit;                                          // the group whose metadata is loaded
    bool qlive = any && advance(qit);

    // diagnostics (enet_hip_diag_trace): per-wave timestamps, tools/timeline.py's
    // 8 x u64 layout [start, metadata, table, barrier B, loop entry, end, HW_ID, groups]
    // (each mark is stored at once: held in registers, the marks cost SGPR spills)
    uint32_t ngroups = 0;
    auto mark = [&](int i) __attribute__((always_inline)) {
        if (TR == 1 && (threadIdx.x & 63u) == 0u) trace[8u * wv + i] = __builtin_amdgcn_s_memrealtime();
    };
    auto trace_end = [&]() __attribute__((always_inline)) {
        if (TR && (threadIdx.x & 63u) == 0u) {
            uint64_t* tr = trace + 8u * wv;
            if (TR == 2) {
                tr[0] = taken;
                tr[1] = last_slot;
            }
            tr[5] = __builtin_amdgcn_s_memrealtime();
            const uint32_t hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);      // HW_ID
            const uint32_t xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20);    // XCC_ID
            tr[6] = hw | (static_cast<uint64_t>(xcc) << 32);
            tr[7] = ngroups;
        }
    };
    if constexpr (BIN != 3) mark(0);                         // (BIN 3: before its sort)

    // ---- prologue: basis row `wave` (waves < 10) and metadata of the first group
    if constexpr (BIN != 3) issue_tables();                  // (BIN 3: before its sort)
    if constexpr (BIN == 1) {                                // the small x^(-8 c) tables: 28 one-KiB chunks
#pragma unroll
        for (uint32_t c = wave; c < static_cast<uint32_t>(kTzSmallDwords / 256); c += kVrW)
            dma16(tb.tz + kTzTableDwords + 256u * c + 4u * lane, kVrTz7 + 1024u * c);
    }
    const uint32_t mbase = kVrMeta + (BIN ? kVrMetaWaveBin : kVrMetaWave) * wave;   // the wave's metadata area
    uint32_t mL = 0;                                         // metadata (read out at group switches)
    uint64_t moff = 0;
    uint32_t midx = 0;                                       // BIN: the record's caller index
    uint32_t mso = 0, mconn = 0;                             // VF: slot offset, connectID
    auto load_meta = [&](const VrIt& it) __attribute__((always_inline)) {
        const auto& B = bl.b[it.b];
        // lane l loads field f = l / kPk of packet l % kPk (lanes past the fields: field
        // 0), the packet clamped to the batch's last (always a valid address; the
        // prologue of a wave with no group at all loads batch 0's last packet)
        const uint64_t bn = umax64(batch_n(it.b), 1u);   // (no kept record at all: record 0, unused)
        const uint64_t base = umin64(group_base(it), bn - 1u);
        const uint64_t left = bn - 1u - base;                // (uniform: scalar select, no VALU)
        const uint32_t l = vr_lane();                       // (recomputed: not a register held across the loop)
        uint32_t f = l / kPk;
        const uint32_t q = min(l & (kPk - 1u), left < 63u ? static_cast<uint32_t>(left) : 63u);
        if constexpr (BIN) {
            f = f < 4u ? f : 0u;
            vr_issue_meta((BIN == 3 ? lrec : reinterpret_cast<uint64_t>(B.off)) + 16u * (base + q) + 4u * f, mbase);
        } else if constexpr (VF) {
            f = f < 5u ? f : 0u;
            const uint64_t la = reinterpret_cast<uint64_t>(B.len + base) + 4u * q;
            const uint64_t oa = reinterpret_cast<uint64_t>(B.off + base) + 8u * q + 4u * (f - 1u);
            const uint64_t va = reinterpret_cast<uint64_t>(f == 3u ? B.slot_off + base : B.connect + base) + 4u * q;
            vr_issue_meta(f == 0u ? la : f < 3u ? oa : va, mbase);
        } else {
            f = f < 3u ? f : 0u;
            const uint64_t la = reinterpret_cast<uint64_t>(B.len + base) + 4u * q;
            const uint64_t oa = reinterpret_cast<uint64_t>(B.off + base) + 8u * q + 4u * (f - 1u);
            vr_issue_meta(f ? oa : la, mbase);
        }
    };
    if constexpr (BIN == 3) {
        // round 0's metadata, put here by the sort; then round 1's over it (its DMA skipped)
        vr_read_meta<BIN, VF, kPk>(mbase, lane_p(), mL, moff, midx, mso, mconn);
        lds_store(mbase + 4u * lane, lds_load(kVrLocalNext + 256u * wave + 4u * lane));
    } else {
        load_meta(any ? pit : VrIt{0u, 0u});                 // (batch 0 exists: count >= 1)
        vr_wait_meta<0, BIN, VF, kPk>(mbase, lane_p(), mL, moff, midx, mso, mconn);   // basis row and metadata landed
    }
    mark(1);

    // ---- producer: window of the group it loads, one stage ahead of the consumer
    // the window start (64-byte aligned) with the packet's first byte in it, plz,
    // in the low 6 bits: one 64-bit register for both; pe = the packet's end
    // EA (the records instance): a packet whose end is 16-byte aligned gets a window
    // that ENDS on its last byte -- nb = ceil(L / 32) blocks, lz = 32 nb - L < 32
    // leading zero bytes -- so no trailing zero bytes (tz = 0: no x^(-8 tz)
    // correction); its start is 16-byte aligned too, so every piece stays an aligned
    // 16-B load, and its partly covered head piece is the granule holding its first
    // byte.  Other packets keep the 64-byte-aligned start.  lz goes to pwl's top 6
    // bits.  Measured: windows ending on ANY packet end (byte-granular 16-B loads)
    // made cfg3 binned 61.6 against 55.9 us (tools/alignprobe.hip: that load shape
    // streams 4.3 against 4.9 TB/s); cfg5's 16-byte-aligned segments gain (vring
    // records 53.5 against 56 us) -- profiles/r03_ea_windows/.
    constexpr bool kEA = BIN != 0;
    constexpr uint64_t kEAMask = (1ull << 58) - 1u;
    uint64_t pwl = 0;
    uint32_t pe = 0;
    constexpr uint32_t kAln = (ABL & 8) ? 128u : 64u;         // window start alignment
    auto plz = [&]() __attribute__((always_inline)) {
        if constexpr (kEA) return static_cast<uint32_t>(pwl >> 58);
        return static_cast<uint32_t>(pwl) & (kAln - 1u);
    };
    auto pws = [&]() __attribute__((always_inline)) -> uint64_t {     // the window start
        if constexpr (kEA) return pwl & kEAMask;
        return pwl & ~static_cast<uint64_t>(kAln - 1u);
    };
    uint32_t pst = 0, pstages = 0;
    uint32_t pidx = 0;                                       // BIN: the first group's caller index (prologue)
    // BIN: the caller indices of the producer's group go to an LDS stash, two slots per
    // wave by group parity, over the basis staging area (free once barrier B is
    // passed; the first group's, taken before it, is stored after it).  The consumer
    // reads its group's slot when it writes the CRCs: no index register held across
    // the ring loop, so the records instance keeps the lane constants live too.
    uint32_t pgn = 0, cgn = 0;                               // groups entered by producer / consumer
    auto stash_addr = [&](uint32_t gn) __attribute__((always_inline)) -> uint32_t {
        return kVrStaging + 4u * kPk * (2u * wave + (gn & 1u)) + 4u * lane_p();
    };
    uint32_t pps = ~0u, pconn = 0;                           // VF: the slot's window position (~0u: none), connectID
    bool pdone = !any;
    auto producer_enter = [&](auto loop_c) __attribute__((always_inline)) {   // group pit; metadata in mL / moff
        const auto& B = bl.b[pit.b];
        if constexpr (BIN) {
            if constexpr (decltype(loop_c)::value) lds_store(stash_addr(pgn), midx);
            else pidx = midx;
            ++pgn;
        }
        const uint64_t rem = batch_n(pit.b) - group_base(pit);   // packets of the batch from the group's first
        const uint32_t L = lane_p() < rem ? mL : 0u;
        const uint64_t a = reinterpret_cast<uint64_t>(B.bytes) + moff;
        const uint32_t lz = static_cast<uint32_t>(a) & (kAln - 1u);
        const uint32_t z = L ? lz : 0u;                      // an empty packet: [0, 0)
        if constexpr (kEA) {
            const uint32_t eb = (L + 31u) & ~31u;            // 32 nb
            const bool ea = ((static_cast<uint32_t>(a) + L) & 15u) == 0u;
            const uint32_t w = ea ? eb - L : z;
            pwl = (a - w) | (static_cast<uint64_t>(w) << 58);
            pe = ea ? eb : z + L;
        } else {
            pwl = (a - lz) | z;
            pe = z + L;
        }
        if constexpr (VF) {                                  // a slot wholly inside the DGRAM, or none
            pps = (L >= 4u && mso <= L - 4u) ? z + mso : ~0u;
            pconn = mconn;
        }
        const uint32_t nb = (pe + 31u) >> 5;
        pstages = max(1u, wave_max_u((nb + P - 1u) >> LG));
        pst = 0;
    };
    // A produce issues the stage's two pieces, preceded -- on a group's first stage,
    // when a next group exists -- by that group's metadata (one LDS-DMA load), a whole
    // group ahead of its use.  The wait for the previous stage (slot WS, WS < 0:
    // none) follows in the same branch, counting the loads just issued (2, or 3
    // with metadata): one issue-and-wait sequence per path, so the in-flight check
    // sees each path's own count.
    auto produce = [&](auto slot_c, auto ws_c) __attribute__((always_inline)) {
        constexpr uint32_t slot = decltype(slot_c)::value;
        constexpr int WS = decltype(ws_c)::value;
        if constexpr ((ABL & 32) != 0) __builtin_amdgcn_s_setprio(3);
        if (!pdone && pst == pstages) {
            if (qlive) {
                // group qit's metadata was issued before the last produce's two stage
                // loads (on this group's first stage, or at the prologue): retired
                // once at most those two are in flight (stores do not count: older)
                vr_wait_meta<2, BIN, VF, kPk>(mbase, lane_p(), mL, moff, midx, mso, mconn);
                pit = qit;
                qlive = advance(qit);
                producer_enter(std::true_type{});
            } else {
                pdone = true;
                pwl = pws();                                 // [0, 0): every piece reads the zero line
                pe = 0;
            }
        }
        const uint32_t q0 = 32u * (lane_k() + P * stage_of(pst, pstages));
        const uint32_t hs16 = lane & 16u;                    // this lane takes the block's halves swapped
        // (ABL & 8, diagnostics: instruction j of a stage reads bytes 16 P j + 16 k)
        const uint32_t a0 = (ABL & 8) ? 32u * P * pst + 16u * lane_k() : q0 + hs16;
        const uint32_t a1 = (ABL & 8) ? a0 + 16u * P : q0 + 16u - hs16;
        const uint32_t lz = plz();
        const uint64_t ws = pws();
        // An interior stage -- window stage >= 1 (past every head piece: lz < 64 <= 32 P)
        // and ending at or before the packet's end in every lane -- has no piece outside
        // [lz, pe): its addresses skip the zero-line selects (wave-uniform branch; about
        // 18 of the stage's VALU, round 5)
        const uint32_t wst = stage_of(pst, pstages);
        constexpr bool kFast = !(ABL & (8 | 64));           // (not the line-shaped / record-order diagnostics)
        const bool inner = !pdone && wst >= 1u && 32u * P * (wst + 1u) <= pe;
        uint64_t s0, s1;
        if (kFast && __builtin_amdgcn_ballot_w64(!inner) == 0u) {
            s0 = ws + a0;
            s1 = ws + a1;
        } else {
            s0 = (a0 < pe && a0 + 16u > lz) ? ws + a0 : zero;
            s1 = (a1 < pe && a1 + 16u > lz) ? ws + a1 : zero;
        }
        // (BIN 3's first produce: the second group's metadata is in LDS already)
        const bool meta = (BIN == 3 && WS < 0) ? false : ((pst == 0u) & qlive & !pdone);
        if (meta) {
            load_meta(qit);
            vr_issue_stage<slot, NT>(s0, s1);
            if constexpr (WS >= 0) vr_wait_stage<(ABL & 4) ? 0 : 3>();   // the metadata load + 2 stage loads younger
        } else {
            vr_issue_stage<slot, NT>(s0, s1);
            if constexpr (WS >= 0) vr_wait_stage<(ABL & 4) ? 0 : 2>();
        }
        if constexpr ((ABL & 32) != 0) __builtin_amdgcn_s_setprio(0);
        ++pst;
    };
    if (any) {
        producer_enter(std::false_type{});
        produce(std::integral_constant<uint32_t, 0>{}, std::integral_constant<int, -1>{});
    }
    if constexpr (BIN == 3) {
        // the wave's record stores (and the table DMAs) have completed before barrier A;
        // only the first stage's two loads stay in flight
        if (any) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }

    // ---- the table image, rebuilt in LDS while stage 0 is in flight.  Wave w
    // writes rows w + 16 i: row j = XOR of basis rows b with bit b of j set (Gray
    // order: one XOR per row), except the INIT and CINV dwords (not linear in j),
    // whose rows < 64 come from basis rows 8 and 9.  Raw s_barrier: no vmcnt drain.
    // the slot counter: slots 0 .. kStatic kVrW - 1 are taken statically; the first dynamic
    // take comes after barrier B (a wave's second group is entered in the loop)
    if (threadIdx.x == 0u) lds_store(BIN ? kVrCtrBin : kVrCtr, kStatic * kVrW);
    __builtin_amdgcn_s_barrier();                            // (A) every basis row has landed
    {
        uint32_t bb[8];
#pragma unroll
        for (int b = 0; b < 8; ++b) bb[b] = lds_load(kVrStaging + 256u * b + 4u * lane);
        const bool nonlin = lane == kInitDword || lane == kCinvDword;
        const uint32_t row8 = kVrStaging + 256u * (lane == kInitDword ? 8u : 9u);
        uint32_t v = 0;
#pragma unroll
        for (int b = 0; b < 4; ++b) v ^= ((wave >> b) & 1u) ? bb[b] : 0u;
#pragma unroll
        for (uint32_t q = 0; q < 16u; ++q) {
            const uint32_t i = q ^ (q >> 1);
            if (q) v ^= bb[4 + __builtin_ctz(q)];
            uint32_t x = v;
            if (i < 4u) {                                    // rows < 64: INIT / CINV
                const uint32_t e = lds_load(row8 + 4u * (wave + 16u * i));
                x = nonlin ? e : x;
            }
            lds_store(256u * (wave + 16u * i) + 4u * lane, x);
        }
    }
    mark(2);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();                            // (B) the image is complete
    mark(3);
    if constexpr (BIN) {                                     // the first group's indices (slot 0)
        if (any) lds_store(stash_addr(0u), pidx);
    }
    if (!any) {
        trace_end();                                         // (the prologue's loads are retired)
        return;
    }

    // ---- consumer
    uint32_t reg = 0, clz = 0, ce = 0, cs = 0, cstages = 0, nedge = ~0u;
    uint32_t rt = 0;                                         // kRot: the last stage's fold
    uint32_t cps = ~0u, cconn = 0, desired = 0;              // VF: slot position, connectID, the slot's bytes
    uint8_t* cok = nullptr;                                  // VF: the keep mask of the group's packets
    uint32_t* cout = nullptr;                                // the CRCs of the group's packets (BIN: the batch's)
    uint64_t crem = 0;                                       // packets of its batch from the group's first
    // first stage >= from holding a partly covered head or tail piece (~0u = none):
    // the per-lane search, one wave reduction per call
    auto next_edge = [&](uint32_t from) __attribute__((always_inline)) -> uint32_t {
        const bool live = ce != clz;
        const uint32_t wh = clz >> 5, wl = (ce - 1u) >> 5;
        uint32_t h = (live && (clz & 15u) && (wh & (P - 1u)) == lane_k()) ? wh >> LG : ~0u;
        uint32_t t = (live && (ce & 15u) && (wl & (P - 1u)) == lane_k()) ? wl >> LG : ~0u;
        h = step_of(h, cstages);
        t = step_of(t, cstages);
        h = h >= from ? h : ~0u;
        t = t >= from ? t : ~0u;
        if constexpr (VF) {                                  // the slot's block(s)
            const uint32_t s0 = cps >> 5, s1 = (cps + 3u) >> 5;
            uint32_t a = (cps != ~0u && (s0 & (P - 1u)) == lane_k()) ? step_of(s0 >> LG, cstages) : ~0u;
            uint32_t b = (cps != ~0u && s1 != s0 && (s1 & (P - 1u)) == lane_k()) ? step_of(s1 >> LG, cstages) : ~0u;
            a = a >= from ? a : ~0u;
            b = b >= from ? b : ~0u;
            h = min(h, min(a, b));
        }
        return wave_min_u(min(h, t));
    };
    // ... and the same from the group's edge-stage mask: bit s = stage s holds such a
    // piece in some lane, bit 31 = some stage >= 31 does.  One wave reduction per
    // group (consumer_enter) instead of one per edge stage; groups of more than 31
    // stages fall back to the search from stage 31 on.
    uint32_t emask = 0;
    auto next_edge_m = [&](uint32_t from) __attribute__((always_inline)) -> uint32_t {
        if (from >= 31u) return (emask >> 31) ? next_edge(from) : ~0u;
        const uint32_t m = emask & (~0u << from);
        if (!m) return ~0u;
        const uint32_t st = static_cast<uint32_t>(__builtin_ctz(m));
        return st < 31u ? st : next_edge(31u);
    };
    // this lane's edge stages as mask bits (stages >= 31 on bit 31)
    auto next_edge_lane_bits = [&]() __attribute__((always_inline)) -> uint32_t {
        const bool live = ce != clz;
        const uint32_t wh = clz >> 5, wl = (ce - 1u) >> 5;
        auto bit = [](uint32_t st) __attribute__((always_inline)) { return st == ~0u ? 0u : 1u << min(st, 31u); };
        uint32_t e = bit((live && (clz & 15u) && (wh & (P - 1u)) == lane_k()) ? step_of(wh >> LG, cstages) : ~0u) |
                     bit((live && (ce & 15u) && (wl & (P - 1u)) == lane_k()) ? step_of(wl >> LG, cstages) : ~0u);
        if constexpr (VF) {                                  // the slot's block(s)
            const uint32_t s0 = cps >> 5, s1 = (cps + 3u) >> 5;
            e |= bit((cps != ~0u && (s0 & (P - 1u)) == lane_k()) ? step_of(s0 >> LG, cstages) : ~0u);
            e |= bit((cps != ~0u && s1 != s0 && (s1 & (P - 1u)) == lane_k()) ? step_of(s1 >> LG, cstages) : ~0u);
        }
        return e;
    };
    // Entered right after the producer has entered the same group (the producer
    // runs exactly one stage ahead), so pit / plz / pe are that group's.
    auto consumer_enter = [&]() __attribute__((always_inline)) {
        clz = plz();
        ce = pe;
        const uint64_t base = group_base(pit);
        // (BIN with ABL & 64, diagnostics: CRCs written in record order, as an unbinned batch)
        cout = bl.b[pit.b].out ? bl.b[pit.b].out + ((BIN && !(ABL & 64)) ? 0u : base) : nullptr;
        if constexpr (VF) {
            cok = bl.b[pit.b].ok + base;
            cps = pps;
            cconn = pconn;
            desired = 0;
        }
        if constexpr (BIN) ++cgn;
        crem = batch_n(pit.b) - base;
        const uint32_t nb = (ce + 31u) >> 5;                 // 0 for an empty packet ([0, 0))
        // the producer's count for this same group (no second wave reduction; the trace
        // instance keeps the reduction: without it, it spilled a VGPR)
        if constexpr (TR == 1) cstages = max(1u, wave_max_u((nb + P - 1u) >> LG));
        else cstages = pstages;
        const uint32_t init = lds_load(init_addr(clz));
        reg = lane_k() == 0u ? (nb ? init : 0xFFFFFFFFu) : 0u;      // packet.cs:144 (empty packet: ~crc = 0)
        // a group whose packets all start and end on 16-byte boundaries has no partly
        // covered piece: one ballot instead of the per-lane search and its wave reduction
        // (cfg2: VALU -4.2 %, profiles/r05_edge_ballot/).  Not in receive verify, whose
        // every packet holds a slot, nor in the records instance, whose length-binned
        // packets of mixed lengths (cfg3) rarely are aligned at both ends (there the
        // ballot only adds work: cfg3 binned -0.7 %)
        constexpr bool kEdgeBallot = !VF && BIN != 1;
        const bool may_edge = ce != clz && ((clz | ce) & 15u) != 0u;
        if (kEdgeBallot && __builtin_amdgcn_ballot_w64(may_edge) == 0u) {
            emask = 0u;
        } else {
            const uint32_t e = next_edge_lane_bits();
            emask = wave_or_u(e);
        }
        nedge = next_edge_m(0);
        cs = 0;
        if (TR) ++ngroups;
    };
    consumer_enter();
    bool done = false;
    auto iteration = [&](auto sc) __attribute__((always_inline)) {
        constexpr uint32_t S = decltype(sc)::value;
        if constexpr (kVrLaneRecompute || kRot || VF) lane = vr_lane();   // (the rt / slot registers need the room)
        produce(std::integral_constant<uint32_t, S ^ 1u>{}, std::integral_constant<int, static_cast<int>(S)>{});
        const uint32_t cst = stage_of(cs, cstages);          // the window stage this step folds
        const bool tail_first = kRot && cs == 0u && cstages > 1u;   // (wave-uniform)
        const uint32_t rin = tail_first ? 0u : reg;
        // the fold of the landed slot S: the fused asm (product instances), or the
        // rotation then the C++ lookups (diagnostics ablations), or -- receive verify's
        // edge stages, whose slot fix-up works on copies -- the copies' fold
        // (not in the verify diagnostics -- tail first, pair rounds, trace -- which then spill)
        constexpr bool kFused = kVrRotateInPlace && !(ABL & (2 | 64)) && !(VF && (kRot || DYN == 2 || TR));
        auto fold = [&]() __attribute__((always_inline)) -> uint32_t {
            if constexpr (kFused) {
                return vr_fold_slot<S>(rin, lane, make_vr_sched(lane));
            } else {
                uint32_t d[8];
                vr_prepare<S, !(ABL & 64)>(rin, lane, d);
                if constexpr (ABL & 2) return xor3(xor3(d[0], d[1], d[2]), xor3(d[3], d[4], d[5]), d[6] ^ d[7]);
                else return vr_lookups(d, make_vr_sched(lane));
            }
        };
        uint32_t nr;
        if (cs == nedge) {                                   // head / tail pieces: keep [clz, ce) only
            const uint32_t q0 = 32u * (lane_k() + P * cst);              // windows < 2 GiB: differences fit int32
            if constexpr (VF) {                              // masked in place, then the slot fix-up on copies
                if constexpr (!(ABL & 1))
                    vr_edge_mask_slot<S>(lane & 16u, static_cast<int32_t>(clz - q0), static_cast<int32_t>(ce - q0));
                u32x4 A, B;
                vr_read_stage<S>(A, B);
                if (cps != ~0u) vr_slot_fix(A, B, make_vr_sched(lane).hs, static_cast<int32_t>(cps - q0), cconn, desired);
                nedge = next_edge_m(cs + 1u);
                uint32_t d[8];
                vr_shuffle(rin, lane, A, B, d);
                if constexpr (ABL & 2) nr = xor3(xor3(d[0], d[1], d[2]), xor3(d[3], d[4], d[5]), d[6] ^ d[7]);
                else nr = vr_lookups(d, make_vr_sched(lane));
            } else {                                         // masked in place, then folded as any stage
                if constexpr (!(ABL & 1))
                    vr_edge_mask_slot<S>(lane & 16u, static_cast<int32_t>(clz - q0), static_cast<int32_t>(ce - q0));
                nedge = next_edge_m(cs + 1u);
                nr = fold();
            }
        } else {
            nr = fold();
        }
        const bool inw = 32u * (lane_k() + P * cst) < ce;           // the lane's block k + P cst is in the window
        if (tail_first) rt = inw ? nr : 0u;
        else reg = inw ? nr : reg;
        if (++cs == cstages) {
            if (kRot && cstages > 1u && 32u * (lane_k() + P * (cstages - 1u)) < ce) {
                // the last-stage block came first: reg = rt ^ reg x^(256 P)
                uint32_t x[4];
#pragma unroll
                for (int b = 0; b < 4; ++b) {
                    const uint32_t sel = 0x0C0C0000u | ((4u + b) << 8);      // byte1 = byte b of reg, byte0 = column
                    x[b] = lds_load(__builtin_amdgcn_perm(reg, col_byte(31u - b), sel));
                }
                reg = xor3(x[0], x[1], x[2]) ^ x[3] ^ rt;
            }
            // lane k is o = (k - nb) mod P blocks past the window end: x^(-256 o)
            const uint32_t nb = (ce + 31u) >> 5;
            const uint32_t o = (lane_k() - nb) & (P - 1u);
            // (lane-uniform byte order: per-lane rotations hoisted out of the loop cost
            // ten VGPRs; four lookups per packet can afford the bank conflicts)
            const uint32_t kk = o ? o : 1u;
            // the four columns free_col(4 (kk - 1) + b) = 32 (kk - 1) + 8 b (+ 4 for kk <= 4),
            // one per byte of `cols`: each lookup's perm takes its column byte from there
            static_assert(kCorrCol == 0u, "column bytes below assume the correction columns start at 0");
            const uint32_t cols = (32u * (kk - 1u) + (kk <= 4u ? 4u : 0u)) * 0x01010101u + 0x18100800u;
            uint32_t x[4];
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                const uint32_t sel = 0x0C0C0000u | ((4u + b) << 8) | static_cast<uint32_t>(b);   // byte1 = byte b of reg, byte0 = column b
                x[b] = lds_load(__builtin_amdgcn_perm(reg, cols, sel));
            }
            const uint32_t corr = xor3(x[0], x[1], x[2]) ^ x[3];
            if constexpr (!(ABL & 16)) reg = o ? corr : reg;
            reg = xor_lanes<0>(LG, reg);
            const uint32_t tz = nb ? 32u * nb - ce : 0u;
            // x^(-8 tz): 16 and 8 zero bytes by the multiplier tables (four lookups each,
            // tz_mul), the rest (< 8) as zero-byte unsteps (the U column, unstep_byte, one
            // lookup and about 6 VALU each).  All unsteps (round 2) cost 96 VALU for cfg2's
            // tz = 16, run whenever any of the wave's packets had a ragged end.
            if constexpr (!(ABL & 16))
                if (lane_k() == 0u) reg = vr_unstep_tz<BIN == 1>(reg, tz, kVrTz);
            if constexpr (VF) {
                desired = xor_lanes<0>(LG, desired);         // the slot's bytes, from at most two lanes
                if (lane_k() == 0u && lane_p() < crem) {
                    const uint32_t comp = cps != ~0u ? finalize(reg) : 0u;
                    cok[lane_p()] = (cps != ~0u && comp == desired) ? 1 : 0;     // protocol.cs:1066-1068
                    if (cout) cout[lane_p()] = comp;
                }
            } else if (lane_k() == 0u && lane_p() < crem) {
                const uint32_t ci = (BIN && !(ABL & 64)) ? lds_load(stash_addr(cgn - 1u)) : lane_p();   // (BIN: the record's index)
                cout[ci] = finalize(reg);                                         // packet.cs:159
            }
            if (pdone) {
                // no newer group entered: the wave is done.  The producer's last loads
                // (zero lines past the end) are dead: retire them before the wave ends
                vr_drain();
                done = true;
                return;
            }
            consumer_enter();
        }
    };
    // each slot's iteration leaves the loop at once when the wave is done, so the
    // loop head is reached only from a completed ring turn (no path with the drained
    // loads of the last turn in flight: tools/isa_inflight_check.py)
    mark(4);                                                 // (streaming starts)
    do {
        iteration(std::integral_constant<uint32_t, 0>{});
        if (!done) iteration(std::integral_constant<uint32_t, 1>{});
    } while (!done);
    trace_end();
}

// ---------------------------------------------------------------- host side

// the instance; dyn = its dynamic-rounds twin where one is built
template <int LG, int TR = 0, int NT = 0, int ABL = 0, int BIN = 0, int WK = 0, int ROT = 0, int VF = 0>
const void* vring_fn(int dyn = 0) {
    // (the dynamic-round twins are diagnostics: the product library's contexts never set
    // vr_dynamic, so it builds none -- ADVICE r4)
#ifdef ENET_HIP_DIAG
    if constexpr (TR != 1 && NT == 0 && ABL == 0 && WK == 0 && ROT == 0) {
        if (dyn == 1) return reinterpret_cast<const void*>(crc32_vring_kernel<LG, TR, NT, ABL, BIN, WK, ROT, VF, 1>);
        if constexpr (!BIN)                                  // (pair rounds: not for the records instance)
            if (dyn == 2) return reinterpret_cast<const void*>(crc32_vring_kernel<LG, TR, NT, ABL, BIN, WK, ROT, VF, 2>);
    }
#endif
    return dyn == 0 ? reinterpret_cast<const void*>(crc32_vring_kernel<LG, TR, NT, ABL, BIN, WK, ROT, VF>) : nullptr;
}
// the dynamic-round mode a variant selects (0: the static deal)
int vring_dyn(const VrVariant& v) { return v.claim ? v.claim_mode : 0; }
// receive verify (8 lanes per packet): the product instance; diagnostics: tail first, end records
const void* vring_pick_v(bool trace, const VrVariant& v) {
    const int dyn = vring_dyn(v);
    if (!trace && !v.nt && !v.abl && !v.walk && !v.tail_first) return vring_fn<3, 0, 0, 0, 0, 0, 0, 1>(dyn);
#ifdef ENET_HIP_DIAG
    if (!trace && !v.nt && !v.abl && !v.walk && v.tail_first) return vring_fn<3, 0, 0, 0, 0, 0, 1, 1>();
    if (trace && v.abl == 128 && !v.nt && !v.walk && !v.tail_first) return vring_fn<3, 2, 0, 0, 0, 0, 0, 1>(dyn);
#endif
    return nullptr;
}
// compact: BIN = 2 (two workgroups per CU).  (diagnostics: abl 2 = no fold lookups, 19 =
// no masks, lookups or end corrections, + 64 = CRCs stored in record order, at 4 lanes)
const void* vring_pick_bin(int lg, int dyn, int abl = 0, bool compact = false, bool trace = false) {
#ifdef ENET_HIP_DIAG
    // the per-wave timeline of the records instance (tools/bin_timeline.py)
    if (trace) {
        if (abl || dyn) return nullptr;
        if (compact) return lg == 2 ? vring_fn<2, 1, 0, 0, 2>() : vring_fn<3, 1, 0, 0, 2>();
        return lg == 2 ? vring_fn<2, 1, 0, 0, 1>() : vring_fn<3, 1, 0, 0, 1>();
    }
#else
    if (trace) return nullptr;
#endif
    if (abl == 0 && compact) return lg == 2 ? vring_fn<2, 0, 0, 0, 2>(dyn) : vring_fn<3, 0, 0, 0, 2>(dyn);
    if (abl == 0) return lg == 2 ? vring_fn<2, 0, 0, 0, 1>(dyn) : vring_fn<3, 0, 0, 0, 1>(dyn);
#ifdef ENET_HIP_DIAG
    if (lg == 2 && dyn == 0 && abl == 2) return compact ? vring_fn<2, 0, 0, 2, 2>() : vring_fn<2, 0, 0, 2, 1>();
    if (lg == 2 && dyn == 0 && abl == 19) return compact ? vring_fn<2, 0, 0, 19, 2>() : vring_fn<2, 0, 0, 19, 1>();
    // 64: the CRCs stored in record order (the scattered out[index] stores priced)
    if (lg == 2 && dyn == 0 && abl == 64 && !compact) return vring_fn<2, 0, 0, 64, 1>();
    if (lg == 2 && dyn == 0 && abl == 83 && !compact) return vring_fn<2, 0, 0, 83, 1>();
#endif
    return nullptr;
}

// the local-tile records instance (BIN = 3); trace = its per-wave timeline twin
// (diagnostics library)
const void* vring_pick_local(int lg, bool trace) {
    if (lg != 2 && lg != 3) return nullptr;
#ifdef ENET_HIP_DIAG
    if (trace) return lg == 2 ? vring_fn<2, 1, 0, 0, 3>() : vring_fn<3, 1, 0, 0, 3>();
#else
    if (trace) return nullptr;
#endif
    return lg == 2 ? vring_fn<2, 0, 0, 0, 3>() : vring_fn<3, 0, 0, 0, 3>();
}

// The product instances: 64 VGPRs (WPE 8), one or two workgroups per CU, stages in
// window order.  The diagnostics library (ENET_HIP_DIAG) adds the sweep variants: a
// trace buffer (per-wave timestamps), nt stage loads, workgroup walks, the tail-first
// stage order and the ablations (wrong CRCs by design).  Null = not built here.
// Measured and not kept: 3 and 4 ring slots and a binned-records variant (its
// record register was copied by hipcc between load and wait).
const void* vring_pick(int lg, bool trace, const VrVariant& v) {
    if (lg != 2 && lg != 3) return nullptr;
    const bool plain = !trace && !v.nt && !v.abl && !v.walk && !v.tail_first;
    const int dyn = vring_dyn(v);
    if (plain) return lg == 2 ? vring_fn<2>(dyn) : vring_fn<3>(dyn);
#ifdef ENET_HIP_DIAG
    const bool nt = v.nt;
    const int abl = v.abl;
    if (v.tail_first) {
        if (abl == 2 && lg == 3 && !trace && !nt && !v.walk) return vring_fn<3, 0, 0, 2, 0, 0, 1>();   // no lookups
        if (trace || abl || v.walk) return nullptr;
        return lg == 2 ? (nt ? vring_fn<2, 0, 1, 0, 0, 0, 1>() : vring_fn<2, 0, 0, 0, 0, 0, 1>())
                       : (nt ? vring_fn<3, 0, 1, 0, 0, 0, 1>() : vring_fn<3, 0, 0, 0, 0, 0, 1>());
    }
    if (v.walk) {
        if (trace || abl) return nullptr;
        return lg == 2 ? (nt ? vring_fn<2, 0, 1, 0, 0, 1>() : vring_fn<2, 0, 0, 0, 0, 1>())
                       : (nt ? vring_fn<3, 0, 1, 0, 0, 1>() : vring_fn<3, 0, 0, 0, 0, 1>());
    }
    if (trace) {
        if (abl == 128 && !nt) return lg == 2 ? vring_fn<2, 2>(dyn) : vring_fn<3, 2>(dyn);   // end records only
        if (abl) return nullptr;
        return lg == 2 ? (nt ? vring_fn<2, 1, 1>() : vring_fn<2, 1>()) : (nt ? vring_fn<3, 1, 1>() : vring_fn<3, 1>());
    }
    if (!abl) return lg == 2 ? vring_fn<2, 0, 1>() : vring_fn<3, 0, 1>();
    if (abl == 8 && lg == 3) return nt ? vring_fn<3, 0, 1, 8>() : vring_fn<3, 0, 0, 8>();
    if (abl == 27 && lg == 3) return nt ? vring_fn<3, 0, 1, 27>() : vring_fn<3, 0, 0, 27>();
    if (abl == 19 && !nt) return lg == 2 ? vring_fn<2, 0, 0, 19>() : vring_fn<3, 0, 0, 19>();
    if (abl == 2 && lg == 3 && !nt) return vring_fn<3, 0, 0, 2>();
    if (abl == 32 && lg == 2) return nt ? vring_fn<2, 0, 3>() : vring_fn<2, 0, 2>();   // sc1 / sc0 sc1
    if (abl == 32 && lg == 3 && !nt) return vring_fn<3, 0, 0, 32>();                     // produce at s_setprio 3
    if (lg == 2 && !nt) {
        switch (abl) {
            case 1: return vring_fn<2, 0, 0, 1>();
            case 2: return vring_fn<2, 0, 0, 2>();
            case 3: return vring_fn<2, 0, 0, 3>();
            case 4: return vring_fn<2, 0, 0, 4>();
            case 6: return vring_fn<2, 0, 0, 6>();
            default: break;
        }
    }
#endif
    return nullptr;
}

int vring_setup() {
    auto set = [](const void* fn, int lds) -> int {
        if (!fn) return 0;
        const hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
        return e == hipSuccess ? 0 : -static_cast<int>(e);
    };
    static const int kAbl[] = {0, 1, 2, 3, 4, 6, 8, 19, 27, 32, 128};
    static uint64_t any_line;                                // (a non-null claim selects the DYN twins)
    for (int d = 0; d < 3; ++d) {
        uint64_t* const claim = d ? &any_line : nullptr;
        for (int t = 0; t < 2; ++t)
            for (int w = 0; w < 2; ++w) {
                VrVariant v;
                v.tail_first = w != 0;
                v.abl = t ? 128 : 0;
                v.claim = claim;
                v.claim_mode = d;
                const int rc = set(vring_pick_v(t != 0, v), kVrLds);
                if (rc) return rc;
            }
        for (int lg = 2; lg <= 3; ++lg) {
            int rc;
            for (int abl : {0, 2, 19, 64, 83}) {
                if ((rc = set(vring_pick_bin(lg, d, abl), kVrLdsBin))) return rc;
                if ((rc = set(vring_pick_bin(lg, d, abl, true), kVrLdsBinC))) return rc;
            }
            if ((rc = set(vring_pick_bin(lg, d, 0, false, true), kVrLdsBin))) return rc;
            if ((rc = set(vring_pick_bin(lg, d, 0, true, true), kVrLdsBinC))) return rc;
            for (bool tr : {false, true})
                if ((rc = set(vring_pick_local(lg, tr), kVrLdsBinC))) return rc;
            for (int t = 0; t < 2; ++t)
                for (int nt = 0; nt < 2; ++nt)
                    for (int abl : kAbl)
                        for (int w = 0; w < 4; ++w) {
                            VrVariant v;
                            v.nt = nt != 0;
                            v.abl = abl;
                            v.walk = (w & 1) != 0;
                            v.tail_first = (w & 2) != 0;
                            v.claim = claim;
                            v.claim_mode = d;
                            if ((rc = set(vring_pick(lg, t != 0, v), kVrLds))) return rc;
                        }
        }
    }
    return 0;
}

int vring_launch_list(int lg, int max_wgs, const VrVariant& v, hipStream_t st, const VrBatches& bl,
                      const KernelTables& tb, const uint32_t* basis2, uint64_t* trace, bool bin) {
    if ((lg != 2 && lg != 3) || bl.count > static_cast<uint32_t>(kVrMaxBatches))
        return -static_cast<int>(hipErrorInvalidValue);
    // empty batches dropped: the kernel may then read any batch's packet n - 1
    VrBatches a{};
    a.claim = v.claim;
    a.claim_gen = v.claim_gen;
    if (bin && (bl.count != 1 || (bl.tile_counts && bl.b[0].n != 1024ull * bl.tiles)))   // records: one batch
        return -static_cast<int>(hipErrorInvalidValue);
    a.tile_counts = bin ? bl.tile_counts : nullptr;
    a.tiles = bin ? bl.tiles : 0u;
    for (uint32_t b = 0; b < bl.count; ++b)
        if (bl.b[b].n) a.b[a.count++] = bl.b[b];
    if (a.count == 0) return 0;
    const uint64_t kpk = 64u >> lg;
    for (uint32_t b = 0; b < a.count; ++b) {                 // the concatenated group space
        a.b[b].g0 = a.groups;
        a.groups += (a.b[b].n + kpk - 1u) / kpk;
    }
    unsigned grid = static_cast<unsigned>(std::max<uint64_t>(
        1, std::min<uint64_t>((a.groups + kVrW - 1) / kVrW, static_cast<uint64_t>(max_wgs))));
    VrVariant w = v;
    if (vring_dyn(w) == 2) {                                 // pairs: an even grid of at least 2 (not binned)
        if (bin || grid < 2 || grid / 2 > static_cast<unsigned>(kVrPairWords)) w.claim = a.claim = nullptr;
        grid &= ~1u;
        grid = std::max(grid, 1u);
    }
    const void* fn = bin ? vring_pick_bin(lg, vring_dyn(w), w.abl, w.compact, trace != nullptr)
                         : vring_pick(lg, trace != nullptr, w);
    if (!fn) return -static_cast<int>(hipErrorInvalidValue);   // a variant this library does not build
    // slots are 32-bit: a workgroup's slot count (rounds x 16) must fit
    if ((a.groups / (static_cast<uint64_t>(grid) * kVrW) + 3u) * kVrW > 0xFFFFFFF0ull)
        return -static_cast<int>(hipErrorInvalidValue);
    void* args[] = {&a, const_cast<KernelTables*>(&tb), const_cast<const uint32_t**>(&basis2), &trace};
    const int lds = bin ? (w.compact ? kVrLdsBinC : kVrLdsBin) : kVrLds;
    const hipError_t e = hipLaunchKernel(fn, dim3(grid), dim3(64 * kVrW), args, lds, st);
    return e == hipSuccess ? 0 : -static_cast<int>(e);
}

int vring_launch_vlist(int max_wgs, const VrVariant& v, hipStream_t st, const VrVBatches& bl, const KernelTables& tb,
                       const uint32_t* basis2, uint64_t* trace) {
    if (bl.count > static_cast<uint32_t>(kVrMaxVBatches)) return -static_cast<int>(hipErrorInvalidValue);
    VrVBatches a{};                                          // empty batches dropped
    a.claim = v.claim;
    a.claim_gen = v.claim_gen;
    for (uint32_t b = 0; b < bl.count; ++b)
        if (bl.b[b].n) a.b[a.count++] = bl.b[b];
    if (a.count == 0) return 0;
    for (uint32_t b = 0; b < a.count; ++b) {                 // the concatenated group space (8 packets a group)
        a.b[b].g0 = a.groups;
        a.groups += (a.b[b].n + 7u) / 8u;
    }
    unsigned grid = static_cast<unsigned>(std::max<uint64_t>(
        1, std::min<uint64_t>((a.groups + kVrW - 1) / kVrW, static_cast<uint64_t>(max_wgs))));
    VrVariant w = v;
    if (vring_dyn(w) == 2) {                                 // pairs: an even grid of at least 2
        if (grid < 2 || grid / 2 > static_cast<unsigned>(kVrPairWords)) w.claim = a.claim = nullptr;
        grid &= ~1u;
        grid = std::max(grid, 1u);
    }
    const void* fn = vring_pick_v(trace != nullptr, w);
    if (!fn) return -static_cast<int>(hipErrorInvalidValue);
    if ((a.groups / (static_cast<uint64_t>(grid) * kVrW) + 3u) * kVrW > 0xFFFFFFF0ull)
        return -static_cast<int>(hipErrorInvalidValue);
    void* args[] = {&a, const_cast<KernelTables*>(&tb), const_cast<const uint32_t**>(&basis2), &trace};
    const hipError_t e = hipLaunchKernel(fn, dim3(grid), dim3(64 * kVrW), args, kVrLds, st);
    return e == hipSuccess ? 0 : -static_cast<int>(e);
}

int vring_launch_local(int lg, int max_wgs, hipStream_t st, const PacketArgs& pa, void* records,
                       const KernelTables& tb, const uint32_t* basis2, uint32_t keep_min) {
    if (pa.n == 0) return 0;
    if ((lg != 2 && lg != 3) || max_wgs < 1 || !records || (reinterpret_cast<uintptr_t>(records) & 15u))
        return -static_cast<int>(hipErrorInvalidValue);
    // T: the packets of a workgroup -- the batch over max_wgs workgroups, in whole groups,
    // at least a group per wave, at most kVrLocalTile (two per thread)
    const uint64_t kpk = 64u >> lg;
    uint64_t T = (pa.n + static_cast<uint64_t>(max_wgs) - 1u) / static_cast<uint64_t>(max_wgs);
    T = std::max<uint64_t>((T + kpk - 1u) / kpk * kpk, kpk * kVrW);
    T = std::min<uint64_t>(T, kVrLocalTile);
    const uint64_t grid = (pa.n + T - 1u) / T;               // (every workgroup has a packet)
    if (grid > static_cast<uint64_t>(max_wgs)) return -static_cast<int>(hipErrorInvalidValue);
    VrBatches a{};
    a.count = 1;
    a.b[0] = VrBatch{pa.bytes, pa.off, pa.len, pa.out, pa.n, 0u};
    a.groups = (pa.n + kpk - 1u) / kpk;
    a.tile_local = static_cast<uint32_t>(T);
    a.local_rec = records;
    a.local_keep_min = keep_min;
    const void* fn = vring_pick_local(lg, pa.trace != nullptr);
    if (!fn) return -static_cast<int>(hipErrorInvalidValue);
    uint64_t* trace = pa.trace;
    void* args[] = {&a, const_cast<KernelTables*>(&tb), const_cast<const uint32_t**>(&basis2), &trace};
    const hipError_t e = hipLaunchKernel(fn, dim3(static_cast<unsigned>(grid)), dim3(64 * kVrW), args, kVrLdsBinC, st);
    return e == hipSuccess ? 0 : -static_cast<int>(e);
}

int vring_launch(int lg, int max_wgs, const VrVariant& v, hipStream_t st, const PacketArgs& pa, const KernelTables& tb,
                 const uint32_t* basis2) {
    if (pa.n == 0) return 0;
    VrBatches bl{};
    bl.count = 1;
    // binned records: the record array rides in the offsets field (BIN instance)
    bl.b[0] = pa.meta4 ? VrBatch{pa.bytes, reinterpret_cast<const uint64_t*>(pa.meta4), nullptr, pa.out, pa.n, 0u}
                       : VrBatch{pa.bytes, pa.off, pa.len, pa.out, pa.n, 0u};
    // (records: the trace instance only in the diagnostics library, where enet_hip_diag_trace
    // can set a trace buffer)
    return vring_launch_list(lg, max_wgs, v, st, bl, tb, basis2, pa.trace, pa.meta4 != nullptr);
}

}  // namespace enethip
