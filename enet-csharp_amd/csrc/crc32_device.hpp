// crc32_device.hpp -- gfx950 device building blocks of the CRC32 kernels
// (included by crc32_kernels.hip and by the measurement-only tools/microbench.hip).
// Reference algorithm: /root/reference/enet-csharp/ENet/c/packet.cs:142-160.
//
// Slicing-by-32 in LDS, conflict-free.  A 32-byte block b_0..b_31 is folded
// into the Sarwate register by   reg' = XOR_m T_{31-m}[b_m ^ reg_m]   (reg_m = byte
// m of reg for m < 4, else 0), T_t[j] = byte j followed by t zero bytes (the
// stream kernel uses T'_t = T_{t+32(P-1)}, see crc32_kernels.hip).  Row j of the
// 64 KiB LDS image is 256 bytes; table t sits in dword column 2t + (t >> 4), so
// the LDS address of a lookup is  j*256 + 8t + 4(t>>4)  -- byte 1 = the data byte,
// byte 0 = a per-lane constant: ONE v_perm_b32 forms it (no shift, no add).  At
// lookup step i lane l handles byte m = i ^ (l & 31) -- an XOR Latin square -- so
// in every ds_read_b32 the 32 lanes of a half-wave read 32 different tables, whose
// columns 2t + (t>>4) are 32 different banks (ds_read_b32 bank = (addr/4) mod 32,
// lanes 0-31 and 32-63 served as separate groups): no conflicts whatever the
// data (tests/test_kernel_model.py proves it).  The 32 dwords per row no table
// uses (columns 2c+1 for c < 16, 2c for c >= 16) hold byte-indexed tables:
// the per-lane overshoot corrections, INIT[] and CINV[].  The
// per-lane byte order costs one dword permutation per block (two bitop3 rounds +
// a half swap).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "crc32_math.hpp"

namespace enethip {

constexpr int kLdsTableBytes = 256 * 256;         // 256 rows x 256 B = 64 KiB
constexpr int kImageDwords = kLdsTableBytes / 4;
constexpr int kCinvEntries = 512;

// Byte offset of slicing table t in a row, and of free column c (the 32 dwords
// per row no slicing table uses).  A free column is a 256-entry table indexed by
// the row, i.e. by a byte value: one v_perm + ds_read per lookup.
__host__ __device__ constexpr uint32_t col_byte(uint32_t t) { return 8u * t + 4u * (t >> 4); }
__host__ __device__ constexpr uint32_t free_col(uint32_t c) { return 4u * (c < 16u ? 2u * c + 1u : 2u * c); }
constexpr uint32_t kCorrCol = 0;    // columns 4(k-1) + b, k = 1..7: (byte b of r) * x^(-256k)
constexpr uint32_t kCorrLanes = 8;  // lanes-per-packet values whose corrections are tabled
constexpr uint32_t kInitCol = 29;   // INIT[r], rows 0..31
constexpr uint32_t kCinvCol = 30;   // CINV[n] = x^(-8n), n < 512: row n & 255 of column 30 + (n >> 8)
__host__ __device__ constexpr uint32_t init_addr(uint32_t r) { return 256u * r + free_col(kInitCol); }
__host__ __device__ constexpr uint32_t cinv_addr(uint32_t n) { return 256u * (n & 255u) + free_col(kCinvCol + (n >> 8)); }
__host__ __device__ constexpr uint32_t corr_col(uint32_t k, uint32_t b) { return free_col(kCorrCol + 4u * (k - 1u) + b); }
// U[h] (free column 28, GF(2)-linear in h): one zero byte undone, reg x^(-8) =
// (reg << 8) ^ U[reg >> 24]; U[t0(b) >> 24] = (t0(b) << 8) | b (the top bytes of the
// Sarwate table are a permutation)
constexpr uint32_t kUnstepCol = 28;
__host__ __device__ constexpr uint32_t unstep_addr(uint32_t h) { return 256u * h + free_col(kUnstepCol); }
constexpr int kXnEntries = 65536;                  // x^(8n) for n < 65536 (+ high part)
// Lean-kernel table basis (crc32_lean.hip): every image column but INIT and CINV
// is GF(2)-linear in the row index, so rows 2^b (b < 8) rebuild it; row 8 holds
// INIT[0..31] | CINV[0..31], the only INIT/CINV rows that kernel reads.
constexpr int kBasisRows = 9;
constexpr int kBasisDwords = kBasisRows * 64;      // per image
constexpr uint32_t kInitDword = free_col(kInitCol) / 4u;
constexpr uint32_t kCinvDword = free_col(kCinvCol) / 4u;

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
// LDS dword addressed by an absolute byte address.  The table is the first thing
// in every kernel's single dynamic LDS array, so it starts at LDS address 0 and
// an integer -> address_space(3) cast feeds the computed address straight to
// ds_read_b32 (a generic `lds + addr` costs one v_add per lookup).
typedef __attribute__((address_space(3))) const uint32_t lds_u32;
typedef __attribute__((address_space(3))) const u32x4 lds_u32x4;

struct KernelTables {
    const uint32_t* image;  // kLdsTableBytes per image (P = 1, 4, 8, 16), copied into LDS
    const uint32_t* xn_lo;  // x^(8n) mod P, n < 65536
    const uint32_t* xn_hi;  // x^(8*65536*q) mod P, q < 65536
    const uint32_t* init;   // INIT[r], r < 32
    const uint8_t* zero;    // 256 zero bytes: DMA source of pieces wholly outside a packet
    const uint32_t* basis;  // kBasisDwords per image (lean kernel)
    const uint32_t* tz;     // kTzTableDwords + kTzSmallDwords: the zero-byte multiplier tables (vring kernel)
};

// Zero-byte multipliers for a packet end's tz correction, reg x^(-8 tz): table k
// (0: 16 zero bytes, 1: 8) byte b, entry v = (v << 8 b) x^(-8 (k ? 8 : 16)), at dword
// 256 (4 k + b) + v.  reg x^(-128) = XOR of four lookups by reg's bytes.
constexpr int kTzTables = 2;
constexpr int kTzTableDwords = kTzTables * 4 * 256;        // 8 KiB
__host__ __device__ constexpr uint32_t tz_addr(uint32_t k, uint32_t b, uint32_t v) {
    return 4u * (256u * (4u * k + b) + v);
}
// ... and for c = 1..7 zero bytes (the vring records instance: tz mod 8 by four lookups
// instead of up to seven unsteps), after them: entry v of byte b = (v << 8 b) x^(-8 c)
// at dword 256 (4 (c - 1) + b) + v of this block
constexpr int kTzSmallTables = 7;
constexpr int kTzSmallDwords = kTzSmallTables * 4 * 256;  // 28 KiB
__host__ __device__ constexpr uint32_t tz_small_addr(uint32_t c, uint32_t b, uint32_t v) {
    return 4u * (256u * (4u * (c - 1u) + b) + v);
}

// ------------------------------------------------------------------ device helpers

__device__ __forceinline__ u32x4 ldg16(const uint8_t* p) {
    u32x4 v;
    __builtin_memcpy(&v, p, 16);  // global_load_dwordx4 (unaligned access mode on gfx950)
    return v;
}

// 16 bytes at a 16-byte aligned GLOBAL address given as an integer (an integer
// cast to a generic pointer would make the compiler emit flat loads, which it
// orders with vmcnt(0) + lgkmcnt(0)).
typedef __attribute__((address_space(1))) const u32x4 global_u32x4;
__device__ __forceinline__ u32x4 ldg16_addr(uint64_t addr) {
    return *reinterpret_cast<global_u32x4*>(static_cast<uintptr_t>(addr));
}

// 16 bytes at A, with bytes in front of the packet start `a` read as zero.
// Precondition: every byte of [max(A,a), A+16) belongs to the packet.
__device__ __forceinline__ u32x4 ldg16_head(const uint8_t* A, const uint8_t* a) {
    if (A >= a) return ldg16(A);
    if (A + 16 <= a) return u32x4{0u, 0u, 0u, 0u};
    uint32_t w[4] = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int b = 0; b < 16; ++b)
        if (A + b >= a) w[b >> 2] |= static_cast<uint32_t>(A[b]) << (8 * (b & 3));
    return u32x4{w[0], w[1], w[2], w[3]};
}

// Zero the first n (0..16) bytes of a 16-byte piece.
__device__ __forceinline__ u32x4 zero_prefix(u32x4 v, uint32_t n) {
    const uint32_t b = n * 8u;
    const uint32_t k0 = b >= 32u ? 0u : (0xFFFFFFFFu << b);
    const uint32_t k1 = b >= 64u ? 0u : (b <= 32u ? 0xFFFFFFFFu : (0xFFFFFFFFu << (b - 32u)));
    const uint32_t k2 = b >= 96u ? 0u : (b <= 64u ? 0xFFFFFFFFu : (0xFFFFFFFFu << (b - 64u)));
    const uint32_t k3 = b >= 128u ? 0u : (b <= 96u ? 0xFFFFFFFFu : (0xFFFFFFFFu << (b - 96u)));
    return u32x4{v.x & k0, v.y & k1, v.z & k2, v.w & k3};
}

// 64-bit unsigned min / max.  HIP's device min<uint64_t> / max<uint64_t> templates go
// through double (v_cvt_f64_u32 ... v_max_f64 ... v_cvt_u32_f64: about 12 VALU, and
// inexact above 2^53); these are a compare and two selects, or scalar ops on uniform values.
__host__ __device__ __forceinline__ constexpr uint64_t umin64(uint64_t a, uint64_t b) { return a < b ? a : b; }
__host__ __device__ __forceinline__ constexpr uint64_t umax64(uint64_t a, uint64_t b) { return a < b ? b : a; }

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

// Per-lane constants of the conflict-free slicing-by-32 schedule.
struct LaneSched {
    uint32_t col[8];  // byte h of col[g]: column byte of the table for step i = 4g + h
    uint32_t sel[4];  // v_perm selector for steps with i & 3 == h
    uint32_t m1, m2;  // all-ones when this lane swaps dwords q <-> q^1 / q <-> q^2
    uint32_t hs;      // all-ones when this lane takes the block's two 16-byte halves swapped
};

__device__ __forceinline__ LaneSched make_sched(uint32_t lane) {
    LaneSched s;
    const uint32_t l5 = lane & 31u;
#pragma unroll
    for (int g = 0; g < 8; ++g) {
        uint32_t r = 0;
#pragma unroll
        for (int h = 0; h < 4; ++h) {
            const uint32_t i = 4u * g + h;
            const uint32_t t = (i ^ l5) ^ 31u;        // table of byte m = i ^ l5
            r |= col_byte(t) << (8 * h);
        }
        s.col[g] = r;
    }
#pragma unroll
    for (int h = 0; h < 4; ++h)
        s.sel[h] = static_cast<uint32_t>(h) | ((4u + (static_cast<uint32_t>(h) ^ (l5 & 3u))) << 8) | 0x0C0C0000u;
    s.m1 = 0u - ((l5 >> 2) & 1u);
    s.m2 = 0u - ((l5 >> 3) & 1u);
    s.hs = 0u - ((l5 >> 4) & 1u);
    return s;
}

// One 32-byte block folded into `reg` (== 32 Sarwate steps, packet.cs:153).
// A, B are the block's halves in LANE order: A = bytes 0-15 and B = 16-31 when
// s.hs == 0, swapped when s.hs is all-ones (the staged kernel swaps them for free
// by its LDS read addresses; fold_block below swaps registers).
__device__ __forceinline__ uint32_t fold_block_lane(uint32_t reg, u32x4 A, u32x4 B, const LaneSched& s) {
    // state enters byte 0-3 of the ORIGINAL block: A.x if no swap, else B.x
    const uint32_t a0 = __builtin_amdgcn_bitop3_b32(A.x, reg, s.hs, 0xB4);   // A ^ (reg & ~hs)
    const uint32_t b0 = __builtin_amdgcn_bitop3_b32(B.x, reg, s.hs, 0x78);   // B ^ (reg & hs)
    const uint32_t w[8] = {a0, A.y, A.z, A.w, b0, B.y, B.z, B.w};
    // d[q] = w[q ^ ((lane >> 2) & 3)]: two rounds of bitwise selects (0xD8 = m ? b : a)
    uint32_t x[8], d[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) x[q] = __builtin_amdgcn_bitop3_b32(w[q], w[q ^ 1], s.m1, 0xD8);
#pragma unroll
    for (int q = 0; q < 8; ++q) d[q] = __builtin_amdgcn_bitop3_b32(x[q], x[q ^ 2], s.m2, 0xD8);
    uint32_t v[32];
#pragma unroll
    for (int i = 0; i < 32; ++i) {
        // v_perm: byte0 = column byte of table t, byte1 = data byte j -> j*256 + col
        const uint32_t addr = __builtin_amdgcn_perm(d[i >> 2], s.col[i >> 2], s.sel[i & 3]);
        v[i] = *reinterpret_cast<lds_u32*>(static_cast<uintptr_t>(addr));
    }
    uint32_t acc = xor3(v[0], v[1], v[2]);
#pragma unroll
    for (int i = 3; i + 1 < 32; i += 2) acc = xor3(acc, v[i], v[i + 1]);
    return acc ^ v[31];
}

// Same, halves given in ORIGINAL order (bytes 0-15, 16-31).
__device__ __forceinline__ uint32_t fold_block(uint32_t reg, u32x4 h0, u32x4 h1, const LaneSched& s) {
    u32x4 A, B;
    A.x = __builtin_amdgcn_bitop3_b32(h0.x, h1.x, s.hs, 0xD8);
    A.y = __builtin_amdgcn_bitop3_b32(h0.y, h1.y, s.hs, 0xD8);
    A.z = __builtin_amdgcn_bitop3_b32(h0.z, h1.z, s.hs, 0xD8);
    A.w = __builtin_amdgcn_bitop3_b32(h0.w, h1.w, s.hs, 0xD8);
    B.x = __builtin_amdgcn_bitop3_b32(h1.x, h0.x, s.hs, 0xD8);
    B.y = __builtin_amdgcn_bitop3_b32(h1.y, h0.y, s.hs, 0xD8);
    B.z = __builtin_amdgcn_bitop3_b32(h1.z, h0.z, s.hs, 0xD8);
    B.w = __builtin_amdgcn_bitop3_b32(h1.w, h0.w, s.hs, 0xD8);
    return fold_block_lane(reg, A, B, s);
}

__device__ __forceinline__ uint32_t mulmod(uint32_t a, uint32_t b) {
    uint32_t p = 0;
#pragma unroll
    for (int j = 0; j < 32; ++j) {
        const uint32_t m = static_cast<uint32_t>(static_cast<int32_t>(a << j) >> 31);
        p = __builtin_amdgcn_bitop3_b32(p, b, m, 0x78);                 // p ^ (b & m)
        const uint32_t r = static_cast<uint32_t>(static_cast<int32_t>(b << 31) >> 31);
        b = __builtin_amdgcn_bitop3_b32(b >> 1, kPoly, r, 0x78);         // (b>>1) ^ (P & r)
    }
    return p;
}

__device__ __forceinline__ uint32_t x8n_dev(uint32_t n, const KernelTables& tb) {
    uint32_t x = tb.xn_lo[n & 0xFFFFu];
    if (n >> 16) x = mulmod(x, tb.xn_hi[n >> 16]);
    return x;
}

__device__ __forceinline__ uint32_t wave_max(uint32_t v) {
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) v = max(v, static_cast<uint32_t>(__shfl_xor(static_cast<int>(v), m)));
    return v;
}

// Cross-lane moves on the DPP network (VALU, no LDS traffic -- ds_bpermute based
// shuffles cost LDS cycles and bank-conflict cycles on gfx950).
template <int CTRL>
__device__ __forceinline__ uint32_t dpp(uint32_t v) {
    return static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), CTRL, 0xF, 0xF, true));
}
constexpr int kDppQuadXor1 = 0xB1;       // quad_perm [1,0,3,2]
constexpr int kDppQuadXor2 = 0x4E;       // quad_perm [2,3,0,1]
constexpr int kDppRowHalfMirror = 0x141;
constexpr int kDppRowMirror = 0x140;
constexpr int kDppRowShl = 0x100;        // + n: lane i reads lane i+n of its row (0 past the row end)

// Wave-uniform max / min of a per-lane value: DPP within each 16-lane row, then
// four v_readlane and scalar ops.
__device__ __forceinline__ uint32_t wave_max_u(uint32_t v) {
    v = max(v, dpp<kDppQuadXor1>(v));
    v = max(v, dpp<kDppQuadXor2>(v));
    v = max(v, dpp<kDppRowHalfMirror>(v));
    v = max(v, dpp<kDppRowMirror>(v));
    const uint32_t a = __builtin_amdgcn_readlane(v, 0), b = __builtin_amdgcn_readlane(v, 16);
    const uint32_t c = __builtin_amdgcn_readlane(v, 32), d = __builtin_amdgcn_readlane(v, 48);
    return __builtin_amdgcn_readfirstlane(max(max(a, b), max(c, d)));   // an SGPR: uniform
}
__device__ __forceinline__ uint32_t wave_or_u(uint32_t v) {
    v |= dpp<kDppQuadXor1>(v);
    v |= dpp<kDppQuadXor2>(v);
    v |= dpp<kDppRowHalfMirror>(v);
    v |= dpp<kDppRowMirror>(v);
    const uint32_t a = __builtin_amdgcn_readlane(v, 0), b = __builtin_amdgcn_readlane(v, 16);
    const uint32_t c = __builtin_amdgcn_readlane(v, 32), d = __builtin_amdgcn_readlane(v, 48);
    return __builtin_amdgcn_readfirstlane(a | b | c | d);   // an SGPR: uniform
}
__device__ __forceinline__ uint32_t wave_min_u(uint32_t v) {
    v = min(v, dpp<kDppQuadXor1>(v));
    v = min(v, dpp<kDppQuadXor2>(v));
    v = min(v, dpp<kDppRowHalfMirror>(v));
    v = min(v, dpp<kDppRowMirror>(v));
    const uint32_t a = __builtin_amdgcn_readlane(v, 0), b = __builtin_amdgcn_readlane(v, 16);
    const uint32_t c = __builtin_amdgcn_readlane(v, 32), d = __builtin_amdgcn_readlane(v, 48);
    return __builtin_amdgcn_readfirstlane(min(min(a, b), min(c, d)));   // an SGPR: uniform
}

// Register after feeding the segment [sp, sp+len) from `reg`, with every block
// loaded straight from global memory (the general path: any offsets, lengths and
// alignments).  The segment is processed as an END-aligned window of nb =
// ceil(len/32) blocks; the rp = 32*nb - len bytes in front of sp read as zero.
//
// Software pipeline over HBM latency: a 4-block register ring.  The loop is
// wave-uniform (trip count = the wave's maximum block count) and every load is
// unconditional -- lanes past their range re-load their last block (or, with no
// block at all, the always-valid `safe` buffer) and keep their register by a
// select -- so the compiler emits counted s_waitcnt vmcnt(N) instead of a full
// drain per block (a predicated load makes it wait vmcnt(0) every block).
__device__ __forceinline__ uint32_t fold_window(uint32_t reg, const uint8_t* sp, uint32_t len,
                                                const LaneSched& s, const uint8_t* safe) {
    const uint32_t nb = (len + 31u) >> 5;
    const uint8_t* W = sp + len - (static_cast<size_t>(nb) << 5);
    const bool head = nb && ((nb << 5) != len);
    const uint32_t jb = head ? 1u : 0u;                 // first ring block
    const uint32_t cnt = nb - jb;                       // ring blocks of this lane
    const uint32_t trips = wave_max(cnt);
    // address of ring block k (clamped into this lane's valid range)
    const uint8_t* base = cnt ? W + 32u * jb : safe;
    const uint32_t last = cnt ? cnt - 1u : 0u;
#define ENH_BLK(k) (base + 32u * min(static_cast<uint32_t>(k), last))
    u32x4 r0a = ldg16(ENH_BLK(0)), r0b = ldg16(ENH_BLK(0) + 16);
    u32x4 r1a = ldg16(ENH_BLK(1)), r1b = ldg16(ENH_BLK(1) + 16);
    u32x4 r2a = ldg16(ENH_BLK(2)), r2b = ldg16(ENH_BLK(2) + 16);
    u32x4 r3a = ldg16(ENH_BLK(3)), r3b = ldg16(ENH_BLK(3) + 16);
    if (head) {
        const u32x4 ha = ldg16_head(W, sp), hb = ldg16_head(W + 16, sp);
        reg = fold_block(reg, ha, hb, s);
    }
    for (uint32_t k = 0; k < trips; k += 4) {
        uint32_t nr;
        nr = fold_block(reg, r0a, r0b, s);
        reg = (k + 0 < cnt) ? nr : reg;
        r0a = ldg16(ENH_BLK(k + 4)); r0b = ldg16(ENH_BLK(k + 4) + 16);
        __builtin_amdgcn_sched_barrier(0);  // keep the reload here: 4 blocks ahead
        nr = fold_block(reg, r1a, r1b, s);
        reg = (k + 1 < cnt) ? nr : reg;
        r1a = ldg16(ENH_BLK(k + 5)); r1b = ldg16(ENH_BLK(k + 5) + 16);
        __builtin_amdgcn_sched_barrier(0);
        nr = fold_block(reg, r2a, r2b, s);
        reg = (k + 2 < cnt) ? nr : reg;
        r2a = ldg16(ENH_BLK(k + 6)); r2b = ldg16(ENH_BLK(k + 6) + 16);
        __builtin_amdgcn_sched_barrier(0);
        nr = fold_block(reg, r3a, r3b, s);
        reg = (k + 3 < cnt) ? nr : reg;
        r3a = ldg16(ENH_BLK(k + 7)); r3b = ldg16(ENH_BLK(k + 7) + 16);
        __builtin_amdgcn_sched_barrier(0);
    }
#undef ENH_BLK
    return reg;
}

}  // namespace enethip
