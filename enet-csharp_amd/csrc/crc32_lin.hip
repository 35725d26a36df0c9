// crc32_lin.hip -- the linear-stream CRC32 kernel for gfx950 (MI355X), round 4.
// Path replaced: ENet.enet_crc32 (/root/reference/enet-csharp/ENet/c/packet.cs:
// 142-160) over a batch of DGRAMs, one CRC per packet (wire order, packet.cs:159).
//
// Why a second shape.  The VGPR-ring kernel (crc32_vring.hip) folds each packet with
// its own lanes, so every wave load instruction reads pieces of 8 packets, and a
// line two packed packets share is fetched by both: that load shape streams at about
// 5.9 TB/s even without the fold.  Here the HBM side is a plain
// linear stream: each wave owns a UNIT of 62 consecutive packets (sorted, not
// overlapping) and moves the unit's contiguous byte span, 8 KiB at a time, into its
// LDS tile by LDS-DMA -- every instruction one contiguous KiB of whole lines, every
// line read once -- while the fold works on the previous tile.
//
// Arithmetic (tests/kernel_model.py lin_unit, checked against the oracle on CPU):
//   * fold, packet-blind: lane c folds super-block c of the tile (128 bytes, 4 blocks
//     of 32) as one serial chain from a zero register, slicing-by-32 in the LDS image:
//     S[q] after q blocks, c = S[4].  The four states go to the wave's STATE area.
//   * boundary pass: a lane per packet start (and the unit's end) that is not on a
//     32-byte boundary folds its block with the bytes before the boundary zeroed:
//     Z = S[q+1] ^ hb = the prefix of the super-block up to the boundary, positioned
//     at the block's end (tb shifted by the 32 - m bytes after it).
//   * head H = c ^ Z x^(8 32 (3-q)) ^ INITS[128 - s'] = reg(~0, SB[s':128]);
//     Horner acc = acc x^(8 128) ^ c_X over the packet's full super-blocks (its lane
//     keeps acc across tiles); tail W = Y ^ acc x^(8 32 (q+1)), then x^(-8 tz) with
//     tz = the 32 - m bytes the block has past the packet end.  A packet inside one
//     super-block: W = Y ^ Z_s x^(8 32 (q_e - q_s)) ^ INITS[32 (q_e+1) - s'].
// Units that are not sorted and non-overlapping (or whose span is far longer than
// their bytes) take a per-lane direct fold from global memory instead (fold_window):
// every input gives the reference's CRCs.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <vector>

#include "context.hpp"
#include "crc32_lin.hpp"

namespace enethip {

constexpr int kLnW = 5;                                   // waves per workgroup, one workgroup per CU
constexpr uint32_t kLnSB = 128;                           // super-block: one lane's chain
constexpr uint32_t kLnTile = 64 * kLnSB;                  // 8 KiB: a wave's tile
constexpr uint32_t kLnRing = kLdsTableBytes;              // kLnW waves x 2 tile slots
constexpr uint32_t kLnState = kLnRing + kLnW * 2 * kLnTile;   // kLnW x 64 lanes x {S1, S2, S3, c}
constexpr uint32_t kLnCtr = kLnState + kLnW * 1024;       // the workgroup's unit counter
constexpr uint32_t kLnMetaBytes = 768;                    // a unit's metadata: 64 offsets | 64 lengths
constexpr uint32_t kLnMeta = kLnCtr + 16;                 // kLnW x 2 buffers
constexpr int kLnLds = kLnMeta + kLnW * 2 * kLnMetaBytes;
static_assert(kLnLds <= 160 * 1024, "LDS");

// Free columns of the lin image (free_col(c), 256 rows, byte-indexed): the
// multipliers M_k = x^(8 32 k) (k = 1..4, columns 4 (k-1) + b: entry v = (v << 8 b) M_k),
// the zero-byte divisors x^(-8 16), x^(-8 8), x^(-8 4) (columns 16 + 4 j + b), U (the
// one-zero-byte unstep, column 28), INITS[n] = ~0 through n zero bytes (column 29) and
// INIT[r], the register r zero bytes carry to ~0 (column 30: the direct-fold path).
constexpr uint32_t kLnMulCol = 0, kLnTzCol = 16, kLnUCol = 28, kLnInitCol = 29, kLnInitInvCol = 30;
static_assert(kLnUCol == kUnstepCol, "the U column of the vring images");

// ------------------------------------------------------------------ host: the image

int lin_image(uint32_t* img) {
    std::fill(img, img + kImageDwords, 0u);
    std::vector<uint32_t> row(256);
    for (uint32_t j = 0; j < 256; ++j) row[j] = crc_table_entry(j);
    for (uint32_t t = 0; t < 32; ++t) {                   // T_t[j] = byte j then t zero bytes
        for (uint32_t j = 0; j < 256; ++j) img[(j * 256 + col_byte(t)) / 4] = row[j];
        for (uint32_t j = 0; j < 256; ++j) row[j] = sarwate_step(row[j], 0);
    }
    // x^-8 = x^-1 to the 8th: from x * x^-1 = 1
    uint32_t xinv = 1u;                                   // x^32 / x = x^31
    for (int i = 1; i < 32; ++i)
        if ((kPoly >> (31 - i)) & 1u) xinv |= 1u << (31 - (i - 1));
    uint32_t xinv8 = kOneReflected;
    for (int i = 0; i < 8; ++i) xinv8 = gf2_mulmod(xinv8, xinv);
    auto xinv_bytes = [&](int n) {
        uint32_t r = kOneReflected;
        for (int i = 0; i < n; ++i) r = gf2_mulmod(r, xinv8);
        return r;
    };
    if (gf2_mulmod(xinv_bytes(1), x8n_modp(1)) != kOneReflected) return -1;
    const uint32_t mul[4] = {x8n_modp(32), x8n_modp(64), x8n_modp(96), x8n_modp(128)};
    const uint32_t div[3] = {xinv_bytes(16), xinv_bytes(8), xinv_bytes(4)};
    for (uint32_t v = 0; v < 256; ++v) {
        for (uint32_t b = 0; b < 4; ++b) {
            for (uint32_t k = 0; k < 4; ++k)
                img[(256u * v + free_col(kLnMulCol + 4u * k + b)) / 4] = gf2_mulmod(v << (8 * b), mul[k]);
            for (uint32_t k = 0; k < 3; ++k)
                img[(256u * v + free_col(kLnTzCol + 4u * k + b)) / 4] = gf2_mulmod(v << (8 * b), div[k]);
        }
        const uint32_t t = crc_table_entry(v);            // U: reg x^(-8) = (reg << 8) ^ U[reg >> 24]
        img[(256u * (t >> 24) + free_col(kLnUCol)) / 4] = (t << 8) | v;
    }
    uint32_t init = 0xFFFFFFFFu, inv = 0xFFFFFFFFu;
    for (uint32_t n = 0; n < 256; ++n) {
        img[(256u * n + free_col(kLnInitCol)) / 4] = init;
        img[(256u * n + free_col(kLnInitInvCol)) / 4] = inv;
        init = sarwate_step(init, 0);
        inv = unstep_zero(inv);
    }
    return 0;
}

// ------------------------------------------------------------------ device helpers

// Tile and image DMA as inline asm: the compiler must not see them (as
// __builtin_amdgcn_global_load_lds it would wait vmcnt(0) before every LDS read that
// might alias the target); they are waited for by explicit counted vmcnt instead.
// M0 = the instruction's LDS base; lane l's 16 bytes land at M0 + 16 l.
template <int NT>
__device__ __forceinline__ void ln_dma16(uint64_t g, uint32_t lds_any) {
    const uint32_t lds = __builtin_amdgcn_readfirstlane(lds_any);   // (wave-uniform: an SGPR)
    if constexpr (NT)
        asm volatile("s_mov_b32 m0, %1\n\tglobal_load_lds_dwordx4 %0, off nt" :: "v"(g), "s"(lds) : "m0", "memory");
    else
        asm volatile("s_mov_b32 m0, %1\n\tglobal_load_lds_dwordx4 %0, off" :: "v"(g), "s"(lds) : "m0", "memory");
}
__device__ __forceinline__ void ln_dma4(uint64_t g, uint32_t lds_any) {
    const uint32_t lds = __builtin_amdgcn_readfirstlane(lds_any);
    asm volatile("s_mov_b32 m0, %1\n\tglobal_load_lds_dword %0, off" :: "v"(g), "s"(lds) : "m0", "memory");
}
template <int N>
__device__ __forceinline__ void ln_wait() {
    asm volatile("s_waitcnt vmcnt(%0)" :: "n"(N) : "memory");
}

// XOR of the four byte-indexed lookups of v in free columns c0 .. c0 + 3 (c0 < 16 or
// >= 16 per block of four): v times the columns' constant.  colw = the four column
// bytes free_col(c0 + b) in bytes b (lane-varying allowed).
__device__ __forceinline__ uint32_t ln_tab4(uint32_t v, uint32_t colw) {
    const uint32_t x0 = lds_load(__builtin_amdgcn_perm(v, colw, 0x0C0C0400u));
    const uint32_t x1 = lds_load(__builtin_amdgcn_perm(v, colw, 0x0C0C0501u));
    const uint32_t x2 = lds_load(__builtin_amdgcn_perm(v, colw, 0x0C0C0602u));
    const uint32_t x3 = lds_load(__builtin_amdgcn_perm(v, colw, 0x0C0C0703u));
    return xor3(x0, x1, x2) ^ x3;
}
__host__ __device__ constexpr uint32_t ln_colw(uint32_t c0) {
    return free_col(c0) | (free_col(c0 + 1) << 8) | (free_col(c0 + 2) << 16) | (free_col(c0 + 3) << 24);
}
// v x^(8 32 k), k = 0..4 per lane
__device__ __forceinline__ uint32_t ln_mulx(uint32_t v, uint32_t k) {
    // columns 4 (k-1) + b < 16: free_col = 8 (4 (k-1) + b) + 4 = 32 (k-1) + 8 b + 4
    const uint32_t colw = 0x1C140C04u + 0x20202020u * (k ? k - 1u : 0u);
    const uint32_t r = ln_tab4(v, colw);
    return k ? r : v;
}
// v x^(-8 tz), tz < 32 per lane: 16, 8, 4 by tables, 2 and 1 by unsteps
__device__ __forceinline__ uint32_t ln_unshift(uint32_t v, uint32_t tz) {
    if (__builtin_amdgcn_ballot_w64((tz & 16u) != 0u)) {
        const uint32_t r = ln_tab4(v, ln_colw(kLnTzCol));
        v = (tz & 16u) ? r : v;
    }
    if (__builtin_amdgcn_ballot_w64((tz & 8u) != 0u)) {
        const uint32_t r = ln_tab4(v, ln_colw(kLnTzCol + 4));
        v = (tz & 8u) ? r : v;
    }
    if (__builtin_amdgcn_ballot_w64((tz & 4u) != 0u)) {
        const uint32_t r = ln_tab4(v, ln_colw(kLnTzCol + 8));
        v = (tz & 4u) ? r : v;
    }
#pragma unroll
    for (uint32_t bit = 2; bit >= 1; bit >>= 1) {
        if (__builtin_amdgcn_ballot_w64((tz & bit) != 0u)) {
#pragma unroll
            for (uint32_t s = 0; s < bit; ++s) {
                const uint32_t r = (v << 8) ^ lds_load(256u * (v >> 24) + free_col(kLnUCol));
                v = (tz & bit) ? r : v;
            }
        }
    }
    return v;
}
__device__ __forceinline__ uint32_t ln_inits(uint32_t n) { return lds_load(256u * n + free_col(kLnInitCol)); }

// One 32-byte block: the 8 dwords in this lane's Latin-square order (register g =
// dword g ^ lx) from LDS at `base` (32-byte aligned + 4 lx: dword g ^ lx lands at
// base ^ 4 g), the register injected into dword 0 (register lx), 32 lookups.
template <int ABL>
__device__ __forceinline__ uint32_t ln_fold(uint32_t reg, uint32_t base, const LaneSched& s, const uint32_t (&inj)[8]) {
    uint32_t d[8];
#pragma unroll
    for (int g = 0; g < 8; ++g) d[g] = lds_load(base ^ (4u * g));
#pragma unroll
    for (int g = 0; g < 8; ++g) d[g] = __builtin_amdgcn_bitop3_b32(d[g], reg, inj[g], 0x78);   // d ^ (reg & inj)
    if constexpr (ABL & 2) {
        return xor3(xor3(d[0], d[1], d[2]), xor3(d[3], d[4], d[5]), d[6] ^ d[7]);
    }
    uint32_t v[32];
#pragma unroll
    for (int i = 0; i < 32; ++i) v[i] = lds_load(__builtin_amdgcn_perm(d[i >> 2], s.col[i >> 2], s.sel[i & 3]));
    uint32_t acc = xor3(v[0], v[1], v[2]);
#pragma unroll
    for (int i = 3; i + 1 < 32; i += 2) acc = xor3(acc, v[i], v[i + 1]);
    return acc ^ v[31];
}
// The same block with bytes < m zeroed and no register: hb = reg(0, block[m:32]).
__device__ __forceinline__ uint32_t ln_suffix(uint32_t base, uint32_t lx, uint32_t m, const LaneSched& s) {
    uint32_t d[8];
#pragma unroll
    for (int g = 0; g < 8; ++g) {
        const uint32_t D = static_cast<uint32_t>(g) ^ lx;
        const int a = static_cast<int>(m) - 4 * static_cast<int>(D);            // bytes of dword D below m
        const uint32_t keep = a <= 0 ? 0xFFFFFFFFu : a >= 4 ? 0u : (0xFFFFFFFFu << (8 * a));
        d[g] = lds_load(base ^ (4u * g)) & keep;
    }
    uint32_t v[32];
#pragma unroll
    for (int i = 0; i < 32; ++i) v[i] = lds_load(__builtin_amdgcn_perm(d[i >> 2], s.col[i >> 2], s.sel[i & 3]));
    uint32_t acc = xor3(v[0], v[1], v[2]);
#pragma unroll
    for (int i = 3; i + 1 < 32; i += 2) acc = xor3(acc, v[i], v[i + 1]);
    return acc ^ v[31];
}


// ------------------------------------------------------------------ the kernel
// ABL (diagnostics, wrong CRCs by design): bit 0 = no boundary / join passes; bit 1 =
// no fold lookups.  NT = nontemporal tile DMA.
template <int ABL, int NT>
__global__ void __launch_bounds__(64 * kLnW) crc32_lin_kernel(VrBatches bl, const uint32_t* image, const uint8_t* zero) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t zaddr = reinterpret_cast<uint64_t>(zero);

    // ---- prologue: the image (64 x 1 KiB DMA over the waves), the unit counter
    for (uint32_t i = wave; i < 64u; i += kLnW)
        ln_dma16<0>(reinterpret_cast<uint64_t>(image) + 1024u * i + 16u * lane, 1024u * i);
    if (threadIdx.x == 0u) lds_store(kLnCtr, 0u);
    ln_wait<0>();
    __syncthreads();

    // the workgroup's units: [u_lo, u_hi) of the launch's concatenated unit space,
    // taken by its waves in turn from the LDS counter
    const uint64_t U = bl.groups;
    const uint64_t u_lo = U * blockIdx.x / gridDim.x, u_hi = U * (blockIdx.x + 1u) / gridDim.x;
    auto take = [&]() __attribute__((always_inline)) -> uint64_t {
        uint32_t sl = 0;
        if (lane == 0u)
            asm volatile("v_mov_b32 %0, 1\n\t"
                         "ds_add_rtn_u32 %0, %1, %0\n\t"
                         "s_waitcnt lgkmcnt(0)"
                         : "=&v"(sl) : "v"(kLnCtr) : "memory");
        sl = __builtin_amdgcn_readfirstlane(sl);
        return u_lo + sl;                                 // >= u_hi: none left
    };
    // a batch's descriptor by a wave-uniform index: scalar loads from the kernel
    // arguments (a vector load would be waited for with the tile DMAs in flight)
    auto batch = [&](uint32_t b) __attribute__((always_inline)) -> VrBatch {
        return bl.b[__builtin_amdgcn_readfirstlane(b)];
    };
    auto locate = [&](uint32_t b, uint64_t u) __attribute__((always_inline)) -> uint32_t {
        while (b + 1u < bl.count && u >= bl.b[__builtin_amdgcn_readfirstlane(b + 1u)].g0) ++b;
        return __builtin_amdgcn_readfirstlane(b);
    };

    // lane constants of the fold: Latin square (register g = dword g ^ lx), the
    // register's injection masks
    const LaneSched sch = make_sched(lane);
    const uint32_t lx = (lane >> 2) & 7u;
    uint32_t inj[8];
#pragma unroll
    for (int g = 0; g < 8; ++g) inj[g] = (static_cast<uint32_t>(g) == lx) ? 0xFFFFFFFFu : 0u;
    // DMA: instruction i of a tile, lane l -> super-block 8 i + (l >> 3), piece
    // (l & 7) ^ 2 ((l >> 3) & 3) of it; i.e. tile byte 1024 i + dofs (whole lines);
    // super-block X's block q then sits at slot byte 128 X + 32 (q ^ (X & 3)), so the
    // fold's dword reads (lane c: 8 (q ^ (c & 3)) + (g ^ lx) mod 32) hit 32 banks
    const uint32_t dofs = 128u * (lane >> 3) + 16u * ((lane & 7u) ^ (2u * ((lane >> 3) & 3u)));
    const uint32_t slot0 = kLnRing + 2u * kLnTile * wave;
    const uint32_t stbase = kLnState + 1024u * wave;
    const uint32_t mbase = kLnMeta + 2u * kLnMetaBytes * wave;
    auto sb_block = [](uint32_t X, uint32_t q) __attribute__((always_inline)) -> uint32_t {
        return 128u * X + 32u * (q ^ (X & 3u));
    };

    // ---- units: lane i = packet i (i < np), lane np = the unit's end boundary
    struct Unit {
        uint32_t b;                  // batch
        uint64_t p0;                 // first packet
        uint32_t np;
        uint64_t A, lo16, E;         // absolute: tile 0's line, first piece's, the span's end
        uint32_t ntiles;
        bool fast;
    };
    // the unit's metadata into meta buffer mb by LDS-DMA: offsets as 128 dwords (two
    // instructions), lengths (one); packet indices clamped to the batch
    auto issue_meta = [&](uint32_t b, uint64_t u, uint32_t mb) __attribute__((always_inline)) {
        const VrBatch B = batch(b);
        const uint64_t p0 = (u - B.g0) * kLnPk, pl = B.n - 1u;
        const uint64_t oa = reinterpret_cast<uint64_t>(B.off), la = reinterpret_cast<uint64_t>(B.len);
        const uint64_t q0 = umin64(p0 + (lane >> 1), pl), q1 = umin64(p0 + 32u + (lane >> 1), pl);
        ln_dma4(oa + 8u * q0 + 4u * (lane & 1u), mb);
        ln_dma4(oa + 8u * q1 + 4u * (lane & 1u), mb + 256u);
        ln_dma4(la + 4u * umin64(p0 + lane, pl), mb + 512u);
    };
    // the unit from its landed metadata: span, tiles, fast or not, lane values
    auto describe = [&](uint32_t b, uint64_t u, uint32_t mb, Unit& un, uint32_t& sr, uint32_t& er,
                        uint32_t& L) __attribute__((always_inline)) {
        const VrBatch B = batch(b);
        un.b = b;
        un.p0 = (u - B.g0) * kLnPk;
        un.np = static_cast<uint32_t>(umin64(kLnPk, B.n - un.p0));
        const uint32_t np = un.np;
        const uint32_t li = min(lane, np - 1u);
        const uint64_t off = static_cast<uint64_t>(lds_load(mb + 8u * li)) |
                             (static_cast<uint64_t>(lds_load(mb + 8u * li + 4u)) << 32);
        const uint32_t len = lds_load(mb + 512u + 4u * li);
        const bool real = lane < np;
        const uint64_t e64 = off + len;
        const uint64_t prev_e = __shfl_up(static_cast<unsigned long long>(e64), 1);
        const uint64_t s64 = real ? off : prev_e;         // lane np: the last packet's end
        L = real ? len : 0u;
        // sorted, not overlapping: e_{i-1} <= s_i
        const bool bad = lane > 0u && lane < np && prev_e > off;
        const bool sorted = __builtin_amdgcn_ballot_w64(bad) == 0ull;
        const uint64_t big = ~0ull;
        uint64_t lo = (real && len) ? s64 : big, hi = (real && len) ? e64 : 0u, tot = real ? len : 0u;
#pragma unroll
        for (int m = 32; m >= 1; m >>= 1) {
            lo = min(lo, static_cast<uint64_t>(__shfl_xor(static_cast<unsigned long long>(lo), m)));
            hi = max(hi, static_cast<uint64_t>(__shfl_xor(static_cast<unsigned long long>(hi), m)));
            tot += static_cast<uint64_t>(__shfl_xor(static_cast<unsigned long long>(tot), m));
        }
        lo = __builtin_amdgcn_readfirstlane(lo);
        hi = __builtin_amdgcn_readfirstlane(hi);
        tot = __builtin_amdgcn_readfirstlane(tot);
        const uint64_t base = reinterpret_cast<uint64_t>(B.bytes);
        sr = er = 0;
        if (lo == big) {                                  // no live packet: no tiles
            un.A = un.lo16 = un.E = 0;
            un.ntiles = 0;
            un.fast = true;
            return;
        }
        un.A = (base + lo) & ~127ull;
        un.lo16 = (base + lo) & ~15ull;
        un.E = base + hi;
        const uint64_t span = un.E - un.A;
        un.fast = sorted && span <= 2u * tot + 8192u && span < (1ull << 31);
        un.ntiles = un.fast ? static_cast<uint32_t>((span + kLnTile - 1u) / kLnTile) : 0u;
        if (un.fast) {
            sr = static_cast<uint32_t>(base + s64 - un.A);
            er = sr + L;
        }
    };
    // tile DMA: tile k of a unit into slot s (pieces wholly outside the unit's
    // packets come from the zero page)
    auto issue_tile = [&](const Unit& x, uint32_t k, uint32_t s) __attribute__((always_inline)) {
        const uint64_t t0 = x.A + static_cast<uint64_t>(kLnTile) * k + dofs;
#pragma unroll
        for (uint32_t i = 0; i < 8u; ++i) {
            const uint64_t g = t0 + 1024u * i;
            const uint64_t src = (g < x.lo16 || g >= x.E) ? zaddr : g;
            ln_dma16<NT>(src, slot0 + kLnTile * s + 1024u * i);
        }
    };
    // results of a finished unit: stored after the next counted wait (a store issued
    // just before one would be waited for with the tile)
    uint32_t pend_val = 0;
    uint64_t pend_ptr = 0;
    bool pend_on = false;
    auto flush = [&]() __attribute__((always_inline)) {
        if (pend_on) *reinterpret_cast<__attribute__((address_space(1))) uint32_t*>(pend_ptr) = pend_val;   // (global_store: in order)
        pend_on = false;
    };

    uint64_t cu = take();
    if (cu >= u_hi) return;                               // (no DMA outstanding)
    uint32_t cb = locate(0u, cu);
    uint32_t mbuf = 0;                                    // the current unit's meta buffer
    issue_meta(cb, cu, mbase);
    ln_wait<0>();
    Unit un;
    uint32_t sr, er, L;
    describe(cb, cu, mbase, un, sr, er, L);
    uint64_t nu = take();                                 // the next unit
    bool nhave = nu < u_hi;
    uint32_t nb = nhave ? locate(cb, nu) : cb;
    bool nmeta = false;                                   // its metadata issued
    uint32_t acc = 0, res = 0, slot = 0, k = 0;
    if (un.fast && un.ntiles) issue_tile(un, 0u, 0u);

    for (;;) {
        const uint32_t nmb = mbase + kLnMetaBytes * (mbuf ^ 1u);
        // ---------------- a unit with no tiles: per-lane direct folds (not sorted, or a
        // span far longer than its bytes), or all packets empty
        if (!(un.fast && un.ntiles)) {
            ln_wait<0>();
            flush();
            if (lane < un.np) {
                const VrBatch B = batch(un.b);
                uint32_t r = 0u;
                if (!un.fast) {
                    // fold_window reads an end-aligned window: rp = 32 nb - L zero bytes in
                    // front, so it starts from INIT[rp], the register they carry to ~0
                    const uint64_t i = un.p0 + lane;
                    const uint32_t Lp = B.len[i];
                    const uint32_t rp = ((Lp + 31u) & ~31u) - Lp;
                    r = finalize(fold_window(lds_load(256u * rp + free_col(kLnInitInvCol)), B.bytes + B.off[i], Lp, sch, zero));
                }
                B.out[un.p0 + lane] = r;                  // (empty packets: finalize(~0) = 0)
            }
            if (!nhave) break;
            if (!nmeta) issue_meta(nb, nu, nmb);
            ln_wait<0>();
            describe(nb, nu, nmb, un, sr, er, L);
            cb = nb;
            mbuf ^= 1u;
            nu = take();
            nhave = nu < u_hi;
            nb = nhave ? locate(cb, nu) : cb;
            nmeta = false;
            acc = res = k = slot = 0;
            if (un.fast && un.ntiles) issue_tile(un, 0u, 0u);
            continue;
        }

        // ---------------- tile k of a fast unit: the next tile's DMA, then this tile's wait
        const bool last = k + 1u == un.ntiles;
        bool nxt = false;                                 // a next tile was issued
        Unit nun;
        uint32_t nsr = 0, ner = 0, nL = 0;
        if (!last) {
            issue_tile(un, k + 1u, slot ^ 1u);
            nxt = true;
        } else if (nhave) {
            // the next unit's first tile: its metadata issued at this unit's first tile
            // (older than this tile's DMA) or now
            if (nmeta) {
                ln_wait<8>();
            } else {
                issue_meta(nb, nu, nmb);
                ln_wait<0>();
            }
            describe(nb, nu, nmb, nun, nsr, ner, nL);
            if (nun.fast && nun.ntiles) {
                issue_tile(nun, 0u, slot ^ 1u);
                nxt = true;
            }
        }
        const bool meta_now = k == 0u && !last && nhave && !nmeta;
        if (meta_now) {
            issue_meta(nb, nu, nmb);
            nmeta = true;
            ln_wait<11>();                                // this tile: all but the next tile + metadata
        } else if (nxt) {
            ln_wait<8>();
        } else {
            ln_wait<0>();
        }
        flush();

        // ---------------- fold: lane c = super-block c of the tile
        const uint32_t sbase = slot0 + kLnTile * slot;
        {
            const uint32_t cq = lane & 3u;
            uint32_t S = 0, st[4];
#pragma unroll
            for (uint32_t q = 0; q < 4u; ++q) {
                S = ln_fold<ABL>(S, sbase + 128u * lane + 32u * (q ^ cq) + 4u * lx, sch, inj);
                st[q] = S;
            }
            *reinterpret_cast<__attribute__((address_space(3))) u32x4*>(static_cast<uintptr_t>(stbase + 16u * lane)) =
                u32x4{st[0], st[1], st[2], st[3]};
        }

        if constexpr (!(ABL & 1)) {
            const uint32_t t_lo = kLnTile * k, t_hi = t_lo + kLnTile;
            // S[q] of tile super-block X, q = 0..4 (S[0] = 0)
            auto S_of = [&](uint32_t X, uint32_t q) __attribute__((always_inline)) -> uint32_t {
                const uint32_t v = lds_load(stbase + 16u * (X & 63u) + 4u * (q ? q - 1u : 0u));   // (X & 63: idle lanes)
                return q ? v : 0u;
            };
            // boundary pass at region offset b (in this tile, b & 31 != 0):
            // Z = S[q+1] ^ reg(0, block[m:32]) = the super-block's prefix to b, at the block end
            auto zpass = [&](uint32_t b) __attribute__((always_inline)) -> uint32_t {
                const uint32_t X = (b - t_lo) >> 7, q = (b >> 5) & 3u, m = b & 31u;
                const uint32_t hb = ln_suffix(sbase + sb_block(X, q) + 4u * lx, lx, m, sch);
                return S_of(X, q + 1u) ^ hb;
            };
            // pass 1: every lane's start (lane np: the unit's end) off a 32-byte boundary
            const bool live = lane <= un.np;
            const bool p1 = live && sr >= t_lo && sr < t_hi && (sr & 31u) != 0u;
            uint32_t Z = 0;
            if (__builtin_amdgcn_ballot_w64(p1)) {
                const uint32_t z = zpass(p1 ? sr : t_lo + 1u);
                Z = p1 ? z : 0u;
            }
            // the next lane's start: this packet's end when the two are one boundary
            const uint32_t Zn = __shfl_down(Z, 1);
            const uint32_t srn = __shfl_down(sr, 1);
            const bool pk = lane < un.np && L != 0u;
            const bool tail = pk && er - 1u >= t_lo && er - 1u < t_hi;
            const bool head = pk && sr >= t_lo && sr < t_hi;
            // pass 2 (gaps): an end off a 32-byte boundary that is not the next start
            uint32_t Y2 = 0;
            const bool p2 = tail && (er & 31u) != 0u && srn != er;
            if (__builtin_amdgcn_ballot_w64(p2)) {
                const uint32_t z = zpass(p2 ? er : t_lo + 1u);
                Y2 = p2 ? z : 0u;
            }
            // heads: H = c ^ Zs x^(8 32 (3 - q)) ^ INITS[128 - s'] (acc at the super-block's
            // end); the start's prefix value: off a block boundary Z, on one S[qs] with
            // one block more (S[0] = 0)
            const uint32_t Xs = (sr - t_lo) >> 7, sp = sr & 127u, qs = sp >> 5, ms = sp & 31u;
            uint32_t Zs = 0, ds = 0;
            if (head) {
                Zs = ms ? Z : S_of(Xs, qs);
                ds = ms ? 0u : 1u;
            }
            // tails: the end's super-block, offset e' in [1, 128], q_e, m_e in [1, 32]
            const uint32_t Xe = ((er - 1u) - t_lo) >> 7;
            const uint32_t ep = er - 128u * ((er - 1u) >> 7);
            const uint32_t qe = (ep - 1u) >> 5, me = ep - 32u * qe;
            const bool same = head && tail && Xs == Xe;
            if (__builtin_amdgcn_ballot_w64(head && !same)) {
                const uint32_t h = S_of(head ? Xs : 0u, 4u) ^ ln_mulx(Zs, 3u - qs + ds) ^ ln_inits(128u - (head ? sp : 0u));
                acc = (head && !same) ? h : acc;
            }
            // Horner over the packet's full super-blocks in this tile, [hs, he]
            uint32_t hs = 64u, he = 0u;
            if (pk && !same && sr < t_hi && er > t_lo) {
                hs = head ? Xs + 1u : 0u;
                he = tail ? (ep == 128u ? Xe + 1u : Xe) : 64u;   // (exclusive)
            }
            // each lane walks its own range (the wave's trip count is the longest range,
            // not the union of the ranges: that is the whole tile at every tile)
            const uint32_t cnt = hs < he ? he - hs : 0u;
            const uint32_t trips = wave_max_u(cnt);
            for (uint32_t t = 0; t < trips; ++t) {
                const uint32_t j = min(hs + t, 63u);
                const uint32_t c = lds_load(stbase + 16u * j + 12u);
                const uint32_t r = ln_tab4(acc, ln_colw(kLnMulCol + 12u)) ^ c;
                acc = t < cnt ? r : acc;
            }
            // tails: W = Y ^ acc x^(8 32 (q_e + 1)) (one super-block: Y ^ Zs x^(8 32 (q_e - q_s))
            // ^ INITS[32 (q_e + 1) - s']), then x^(-8 (32 - m_e))
            if (__builtin_amdgcn_ballot_w64(tail)) {
                const bool mid = tail && ep != 128u;
                const uint32_t Y = me == 32u ? S_of(mid ? Xe : 0u, qe + 1u) : (srn == er ? Zn : Y2);
                const uint32_t W1 = Y ^ ln_mulx(Zs, qe - qs + ds) ^ ln_inits(32u * (qe + 1u) - (same ? sp : 0u));
                const uint32_t W2 = Y ^ ln_mulx(acc, qe + 1u);
                const uint32_t W = same ? W1 : W2;
                const uint32_t st_mid = ln_unshift(mid ? W : 0u, mid ? 32u - me : 0u);
                // ending on a super-block end: acc (Horner took the super-block), or the
                // head of a packet inside one super-block
                const uint32_t st_end = same ? (S_of(Xs, 4u) ^ ln_mulx(Zs, 3u - qs + ds) ^ ln_inits(128u - sp)) : acc;
                if (tail) res = finalize(mid ? st_mid : st_end);
            }
        } else {
            res = lds_load(stbase + 16u * lane + 12u);    // (ablation: the fold alone)
        }

        // ---------------- advance
        if (!last) {
            ++k;
            slot ^= 1u;
            continue;
        }
        // the unit is done: its results go out after the next counted wait
        if (lane < un.np) {
            pend_val = L ? res : 0u;
            pend_ptr = reinterpret_cast<uint64_t>(batch(un.b).out + un.p0 + lane);
            pend_on = true;
        }
        if (!nhave) break;
        cb = nb;
        mbuf ^= 1u;
        un = nun;
        sr = nsr;
        er = ner;
        L = nL;
        nu = take();
        nhave = nu < u_hi;
        nb = nhave ? locate(cb, nu) : cb;
        nmeta = false;
        acc = res = k = 0;
        slot ^= 1u;
        if (!nxt) {                                       // (the next unit has no tiles)
            ln_wait<0>();
            flush();
            slot = 0;
        }
    }
    ln_wait<0>();
    flush();
    ln_wait<0>();
}

// ------------------------------------------------------------------ host

namespace {
template <int ABL, int NT>
int ln_set() {
    return herr(hipFuncSetAttribute(reinterpret_cast<const void*>(crc32_lin_kernel<ABL, NT>),
                                    hipFuncAttributeMaxDynamicSharedMemorySize, kLnLds));
}
}  // namespace

// The linear kernel is a diagnostics-library path (kernel paths 22 / 23; DESIGN.md
// 6.0e): correct on every input, slower than the VGPR-ring kernel, so the product
// library builds no instance of it.
int lin_setup() {
    int rc = 0;
#ifdef ENET_HIP_DIAG
    rc = ln_set<0, 1>();
    if (!rc) rc = ln_set<0, 0>();
    if (!rc) rc = ln_set<1, 1>();
    if (!rc) rc = ln_set<3, 1>();
#endif
    return rc;
}

int lin_launch_list(int max_wgs, hipStream_t st, const VrBatches& bl, const uint32_t* image, const uint8_t* zero,
                    int abl, bool nt) {
    if (bl.count > static_cast<uint32_t>(kVrMaxBatches)) return -static_cast<int>(hipErrorInvalidValue);
    VrBatches a{};
    a.count = 0;
    uint64_t U = 0;
    for (uint32_t i = 0; i < bl.count; ++i) {
        if (bl.b[i].n == 0) continue;                     // (no units)
        a.b[a.count] = bl.b[i];
        a.b[a.count].g0 = U;
        U += (bl.b[i].n + kLnPk - 1u) / kLnPk;
        ++a.count;
    }
    if (U == 0) return 0;
    a.groups = U;
    const unsigned grid = static_cast<unsigned>(std::min<uint64_t>(static_cast<uint64_t>(max_wgs), (U + kLnW - 1) / kLnW));
    const void* fn = nullptr;
#ifdef ENET_HIP_DIAG
    if (abl == 0) fn = nt ? reinterpret_cast<const void*>(crc32_lin_kernel<0, 1>)
                          : reinterpret_cast<const void*>(crc32_lin_kernel<0, 0>);
    else if (abl == 1) fn = reinterpret_cast<const void*>(crc32_lin_kernel<1, 1>);
    else if (abl == 3) fn = reinterpret_cast<const void*>(crc32_lin_kernel<3, 1>);
#else
    (void)abl;
    (void)nt;
#endif
    if (!fn) return -static_cast<int>(hipErrorInvalidValue);
    void* args[] = {&a, const_cast<uint32_t**>(&image), const_cast<uint8_t**>(&zero)};
    return herr(hipLaunchKernel(fn, dim3(grid), dim3(64 * kLnW), args, kLnLds, st));
}

}  // namespace enethip
