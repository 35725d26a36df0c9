// gather_join.hpp -- the per-DGRAM side of enet_hip_crc32_gather_binned_device
// (send-side gather lists, c/protocol.cs:1690-1698 per DGRAM; packet.cs:142-160 over
// the concatenated ENetBuffers).  Shared by crc32_kernels.hip (the one-pass join)
// and crc32_lean.hip (the pre-join that runs beside the length-binning tiles).
#pragma once
#include <hip/hip_runtime.h>

#include "crc32_device.hpp"
#include "crc32_math.hpp"

namespace enethip {

// Gather segments of at most this many bytes are folded by the per-DGRAM pass, not by
// the binned checksum pass (an ENet DGRAM's protocol header and command headers:
// 4-8 and 4-48 B)
constexpr uint32_t kGatherSmall = 48;

struct GatherArgs {
    const uint8_t* bytes;
    const uint64_t* seg_off;
    const uint32_t* seg_len;
    const uint32_t* seg_first;
    uint64_t n;
    uint32_t* out;
    uint64_t segs;      // segments with a CRC in seg_crc (the join's bound; the host's segCount)
};

// A short segment's 4-byte steps are slicing-by-4 on the dword v_alignbyte cuts at its
// offset, its last L mod 4 bytes Sarwate steps (T_3 .. T_0 = columns 6, 4, 2, 0 of the
// P = 1 image, 4 KiB in LDS).  Restated in tests/kernel_model.py (fold_small).
constexpr int kSmallDwords = (3 + static_cast<int>(kGatherSmall) + 3) / 4;
static_assert(15 + kGatherSmall <= 16 * ((kSmallDwords + 1 + 3) / 4), "a short segment's aligned lines fit the join's loads");

// p[i] as a GLOBAL load (a generic pointer makes hipcc emit a flat load)
template <class T>
__device__ __forceinline__ T gload(const T* p, uint64_t i) {
    return *reinterpret_cast<__attribute__((address_space(1))) const T*>(reinterpret_cast<uintptr_t>(p + i));
}

__device__ __forceinline__ void load_small(const uint8_t* a, uint32_t L, uint32_t (&d)[kSmallDwords + 1]) {
    const uint32_t sh = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(a)) & 3u;
    const uint32_t* w = reinterpret_cast<const uint32_t*>(reinterpret_cast<uintptr_t>(a) & ~static_cast<uintptr_t>(3));
    const uint32_t nd = (sh + L + 3u) >> 2;
    // global loads (through a generic pointer hipcc emits flat loads, counted in lgkmcnt
    // too: round 3's form, within noise of this one -- DESIGN.md 4.4)
#pragma unroll
    for (int k = 0; k < kSmallDwords; ++k) d[k] = static_cast<uint32_t>(k) < nd ? gload(w, k) : 0u;
    d[kSmallDwords] = 0u;
}

__device__ __forceinline__ uint32_t fold_small(uint32_t reg, uint32_t sh, uint32_t L,
                                               const uint32_t (&d)[kSmallDwords + 1], const uint32_t (*t4)[256]) {
    const uint32_t nf = L >> 2;
    uint32_t tail = 0;
#pragma unroll
    for (int i = 0; i < kSmallDwords - 1; ++i) {
        const uint32_t v = __builtin_amdgcn_alignbyte(d[i + 1], d[i], sh);
        if (static_cast<uint32_t>(i) < nf) {
            const uint32_t x = reg ^ v;
            reg = t4[3][x & 0xFFu] ^ t4[2][(x >> 8) & 0xFFu] ^ t4[1][(x >> 16) & 0xFFu] ^ t4[0][x >> 24];
        }
        tail = static_cast<uint32_t>(i) == nf ? v : tail;
    }
    for (uint32_t j = 0; j < (L & 3u); ++j) reg = t4[0][(reg ^ (tail >> (8u * j))) & 0xFFu] ^ (reg >> 8);
    return reg;
}

// The T_3 .. T_0 tables of fold_small, from the P = 1 image (columns 6, 4, 2, 0)
template <int NT>
__device__ __forceinline__ void fill_t4(uint32_t (*t4)[256], const uint32_t* image) {
    for (uint32_t i = threadIdx.x; i < 1024u; i += NT) t4[i >> 8][i & 255u] = image[64u * (i & 255u) + 2u * (i >> 8)];
    __syncthreads();
}

// ---------------------------------------------------------------- the split join
//
// The Sarwate register over a DGRAM is affine in every long segment's own register
// R_q = reg(0xFFFFFFFF, B_q) (what the records pass computes; seg_crc[q] =
// finalize(R_q)).  From reg = 0xFFFFFFFF, a long segment steps
// reg' = (reg ^ 0xFFFFFFFF) x^(8 L) ^ R_q and a short one reg' = fold(reg, B), both
// linear in reg plus a constant, so
//     reg(DGRAM) = A ^ XOR_q R_q x^(8 after_q),
// A = the same walk with every R_q = 0, after_q = the bytes of the segments after q.
// And finalize(A ^ c) = finalize(A) ^ bswap(c).  So:
//   * the pre-join (one thread per DGRAM, launched beside the length-binning tiles,
//     before the records pass) folds the short segments, writes out[d] = finalize(A)
//     and, for each long segment q, info[q] = {d, x^(8 after_q)};
//   * the post-join (one thread per segment, after the records pass) XORs
//     bswap(R_q x^(8 after_q)) into out[info[q].x] -- for the usual last long segment
//     (after = 0) that is ~seg_crc[q].
// segFirst must be non-decreasing (each segment in at most one DGRAM): then exactly
// the segments segFirst[0] <= q < segFirst[n] carry a fresh info entry.  Restated in
// tests/kernel_model.py (gather_split_join).
constexpr int kJoinQ = 4;                                  // segments in flight per thread

__device__ __forceinline__ void gather_prejoin_dgram(const GatherArgs& ga, uint2* info, const KernelTables& tb,
                                                     uint32_t small, uint64_t d, const uint32_t (*t4)[256]) {
    const uint32_t s1 = static_cast<uint32_t>(umin64(ga.seg_first[d + 1], ga.segs));
    const uint32_t s0 = min(ga.seg_first[d], s1);
    // the DGRAM's length first when its segments span more than one round of loads
    uint32_t total = 0;
    if (s1 - s0 > static_cast<uint32_t>(kJoinQ))
        for (uint32_t q = s0; q < s1; ++q) total += ga.seg_len[q];
    uint32_t reg = 0xFFFFFFFFu, pos = 0;
    for (uint32_t q0 = s0; q0 < s1; q0 += kJoinQ) {
        uint32_t L[kJoinQ];
        const uint8_t* A[kJoinQ];
#pragma unroll
        for (int i = 0; i < kJoinQ; ++i) {
            const bool in = q0 + i < s1;
            L[i] = in ? ga.seg_len[q0 + i] : 0u;
            A[i] = ga.bytes + (in ? ga.seg_off[q0 + i] : 0u);
        }
        if (s1 - s0 <= static_cast<uint32_t>(kJoinQ)) total = L[0] + L[1] + L[2] + L[3];
        uint32_t D[kJoinQ][kSmallDwords + 1], X[kJoinQ];
#pragma unroll
        for (int i = 0; i < kJoinQ; ++i) {
            if (L[i] != 0u && L[i] <= small) load_small(A[i], L[i], D[i]);
            else
#pragma unroll
                for (int k = 0; k <= kSmallDwords; ++k) D[i][k] = 0u;
            X[i] = L[i] > small ? tb.xn_lo[L[i] & 0xFFFFu] : 0u;
        }
#pragma unroll
        for (int i = 0; i < kJoinQ; ++i) {
            if (L[i] == 0u) continue;
            pos += L[i];
            if (L[i] <= small) {
                reg = fold_small(reg, static_cast<uint32_t>(reinterpret_cast<uintptr_t>(A[i])) & 3u, L[i], D[i], t4);
            } else {
                const uint32_t x = (L[i] >> 16) ? mulmod(X[i], tb.xn_hi[L[i] >> 16]) : X[i];
                reg = reg == 0xFFFFFFFFu ? 0u : mulmod(reg ^ 0xFFFFFFFFu, x);
                const uint32_t after = total - pos;
                info[q0 + i] = make_uint2(static_cast<uint32_t>(d), after ? x8n_dev(after, tb) : kOneReflected);
            }
        }
    }
    ga.out[d] = finalize(reg);
}

}  // namespace enethip
