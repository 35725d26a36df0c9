// crc32_stream_common.hpp -- device pieces shared by the streamed CRC32 kernels
// (crc32_kernels.hip, crc32_lean.hip): kernel arguments, LDS-DMA and counted
// vmcnt helpers, the per-packet window / task of the strided-lane scheme, the
// head/tail/slot fix-ups and the end-of-packet finish.  Derivation: DESIGN.md 4,
// restated and checked against the oracle in tests/kernel_model.py.
// Reference: /root/reference/enet-csharp/ENet/c/packet.cs:142-160 (crc),
// c/protocol.cs:1052-1068 (receive verify).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "crc32_device.hpp"
#include "crc32_math.hpp"

namespace enethip {

struct PacketArgs {
    const uint8_t* bytes;
    const uint64_t* off;
    const uint32_t* len;
    uint64_t n;
    uint32_t lg;  // log2(lanes per packet)
    uint32_t* out;
    // verify mode
    const uint32_t* slot_off;
    const uint32_t* connect;
    uint8_t* ok;
    uint64_t* trace;  // diagnostics: per-wave timeline (enet_hip_diag_trace) or null
    uint32_t prio;    // lean kernel: raise the issue priority of lagging waves (tuning)
    // lean kernel: packet metadata pre-ordered by length bin, one record per packet
    // in the kernel's metadata field order -- MODE 0 {len, off_lo, off_hi, index},
    // MODE 1 {len, off_lo, off_hi, slot_off, connect, index, 0, 0} (the *_binned
    // entry points); out/ok[index] receive the results.  Null = read the arrays.
    const uint32_t* meta4;
};

__device__ __forceinline__ uint32_t lds_load(uint32_t addr) { return *reinterpret_cast<lds_u32*>(static_cast<uintptr_t>(addr)); }
__device__ __forceinline__ u32x4 lds_load16(uint32_t addr) { return *reinterpret_cast<lds_u32x4*>(static_cast<uintptr_t>(addr)); }
__device__ __forceinline__ void lds_store(uint32_t addr, uint32_t v) {
    *reinterpret_cast<__attribute__((address_space(3))) uint32_t*>(static_cast<uintptr_t>(addr)) = v;
}

// s_waitcnt vmcnt(min(n, 63)): the immediate picked by a balanced scalar
// branch tree (n is wave-uniform).
template <int Lo, int Hi>
__device__ __forceinline__ void wait_vm_tree(uint32_t n) {
    if constexpr (Lo == Hi) {
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(Lo) : "memory");
    } else {
        constexpr int Mid = (Lo + Hi) / 2;
        if (n <= static_cast<uint32_t>(Mid)) wait_vm_tree<Lo, Mid>(n);
        else wait_vm_tree<Mid + 1, Hi>(n);
    }
}
__device__ __forceinline__ void wait_vm(uint32_t n) { wait_vm_tree<0, 63>(__builtin_amdgcn_readfirstlane(n)); }

__device__ __forceinline__ void dma16(const void* g, uint32_t lds_addr) {
    __builtin_amdgcn_global_load_lds(g, reinterpret_cast<__attribute__((address_space(3))) void*>(
                                            static_cast<uintptr_t>(lds_addr)), 16, 0, 0);
}
// cache-policy variant (AUX = the instruction's cpol immediate: 2 = nt)
template <int AUX>
__device__ __forceinline__ void dma16_pol(const void* g, uint32_t lds_addr) {
    __builtin_amdgcn_global_load_lds(g, reinterpret_cast<__attribute__((address_space(3))) void*>(
                                            static_cast<uintptr_t>(lds_addr)), 16, 0, AUX);
}
__device__ __forceinline__ void dma4(const void* g, uint32_t lds_addr) {
    __builtin_amdgcn_global_load_lds(g, reinterpret_cast<__attribute__((address_space(3))) void*>(
                                            static_cast<uintptr_t>(lds_addr)), 4, 0, 0);
}

// One packet's window, seen from any lane.
struct Window {
    uint64_t ws;        // first window byte (16-byte aligned)
    uint32_t L, lz, nb, tz, r;
    bool active;
};

// Consumer side: this lane's task of the group.
struct Task {
    uint64_t pk;
    uint32_t k, w0, nb, lz, tz, cnt, reg;
    uint32_t e0, e1, e2, e3;   // block ordinals needing head/tail/slot fix-ups (~0u = none)
    bool active;
    int32_t ps;                // verify: window position of the slot
    uint32_t connect;
    bool slot_ok;
};

// First stage >= from holding a fix-up block of any lane (wave-uniform; ~0u =
// none); a stage is 2^LSB block ordinals.
template <uint32_t LSB>
__device__ __forceinline__ uint32_t next_edge_stage_l(const Task& t, uint32_t from) {
    uint32_t m = ~0u;
    const uint32_t e[4] = {t.e0, t.e1, t.e2, t.e3};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const uint32_t st = e[i] == ~0u ? ~0u : e[i] >> LSB;
        if (st >= from) m = min(m, st);
    }
    return wave_min_u(m);
}

// Keep bytes [lo, hi) of dword q (bytes 4q .. 4q+3 of the block).
__device__ __forceinline__ uint32_t keep_mask(int lo, int hi, int q) {
    const int a = lo - 4 * q, b = hi - 4 * q;
    const uint32_t ma = a <= 0 ? 0xFFFFFFFFu : a >= 4 ? 0u : (0xFFFFFFFFu << (8 * a));
    const uint32_t mb = b >= 4 ? 0xFFFFFFFFu : b <= 0 ? 0u : (0xFFFFFFFFu >> (32 - 8 * b));
    return ma & mb;
}

// Head/tail zeroing and (verify) slot substitution of block w, words in LANE
// order (A, B swapped when hs).
template <int MODE>
__device__ __forceinline__ void edge_fix(u32x4& A, u32x4& B, uint32_t hs, const Task& t, uint32_t w,
                                         uint32_t& desired) {
    uint32_t v[8];
    const bool sw = hs != 0;
    const u32x4 h0 = sw ? B : A, h1 = sw ? A : B;
    v[0] = h0.x; v[1] = h0.y; v[2] = h0.z; v[3] = h0.w;
    v[4] = h1.x; v[5] = h1.y; v[6] = h1.z; v[7] = h1.w;
    const int lo = (w == 0) ? static_cast<int>(t.lz) : 0;
    const int hi = (w + 1 == t.nb) ? 32 - static_cast<int>(t.tz) : 32;
#pragma unroll
    for (int q = 0; q < 8; ++q) v[q] &= keep_mask(lo, hi, q);
    if (MODE) {
        const int rel = t.ps - 32 * static_cast<int>(w);
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const int d = rel - 4 * q;
            if (d > -4 && d < 4) {
                uint32_t M, C;
                if (d >= 0) {
                    M = 0xFFFFFFFFu << (8 * d);
                    C = t.connect << (8 * d);
                    desired |= v[q] >> (8 * d);
                } else {
                    M = 0xFFFFFFFFu >> (-8 * d);
                    C = t.connect >> (-8 * d);
                    desired |= (v[q] & M) << (-8 * d);
                }
                v[q] = (v[q] & ~M) | (C & M);
            }
        }
    }
    const u32x4 n0 = {v[0], v[1], v[2], v[3]}, n1 = {v[4], v[5], v[6], v[7]};
    A = sw ? n1 : n0;
    B = sw ? n0 : n1;
}

// XOR of the P registers of each packet into its lane k == 0 (DPP tree inside a
// 16-lane row: lane k takes lane k + 2^l at level l).
template <int LVL>
__device__ __forceinline__ uint32_t xor_lanes(uint32_t lg, uint32_t v) {
    if constexpr (LVL < 4) {
        if (LVL < static_cast<int>(lg)) return xor_lanes<LVL + 1>(lg, v ^ dpp<kDppRowShl + (1 << LVL)>(v));
    }
    return v;
}

template <int I, int N, class F>
__device__ __forceinline__ void static_for(F&& f) {
    if constexpr (I < N) {
        f(std::integral_constant<int, I>{});
        static_for<I + 1, N>(f);
    }
}

// One zero byte undone: reg x^(-8) = (reg << 8) ^ U[reg >> 24] (U in free column
// kUnstepCol of the image, unstep_addr).  In asm with immediate constants: written
// in C++, hipcc hoisted the address constants into VGPRs and spilled one.
__device__ __forceinline__ uint32_t unstep_byte(uint32_t reg) {
    uint32_t t;
    static_assert(unstep_addr(0) == 0xe0u, "the U column's byte offset in a row");
    asm volatile("v_lshrrev_b32 %[t], 16, %[r]\n\t"
                 "v_and_b32 %[t], 0xff00, %[t]\n\t"
                 "v_or_b32 %[t], 0xe0, %[t]\n\t"
                 "ds_read_b32 %[t], %[t]\n\t"
                 "v_lshlrev_b32 %[r], 8, %[r]\n\t"
                 "s_waitcnt lgkmcnt(0)\n\t"
                 "v_xor_b32 %[r], %[r], %[t]"
                 : [r] "+v"(reg), [t] "=&v"(t) :: "memory");
    return reg;
}

// reg x^(-8 tz), tz < 32: tz zero-byte unsteps, straight-line by the bits of tz
// (the wave runs a block when any lane needs it; about 6 VALU per byte against ~160
// for a bit-serial multiply by CINV[tz])
__device__ __forceinline__ uint32_t unstep_bytes(uint32_t reg, uint32_t tz) {
    static_for<0, 5>([&](auto bc) __attribute__((always_inline)) {
        constexpr int bit = 4 - decltype(bc)::value;
        if (tz & (1u << bit)) {
#pragma unroll
            for (int j = 0; j < (1 << bit); ++j) reg = unstep_byte(reg);
        }
    });
    return reg;
}

// End of a group: lane k sits 32k + tz bytes past the data end.  Undo the 32k
// by x^(-256k) -- four byte-indexed lookups in the image's correction columns
// (each lane starts at a different byte so the lanes sharing k spread over four
// columns), XOR the P lanes, then undo tz (unaligned packet ends only).  Lane
// k == 0 of each packet returns the packet's register.
__device__ __forceinline__ uint32_t finish_packet(uint32_t lg, uint32_t k, uint32_t tz, uint32_t lane, uint32_t reg) {
    if ((1u << lg) <= kCorrLanes) {
        const uint32_t kk = k ? k : 1u;
        const uint32_t rot = (lane >> lg) & 3u;
        uint32_t x[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const uint32_t b = (static_cast<uint32_t>(i) + rot) & 3u;
            const uint32_t sel = 0x0C0C0000u | ((4u + b) << 8);      // byte1 = byte b of reg, byte0 = column
            x[i] = lds_load(__builtin_amdgcn_perm(reg, corr_col(kk, b), sel));
        }
        const uint32_t c = xor3(x[0], x[1], x[2]) ^ x[3];
        reg = k ? c : reg;
    } else {
        reg = mulmod(reg, lds_load(cinv_addr(32u * k)));
    }
    reg = xor_lanes<0>(lg, reg);
    if (k == 0) reg = unstep_bytes(reg, tz);                 // x^(-8 tz), tz < 16 here
    return reg;
}


template <int N, class F>
__device__ __forceinline__ void unroll_slots(F&& f) {
    if constexpr (N > 0) {
        unroll_slots<N - 1>(f);
        f(std::integral_constant<uint32_t, N - 1>{});
    }
}

}  // namespace enethip
