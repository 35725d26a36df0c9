// ringprobe.hip -- measurement only: the loader-wave shape for the
// cfg2 checksum.  One workgroup per CU: F folder waves + ONE loader wave.  The loader
// moves every folder's next stage into an LDS ring by LDS-DMA (global_load_lds_dwordx4,
// per-lane source addresses), keeps D-1 rounds in flight and publishes a round with
// one s_barrier; the folders fold from the ring.  A folder owns a group of 64 packets,
// ONE LANE PER PACKET (P = 1): a stage is SB 32-byte blocks of each packet's window,
// so the per-packet work (head mask, INIT, tail mask, tz correction) is paid once per
// lane per packet instead of once per lane per 150 bytes as at 8 lanes per packet.
// Path replaced: ENet.enet_crc32, /root/reference/enet-csharp/ENet/c/packet.cs:142-160.
//
// Modes: 0 = folders only pass the barriers (the DMA + handshake alone), 1 = skeleton
// (the folders read every data dword of the ring and XOR them), 2 = the real fold
// (slicing-by-32 in the conflict-free 64 KiB image, head/tail masks, INIT, tz), whose
// CRCs are checked against a CPU Sarwate loop.
//   hipcc --offload-arch=gfx950 -O3 -I enet-csharp_amd/csrc -o tools/ringprobe tools/ringprobe.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "crc32_device.hpp"
#include "crc32_math.hpp"

using namespace enethip;

#define HC(x)                                                                    \
    do {                                                                         \
        hipError_t e_ = (x);                                                     \
        if (e_ != hipSuccess) {                                                  \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(2);                                                             \
        }                                                                        \
    } while (0)

constexpr uint32_t kRing = kLdsTableBytes;

template <int N>
__device__ __forceinline__ void wait_vm() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
__device__ __forceinline__ void barrier_raw() { asm volatile("s_barrier" ::: "memory"); }

template <int NT>
__device__ __forceinline__ void dma16(uint32_t voff, uint64_t sbase, uint32_t m0) {
    if constexpr (NT)
        asm volatile("s_mov_b32 m0, %2\n\tglobal_load_lds_dwordx4 %0, %1 offset:0 nt" ::"v"(voff), "s"(sbase), "s"(m0)
                     : "memory");
    else
        asm volatile("s_mov_b32 m0, %2\n\tglobal_load_lds_dwordx4 %0, %1 offset:0" ::"v"(voff), "s"(sbase), "s"(m0)
                     : "memory");
}

// block swizzle of packet p's LDS region (ds_read_b32 conflict-free, see the header)
template <int SB>
__host__ __device__ constexpr uint32_t swz(uint32_t p) {
    return SB == 4 ? (p & 3u) : SB == 2 ? ((p >> 1) & 1u) : 0u;
}

struct Args {
    const uint8_t* base;
    uint32_t npk, pklen, nb;   // nb: every packet's window has nb blocks (checked on the host)
    const uint32_t* image;
    uint32_t* out;
};

template <int F, int SB, int D, int MODE, int NT>
__global__ void __launch_bounds__(64 * (F + 1)) ring_kernel(Args a) {
    constexpr uint32_t kSlot = 64u * 32u * SB;     // one folder's stage: 64 packets x SB blocks
    constexpr uint32_t IPR = F * 2 * SB;           // DMA instructions per round
    static_assert((D - 2) * IPR <= 63, "vmcnt");
    static_assert(kRing + F * D * kSlot <= 160 * 1024, "LDS");
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    // image: 64 x 1 KiB over the waves
    for (uint32_t i = wave; i < 64u; i += F + 1) {
        const uint64_t g = reinterpret_cast<uint64_t>(a.image) + 1024u * i + 16u * lane;
        const uint32_t m0 = __builtin_amdgcn_readfirstlane(1024u * i);
        asm volatile("s_mov_b32 m0, %1\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(g), "s"(m0) : "memory");
    }
    wait_vm<0>();
    barrier_raw();

    const uint32_t groups = a.npk / 64u;
    const uint32_t folders = gridDim.x * F;
    const uint32_t gpf = (groups + folders - 1u) / folders;
    const uint32_t nb = a.nb;
    const uint32_t nst = (nb + SB - 1u) / SB;
    const uint32_t R = gpf * nst;
    auto gidx = [&](uint32_t f, uint32_t k) -> uint32_t { return (blockIdx.x * F + f) + k * folders; };

    if (wave == F) {
        // ------------------------------------------------------------ loader
        __builtin_amdgcn_s_setprio(3);
        uint32_t voff[F][2 * SB];
        auto set_groups = [&](uint32_t k) __attribute__((always_inline)) {
#pragma unroll
            for (int f = 0; f < F; ++f) {
                const uint32_t g = gidx(f, k);
                const bool ok = g < groups;
#pragma unroll
                for (int i = 0; i < 2 * SB; ++i) {
                    const uint32_t pi = i * (32 / SB) + lane / (2 * SB), pos = lane % (2 * SB);
                    const uint32_t P = ok ? 64u * g + pi : 0u;
                    const uint32_t off = a.pklen * P;
                    const uint32_t ks = pos ^ (2u * swz<SB>(pi));
                    voff[f][i] = (off & ~31u) + 16u * ks;
                }
            }
        };
        auto issue = [&](uint32_t r) __attribute__((always_inline)) {
            const uint32_t s = r % nst, k = r / nst;
            if (s == 0u) set_groups(k);
            const uint64_t sb = reinterpret_cast<uint64_t>(a.base) + 32u * SB * s;
            const uint32_t slot = r % D;
#pragma unroll
            for (int f = 0; f < F; ++f)
#pragma unroll
                for (int i = 0; i < 2 * SB; ++i)
                    dma16<NT>(voff[f][i], sb, __builtin_amdgcn_readfirstlane(kRing + (f * D + slot) * kSlot + 1024u * i));
        };
        for (uint32_t r = 0; r < D - 1 && r < R; ++r) issue(r);
        for (uint32_t r = 0; r < R; ++r) {
            const uint32_t inflight = min(static_cast<uint32_t>(D - 2), R - 1u - r);   // rounds after r
            switch (inflight) {
                case 0: wait_vm<0>(); break;
                case 1: wait_vm<(D >= 3 ? IPR : 0)>(); break;
                case 2: wait_vm<(D >= 4 ? 2 * IPR : 0)>(); break;
                default: wait_vm<(D >= 5 ? 3 * IPR : 0)>(); break;
            }
            barrier_raw();
            if (r + D - 1 < R) issue(r + D - 1);
        }
        wait_vm<0>();
        return;
    }
    // ---------------------------------------------------------------- folders
    const uint32_t f = wave;
    const LaneSched sch = make_sched(lane);
    const uint32_t rp = ((lane & 31u) >> 2) & 7u;
    uint32_t inj[8];
#pragma unroll
    for (int g = 0; g < 8; ++g) inj[g] = (static_cast<uint32_t>(g) == rp) ? 0xFFFFFFFFu : 0u;
    uint32_t A[SB][8];
    const uint32_t abase = kRing + f * D * kSlot + 32u * SB * lane;
    const uint32_t cx = 32u * swz<SB>(lane) + 4u * rp;
#pragma unroll
    for (int q = 0; q < SB; ++q)
#pragma unroll
        for (int g = 0; g < 8; ++g) A[q][g] = abase + ((32u * q + 4u * g) ^ cx);
    uint32_t reg = 0, acc = 0, e = 0;
    const uint32_t L = a.pklen;
    for (uint32_t r0 = 0; r0 < R; r0 += D) {
#pragma unroll
        for (int u = 0; u < D; ++u) {
            const uint32_t r = r0 + u;
            if (r >= R) break;
            barrier_raw();
            const uint32_t s = r % nst, k = r / nst;
            const uint32_t grp = gidx(f, k);
            if (grp >= groups) continue;
            if (MODE == 2 && s == 0u) {
                e = (a.pklen * (64u * grp + lane)) & 31u;
                reg = *reinterpret_cast<lds_u32*>(static_cast<uintptr_t>(init_addr(e)));
            }
#pragma unroll
            for (int q = 0; q < SB; ++q) {
                const uint32_t b = SB * s + q;
                if (b >= nb) break;                    // (uniform: every window has nb blocks)
                uint32_t d[8];
#pragma unroll
                for (int g = 0; g < 8; ++g)
                    d[g] = *reinterpret_cast<lds_u32*>(static_cast<uintptr_t>(A[q][g] + u * kSlot));
                if constexpr (MODE == 1) {
                    acc ^= xor3(xor3(d[0], d[1], d[2]), xor3(d[3], d[4], d[5]), d[6] ^ d[7]);
                } else if constexpr (MODE == 2) {
                    if (b == 0u) {                     // bytes before the packet start
#pragma unroll
                        for (int g = 0; g < 8; ++g) {
                            const int Dw = static_cast<int>(g ^ rp), n = static_cast<int>(e) - 4 * Dw;
                            const uint32_t keep = n >= 4 ? 0u : n <= 0 ? ~0u : (~0u << (8 * n));
                            d[g] &= keep;
                        }
                    }
                    if (b == nb - 1u) {                // bytes past the packet end
                        const int end = static_cast<int>(e + L - 32u * (nb - 1u));
#pragma unroll
                        for (int g = 0; g < 8; ++g) {
                            const int Dw = static_cast<int>(g ^ rp), n = end - 4 * Dw;
                            const uint32_t keep = n >= 4 ? ~0u : n <= 0 ? 0u : (~0u >> (8 * (4 - n)));
                            d[g] &= keep;
                        }
                    }
#pragma unroll
                    for (int g = 0; g < 8; ++g) d[g] = __builtin_amdgcn_bitop3_b32(d[g], reg, inj[g], 0x78);
                    uint32_t v[32];
#pragma unroll
                    for (int i = 0; i < 32; ++i)
                        v[i] = *reinterpret_cast<lds_u32*>(
                            static_cast<uintptr_t>(__builtin_amdgcn_perm(d[i >> 2], sch.col[i >> 2], sch.sel[i & 3])));
                    uint32_t x = xor3(v[0], v[1], v[2]);
#pragma unroll
                    for (int i = 3; i + 1 < 32; i += 2) x = xor3(x, v[i], v[i + 1]);
                    reg = x ^ v[31];
                }
            }
            if (s == nst - 1u) {
                uint32_t res = acc;
                if constexpr (MODE == 2) {
                    const uint32_t tz = 32u * nb - (e + L);
                    res = finalize(tz ? mulmod(reg, *reinterpret_cast<lds_u32*>(static_cast<uintptr_t>(cinv_addr(tz))))
                                      : reg);
                }
                a.out[64u * grp + lane] = res;
                acc = 0;
            }
        }
    }
}


// Loader-only DMA probe: the workgroup's contiguous range split into S contiguous
// streams; a round moves B bytes of every stream (S x B bytes) into the next ring slot,
// D - 1 rounds in flight, one s_barrier per round with W - 1 idle waves.  Maps the
// HBM rate of the loader-wave DMA against streams per CU and bytes per stream-step.
template <int S, int B, int D, int NT, int W>
__global__ void __launch_bounds__(64 * W) stream_kernel(const uint8_t* base, uint64_t bytes, uint32_t* sink) {
    constexpr uint32_t RS = S * B, IPR = RS / 1024u;
    static_assert(RS % 1024 == 0 && (D - 2) * IPR <= 63 && kRing + D * RS <= 160 * 1024, "shape");
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t per_wg = (bytes / gridDim.x) & ~static_cast<uint64_t>(RS - 1);
    const uint64_t per_stream = per_wg / S;
    const uint32_t R = static_cast<uint32_t>(per_stream / B);
    if (wave == 0) {
        __builtin_amdgcn_s_setprio(3);
        uint32_t voff[IPR];
#pragma unroll
        for (int i = 0; i < static_cast<int>(IPR); ++i) {
            uint32_t st, o;
            if constexpr (B >= 1024) {
                st = i / (B / 1024);
                o = 1024u * (i % (B / 1024)) + 16u * lane;
            } else {
                st = i * (1024 / B) + lane / (B / 16);
                o = 16u * (lane % (B / 16));
            }
            voff[i] = static_cast<uint32_t>(st * per_stream) + o;
        }
        const uint64_t wb = reinterpret_cast<uint64_t>(base) + per_wg * blockIdx.x;
        auto issue = [&](uint32_t r) __attribute__((always_inline)) {
            const uint64_t sb = wb + static_cast<uint64_t>(B) * r;
            const uint32_t slot = r % D;
#pragma unroll
            for (int i = 0; i < static_cast<int>(IPR); ++i)
                dma16<NT>(voff[i], sb, __builtin_amdgcn_readfirstlane(kRing + slot * RS + 1024u * i));
        };
        for (uint32_t r = 0; r < D - 1 && r < R; ++r) issue(r);
        for (uint32_t r = 0; r < R; ++r) {
            const uint32_t inflight = min(static_cast<uint32_t>(D - 2), R - 1u - r);
            switch (inflight) {
                case 0: wait_vm<0>(); break;
                case 1: wait_vm<(D >= 3 ? IPR : 0)>(); break;
                case 2: wait_vm<(D >= 4 ? 2 * IPR : 0)>(); break;
                default: wait_vm<(D >= 5 ? 3 * IPR : 0)>(); break;
            }
            barrier_raw();
            if (r + D - 1 < R) issue(r + D - 1);
        }
        wait_vm<0>();
        return;
    }
    uint32_t acc = 0;
    for (uint32_t r = 0; r < R; ++r) {
        barrier_raw();
        acc ^= *reinterpret_cast<lds_u32*>(static_cast<uintptr_t>(kRing + (r % D) * RS + 4u * (threadIdx.x & 255u)));
    }
    if (acc == 0x12345679u) sink[0] = acc;
}


// P = 1 with LINE-aligned windows: a packet's stages are the 128-byte lines it touches,
// so every DMA instruction moves 8 whole lines.  NTM: 0 = default policy, 1 = nt,
// 2 = nt on body stages only (stage 0 and the last two stages keep the default policy,
// so a boundary line, read by both neighbours, can be served from the cache the second
// time).  MODE 3 = the split fold: fold0(block) (32 lookups, no register) and the
// chain reg' = adv32(reg) ^ fold0 (4 lookups in copies of T_31..T_28, free columns
// 4k + m), so only 4 lookups per block wait on the previous block.
template <int F, int D, int MODE, int NTM>
__global__ void __launch_bounds__(64 * (F + 1)) line_kernel(Args a, uint32_t nst) {
    constexpr uint32_t kSlot = 64u * 128u;
    constexpr uint32_t IPR = F * 8;
    static_assert((D - 2) * IPR <= 63, "vmcnt");
    static_assert(kRing + F * D * kSlot <= 160 * 1024, "LDS");
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    for (uint32_t i = wave; i < 64u; i += F + 1) {
        const uint64_t g = reinterpret_cast<uint64_t>(a.image) + 1024u * i + 16u * lane;
        const uint32_t m0 = __builtin_amdgcn_readfirstlane(1024u * i);
        asm volatile("s_mov_b32 m0, %1\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(g), "s"(m0) : "memory");
    }
    wait_vm<0>();
    barrier_raw();
    const uint32_t groups = a.npk / 64u;
    const uint32_t folders = gridDim.x * F;
    const uint32_t gpf = (groups + folders - 1u) / folders;
    const uint32_t R = gpf * nst;
    auto gidx = [&](uint32_t f, uint32_t k) -> uint32_t { return (blockIdx.x * F + f) + k * folders; };
    if (wave == F) {
        __builtin_amdgcn_s_setprio(3);
        uint32_t voff[F][8];
        uint32_t s = 0, k = 0, slot = 0;
        auto issue = [&]() __attribute__((always_inline)) {
            if (s == 0u) {
#pragma unroll
                for (int f = 0; f < F; ++f) {
                    const uint32_t g = gidx(f, k);
                    const bool ok = g < groups;
#pragma unroll
                    for (int i = 0; i < 8; ++i) {
                        const uint32_t pi = 8u * i + (lane >> 3), pos = lane & 7u;
                        const uint32_t off = ok ? a.pklen * (64u * g + pi) : 0u;
                        voff[f][i] = (off & ~127u) + 16u * (pos ^ (2u * (pi & 3u)));
                    }
                }
            }
            const uint64_t sb = reinterpret_cast<uint64_t>(a.base) + 128u * s;
            const bool nt = NTM == 1 || (NTM == 2 && s >= 1u && s + 2u < nst);
            if (nt) {
#pragma unroll
                for (int f = 0; f < F; ++f)
#pragma unroll
                    for (int i = 0; i < 8; ++i)
                        dma16<1>(voff[f][i], sb, __builtin_amdgcn_readfirstlane(kRing + (f * D + slot) * kSlot + 1024u * i));
            } else {
#pragma unroll
                for (int f = 0; f < F; ++f)
#pragma unroll
                    for (int i = 0; i < 8; ++i)
                        dma16<0>(voff[f][i], sb, __builtin_amdgcn_readfirstlane(kRing + (f * D + slot) * kSlot + 1024u * i));
            }
            if (++s == nst) { s = 0; ++k; }
            if (++slot == D) slot = 0;
        };
        for (uint32_t r = 0; r < D - 1 && r < R; ++r) issue();
        for (uint32_t r = 0; r < R; ++r) {
            const uint32_t inflight = min(static_cast<uint32_t>(D - 2), R - 1u - r);
            switch (inflight) {
                case 0: wait_vm<0>(); break;
                case 1: wait_vm<(D >= 3 ? IPR : 0)>(); break;
                default: wait_vm<(D >= 4 ? 2 * IPR : 0)>(); break;
            }
            barrier_raw();
            if (r + D - 1 < R) issue();
        }
        wait_vm<0>();
        return;
    }
    const uint32_t f = wave;
    const LaneSched sch = make_sched(lane);
    const uint32_t l5 = lane & 31u, rp = (l5 >> 2) & 7u;
    uint32_t inj[8];
#pragma unroll
    for (int g = 0; g < 8; ++g) inj[g] = (static_cast<uint32_t>(g) == rp) ? 0xFFFFFFFFu : 0u;
    // adv32 by copies: step i reads byte m = i ^ (l & 3) of reg in copy (l >> 3) & 3
    uint32_t acol[4], asel[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const uint32_t m = static_cast<uint32_t>(i) ^ (l5 & 3u), kc = (l5 >> 3) & 3u;
        acol[i] = free_col(4u * kc + m);                  // v_perm src1: byte 0 = the column byte
        asel[i] = ((4u + m) << 8) | 0x0C0C0000u;          // byte0 <- src1 byte 0, byte1 <- reg byte m
    }
    uint32_t A[4][8];
    const uint32_t abase = kRing + f * D * kSlot + 128u * lane;
    const uint32_t cx = 32u * (lane & 3u) + 4u * rp;
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int g = 0; g < 8; ++g) A[q][g] = abase + ((32u * q + 4u * g) ^ cx);
    uint32_t reg = 0, acc = 0, e = 0, fb = 0, lb = 0, rel_end = 0;
    const uint32_t L = a.pklen;
    uint32_t s = 0, k = 0;
    for (uint32_t r0 = 0; r0 < R; r0 += D) {
#pragma unroll
        for (int u = 0; u < D; ++u) {
            if (r0 + u >= R) break;
            barrier_raw();
            const uint32_t grp = gidx(f, k);
            if (grp < groups) {
                if (s == 0u) {
                    const uint32_t off = a.pklen * (64u * grp + lane);
                    e = off & 31u;
                    fb = (off & 127u) >> 5;
                    rel_end = (off & 127u) + L;
                    lb = (rel_end - 1u) >> 5;
                    reg = *reinterpret_cast<lds_u32*>(static_cast<uintptr_t>(init_addr(e)));
                }
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const uint32_t j = 4u * s + q;
                    uint32_t d[8];
#pragma unroll
                    for (int g = 0; g < 8; ++g)
                        d[g] = *reinterpret_cast<lds_u32*>(static_cast<uintptr_t>(A[q][g] + u * kSlot));
                    if constexpr (MODE == 1) {
                        acc ^= xor3(xor3(d[0], d[1], d[2]), xor3(d[3], d[4], d[5]), d[6] ^ d[7]);
                    } else if constexpr (MODE >= 2) {
                        const bool first = j == fb, last = j == lb, active = j >= fb && j <= lb;
                        if (__builtin_amdgcn_ballot_w64(first)) {
#pragma unroll
                            for (int g = 0; g < 8; ++g) {
                                const int Dw = static_cast<int>(g ^ rp), n = static_cast<int>(e) - 4 * Dw;
                                const uint32_t keep = n >= 4 ? 0u : n <= 0 ? ~0u : (~0u << (8 * n));
                                d[g] &= first ? keep : ~0u;
                            }
                        }
                        if (__builtin_amdgcn_ballot_w64(last)) {
                            const int end = static_cast<int>(rel_end - 32u * lb);
#pragma unroll
                            for (int g = 0; g < 8; ++g) {
                                const int Dw = static_cast<int>(g ^ rp), n = end - 4 * Dw;
                                const uint32_t keep = n >= 4 ? ~0u : n <= 0 ? 0u : (~0u >> (8 * (4 - n)));
                                d[g] &= last ? keep : ~0u;
                            }
                        }
                        if (__builtin_amdgcn_ballot_w64(active)) {
                            uint32_t nr;
                            if constexpr (MODE == 2) {
#pragma unroll
                                for (int g = 0; g < 8; ++g) d[g] = __builtin_amdgcn_bitop3_b32(d[g], reg, inj[g], 0x78);
                            }
                            uint32_t v[32];
#pragma unroll
                            for (int i = 0; i < 32; ++i)
                                v[i] = *reinterpret_cast<lds_u32*>(static_cast<uintptr_t>(
                                    __builtin_amdgcn_perm(d[i >> 2], sch.col[i >> 2], sch.sel[i & 3])));
                            uint32_t x = xor3(v[0], v[1], v[2]);
#pragma unroll
                            for (int i = 3; i + 1 < 32; i += 2) x = xor3(x, v[i], v[i + 1]);
                            x ^= v[31];
                            if constexpr (MODE == 3) {
                                uint32_t w[4];
#pragma unroll
                                for (int i = 0; i < 4; ++i)
                                    w[i] = *reinterpret_cast<lds_u32*>(
                                        static_cast<uintptr_t>(__builtin_amdgcn_perm(reg, acol[i], asel[i])));
                                nr = xor3(x, w[0], w[1]) ^ xor3(w[2], w[3], 0u);
                            } else {
                                nr = x;
                            }
                            reg = active ? nr : reg;
                        }
                    }
                }
                if (s == nst - 1u) {
                    uint32_t res = acc;
                    if constexpr (MODE >= 2) {
                        const uint32_t tz = 32u * (lb + 1u) - rel_end;
                        res = finalize(tz ? mulmod(reg, *reinterpret_cast<lds_u32*>(static_cast<uintptr_t>(cinv_addr(tz))))
                                          : reg);
                    }
                    a.out[64u * grp + lane] = res;
                    acc = 0;
                }
            }
            if (++s == nst) { s = 0; ++k; }
        }
    }
}

// P = 4 with line-aligned windows: F folder waves of 16 packets (4 lanes each; lane k
// folds block k of every line with the advancing tables T'_t = T_{t+96}), one loader.
// A packet's window is the lines it touches: lz = a mod 128 leading bytes (masked;
// lane 0 starts at INIT[lz]), the packet, then tz < 128 bytes (masked), undone at the
// end by x^(-8 tz).  Lanes past their packet's last line keep their register.
template <int F, int D, int MODE, int NTM>
__global__ void __launch_bounds__(64 * (F + 1)) line4_kernel(Args a, uint32_t nst) {
    constexpr uint32_t kSlot = 16u * 128u;
    constexpr uint32_t IPR = F * 2;
    static_assert((D - 2) * IPR <= 63, "vmcnt");
    static_assert(kRing + F * D * kSlot <= 160 * 1024, "LDS");
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    for (uint32_t i = wave; i < 64u; i += F + 1) {
        const uint64_t g = reinterpret_cast<uint64_t>(a.image) + 1024u * i + 16u * lane;
        const uint32_t m0 = __builtin_amdgcn_readfirstlane(1024u * i);
        asm volatile("s_mov_b32 m0, %1\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(g), "s"(m0) : "memory");
    }
    wait_vm<0>();
    barrier_raw();
    const uint32_t groups = a.npk / 16u;
    const uint32_t folders = gridDim.x * F;
    const uint32_t gpf = (groups + folders - 1u) / folders;
    const uint32_t R = gpf * nst;
    auto gidx = [&](uint32_t f, uint32_t k) -> uint32_t { return (blockIdx.x * F + f) + k * folders; };
    if (wave == F) {
        __builtin_amdgcn_s_setprio(3);
        uint32_t voff[F][2];
        uint32_t s = 0, k = 0, slot = 0;
        auto issue = [&]() __attribute__((always_inline)) {
            if (s == 0u) {
#pragma unroll
                for (int f = 0; f < F; ++f) {
                    const uint32_t g = gidx(f, k);
                    const bool ok = g < groups;
#pragma unroll
                    for (int i = 0; i < 2; ++i) {
                        const uint32_t pi = 8u * i + (lane >> 3);
                        const uint32_t off = ok ? a.pklen * (16u * g + pi) : 0u;
                        voff[f][i] = (off & ~127u) + 16u * (lane & 7u);
                    }
                }
            }
            const uint64_t sb = reinterpret_cast<uint64_t>(a.base) + 128u * s;
            const bool nt = NTM == 1 || (NTM == 2 && s >= 1u && s + 2u < nst);
            if (NTM == 3) {
            } else
            if (nt) {
#pragma unroll
                for (int f = 0; f < F; ++f)
#pragma unroll
                    for (int i = 0; i < 2; ++i)
                        dma16<1>(voff[f][i], sb, __builtin_amdgcn_readfirstlane(kRing + (f * D + slot) * kSlot + 1024u * i));
            } else {
#pragma unroll
                for (int f = 0; f < F; ++f)
#pragma unroll
                    for (int i = 0; i < 2; ++i)
                        dma16<0>(voff[f][i], sb, __builtin_amdgcn_readfirstlane(kRing + (f * D + slot) * kSlot + 1024u * i));
            }
            if (++s == nst) { s = 0; ++k; }
            if (++slot == D) slot = 0;
        };
        for (uint32_t r = 0; r < D - 1 && r < R; ++r) issue();
        for (uint32_t r = 0; r < R; ++r) {
            const uint32_t inflight = min(static_cast<uint32_t>(D - 2), R - 1u - r);
            switch (inflight) {
                case 0: wait_vm<0>(); break;
                case 1: wait_vm<(D >= 3 ? IPR : 0)>(); break;
                default: wait_vm<(D >= 4 ? 2 * IPR : 0)>(); break;
            }
            barrier_raw();
            if (r + D - 1 < R) issue();
        }
        wait_vm<0>();
        return;
    }
    const uint32_t f = wave;
    const LaneSched sch = make_sched(lane);
    const uint32_t l5 = lane & 31u, rp = (l5 >> 2) & 7u, kl = lane & 3u;
    uint32_t inj[8];
#pragma unroll
    for (int g = 0; g < 8; ++g) inj[g] = (static_cast<uint32_t>(g) == rp) ? 0xFFFFFFFFu : 0u;
    uint32_t A[8];
    const uint32_t abase = kRing + f * D * kSlot + 32u * lane;     // packet lane>>2's line, block k
#pragma unroll
    for (int g = 0; g < 8; ++g) A[g] = abase + 4u * (static_cast<uint32_t>(g) ^ rp);
    uint32_t reg = 0, acc = 0, lz = 0, nl = 0, rel_end = 0;
    const uint32_t L = a.pklen;
    uint32_t s = 0, k = 0;
    for (uint32_t r0 = 0; r0 < R; r0 += D) {
#pragma unroll
        for (int u = 0; u < D; ++u) {
            if (r0 + u >= R) break;
            barrier_raw();
            const uint32_t grp = gidx(f, k);
            if (grp < groups) {
                if (s == 0u) {
                    const uint32_t off = a.pklen * (16u * grp + (lane >> 2));
                    lz = off & 127u;
                    rel_end = lz + L;
                    nl = (rel_end + 127u) >> 7;
                    reg = kl == 0u ? *reinterpret_cast<lds_u32*>(static_cast<uintptr_t>(256u * lz + free_col(kInitCol))) : 0u;
                }
                uint32_t d[8];
#pragma unroll
                for (int g = 0; g < 8; ++g) d[g] = *reinterpret_cast<lds_u32*>(static_cast<uintptr_t>(A[g] + u * kSlot));
                if constexpr (MODE == 1) {
                    acc ^= xor3(xor3(d[0], d[1], d[2]), xor3(d[3], d[4], d[5]), d[6] ^ d[7]);
                } else if constexpr (MODE == 2) {
                    const bool active = s < nl;
                    if (s == 0u) {                        // bytes before the packet start
                        const int hb = static_cast<int>(lz) - 32 * static_cast<int>(kl);
#pragma unroll
                        for (int g = 0; g < 8; ++g) {
                            const int n = hb - 4 * static_cast<int>(g ^ rp);
                            d[g] &= n >= 4 ? 0u : n <= 0 ? ~0u : (~0u << (8 * n));
                        }
                    }
                    const bool last = s + 1u == nl;
                    if (__builtin_amdgcn_ballot_w64(last)) {   // bytes past the packet end
                        const int eb = static_cast<int>(rel_end - 128u * s) - 32 * static_cast<int>(kl);
#pragma unroll
                        for (int g = 0; g < 8; ++g) {
                            const int n = eb - 4 * static_cast<int>(g ^ rp);
                            const uint32_t keep = n >= 4 ? ~0u : n <= 0 ? 0u : (~0u >> (8 * (4 - n)));
                            d[g] &= last ? keep : ~0u;
                        }
                    }
#pragma unroll
                    for (int g = 0; g < 8; ++g) d[g] = __builtin_amdgcn_bitop3_b32(d[g], reg, inj[g], 0x78);
                    uint32_t v[32];
#pragma unroll
                    for (int i = 0; i < 32; ++i)
                        v[i] = *reinterpret_cast<lds_u32*>(
                            static_cast<uintptr_t>(__builtin_amdgcn_perm(d[i >> 2], sch.col[i >> 2], sch.sel[i & 3])));
                    uint32_t x = xor3(v[0], v[1], v[2]);
#pragma unroll
                    for (int i = 3; i + 1 < 32; i += 2) x = xor3(x, v[i], v[i + 1]);
                    x ^= v[31];
                    reg = active ? x : reg;
                }
                if (s == nst - 1u) {
                    uint32_t res = acc;
                    if constexpr (MODE == 2) {
                        // lane k sits k blocks past the window end: x^(-256 k), then the quad XOR
                        uint32_t c = reg;
                        if (kl) {
                            uint32_t y = 0;
#pragma unroll
                            for (int b = 0; b < 4; ++b)
                                y ^= *reinterpret_cast<lds_u32*>(static_cast<uintptr_t>(
                                    256u * ((reg >> (8 * b)) & 255u) + corr_col(kl, static_cast<uint32_t>(b))));
                            c = y;
                        }
                        c ^= dpp<kDppQuadXor1>(c);
                        c ^= dpp<kDppQuadXor2>(c);
                        const uint32_t tz = 128u * nl - rel_end;
                        res = finalize(tz ? mulmod(c, *reinterpret_cast<lds_u32*>(static_cast<uintptr_t>(cinv_addr(tz)))) : c);
                    }
                    if (kl == 0u) a.out[16u * grp + (lane >> 2)] = res;
                    acc = 0;
                }
            }
            if (++s == nst) { s = 0; ++k; }
        }
    }
}

// The same P = 4 line shape with the per-round s_barrier replaced by LDS handshake
// words, so folder waves drift out of phase (LDS and VALU phases overlap) and only
// wait when the ring is empty: word 0 = rounds published by the loader (written after
// its counted vmcnt wait), word 1 + s = folders done reading slot s (ds_add after
// their data reads returned).  The loader issues a round when its slot is free and
// fewer than D - 1 rounds are in flight, otherwise publishes the oldest in flight.
// Head and tail masks are v_perm selectors built once per packet.  MODE 4 = the fold
// with the table lookups replaced by the XOR of the lookup addresses (diagnostic).
__device__ __forceinline__ uint32_t lds_vload(uint32_t addr) {
    return *reinterpret_cast<volatile __attribute__((address_space(3))) uint32_t*>(static_cast<uintptr_t>(addr));
}
__device__ __forceinline__ void lds_add(uint32_t addr, uint32_t v) {
    __hip_atomic_fetch_add(reinterpret_cast<__attribute__((address_space(3))) uint32_t*>(static_cast<uintptr_t>(addr)), v,
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ uint32_t head_sel(int n) {   // keep bytes >= n of a dword
    const uint32_t id = 0x07060504u, z = 0x0C0C0C0Cu;
    if (n <= 0) return id;
    if (n >= 4) return z;
    const uint32_t m = ~0u << (8 * n);
    return (id & m) | (z & ~m);
}
__device__ __forceinline__ uint32_t tail_sel(int n) {   // keep bytes < n of a dword
    const uint32_t id = 0x07060504u, z = 0x0C0C0C0Cu;
    if (n >= 4) return id;
    if (n <= 0) return z;
    const uint32_t m = ~0u << (8 * n);
    return (id & ~m) | (z & m);
}

template <int F, int D, int MODE, int NTM>
__global__ void __launch_bounds__(64 * (F + 1)) hs4_kernel(Args a, uint32_t nst) {
    constexpr uint32_t kSlot = 16u * 128u;
    constexpr uint32_t IPR = F * 2, K = D - 1;
    constexpr uint32_t kHs = kRing + F * D * kSlot;
    static_assert((K - 1) * IPR <= 63 && K <= 3, "vmcnt");
    static_assert(kHs + 64 <= 160 * 1024, "LDS");
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    for (uint32_t i = wave; i < 64u; i += F + 1) {
        const uint64_t g = reinterpret_cast<uint64_t>(a.image) + 1024u * i + 16u * lane;
        const uint32_t m0 = __builtin_amdgcn_readfirstlane(1024u * i);
        asm volatile("s_mov_b32 m0, %1\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(g), "s"(m0) : "memory");
    }
    if (threadIdx.x <= D) *reinterpret_cast<__attribute__((address_space(3))) uint32_t*>(static_cast<uintptr_t>(kHs + 4u * threadIdx.x)) = 0u;
    wait_vm<0>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    barrier_raw();
    const uint32_t groups = a.npk / 16u;
    const uint32_t folders = gridDim.x * F;
    const uint32_t gpf = (groups + folders - 1u) / folders;
    const uint32_t R = gpf * nst;
    auto gidx = [&](uint32_t f, uint32_t k) -> uint32_t { return (blockIdx.x * F + f) + k * folders; };
    if (wave == F) {
        __builtin_amdgcn_s_setprio(3);
        uint32_t voff[F][2];
        uint32_t s = 0, k = 0, slot = 0;
        auto issue = [&]() __attribute__((always_inline)) {
            if (s == 0u) {
#pragma unroll
                for (int f = 0; f < F; ++f) {
                    const uint32_t g = gidx(f, k);
                    const bool ok = g < groups;
#pragma unroll
                    for (int i = 0; i < 2; ++i) {
                        const uint32_t pi = 8u * i + (lane >> 3);
                        const uint32_t off = ok ? a.pklen * (16u * g + pi) : 0u;
                        voff[f][i] = (off & ~127u) + 16u * (lane & 7u);
                    }
                }
            }
            const uint64_t sb = reinterpret_cast<uint64_t>(a.base) + 128u * s;
            const bool nt = NTM == 1 || (NTM == 2 && s >= 1u && s + 2u < nst);
            if (NTM == 3) {
            } else
            if (nt) {
#pragma unroll
                for (int f = 0; f < F; ++f)
#pragma unroll
                    for (int i = 0; i < 2; ++i)
                        dma16<1>(voff[f][i], sb, __builtin_amdgcn_readfirstlane(kRing + (f * D + slot) * kSlot + 1024u * i));
            } else {
#pragma unroll
                for (int f = 0; f < F; ++f)
#pragma unroll
                    for (int i = 0; i < 2; ++i)
                        dma16<0>(voff[f][i], sb, __builtin_amdgcn_readfirstlane(kRing + (f * D + slot) * kSlot + 1024u * i));
            }
            if (++s == nst) { s = 0; ++k; }
            if (++slot == D) slot = 0;
        };
        uint32_t issued = 0, published = 0;
        while (published < R) {
            if (issued < R && issued - published < K) {
                const uint32_t need = F * (issued / D);
                if (issued < D || lds_vload(kHs + 4u + 4u * (issued % D)) >= need) {
                    issue();
                    ++issued;
                    continue;
                }
            }
            if (issued > published) {
                switch (issued - published - 1u) {
                    case 0: wait_vm<0>(); break;
                    case 1: wait_vm<IPR>(); break;
                    default: wait_vm<(K >= 3 ? 2 * IPR : 0)>(); break;
                }
                ++published;
                *reinterpret_cast<volatile __attribute__((address_space(3))) uint32_t*>(static_cast<uintptr_t>(kHs)) = published;
            } else {
                __builtin_amdgcn_s_sleep(1);
            }
        }
        wait_vm<0>();
        return;
    }
    const uint32_t f = wave;
    const LaneSched sch = make_sched(lane);
    const uint32_t l5 = lane & 31u, rp = (l5 >> 2) & 7u, kl = lane & 3u;
    uint32_t inj[8];
#pragma unroll
    for (int g = 0; g < 8; ++g) inj[g] = (static_cast<uint32_t>(g) == rp) ? 0xFFFFFFFFu : 0u;
    uint32_t A[8];
    const uint32_t abase = kRing + f * D * kSlot + 32u * lane;
#pragma unroll
    for (int g = 0; g < 8; ++g) A[g] = abase + 4u * (static_cast<uint32_t>(g) ^ rp);
    uint32_t reg = 0, acc = 0, lz = 0, nl = 0, rel_end = 0, known = 0;
    uint32_t hsel[8], tsel[8];
    const uint32_t L = a.pklen;
    uint32_t s = 0, k = 0;
    for (uint32_t r0 = 0; r0 < R; r0 += D) {
#pragma unroll
        for (int u = 0; u < D; ++u) {
            const uint32_t r = r0 + u;
            if (r >= R) break;
            if (r >= known) {
                known = lds_vload(kHs);
                while (known <= r) {
                    __builtin_amdgcn_s_sleep(1);
                    known = lds_vload(kHs);
                }
            }
            const uint32_t grp = gidx(f, k);
            uint32_t d[8];
#pragma unroll
            for (int g = 0; g < 8; ++g) d[g] = *reinterpret_cast<lds_u32*>(static_cast<uintptr_t>(A[g] + u * kSlot));
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            if (lane == 0u) lds_add(kHs + 4u + 4u * u, 1u);
            if (grp < groups) {
                if (s == 0u) {
                    const uint32_t off = a.pklen * (16u * grp + (lane >> 2));
                    lz = off & 127u;
                    rel_end = lz + L;
                    nl = (rel_end + 127u) >> 7;
                    const int hb = static_cast<int>(lz) - 32 * static_cast<int>(kl);
                    const int eb = static_cast<int>(rel_end - 128u * (nl - 1u)) - 32 * static_cast<int>(kl);
#pragma unroll
                    for (int g = 0; g < 8; ++g) {
                        hsel[g] = head_sel(hb - 4 * static_cast<int>(g ^ rp));
                        tsel[g] = tail_sel(eb - 4 * static_cast<int>(g ^ rp));
                    }
                    reg = kl == 0u ? *reinterpret_cast<lds_u32*>(static_cast<uintptr_t>(256u * lz + free_col(kInitCol))) : 0u;
                }
                if constexpr (MODE == 1) {
                    acc ^= xor3(xor3(d[0], d[1], d[2]), xor3(d[3], d[4], d[5]), d[6] ^ d[7]);
                } else if constexpr (MODE >= 2) {
                    const bool active = s < nl;
                    if (MODE != 5 && s == 0u) {
#pragma unroll
                        for (int g = 0; g < 8; ++g) d[g] = __builtin_amdgcn_perm(d[g], 0u, hsel[g]);
                    }
                    const bool last = s + 1u == nl;
                    if (MODE != 5 && __builtin_amdgcn_ballot_w64(last)) {
#pragma unroll
                        for (int g = 0; g < 8; ++g) d[g] = __builtin_amdgcn_perm(d[g], 0u, last ? tsel[g] : 0x07060504u);
                    }
#pragma unroll
                    for (int g = 0; g < 8; ++g) d[g] = MODE == 6 ? d[g] : __builtin_amdgcn_bitop3_b32(d[g], reg, inj[g], 0x78);
                    uint32_t v[32];
#pragma unroll
                    for (int i = 0; i < 32; ++i) {
                        const uint32_t ad = __builtin_amdgcn_perm(d[i >> 2], sch.col[i >> 2], sch.sel[i & 3]);
                        v[i] = MODE == 4 ? ad : *reinterpret_cast<lds_u32*>(static_cast<uintptr_t>(ad));
                    }
                    uint32_t x = xor3(v[0], v[1], v[2]);
#pragma unroll
                    for (int i = 3; i + 1 < 32; i += 2) x = xor3(x, v[i], v[i + 1]);
                    x ^= v[31];
                    reg = active ? x : reg;
                }
                if (s == nst - 1u) {
                    uint32_t res = acc;
                    if constexpr (MODE >= 2) {
                        uint32_t c = reg;
                        if (kl) {
                            uint32_t y = 0;
#pragma unroll
                            for (int b = 0; b < 4; ++b)
                                y ^= *reinterpret_cast<lds_u32*>(static_cast<uintptr_t>(
                                    256u * ((reg >> (8 * b)) & 255u) + corr_col(kl, static_cast<uint32_t>(b))));
                            c = y;
                        }
                        c ^= dpp<kDppQuadXor1>(c);
                        c ^= dpp<kDppQuadXor2>(c);
                        const uint32_t tz = 128u * nl - rel_end;
                        res = MODE == 5 ? c : finalize(tz ? mulmod(c, *reinterpret_cast<lds_u32*>(static_cast<uintptr_t>(cinv_addr(tz)))) : c);
                    }
                    if (kl == 0u) a.out[16u * grp + (lane >> 2)] = res;
                    acc = 0;
                }
            }
            if (++s == nst) { s = 0; ++k; }
        }
    }
}

// ------------------------------------------------------------------ host

static std::vector<uint32_t> p4_image() {
    // T'_t = T_{t+96}; corrections x^(-256 k), k = 1..3; INIT rows 0..127; CINV
    std::vector<uint32_t> img(kImageDwords, 0u);
    std::vector<uint32_t> row(256);
    for (uint32_t j = 0; j < 256; ++j) {
        uint32_t r = crc_table_entry(j);
        for (int z = 0; z < 96; ++z) r = sarwate_step(r, 0);
        row[j] = r;
    }
    for (uint32_t t = 0; t < 32; ++t) {
        for (uint32_t j = 0; j < 256; ++j) img[(j * 256 + col_byte(t)) / 4] = row[j];
        for (uint32_t j = 0; j < 256; ++j) row[j] = sarwate_step(row[j], 0);
    }
    uint32_t xinv = 1u;
    for (int i = 1; i < 32; ++i)
        if ((kPoly >> (31 - i)) & 1u) xinv |= 1u << (31 - (i - 1));
    uint32_t xinv8 = kOneReflected;
    for (int i = 0; i < 8; ++i) xinv8 = gf2_mulmod(xinv8, xinv);
    std::vector<uint32_t> cinv(512);
    cinv[0] = kOneReflected;
    for (int i = 1; i < 512; ++i) cinv[i] = gf2_mulmod(cinv[i - 1], xinv8);
    for (uint32_t k = 1; k < 4; ++k)
        for (uint32_t b = 0; b < 4; ++b)
            for (uint32_t v = 0; v < 256; ++v) img[(256u * v + corr_col(k, b)) / 4] = gf2_mulmod(v << (8 * b), cinv[32 * k]);
    uint32_t init = 0xFFFFFFFFu;
    for (uint32_t r = 0; r < 256; ++r) {
        img[(256u * r + free_col(kInitCol)) / 4] = init;
        init = unstep_zero(init);
    }
    for (uint32_t i = 0; i < 512; ++i) img[cinv_addr(i) / 4] = cinv[i];
    return img;
}

static std::vector<uint32_t> p1_image() {
    std::vector<uint32_t> img(kImageDwords, 0u);
    std::vector<uint32_t> row(256);
    for (uint32_t j = 0; j < 256; ++j) row[j] = crc_table_entry(j);
    for (uint32_t t = 0; t < 32; ++t) {
        for (uint32_t j = 0; j < 256; ++j) img[(j * 256 + col_byte(t)) / 4] = row[j];
        for (uint32_t j = 0; j < 256; ++j) row[j] = sarwate_step(row[j], 0);
    }
    for (uint32_t k = 0; k < 4; ++k)                      // copies of T_31..T_28 (line_kernel MODE 3)
        for (uint32_t m = 0; m < 4; ++m)
            for (uint32_t j = 0; j < 256; ++j) img[(j * 256 + free_col(4 * k + m)) / 4] = img[(j * 256 + col_byte(31 - m)) / 4];
    uint32_t init = 0xFFFFFFFFu;
    for (uint32_t r = 0; r < 64; ++r) {
        img[init_addr(r) / 4] = init;
        init = unstep_zero(init);
    }
    uint32_t xinv = 1u;
    for (int i = 1; i < 32; ++i)
        if ((kPoly >> (31 - i)) & 1u) xinv |= 1u << (31 - (i - 1));
    uint32_t xinv8 = kOneReflected;
    for (int i = 0; i < 8; ++i) xinv8 = gf2_mulmod(xinv8, xinv);
    uint32_t c = kOneReflected;
    for (uint32_t i = 0; i < 512; ++i) {
        img[cinv_addr(i) / 4] = c;
        c = gf2_mulmod(c, xinv8);
    }
    return img;
}

int main(int argc, char** argv) {
    const uint32_t pklen = argc > 1 ? static_cast<uint32_t>(atoi(argv[1])) : 1200u;
    const uint32_t npk = 5u * 65536u;
    const uint64_t bytes = static_cast<uint64_t>(npk) * pklen;
    std::vector<uint8_t> h(bytes + 4096);
    uint64_t s = 0x9E3779B97F4A7C15ull;
    for (uint64_t i = 0; i < h.size(); i += 8) {
        s ^= s << 13; s ^= s >> 7; s ^= s << 17;
        memcpy(&h[i], &s, std::min<uint64_t>(8, h.size() - i));
    }
    std::vector<uint32_t> ref(npk);
    for (uint32_t p = 0; p < npk; ++p) {
        uint32_t r = 0xFFFFFFFFu;
        const uint8_t* q = h.data() + static_cast<uint64_t>(p) * pklen;
        for (uint32_t i = 0; i < pklen; ++i) r = sarwate_step(r, q[i]);
        ref[p] = finalize(r);
    }
    uint8_t* d;
    uint32_t *dimg, *dout;
    HC(hipMalloc(&d, h.size()));
    HC(hipMemcpy(d, h.data(), h.size(), hipMemcpyHostToDevice));
    const std::vector<uint32_t> img = p1_image();
    HC(hipMalloc(&dimg, kLdsTableBytes));
    HC(hipMemcpy(dimg, img.data(), kLdsTableBytes, hipMemcpyHostToDevice));
    HC(hipMalloc(&dout, 4u * npk));
    int cus = 0;
    HC(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    hipEvent_t e0, e1;
    HC(hipEventCreate(&e0));
    HC(hipEventCreate(&e1));
    uint32_t nb = 0;
    for (uint32_t p = 0; p < 64; ++p) {
        const uint32_t e = (pklen * p) & 31u, n = (e + pklen + 31u) / 32u;
        if (nb && n != nb) {
            printf("# windows of %u-byte packets differ in block count: the probe needs one count\n", pklen);
            return 1;
        }
        nb = n;
    }
    Args a{d, npk, pklen, nb, dimg, dout};
    printf("# %u packets x %u B = %.1f MB per launch, %d CUs\n", npk, pklen, bytes / 1e6, cus);
    auto run = [&](auto kern, int F, int SB, int D, int MODE, int NT, int lds) {
        HC(hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, lds));
        HC(hipMemset(dout, 0, 4u * npk));
        auto launch = [&] { hipLaunchKernelGGL(kern, dim3(cus), dim3(64 * (F + 1)), lds, 0, a); };
        for (int w = 0; w < 3; ++w) launch();
        HC(hipDeviceSynchronize());
        const int reps = 20;
        HC(hipEventRecord(e0));
        for (int i = 0; i < reps; ++i) launch();
        HC(hipEventRecord(e1));
        HC(hipEventSynchronize(e1));
        float ms = 0;
        HC(hipEventElapsedTime(&ms, e0, e1));
        const double us = ms * 1e3 / reps, tbs = bytes / (us * 1e-6) / 1e12;
        const char* ok = "-";
        if (MODE == 2) {
            std::vector<uint32_t> o(npk);
            HC(hipMemcpy(o.data(), dout, 4u * npk, hipMemcpyDeviceToHost));
            uint32_t bad = 0;
            for (uint32_t p = 0; p < npk; ++p) bad += o[p] != ref[p];
            ok = bad ? "MISMATCH" : "exact";
            if (bad) printf("#   %u mismatches, e.g. p0 %08x vs %08x\n", bad, o[0], ref[0]);
        }
        printf("F=%d SB=%d D=%d mode=%d nt=%d: %8.2f us per launch  %.3f TB/s = %.3f of 8  %s\n", F, SB, D, MODE, NT, us,
               tbs, tbs / 8.0, ok);
        fflush(stdout);
    };
#define RUN(F, SB, D, M, NT) run(ring_kernel<F, SB, D, M, NT>, F, SB, D, M, NT, kRing + F * D * 64 * 32 * SB)

    auto srun = [&](auto kern, int S, int B, int D, int NT, int W, int lds) {
        HC(hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, lds));
        auto launch = [&] { hipLaunchKernelGGL(kern, dim3(cus), dim3(64 * W), lds, 0, d, bytes, dout); };
        for (int w = 0; w < 3; ++w) launch();
        HC(hipDeviceSynchronize());
        const int reps = 20;
        HC(hipEventRecord(e0));
        for (int i = 0; i < reps; ++i) launch();
        HC(hipEventRecord(e1));
        HC(hipEventSynchronize(e1));
        float ms = 0;
        HC(hipEventElapsedTime(&ms, e0, e1));
        const uint64_t moved = ((bytes / cus) & ~static_cast<uint64_t>(S * B - 1)) * cus;
        const double us = ms * 1e3 / reps, tbs = moved / (us * 1e-6) / 1e12;
        printf("streams S=%3d B=%5d D=%d nt=%d waves=%d: %8.2f us  %.3f TB/s = %.3f of 8\n", S, B, D, NT, W, us, tbs, tbs / 8.0);
        fflush(stdout);
    };
#define SRUN(S, B, D, NT, W) srun(stream_kernel<S, B, D, NT, W>, S, B, D, NT, W, kRing + D * S * B)
    uint32_t nst = 0;
    for (uint32_t p = 0; p < npk; ++p) {
        const uint64_t off = static_cast<uint64_t>(pklen) * p;
        nst = std::max<uint32_t>(nst, static_cast<uint32_t>(((off + pklen - 1) >> 7) - (off >> 7) + 1));
    }
    auto lrun = [&](auto kern, int F, int D, int MODE, int NTM, int lds) {
        HC(hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, lds));
        HC(hipMemset(dout, 0, 4u * npk));
        auto launch = [&] { hipLaunchKernelGGL(kern, dim3(cus), dim3(64 * (F + 1)), lds, 0, a, nst); };
        for (int w = 0; w < 3; ++w) launch();
        HC(hipDeviceSynchronize());
        const int reps = 20;
        HC(hipEventRecord(e0));
        for (int i = 0; i < reps; ++i) launch();
        HC(hipEventRecord(e1));
        HC(hipEventSynchronize(e1));
        float ms = 0;
        HC(hipEventElapsedTime(&ms, e0, e1));
        const double us = ms * 1e3 / reps, tbs = bytes / (us * 1e-6) / 1e12;
        const char* ok = "-";
        if (MODE >= 2) {
            std::vector<uint32_t> o(npk);
            HC(hipMemcpy(o.data(), dout, 4u * npk, hipMemcpyDeviceToHost));
            uint32_t bad = 0;
            for (uint32_t p = 0; p < npk; ++p) bad += o[p] != ref[p];
            ok = bad ? "MISMATCH" : "exact";
            if (bad) printf("#   %u mismatches, e.g. p0 %08x vs %08x\n", bad, o[0], ref[0]);
        }
        printf("lines F=%d D=%d mode=%d ntm=%d (%u stages): %8.2f us  %.3f TB/s = %.3f of 8  %s\n", F, D, MODE, NTM, nst, us, tbs,
               tbs / 8.0, ok);
        fflush(stdout);
    };
#define LRUN(F, D, M, NTM) lrun(line_kernel<F, D, M, NTM>, F, D, M, NTM, kRing + F * D * 8192)
    uint32_t* dimg4;
    {
        const std::vector<uint32_t> img4 = p4_image();
        HC(hipMalloc(&dimg4, kLdsTableBytes));
        HC(hipMemcpy(dimg4, img4.data(), kLdsTableBytes, hipMemcpyHostToDevice));
    }
    auto l4run = [&](auto kern, int F, int D, int MODE, int NTM, int lds) {
        HC(hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, lds));
        HC(hipMemset(dout, 0, 4u * npk));
        Args a4 = a;
        a4.image = dimg4;
        auto launch = [&] { hipLaunchKernelGGL(kern, dim3(cus), dim3(64 * (F + 1)), lds, 0, a4, nst); };
        for (int w = 0; w < 3; ++w) launch();
        HC(hipDeviceSynchronize());
        const int reps = 20;
        HC(hipEventRecord(e0));
        for (int i = 0; i < reps; ++i) launch();
        HC(hipEventRecord(e1));
        HC(hipEventSynchronize(e1));
        float ms = 0;
        HC(hipEventElapsedTime(&ms, e0, e1));
        const double us = ms * 1e3 / reps, tbs = bytes / (us * 1e-6) / 1e12;
        const char* ok = "-";
        if (MODE >= 2) {
            std::vector<uint32_t> o(npk);
            HC(hipMemcpy(o.data(), dout, 4u * npk, hipMemcpyDeviceToHost));
            uint32_t bad = 0;
            for (uint32_t p = 0; p < npk; ++p) bad += o[p] != ref[p];
            ok = bad ? "MISMATCH" : "exact";
            if (bad) printf("#   %u mismatches, e.g. p0 %08x vs %08x\n", bad, o[0], ref[0]);
        }
        printf("lines4 F=%d D=%d mode=%d ntm=%d (%u stages): %8.2f us  %.3f TB/s = %.3f of 8  %s\n", F, D, MODE, NTM, nst, us,
               tbs, tbs / 8.0, ok);
        fflush(stdout);
    };
#define L4RUN(F, D, M, NTM) l4run(line4_kernel<F, D, M, NTM>, F, D, M, NTM, kRing + F * D * 2048)
#define H4RUN(F, D, M, NTM) l4run(hs4_kernel<F, D, M, NTM>, F, D, M, NTM, kRing + F * D * 2048 + 64)
    if (argc > 2 && atoi(argv[2]) == 6) {
        for (int rep = 0; rep < 2; ++rep) {
            H4RUN(15, 3, 2, 3); H4RUN(15, 3, 5, 3); H4RUN(15, 3, 6, 3);
            H4RUN(15, 3, 2, 2); H4RUN(15, 3, 5, 2); H4RUN(15, 3, 6, 2);
            H4RUN(12, 3, 5, 3); H4RUN(12, 3, 5, 2);
        }
        return 0;
    }
    if (argc > 2 && atoi(argv[2]) == 5) {
        for (int rep = 0; rep < 2; ++rep) {
            H4RUN(15, 3, 2, 3); H4RUN(15, 3, 4, 3); H4RUN(15, 3, 1, 3); H4RUN(15, 3, 2, 2);
            H4RUN(12, 3, 2, 3); H4RUN(12, 3, 4, 3);
            L4RUN(12, 3, 2, 3); L4RUN(12, 3, 1, 3); L4RUN(12, 3, 2, 2);
            // one cold launch after an idle gap
            hipDeviceSynchronize();
        }
        return 0;
    }
    if (argc > 2 && atoi(argv[2]) == 4) {
        for (int rep = 0; rep < 2; ++rep) {
            H4RUN(15, 3, 0, 2); H4RUN(15, 3, 1, 2); H4RUN(15, 3, 2, 2); H4RUN(15, 3, 4, 2); H4RUN(15, 3, 2, 0);
            H4RUN(12, 3, 0, 2); H4RUN(12, 3, 2, 2); H4RUN(11, 4, 0, 2); H4RUN(11, 4, 2, 2); H4RUN(8, 4, 2, 2);
            L4RUN(12, 3, 2, 2);
        }
        return 0;
    }
    if (argc > 2 && atoi(argv[2]) == 3) {
        for (int rep = 0; rep < 2; ++rep) {
            L4RUN(15, 3, 0, 2); L4RUN(15, 3, 1, 2); L4RUN(15, 3, 2, 2); L4RUN(15, 3, 2, 0); L4RUN(15, 3, 2, 1);
            L4RUN(12, 4, 0, 2); L4RUN(12, 4, 1, 2); L4RUN(12, 4, 2, 2); L4RUN(12, 4, 2, 0);
            L4RUN(8, 4, 2, 2); L4RUN(12, 3, 2, 2);
        }
        return 0;
    }
    if (argc > 2 && atoi(argv[2]) == 2) {
        for (int rep = 0; rep < 2; ++rep) {
            LRUN(4, 3, 0, 0); LRUN(4, 3, 0, 1); LRUN(4, 3, 0, 2);
            LRUN(4, 3, 1, 0); LRUN(4, 3, 1, 1); LRUN(4, 3, 1, 2);
            LRUN(4, 3, 2, 0); LRUN(4, 3, 2, 1); LRUN(4, 3, 2, 2);
            LRUN(4, 3, 3, 0); LRUN(4, 3, 3, 1); LRUN(4, 3, 3, 2);
        }
        return 0;
    }
    if (argc > 2 && atoi(argv[2]) == 1) {
        for (int nt = 0; nt < 2; ++nt) {
            if (nt) {
                SRUN(1, 32768, 3, 1, 5); SRUN(4, 8192, 3, 1, 5); SRUN(16, 2048, 3, 1, 5); SRUN(32, 1024, 3, 1, 5);
                SRUN(64, 512, 3, 1, 5); SRUN(128, 256, 3, 1, 5); SRUN(256, 128, 3, 1, 5);
                SRUN(16, 1024, 5, 1, 5); SRUN(64, 256, 5, 1, 5); SRUN(1, 16384, 5, 1, 5); SRUN(1, 32768, 3, 1, 1);
            } else {
                SRUN(1, 32768, 3, 0, 5); SRUN(4, 8192, 3, 0, 5); SRUN(16, 2048, 3, 0, 5); SRUN(32, 1024, 3, 0, 5);
                SRUN(64, 512, 3, 0, 5); SRUN(128, 256, 3, 0, 5); SRUN(256, 128, 3, 0, 5);
                SRUN(16, 1024, 5, 0, 5); SRUN(64, 256, 5, 0, 5); SRUN(1, 16384, 5, 0, 5); SRUN(1, 32768, 3, 0, 1);
            }
        }
        RUN(4, 4, 3, 0, 0); RUN(4, 4, 3, 1, 0); RUN(4, 2, 4, 0, 0); RUN(4, 2, 4, 1, 0);
        return 0;
    }
    for (int rep = 0; rep < 2; ++rep) {
        RUN(4, 4, 3, 0, 1); RUN(4, 4, 3, 1, 1); RUN(4, 4, 3, 2, 1); RUN(4, 4, 3, 2, 0);
        RUN(4, 2, 5, 0, 1); RUN(4, 2, 5, 1, 1); RUN(4, 2, 5, 2, 1); RUN(4, 2, 5, 2, 0);
        RUN(8, 2, 3, 0, 1); RUN(8, 2, 3, 1, 1); RUN(8, 2, 3, 2, 1); RUN(8, 2, 3, 2, 0);
        RUN(8, 1, 5, 0, 1); RUN(8, 1, 5, 1, 1); RUN(8, 1, 5, 2, 1); RUN(8, 1, 5, 2, 0);
        RUN(4, 2, 4, 2, 0); RUN(4, 1, 5, 2, 0);
    }
    return 0;
}
