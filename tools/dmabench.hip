// dmabench.hip -- measurement-only (NOT part of libenethip): the memory-side
// ceiling of an LDS-DMA streamed persistent kernel on gfx950, as a function of
// waves per CU, ring depth, per-instruction access pattern and cache policy.
// Every wave streams 2 KiB "stages" (two global_load_lds_dwordx4) through a ring
// of NB LDS slots with a CONSTANT s_waitcnt vmcnt((NB-1)*2), reads the landed
// stage back with two ds_read_b128 per lane and XORs it (minimal compute).
//   PAT 0: instruction i covers 1 KiB contiguous (lane l: +1024 i + 16 l)
//   PAT 1: instruction h covers every other 16-B piece (lane l: +32 l + 16 h)
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int N>
__device__ __forceinline__ void waitvm() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }

template <int W, int NB, int PAT, int AUX>
__global__ void __launch_bounds__(64 * W) k_dma(const uint8_t* buf, uint64_t units, uint32_t* sink, uint64_t* trace,
                                                const uint8_t* zero) {
    const uint64_t t_start = __builtin_amdgcn_s_memrealtime();
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t wv = (uint64_t)blockIdx.x * W + wave, wt = (uint64_t)gridDim.x * W;
    // PAT >= 2: units = groups, J = stages
    constexpr uint64_t kStg = PAT == 4 ? 3u : PAT >= 2 ? 5u : 1u;
    const uint64_t J = (wv < units ? (units - 1 - wv) / wt + 1 : 0) * kStg;
    const uint32_t ring = wave * NB * 2048u;
    auto issue = [&](uint64_t j, uint32_t slot) __attribute__((always_inline)) {
        const uint64_t jj = min(j, J - 1);
        const uint64_t u = wv + jj * wt;      // clamped: constant op count
        const uint8_t* base = buf + u * 2048u;
        // PAT >= 2: lean-kernel-like packet chunks.  Groups of 64/PL packets of
        // 1200 B packed; a group takes STG stages; stage s of packet p reads the
        // PL*32-byte chunk s of its window (window = lean's 16-B-aligned end, or for
        // PAT 3 a 128-B-aligned start); pieces wholly outside read a zero line.
        constexpr uint32_t PL = PAT == 4 ? 16u : 8u, NPK = 64u / PL;
        constexpr uint32_t NBW = PAT == 3 ? 40u : PAT == 5 ? 39u : 38u;   // window blocks of a 1200-B packet
        constexpr uint32_t STG = (NBW + PL - 1) / PL;
        const uint64_t grp = wv + (jj / STG) * wt, s = jj % STG;
        const uint32_t p = lane / PL, k = lane % PL;
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const uint8_t* g;
            if constexpr (PAT >= 2) {
                const uint64_t start = (grp * NPK + p) * 1200u;
                const uint64_t ws = PAT == 3 ? (start & ~127ull) : PAT == 5 ? (start & ~63ull) : (start >= 16u ? start - 16u : 0u);
                const uint32_t piece = (uint32_t)s * 2u * PL + i * PL + k;
                g = piece < 2u * NBW ? buf + ws + 16u * piece : zero;
            } else {
                g = PAT == 0 ? base + 1024u * i + 16u * lane : base + 32u * lane + 16u * i;
            }
            __builtin_amdgcn_global_load_lds(g, (__attribute__((address_space(3))) void*)(uintptr_t)(ring + slot * 2048u + 1024u * i),
                                             16, 0, AUX);
        }
    };
    if (!J) return;
    u32x4 acc = {0, 0, 0, 0};
#pragma unroll
    for (int s = 0; s < NB - 1; ++s) issue(s, s);
    uint64_t j = 0;
    for (;;) {
#pragma unroll
        for (int s = 0; s < NB; ++s) {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            issue(j + NB - 1, (s + NB - 1) % NB);
            waitvm<(NB - 1) * 2>();
            const uint32_t a0 = ring + s * 2048u + 16u * lane;
            acc ^= *(__attribute__((address_space(3))) const u32x4*)(uintptr_t)a0;
            acc ^= *(__attribute__((address_space(3))) const u32x4*)(uintptr_t)(a0 + 1024u);
            if (++j == J) goto done;
        }
    }
done:
    waitvm<0>();
    if (trace && (threadIdx.x & 63u) == 0u) {
        uint64_t* tr = trace + 4u * wv;
        tr[0] = t_start;
        tr[1] = t_start;
        tr[2] = __builtin_amdgcn_s_memrealtime();
        tr[3] = __builtin_amdgcn_s_getreg((31 << 11) | 4) | ((uint64_t)__builtin_amdgcn_s_getreg((31 << 11) | 20) << 32);
    }
    const uint32_t x = acc.x ^ acc.y ^ acc.z ^ acc.w;
    if (x == 0x9E3779B9u) sink[0] = x;
}

// plain coalesced probe (VGPR loads), persistent or oversubscribed grid
template <int T, int U>
__global__ void __launch_bounds__(T) k_probe(const uint8_t* b, uint64_t nvec, uint32_t* sink) {
    const u32x4* p = reinterpret_cast<const u32x4*>(b);
    u32x4 acc = {0u, 0u, 0u, 0u};
    const uint64_t stride = (uint64_t)gridDim.x * T;
    uint64_t i = (uint64_t)blockIdx.x * T + threadIdx.x;
    for (; i + (U - 1) * stride < nvec; i += U * stride) {
        u32x4 v[U];
#pragma unroll
        for (int k = 0; k < U; ++k) v[k] = p[i + k * stride];
#pragma unroll
        for (int k = 0; k < U; ++k) acc ^= v[k];
    }
    for (; i < nvec; i += stride) acc ^= p[i];
    const uint32_t x = acc.x ^ acc.y ^ acc.z ^ acc.w;
    if (x == 0x9E3779B9u) sink[0] = x;
}

static uint64_t* g_trace = nullptr;
extern "C" void db_trace(uint64_t* t) { g_trace = t; }
template <int W, int NB, int PAT, int AUX>
static int launch_dma(const void* buf, uint64_t bytes, int grid, uint32_t* sink, hipStream_t s) {
    const int lds = W * NB * 2048;
    static bool set = false;
    if (!set) {
        hipFuncSetAttribute((const void*)k_dma<W, NB, PAT, AUX>, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
        set = true;
    }
    static uint8_t* zero = nullptr;
    if (!zero) {
        hipMalloc(&zero, 4096);
        hipMemset(zero, 0, 4096);
    }
    const uint64_t units = PAT == 4 ? bytes / 4800 : PAT >= 2 ? bytes / 9600 : bytes / 2048;
    hipLaunchKernelGGL((k_dma<W, NB, PAT, AUX>), dim3(grid), dim3(64 * W), lds, s, (const uint8_t*)buf, units,
                       sink, g_trace, zero);
    return (int)hipGetLastError();
}

#define CASE(id, W, NB, PAT, AUX) \
    case id: return launch_dma<W, NB, PAT, AUX>(buf, bytes, grid, sink, s);

extern "C" int db_dma(int cfg, const void* buf, uint64_t bytes, int grid, uint32_t* sink, void* st) {
    hipStream_t s = (hipStream_t)st;
    switch (cfg) {
        CASE(0, 16, 2, 0, 0)
        CASE(1, 16, 3, 0, 0)
        CASE(2, 16, 4, 0, 0)
        CASE(3, 8, 4, 0, 0)
        CASE(4, 8, 6, 0, 0)
        CASE(5, 16, 2, 1, 0)
        CASE(6, 16, 3, 1, 0)
        CASE(7, 16, 4, 1, 0)
        CASE(8, 16, 3, 0, 2)
        CASE(9, 16, 3, 1, 2)
        CASE(10, 12, 4, 0, 0)
        CASE(11, 12, 4, 1, 0)
        CASE(12, 4, 8, 0, 0)
        CASE(13, 8, 8, 0, 0)
        CASE(14, 16, 2, 2, 0)
        CASE(15, 16, 2, 3, 0)
        CASE(16, 16, 2, 4, 0)
        CASE(17, 16, 2, 0, 2)
        CASE(18, 16, 2, 2, 2)
        CASE(19, 16, 2, 3, 2)
        CASE(20, 16, 3, 2, 0)
        CASE(21, 16, 3, 3, 0)
        CASE(22, 16, 2, 5, 0)
        CASE(23, 16, 3, 5, 0)
        CASE(24, 14, 3, 2, 0)
        CASE(25, 10, 4, 2, 0)
        default: return -1;
    }
}
extern "C" int db_ncfg() { return 26; }
extern "C" const char* db_name(int cfg) {
    static const char* n[] = {"W16 NB2 dense", "W16 NB3 dense", "W16 NB4 dense", "W8 NB4 dense", "W8 NB6 dense",
                              "W16 NB2 half", "W16 NB3 half", "W16 NB4 half", "W16 NB3 dense nt", "W16 NB3 half nt",
                              "W12 NB4 dense", "W12 NB4 half", "W4 NB8 dense", "W8 NB8 dense",
                              "W16 NB2 lean8", "W16 NB2 lean8 a128", "W16 NB2 lean16", "W16 NB2 dense nt",
                              "W16 NB2 lean8 nt", "W16 NB2 lean8 a128 nt", "W16 NB3 lean8", "W16 NB3 lean8 a128",
                              "W16 NB2 lean8 a64", "W16 NB3 lean8 a64", "W14 NB3 lean8", "W10 NB4 lean8"};
    return cfg < 26 ? n[cfg] : "?";
}

extern "C" int db_probe(int cfg, const void* buf, uint64_t bytes, int grid, uint32_t* sink, void* st) {
    hipStream_t s = (hipStream_t)st;
    const uint64_t nvec = bytes / 16;
    switch (cfg) {
        case 0: hipLaunchKernelGGL((k_probe<512, 4>), dim3(grid), dim3(512), 0, s, (const uint8_t*)buf, nvec, sink); break;
        case 1: hipLaunchKernelGGL((k_probe<1024, 4>), dim3(grid), dim3(1024), 0, s, (const uint8_t*)buf, nvec, sink); break;
        case 2: hipLaunchKernelGGL((k_probe<1024, 8>), dim3(grid), dim3(1024), 0, s, (const uint8_t*)buf, nvec, sink); break;
        case 3: hipLaunchKernelGGL((k_probe<256, 4>), dim3(grid), dim3(256), 0, s, (const uint8_t*)buf, nvec, sink); break;
        default: return -1;
    }
    return (int)hipGetLastError();
}
