// pipebench.hip -- measurement-only (NOT part of libenethip): the lean CRC
// kernel's memory pipeline with a realistic consumer, stripped of packet edges,
// to choose ring depth, table layout and window alignment on gfx950.
//
// Work = cfg2 (65536 packets x 1200 B packed); a group = 8 packets x 8 lanes;
// stage s of packet p = its window chunk s (256 B = pieces 16s..16s+15, lane k of
// the packet DMAs pieces k and 8 + k).  Consumer per stage and lane: 8
// ds_read_b32 of its 32-byte block (conflict-free dword permutation), then the
// slicing-by-32 fold (32 table lookups), exactly the lean kernel's op mix.
//   PAT 0: window = lean's (end on a 16-B granule: lz = 16 for cfg2)  5 stages
//   PAT 1: window start on a 64-B boundary                            5 stages
//   PAT 2: window start on a 128-B boundary                           6 stages
//   PAT 3: dense (stage = 2 KiB contiguous, no packet geometry)      5 stages
//   TB 0: 64 KiB image, address = one v_perm (the lean kernel's)
//   TB 1: 32 KiB image (row = 128 B), address = bfe + lshl_or
//   TB 2: no lookups (fold = XOR of the data)
//   META 1: each lane first loads its packets' offsets (the dependent metadata
//           read at the head of the lean kernel) and addresses from them
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) const uint32_t lds_u32;

template <int N>
__device__ __forceinline__ void waitvm() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }

__device__ __forceinline__ void dma16(const void* g, uint32_t lds_addr) {
    __builtin_amdgcn_global_load_lds(g, reinterpret_cast<__attribute__((address_space(3))) void*>(
                                            static_cast<uintptr_t>(lds_addr)), 16, 0, 0);
}
__device__ __forceinline__ uint32_t ldsr(uint32_t a) { return *reinterpret_cast<lds_u32*>(static_cast<uintptr_t>(a)); }
__device__ __forceinline__ void ldsw(uint32_t a, uint32_t v) {
    *reinterpret_cast<__attribute__((address_space(3))) uint32_t*>(static_cast<uintptr_t>(a)) = v;
}
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

constexpr uint32_t kPkt = 1200, kPk = 8, kP = 8;

template <int N, class F>
__device__ __forceinline__ void unroll_slots(F&& f) {
    if constexpr (N > 0) {
        unroll_slots<N - 1>(f);
        f(std::integral_constant<uint32_t, N - 1>{});
    }
}

// one 32-byte block: 32 lookups (TB 0/1) or a plain XOR (TB 2)
template <int TB>
__device__ __forceinline__ uint32_t fold(uint32_t reg, const uint32_t (&x)[8], const uint32_t (&col)[8],
                                         const uint32_t (&sel)[4]) {
    if constexpr (TB == 2) {
        return xor3(reg ^ x[0] ^ x[1], x[2] ^ x[3] ^ x[4], x[5] ^ x[6] ^ x[7]);
    } else {
        uint32_t d[8];
#pragma unroll
        for (int r = 0; r < 8; ++r) d[r] = r == 0 ? x[0] ^ reg : x[r];
        uint32_t v[32];
#pragma unroll
        for (int i = 0; i < 32; ++i) {
            uint32_t a;
            if constexpr (TB == 0) {
                a = __builtin_amdgcn_perm(d[i >> 2], col[i >> 2], sel[i & 3]);
            } else {
                const uint32_t c = (col[i >> 2] >> (8 * (i & 3))) & 0xFFu;
                a = (__builtin_amdgcn_ubfe(d[i >> 2], 8 * (i & 3), 8) << 7) | c;
            }
            v[i] = ldsr(a);
        }
        uint32_t acc = xor3(v[0], v[1], v[2]);
#pragma unroll
        for (int i = 3; i + 1 < 32; i += 2) acc = xor3(acc, v[i], v[i + 1]);
        return acc ^ v[31];
    }
}

template <int W, int NB, int PAT, int TB, int META>
struct Geo {
    static constexpr uint32_t kTable = TB == 0 ? 65536u : TB == 1 ? 32768u : 0u;
    static constexpr uint32_t kStg = PAT == 2 ? 6u : 5u;
    static constexpr uint32_t kLds = kTable + W * NB * 2048u;
    static_assert(kLds <= 160u * 1024u, "LDS");
};

template <int W, int NB, int PAT, int TB, int META>
__global__ void __launch_bounds__(64 * W) k_pipe(const uint8_t* buf, const uint64_t* offs, uint64_t ngroups,
                                                 const uint8_t* zero, uint32_t* sink) {
    using G = Geo<W, NB, PAT, TB, META>;
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t wv = (uint64_t)blockIdx.x * W + wave, wt = (uint64_t)gridDim.x * W;
    const uint32_t J = wv < ngroups ? (uint32_t)((ngroups - 1 - wv) / wt) + 1u : 0u;
    const uint32_t ring = G::kTable + wave * NB * 2048u;
    const uint32_t p = lane >> 3, k = lane & 7u;

    // metadata: this lane's packet start for each of its groups (J <= 2 here)
    // (named registers: a dynamically indexed private array gets promoted to
    // static LDS, which would sit under the absolute-addressed table and ring)
    auto start_of = [&](uint32_t j) __attribute__((always_inline)) -> uint64_t {
        const uint64_t g = wv + (uint64_t)min(j, J ? J - 1u : 0u) * wt;
        return META ? offs[g * kPk + p] : (g * kPk + p) * kPkt;
    };
    const uint64_t st0 = start_of(0), st1 = start_of(1);     // cfg2: J == 2 for every wave
    if (META) waitvm<0>();

    // table: every wave writes its share (stands in for the basis rebuild)
    if (TB != 2) {
        for (uint32_t i = threadIdx.x; i < G::kTable / 4u; i += 64u * W) ldsw(4u * i, i * 0x9E3779B1u);
    }

    auto issue = [&](uint32_t it, uint32_t slot) __attribute__((always_inline)) {
        const uint32_t jj = min(it, J * G::kStg - 1u);
        const uint32_t j = jj / G::kStg, s = jj % G::kStg;
        const uint64_t start = j ? st1 : st0;
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const uint8_t* g;
            if constexpr (PAT == 3) {
                const uint64_t grp = wv + (uint64_t)j * wt;
                g = buf + grp * kPk * kPkt + 2048u * s + 1024u * i + 16u * lane;
            } else {
                const uint64_t ws = PAT == 1 ? (start & ~63ull) : PAT == 2 ? (start & ~127ull)
                                                                            : (start >= 16u ? start - 16u : 0u);
                const uint64_t a = ws + 16u * (s * 16u + i * 8u + k);
                g = (a + 16u > start && a < start + kPkt) ? buf + a : zero;
            }
            dma16(g, ring + slot * 2048u + 1024u * i);
        }
    };
    if (!J || J > 2u) return;                        // st0/st1 cover two groups (cfg2: J == 2)
    const uint32_t total = J * G::kStg;
#pragma unroll
    for (int s = 0; s < NB - 1; ++s) issue(s, s);
    __syncthreads();                                   // table written

    // lane constants: conflict-free data dword permutation D, lookup columns
    const uint32_t l5 = lane & 31u;
    const uint32_t D = (lane >> 2) & 7u;
    uint32_t col[8], sel[4];
#pragma unroll
    for (int g = 0; g < 8; ++g) {
        uint32_t r = 0;
#pragma unroll
        for (int h = 0; h < 4; ++h) {
            const uint32_t t = ((4u * g + h) ^ l5) ^ 31u;
            r |= (TB == 0 ? (8u * t + 4u * (t >> 4)) : 4u * t) << (8 * h);
        }
        col[g] = r;
    }
#pragma unroll
    for (int h = 0; h < 4; ++h) sel[h] = (uint32_t)h | ((4u + (uint32_t)h) << 8) | 0x0C0C0000u;
    // the lane's block in a stage: packet p, block k of the 256-B chunk (pieces 2k, 2k+1
    // sit at 1024*(2k>=8) + 16*(8p + (2k & 7)))
    const uint32_t blk = 1024u * ((2u * k) >> 3) + 16u * (8u * p + ((2u * k) & 7u));

    uint32_t reg = 0xFFFFFFFFu;
    uint32_t it = 0;
    bool fin = false;
    auto iteration = [&](auto sc) __attribute__((always_inline)) {
        constexpr uint32_t S = decltype(sc)::value;
        if (fin) return;
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        issue(it + NB - 1, (S + NB - 1) % NB);
        waitvm<(NB - 1) * 2>();
        uint32_t x[8];
#pragma unroll
        for (int r = 0; r < 8; ++r) x[r] = ldsr(ring + S * 2048u + blk + 4u * ((r ^ D) & 3u) + 16u * ((r ^ D) >> 2));
        reg = fold<TB>(reg, x, col, sel);
        if (++it == total) fin = true;
    };
    while (!fin) unroll_slots<NB>(iteration);
    waitvm<0>();
    if (reg == 0x9E3779B9u) sink[0] = reg;
}

// VGPR ring variant: lane (p, k) loads its own 32-byte block k of the stage
// chunk straight into registers (two global_load_dwordx4, one ring slot = 8
// VGPRs), so LDS serves the table lookups only.  PAT as above (0..2).
typedef __attribute__((address_space(1))) const u32x4 gu32x4;
__device__ __forceinline__ u32x4 gld16(uint64_t a) { return *reinterpret_cast<gu32x4*>(static_cast<uintptr_t>(a)); }

template <int W, int NB, int PAT, int TB, int PERM>
__global__ void __launch_bounds__(64 * W) k_vpipe(const uint8_t* buf, const uint64_t* offs, uint64_t ngroups,
                                                  const uint8_t* zero, uint32_t* sink) {
    constexpr uint32_t kTable = TB == 0 ? 65536u : TB == 1 ? 32768u : 0u;
    constexpr uint32_t kStg = PAT == 2 ? 6u : 5u;
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t wv = (uint64_t)blockIdx.x * W + wave, wt = (uint64_t)gridDim.x * W;
    const uint32_t J = wv < ngroups ? (uint32_t)((ngroups - 1 - wv) / wt) + 1u : 0u;
    const uint32_t p = lane >> 3, k = lane & 7u;
    auto start_of = [&](uint32_t j) __attribute__((always_inline)) -> uint64_t {
        const uint64_t g = wv + (uint64_t)min(j, J ? J - 1u : 0u) * wt;
        return offs[g * kPk + p];
    };
    const uint64_t st0 = start_of(0), st1 = start_of(1);
    if (TB != 2) {
        for (uint32_t i = threadIdx.x; i < kTable / 4u; i += 64u * W) ldsw(4u * i, i * 0x9E3779B1u);
    }
    if (!J || J > 2u) return;
    const uint32_t total = J * kStg;
    u32x4 ra[NB], rb[NB];
    auto issue = [&](uint32_t it, auto slot_c) __attribute__((always_inline)) {
        constexpr uint32_t slot = decltype(slot_c)::value;
        const uint32_t jj = min(it, total - 1u);
        const uint32_t j = jj / kStg, s = jj % kStg;
        const uint64_t start = j ? st1 : st0;
        const uint64_t ws = PAT == 1 ? (start & ~63ull) : PAT == 2 ? (start & ~127ull) : (start >= 16u ? start - 16u : 0u);
        const uint64_t a = ws + 256u * s + 32u * k;
        const uint64_t base = reinterpret_cast<uint64_t>(buf);
        const uint64_t src = (a + 32u > start && a < start + kPkt) ? base + a : reinterpret_cast<uint64_t>(zero);
        ra[slot] = gld16(src);
        rb[slot] = gld16(src + 16u);
    };
    unroll_slots<NB - 1>([&](auto sc) __attribute__((always_inline)) { issue(decltype(sc)::value, sc); });
    __syncthreads();
    const uint32_t l5 = lane & 31u;
    uint32_t col[8], sel[4];
#pragma unroll
    for (int g = 0; g < 8; ++g) {
        uint32_t r = 0;
#pragma unroll
        for (int h = 0; h < 4; ++h) {
            const uint32_t t = ((4u * g + h) ^ l5) ^ 31u;
            r |= (TB == 0 ? (8u * t + 4u * (t >> 4)) : 4u * t) << (8 * h);
        }
        col[g] = r;
    }
#pragma unroll
    for (int h = 0; h < 4; ++h) sel[h] = (uint32_t)h | ((4u + (uint32_t)h) << 8) | 0x0C0C0000u;
    const uint32_t m1 = 0u - ((lane >> 2) & 1u), m2 = 0u - ((lane >> 3) & 1u);
    uint32_t reg = 0xFFFFFFFFu;
    uint32_t it = 0;
    bool fin = false;
    auto iteration = [&](auto sc) __attribute__((always_inline)) {
        constexpr uint32_t S = decltype(sc)::value;
        if (fin) return;
        issue(it + NB - 1, std::integral_constant<uint32_t, (S + NB - 1) % NB>{});
        uint32_t x[8] = {ra[S].x, ra[S].y, ra[S].z, ra[S].w, rb[S].x, rb[S].y, rb[S].z, rb[S].w};
        if constexpr (PERM) {
            // lane dword permutation x'[q] = x[q ^ D], D bits 0-1 by two select rounds
            // (bit 2 = which 16-B half is loaded first: free through the load address)
            uint32_t y[8];
#pragma unroll
            for (int q = 0; q < 8; ++q) y[q] = __builtin_amdgcn_bitop3_b32(x[q], x[q ^ 1], m1, 0xD8);
#pragma unroll
            for (int q = 0; q < 8; ++q) x[q] = __builtin_amdgcn_bitop3_b32(y[q], y[q ^ 2], m2, 0xD8);
        }
        reg = fold<TB>(reg, x, col, sel);
        if (++it == total) fin = true;
    };
    while (!fin) unroll_slots<NB>(iteration);
    if (reg == 0x9E3779B9u) sink[0] = reg;
}

template <int W, int NB, int PAT, int TB, int GRID, int PERM = 0>
static int vlaunch(const void* buf, const void* offs, uint64_t ngroups, const void* zero, uint32_t* sink,
                   hipStream_t s) {
    constexpr uint32_t kTable = TB == 0 ? 65536u : TB == 1 ? 32768u : 0u;
    static bool set = false;
    if (!set) {
        (void)hipFuncSetAttribute((const void*)k_vpipe<W, NB, PAT, TB, PERM>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  kTable);
        set = true;
    }
    hipLaunchKernelGGL((k_vpipe<W, NB, PAT, TB, PERM>), dim3(GRID), dim3(64 * W), kTable, s, (const uint8_t*)buf,
                       (const uint64_t*)offs, ngroups, (const uint8_t*)zero, sink);
    return (int)hipGetLastError();
}

template <int W, int NB, int PAT, int TB, int META>
static int launch(const void* buf, const void* offs, uint64_t ngroups, const void* zero, uint32_t* sink,
                  hipStream_t s) {
    using G = Geo<W, NB, PAT, TB, META>;
    static bool set = false;
    if (!set) {
        (void)hipFuncSetAttribute((const void*)k_pipe<W, NB, PAT, TB, META>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  G::kLds);
        set = true;
    }
    hipLaunchKernelGGL((k_pipe<W, NB, PAT, TB, META>), dim3(256), dim3(64 * W), G::kLds, s, (const uint8_t*)buf,
                       (const uint64_t*)offs, ngroups, (const uint8_t*)zero, sink);
    return (int)hipGetLastError();
}

#define VARIANTS(X)                        \
    X(0, 16, 2, 0, 0, 1, "lean-like")      \
    X(1, 16, 2, 0, 2, 1, "no lookups")     \
    X(2, 16, 2, 1, 0, 1, "a64")            \
    X(3, 16, 2, 2, 0, 1, "a128")           \
    X(4, 16, 2, 0, 0, 0, "no meta")        \
    X(5, 16, 3, 0, 1, 1, "T32K NB3")       \
    X(6, 16, 4, 0, 1, 1, "T32K NB4")       \
    X(7, 16, 3, 1, 1, 1, "a64 T32K NB3")   \
    X(8, 16, 4, 1, 1, 1, "a64 T32K NB4")   \
    X(9, 16, 2, 0, 1, 1, "T32K NB2")       \
    X(10, 16, 2, 3, 0, 0, "dense")         \
    X(11, 16, 3, 3, 1, 0, "dense T32K NB3") \
    X(12, 16, 3, 0, 0, 1, "NB3")           \
    X(13, 16, 3, 1, 0, 1, "a64 NB3")       \
    X(14, 16, 3, 3, 2, 0, "dense nolookup NB3")

#define VVARIANTS(X)                           \
    X(15, 16, 2, 1, 0, 256, "vgpr a64")        \
    X(16, 16, 3, 1, 0, 256, "vgpr a64")        \
    X(17, 16, 4, 1, 0, 256, "vgpr a64")        \
    X(18, 16, 3, 0, 0, 256, "vgpr lean")       \
    X(19, 8, 4, 1, 0, 512, "vgpr a64 2wg")     \
    X(20, 16, 3, 1, 2, 256, "vgpr a64 nolookup") \
    X(21, 8, 6, 1, 0, 512, "vgpr a64 2wg")     \
    X(22, 16, 6, 1, 0, 256, "vgpr a64")        \
    X(23, 16, 2, 1, 0, 256, "vgpr a64 perm")   \
    X(24, 16, 3, 1, 0, 256, "vgpr a64 perm")   \
    X(25, 16, 2, 1, 0, 512, "vgpr a64 2wg")    \
    X(26, 16, 3, 1, 0, 512, "vgpr a64 2wg")    \
    X(27, 16, 2, 1, 0, 512, "vgpr a64 perm 2wg") \
    X(28, 16, 3, 1, 0, 512, "vgpr a64 perm 2wg")

#define CASE(id, W, NB, PAT, TB, META, name) \
    case id: return launch<W, NB, PAT, TB, META>(buf, offs, ngroups, zero, sink, s);
#define NAME(id, W, NB, PAT, TB, META, name) name " W" #W " NB" #NB,
#define VCASE(id, W, NB, PAT, TB, GRID, name) \
    case id: return vlaunch<W, NB, PAT, TB, GRID, id == 23 || id == 24 || id >= 27>(buf, offs, ngroups, zero, sink, s);
#define VNAME(id, W, NB, PAT, TB, GRID, name) name " W" #W " NB" #NB " grid" #GRID,

extern "C" int pb_run(int cfg, const void* buf, const void* offs, uint64_t ngroups, const void* zero, uint32_t* sink,
                      void* st) {
    hipStream_t s = (hipStream_t)st;
    switch (cfg) {
        VARIANTS(CASE)
        VVARIANTS(VCASE)
        default: return -1;
    }
}
static const char* kNames[] = {VARIANTS(NAME) VVARIANTS(VNAME)};
extern "C" int pb_ncfg() { return (int)(sizeof(kNames) / sizeof(kNames[0])); }
extern "C" const char* pb_name(int cfg) { return cfg < pb_ncfg() ? kNames[cfg] : "?"; }
