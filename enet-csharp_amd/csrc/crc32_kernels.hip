// crc32_kernels.hip -- gfx950 (MI355X, CDNA4) kernels of libenethip and the
// C-ABI entry points that launch them.  See DESIGN.md for the derivation.
//
// Path replaced: ENet.enet_crc32 (/root/reference/enet-csharp/ENet/c/packet.cs:142-160)
// applied to a whole batch of DGRAMs at once.  Bit-exact with the reference: the
// kernels compute the same Sarwate register (packet.cs:153) by a different but
// algebraically identical route.
//
// Work decomposition (one launch, persistent grid):
//   * a TASK is one lane x one packet segment: packet p is split over P = 2^lg
//     consecutive lanes (lanes_per_packet); each lane runs its share of the
//     packet's 32-byte blocks, then the P partial registers are combined with
//     the GF(2) carry-combine  reg(A||B) = reg(A) (*) x^(8|B|)  ^  reg(B)
//     and an XOR across the P lanes (__shfl_xor).
//   * a packet of L bytes is processed as an END-aligned window of nb = ceil(L/32)
//     blocks; the r' = 32*nb - L bytes in front of the packet are treated as zero
//     and the register starts at INIT[r'] (the state that r' zero bytes carry to
//     0xFFFFFFFF, packet.cs:144), so no per-packet tail loop is needed.
//   * each 32-byte block is folded with slicing-by-32: 32 independent table
//     lookups T_{31-m}[byte_m ^ state_m] XORed together.  The 32 tables live in
//     LDS (64 KiB) in a layout where, for every lookup instruction, the 32 lanes
//     of a half-wave hit 32 different banks (conflict-free; DESIGN.md "LDS table
//     layout"): lane l handles byte m = i ^ (l & 15) at step i, table t = m ^ 31
//     sits in bank column 2t + ((l >> 4) & 1) of a 256-byte row indexed by the
//     byte value, and one v_perm_b32 builds the LDS address from the data byte.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

#include "crc32_math.hpp"
#include "enet_hip.h"

namespace enethip {

constexpr int kThreads = 512;                      // workgroup size (8 waves)
constexpr int kLdsImageBytes = 256 * 64 * 4;       // 256 rows x 64 dwords = 64 KiB
constexpr int kXnEntries = 65536;                  // x^(8n) for n < 65536 (+ high part)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

struct KernelTables {
    const uint32_t* image;  // kLdsImageBytes, copied into LDS by every workgroup
    const uint32_t* xn_lo;  // x^(8n) mod P, n < 65536
    const uint32_t* xn_hi;  // x^(8*65536*q) mod P, q < 65536
    const uint32_t* init;   // INIT[r], r < 32
};

// ------------------------------------------------------------------ device helpers

__device__ __forceinline__ u32x4 ldg16(const uint8_t* p) {
    u32x4 v;
    __builtin_memcpy(&v, p, 16);  // global_load_dwordx4 (unaligned access mode on gfx950)
    return v;
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

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

// Per-lane constants of the conflict-free slicing-by-32 schedule.
struct LaneSched {
    uint32_t col[8];  // byte h of col[g]: LDS column byte offset for step i = 4g + h
    uint32_t sel[4];  // v_perm selector for steps with i & 3 == h
    bool swap1, swap2;
};

__device__ __forceinline__ LaneSched make_sched(uint32_t lane) {
    LaneSched s;
    const uint32_t v = lane & 15u, c = (lane >> 4) & 1u;
#pragma unroll
    for (int g = 0; g < 8; ++g) {
        uint32_t r = 0;
#pragma unroll
        for (int h = 0; h < 4; ++h) {
            const uint32_t i = 4u * g + h;
            const uint32_t t = (i ^ v) ^ 31u;        // table of byte m = i ^ v
            r |= (8u * t + 4u * c) << (8 * h);       // dword column 2t + c
        }
        s.col[g] = r;
    }
#pragma unroll
    for (int h = 0; h < 4; ++h)
        s.sel[h] = static_cast<uint32_t>(h) | ((4u + (static_cast<uint32_t>(h) ^ (v & 3u))) << 8) | 0x0C0C0000u;
    s.swap1 = (v >> 2) & 1u;
    s.swap2 = (v >> 3) & 1u;
    return s;
}

// One 32-byte block folded into register `reg` (== 32 Sarwate steps, packet.cs:153).
__device__ __forceinline__ uint32_t fold_block(uint32_t reg, u32x4 h0, u32x4 h1, const uint8_t* lds,
                                               const LaneSched& s) {
    uint32_t w[8] = {h0.x ^ reg, h0.y, h0.z, h0.w, h1.x, h1.y, h1.z, h1.w};
    uint32_t x[8], d[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) x[q] = s.swap1 ? w[q ^ 1] : w[q];
#pragma unroll
    for (int q = 0; q < 8; ++q) d[q] = s.swap2 ? x[q ^ 2] : x[q];
    uint32_t v[32];
#pragma unroll
    for (int i = 0; i < 32; ++i) {
        const uint32_t addr = __builtin_amdgcn_perm(d[i >> 2], s.col[i >> 2], s.sel[i & 3]);
        v[i] = *reinterpret_cast<const uint32_t*>(lds + addr);
    }
    uint32_t acc = xor3(v[0], v[1], v[2]);
#pragma unroll
    for (int i = 3; i + 1 < 32; i += 2) acc = xor3(acc, v[i], v[i + 1]);
    return acc ^ v[31];
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

// Register after feeding blocks [j0, j1) of the end-aligned window of packet
// bytes [a, a+L), starting from `reg`.  nb = ceil(L/32), rp = 32*nb - L.
// 4-deep register prefetch ring (software pipeline over HBM latency).
__device__ __forceinline__ uint32_t fold_window(uint32_t reg, const uint8_t* a, uint32_t L, uint32_t nb,
                                                uint32_t j0, uint32_t j1, const uint8_t* lds,
                                                const LaneSched& s) {
    const uint8_t* W = a + L - (static_cast<size_t>(nb) << 5);
    uint32_t j = j0;
    const bool head = (j == 0) && (j < j1) && ((nb << 5) != L);
    if (head) j = 1;
    u32x4 r0a = {}, r0b = {}, r1a = {}, r1b = {}, r2a = {}, r2b = {}, r3a = {}, r3b = {};
    if (j + 0 < j1) { r0a = ldg16(W + 32 * (j + 0)); r0b = ldg16(W + 32 * (j + 0) + 16); }
    if (j + 1 < j1) { r1a = ldg16(W + 32 * (j + 1)); r1b = ldg16(W + 32 * (j + 1) + 16); }
    if (j + 2 < j1) { r2a = ldg16(W + 32 * (j + 2)); r2b = ldg16(W + 32 * (j + 2) + 16); }
    if (j + 3 < j1) { r3a = ldg16(W + 32 * (j + 3)); r3b = ldg16(W + 32 * (j + 3) + 16); }
    if (head) {
        const u32x4 ha = ldg16_head(W, a), hb = ldg16_head(W + 16, a);
        reg = fold_block(reg, ha, hb, lds, s);
    }
    while (j < j1) {
        reg = fold_block(reg, r0a, r0b, lds, s);
        if (j + 4 < j1) { r0a = ldg16(W + 32 * (j + 4)); r0b = ldg16(W + 32 * (j + 4) + 16); }
        if (++j >= j1) break;
        reg = fold_block(reg, r1a, r1b, lds, s);
        if (j + 4 < j1) { r1a = ldg16(W + 32 * (j + 4)); r1b = ldg16(W + 32 * (j + 4) + 16); }
        if (++j >= j1) break;
        reg = fold_block(reg, r2a, r2b, lds, s);
        if (j + 4 < j1) { r2a = ldg16(W + 32 * (j + 4)); r2b = ldg16(W + 32 * (j + 4) + 16); }
        if (++j >= j1) break;
        reg = fold_block(reg, r3a, r3b, lds, s);
        if (j + 4 < j1) { r3a = ldg16(W + 32 * (j + 4)); r3b = ldg16(W + 32 * (j + 4) + 16); }
        ++j;
    }
    return reg;
}

__device__ __forceinline__ void fill_lds(uint8_t* lds, const uint32_t* image) {
    const u32x4* src = reinterpret_cast<const u32x4*>(image);
    u32x4* dst = reinterpret_cast<u32x4*>(lds);
#pragma unroll 4
    for (int i = threadIdx.x; i < kLdsImageBytes / 16; i += kThreads) dst[i] = src[i];
    __syncthreads();
}

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
};

// MODE 0: out[p] = enet_crc32(packet p).  MODE 1: receive verify.
template <int MODE>
__global__ void __launch_bounds__(kThreads) crc32_packets_kernel(PacketArgs pa, KernelTables tb) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    fill_lds(lds, tb.image);
    const uint32_t lane = threadIdx.x & 63u;
    const LaneSched s = make_sched(lane);
    const uint32_t P = 1u << pa.lg;
    const uint64_t total = pa.n << pa.lg;
    const uint64_t stride = static_cast<uint64_t>(gridDim.x) * kThreads;
    for (uint64_t base = static_cast<uint64_t>(blockIdx.x) * kThreads + (threadIdx.x & ~63u); base < total;
         base += stride) {
        const uint64_t t = base + lane;
        const bool active = t < total;
        const uint64_t pk = t >> pa.lg;
        const uint32_t k = static_cast<uint32_t>(t) & (P - 1u);
        uint32_t L = 0;
        const uint8_t* a = pa.bytes;
        if (active) {
            L = pa.len[pk];
            a = pa.bytes + pa.off[pk];
        }
        const uint32_t nb = (L + 31u) >> 5;
        const uint32_t rp = (nb << 5) - L;
        const uint32_t per = nb >> pa.lg, rem = nb & (P - 1u);
        const uint32_t j0 = k * per + min(k, rem);
        const uint32_t j1 = j0 + per + (k < rem ? 1u : 0u);
        uint32_t reg = (k == 0) ? tb.init[rp] : 0u;
        reg = fold_window(reg, a, L, nb, j0, j1, lds, s);
        const uint32_t after = nb - j1;
        if (after) reg = mulmod(reg, x8n_dev(after << 5, tb));
        for (uint32_t m = 1; m < P; m <<= 1) reg ^= __shfl_xor(reg, static_cast<int>(m));
        if (active && k == 0) {
            if (MODE == 0) {
                pa.out[pk] = finalize(reg);
            } else {
                // protocol.cs:1052-1068: desired = slot; slot := connectID; crc over the
                // DGRAM; keep iff equal.  By linearity the substitution adds
                // (slot ^ connectID) fed at byte offset so, followed by L-so zero bytes.
                const uint32_t so = pa.slot_off[pk];
                uint32_t comp = 0;
                uint8_t okv = 0;
                if (so <= L && L - so >= 4u) {
                    uint32_t desired;
                    __builtin_memcpy(&desired, a + so, 4);
                    const uint32_t delta = desired ^ pa.connect[pk];
                    const uint32_t fixed = reg ^ mulmod(delta, x8n_dev(L - so, tb));
                    comp = finalize(fixed);
                    okv = (comp == desired) ? 1 : 0;
                }
                pa.ok[pk] = okv;
                if (pa.out) pa.out[pk] = comp;
            }
        }
    }
}

struct GatherArgs {
    const uint8_t* bytes;
    const uint64_t* seg_off;
    const uint32_t* seg_len;
    const uint32_t* seg_first;
    uint64_t n;
    uint32_t* out;
};

// One lane per DGRAM; segments folded in order and joined by the carry-combine.
__global__ void __launch_bounds__(kThreads) crc32_gather_kernel(GatherArgs ga, KernelTables tb) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    fill_lds(lds, tb.image);
    const LaneSched s = make_sched(threadIdx.x & 63u);
    const uint64_t stride = static_cast<uint64_t>(gridDim.x) * kThreads;
    for (uint64_t d = static_cast<uint64_t>(blockIdx.x) * kThreads + threadIdx.x; d < ga.n; d += stride) {
        const uint32_t s0 = ga.seg_first[d], s1 = ga.seg_first[d + 1];
        uint32_t reg = 0xFFFFFFFFu;
        bool first = true;
        for (uint32_t q = s0; q < s1; ++q) {
            const uint32_t L = ga.seg_len[q];
            if (L == 0) continue;
            const uint8_t* a = ga.bytes + ga.seg_off[q];
            const uint32_t nb = (L + 31u) >> 5;
            const uint32_t rp = (nb << 5) - L;
            if (first) {
                reg = fold_window(tb.init[rp], a, L, nb, 0, nb, lds, s);
                first = false;
            } else {
                const uint32_t part = fold_window(0u, a, L, nb, 0, nb, lds, s);
                reg = mulmod(reg, x8n_dev(L, tb)) ^ part;
            }
        }
        ga.out[d] = finalize(reg);
    }
}

// Read-roofline probe: every byte loaded once by 16-byte coalesced loads,
// 4 loads in flight per lane, XOR-folded so nothing is dead code.
__global__ void __launch_bounds__(kThreads) read_probe_kernel(const uint8_t* bytes, uint64_t nvec, uint32_t* sink) {
    const u32x4* p = reinterpret_cast<const u32x4*>(bytes);
    u32x4 acc = {0u, 0u, 0u, 0u};
    const uint64_t stride = static_cast<uint64_t>(gridDim.x) * kThreads;
    uint64_t i = static_cast<uint64_t>(blockIdx.x) * kThreads + threadIdx.x;
    for (; i + 3 * stride < nvec; i += 4 * stride) {
        const u32x4 a = p[i], b = p[i + stride], c = p[i + 2 * stride], d = p[i + 3 * stride];
        acc ^= a ^ b ^ c ^ d;
    }
    for (; i < nvec; i += stride) acc ^= p[i];
    const uint32_t x = acc.x ^ acc.y ^ acc.z ^ acc.w;
    if (x == 0x9E3779B9u) sink[0] = x;  // practically never taken; keeps the loads live
}

}  // namespace enethip

// =================================================================== host side

using namespace enethip;

struct enet_hip_context {
    int device = 0;
    int num_cus = 256;
    hipStream_t stream = nullptr;
    uint32_t* d_image = nullptr;
    uint32_t* d_xn = nullptr;    // lo[65536] | hi[65536]
    uint32_t* d_init = nullptr;  // 32
    int lanes_per_packet = 0;    // 0 = auto
    int wgs_per_cu = 0;          // 0 = auto
    // staging for the host-memory entry points
    std::mutex mu;
    uint8_t* d_bytes = nullptr;
    size_t d_bytes_cap = 0;
    uint8_t* d_meta = nullptr;  // off | len | out
    size_t d_meta_cap = 0;
};

namespace {

int herr(hipError_t e) { return e == hipSuccess ? 0 : -static_cast<int>(e); }

#define ENH_CHECK(expr)                 \
    do {                                \
        hipError_t e_ = (expr);         \
        if (e_ != hipSuccess) return herr(e_); \
    } while (0)

struct HostTables {
    std::vector<uint32_t> image, xn, init;
    HostTables() : image(kLdsImageBytes / 4), xn(2 * kXnEntries), init(32) {
        // slicing tables T_t[j] = byte j followed by t zero bytes (t < 32)
        static uint32_t T[32][256];
        for (uint32_t j = 0; j < 256; ++j) T[0][j] = crc_table_entry(j);
        for (int t = 1; t < 32; ++t)
            for (uint32_t j = 0; j < 256; ++j) T[t][j] = (T[t - 1][j] >> 8) ^ T[0][T[t - 1][j] & 0xFFu];
        for (uint32_t j = 0; j < 256; ++j)
            for (uint32_t t = 0; t < 32; ++t)
                for (uint32_t c = 0; c < 2; ++c) image[j * 64 + 2 * t + c] = T[t][j];
        // x^(8n) for n < 65536: one zero-byte step per n
        xn[0] = kOneReflected;
        for (int n = 1; n < kXnEntries; ++n) xn[n] = sarwate_step(xn[n - 1], 0);
        const uint32_t x64k = sarwate_step(xn[kXnEntries - 1], 0);  // x^(8*65536)
        xn[kXnEntries] = kOneReflected;
        for (int q = 1; q < kXnEntries; ++q) xn[kXnEntries + q] = gf2_mulmod(xn[kXnEntries + q - 1], x64k);
        init[0] = 0xFFFFFFFFu;
        for (int r = 1; r < 32; ++r) init[r] = unstep_zero(init[r - 1]);
    }
};

const HostTables& host_tables() {
    static const HostTables t;
    return t;
}

int auto_lanes(const enet_hip_context* ctx) { return ctx->lanes_per_packet > 0 ? ctx->lanes_per_packet : 4; }

int log2i(int v) {
    int l = 0;
    while ((1 << l) < v) ++l;
    return l;
}

KernelTables tables_of(const enet_hip_context* ctx) {
    return KernelTables{ctx->d_image, ctx->d_xn, ctx->d_xn + kXnEntries, ctx->d_init};
}

unsigned grid_for(const enet_hip_context* ctx, uint64_t tasks) {
    const int per_cu = ctx->wgs_per_cu > 0 ? ctx->wgs_per_cu : 2;
    const uint64_t cap = static_cast<uint64_t>(ctx->num_cus) * per_cu;
    const uint64_t need = (tasks + kThreads - 1) / kThreads;
    return static_cast<unsigned>(std::max<uint64_t>(1, std::min(need, cap)));
}

int launch_packets(enet_hip_context* ctx, int mode, const PacketArgs& pa, hipStream_t st) {
    if (pa.n == 0) return 0;
    const uint64_t tasks = pa.n << pa.lg;
    const unsigned grid = grid_for(ctx, tasks);
    if (mode == 0)
        hipLaunchKernelGGL(crc32_packets_kernel<0>, dim3(grid), dim3(kThreads), kLdsImageBytes, st, pa, tables_of(ctx));
    else
        hipLaunchKernelGGL(crc32_packets_kernel<1>, dim3(grid), dim3(kThreads), kLdsImageBytes, st, pa, tables_of(ctx));
    return herr(hipGetLastError());
}

int ensure(uint8_t** p, size_t* cap, size_t need) {
    if (*cap >= need) return 0;
    if (*p) ENH_CHECK(hipFree(*p));
    *p = nullptr;
    *cap = 0;
    size_t sz = std::max<size_t>(need, 1 << 20);
    ENH_CHECK(hipMalloc(reinterpret_cast<void**>(p), sz));
    *cap = sz;
    return 0;
}

}  // namespace

extern "C" {

int enet_hip_device_count(int* count) {
    if (!count) return -static_cast<int>(hipErrorInvalidValue);
    int c = 0;
    hipError_t e = hipGetDeviceCount(&c);
    *count = (e == hipSuccess) ? c : 0;
    return herr(e);
}

const char* enet_hip_error_string(int code) {
    if (code == 0) return "success";
    if (code > 0) return "unknown";
    return hipGetErrorString(static_cast<hipError_t>(-code));
}

int enet_hip_context_create(int device, enet_hip_context** out) {
    if (!out) return -static_cast<int>(hipErrorInvalidValue);
    *out = nullptr;
    int ndev = 0;
    ENH_CHECK(hipGetDeviceCount(&ndev));
    if (device < 0 || device >= ndev) return -static_cast<int>(hipErrorInvalidDevice);
    ENH_CHECK(hipSetDevice(device));
    auto* ctx = new enet_hip_context();
    ctx->device = device;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) == hipSuccess && prop.multiProcessorCount > 0)
        ctx->num_cus = prop.multiProcessorCount;
    const HostTables& ht = host_tables();
    int rc = 0;
    do {
        if ((rc = herr(hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking)))) break;
        if ((rc = herr(hipMalloc(reinterpret_cast<void**>(&ctx->d_image), kLdsImageBytes)))) break;
        if ((rc = herr(hipMalloc(reinterpret_cast<void**>(&ctx->d_xn), ht.xn.size() * 4)))) break;
        if ((rc = herr(hipMalloc(reinterpret_cast<void**>(&ctx->d_init), 32 * 4)))) break;
        if ((rc = herr(hipMemcpy(ctx->d_image, ht.image.data(), kLdsImageBytes, hipMemcpyHostToDevice)))) break;
        if ((rc = herr(hipMemcpy(ctx->d_xn, ht.xn.data(), ht.xn.size() * 4, hipMemcpyHostToDevice)))) break;
        if ((rc = herr(hipMemcpy(ctx->d_init, ht.init.data(), 32 * 4, hipMemcpyHostToDevice)))) break;
        if ((rc = herr(hipFuncSetAttribute(reinterpret_cast<const void*>(crc32_packets_kernel<0>),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, kLdsImageBytes)))) break;
        if ((rc = herr(hipFuncSetAttribute(reinterpret_cast<const void*>(crc32_packets_kernel<1>),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, kLdsImageBytes)))) break;
        if ((rc = herr(hipFuncSetAttribute(reinterpret_cast<const void*>(crc32_gather_kernel),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, kLdsImageBytes)))) break;
    } while (0);
    if (rc) {
        enet_hip_context_destroy(ctx);
        return rc;
    }
    *out = ctx;
    return 0;
}

int enet_hip_context_destroy(enet_hip_context* ctx) {
    if (!ctx) return 0;
    (void)hipSetDevice(ctx->device);
    if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
    (void)hipFree(ctx->d_image);
    (void)hipFree(ctx->d_xn);
    (void)hipFree(ctx->d_init);
    (void)hipFree(ctx->d_bytes);
    (void)hipFree(ctx->d_meta);
    if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
    delete ctx;
    return 0;
}

int enet_hip_set_tuning(enet_hip_context* ctx, int lanes_per_packet, int workgroups_per_cu) {
    if (!ctx) return -static_cast<int>(hipErrorInvalidValue);
    if (lanes_per_packet < 0 || lanes_per_packet > 64 || (lanes_per_packet & (lanes_per_packet - 1)))
        return -static_cast<int>(hipErrorInvalidValue);
    if (workgroups_per_cu < 0 || workgroups_per_cu > 8) return -static_cast<int>(hipErrorInvalidValue);
    ctx->lanes_per_packet = lanes_per_packet;
    ctx->wgs_per_cu = workgroups_per_cu;
    return 0;
}

int enet_hip_crc32_batch_device(enet_hip_context* ctx, const uint8_t* bytes, const uint64_t* offsets,
                                const uint32_t* lengths, size_t count, uint32_t* out, void* stream) {
    if (!ctx) return -static_cast<int>(hipErrorInvalidValue);
    if (count == 0) return 0;
    if (!bytes || !offsets || !lengths || !out) return -static_cast<int>(hipErrorInvalidValue);
    ENH_CHECK(hipSetDevice(ctx->device));
    PacketArgs pa{};
    pa.bytes = bytes;
    pa.off = offsets;
    pa.len = lengths;
    pa.n = count;
    pa.lg = static_cast<uint32_t>(log2i(auto_lanes(ctx)));
    pa.out = out;
    return launch_packets(ctx, 0, pa, stream ? static_cast<hipStream_t>(stream) : ctx->stream);
}

int enet_hip_verify_batch_device(enet_hip_context* ctx, const uint8_t* bytes, const uint64_t* offsets,
                                 const uint32_t* lengths, const uint32_t* slotOffsets, const uint32_t* connectIds,
                                 size_t count, uint8_t* ok, uint32_t* computed, void* stream) {
    if (!ctx) return -static_cast<int>(hipErrorInvalidValue);
    if (count == 0) return 0;
    if (!bytes || !offsets || !lengths || !slotOffsets || !connectIds || !ok)
        return -static_cast<int>(hipErrorInvalidValue);
    ENH_CHECK(hipSetDevice(ctx->device));
    PacketArgs pa{};
    pa.bytes = bytes;
    pa.off = offsets;
    pa.len = lengths;
    pa.n = count;
    pa.lg = static_cast<uint32_t>(log2i(auto_lanes(ctx)));
    pa.out = computed;
    pa.slot_off = slotOffsets;
    pa.connect = connectIds;
    pa.ok = ok;
    return launch_packets(ctx, 1, pa, stream ? static_cast<hipStream_t>(stream) : ctx->stream);
}

int enet_hip_crc32_gather_device(enet_hip_context* ctx, const uint8_t* bytes, const uint64_t* segOffsets,
                                 const uint32_t* segLengths, const uint32_t* segFirst, size_t dgramCount,
                                 uint32_t* out, void* stream) {
    if (!ctx) return -static_cast<int>(hipErrorInvalidValue);
    if (dgramCount == 0) return 0;
    if (!bytes || !segOffsets || !segLengths || !segFirst || !out) return -static_cast<int>(hipErrorInvalidValue);
    ENH_CHECK(hipSetDevice(ctx->device));
    GatherArgs ga{bytes, segOffsets, segLengths, segFirst, dgramCount, out};
    const unsigned grid = grid_for(ctx, dgramCount);
    hipLaunchKernelGGL(crc32_gather_kernel, dim3(grid), dim3(kThreads), kLdsImageBytes,
                       stream ? static_cast<hipStream_t>(stream) : ctx->stream, ga, tables_of(ctx));
    return herr(hipGetLastError());
}

int enet_hip_crc32_batch_host(enet_hip_context* ctx, const uint8_t* bytes, size_t byteCount,
                              const uint64_t* offsets, const uint32_t* lengths, size_t count, uint32_t* out) {
    if (!ctx) return -static_cast<int>(hipErrorInvalidValue);
    if (count == 0) return 0;
    if (!bytes || !offsets || !lengths || !out) return -static_cast<int>(hipErrorInvalidValue);
    for (size_t i = 0; i < count; ++i)  // host-side shape check before any launch
        if (offsets[i] > byteCount || lengths[i] > byteCount - offsets[i]) return -static_cast<int>(hipErrorInvalidValue);
    std::lock_guard<std::mutex> lk(ctx->mu);
    ENH_CHECK(hipSetDevice(ctx->device));
    int rc;
    if ((rc = ensure(&ctx->d_bytes, &ctx->d_bytes_cap, byteCount + 16))) return rc;
    const size_t meta = count * (8 + 4 + 4) + 64;
    if ((rc = ensure(&ctx->d_meta, &ctx->d_meta_cap, meta))) return rc;
    uint64_t* d_off = reinterpret_cast<uint64_t*>(ctx->d_meta);
    uint32_t* d_len = reinterpret_cast<uint32_t*>(ctx->d_meta + count * 8);
    uint32_t* d_out = reinterpret_cast<uint32_t*>(ctx->d_meta + count * 12);
    hipStream_t st = ctx->stream;
    ENH_CHECK(hipMemcpyAsync(ctx->d_bytes, bytes, byteCount, hipMemcpyHostToDevice, st));
    ENH_CHECK(hipMemcpyAsync(d_off, offsets, count * 8, hipMemcpyHostToDevice, st));
    ENH_CHECK(hipMemcpyAsync(d_len, lengths, count * 4, hipMemcpyHostToDevice, st));
    PacketArgs pa{};
    pa.bytes = ctx->d_bytes;
    pa.off = d_off;
    pa.len = d_len;
    pa.n = count;
    pa.lg = static_cast<uint32_t>(log2i(auto_lanes(ctx)));
    pa.out = d_out;
    if ((rc = launch_packets(ctx, 0, pa, st))) return rc;
    ENH_CHECK(hipMemcpyAsync(out, d_out, count * 4, hipMemcpyDeviceToHost, st));
    ENH_CHECK(hipStreamSynchronize(st));
    return 0;
}

int enet_hip_crc32_batch_multi(enet_hip_context* const* contexts, int contextCount, const uint8_t* bytes,
                               size_t byteCount, const uint64_t* offsets, const uint32_t* lengths, size_t count,
                               uint32_t* out) {
    if (!contexts || contextCount <= 0) return -static_cast<int>(hipErrorInvalidValue);
    if (count == 0) return 0;
    if (!bytes || !offsets || !lengths || !out) return -static_cast<int>(hipErrorInvalidValue);
    for (int i = 0; i < contextCount; ++i)
        if (!contexts[i]) return -static_cast<int>(hipErrorInvalidValue);
    std::vector<int> rcs(contextCount, 0);
    std::vector<std::thread> th;
    for (int i = 0; i < contextCount; ++i) {
        th.emplace_back([&, i]() {
            const size_t lo = count * static_cast<size_t>(i) / contextCount;
            const size_t hi = count * static_cast<size_t>(i + 1) / contextCount;
            if (hi == lo) return;
            // rebase this shard's offsets onto the byte span it touches
            uint64_t bmin = UINT64_MAX, bmax = 0;
            for (size_t p = lo; p < hi; ++p) {
                bmin = std::min<uint64_t>(bmin, offsets[p]);
                bmax = std::max<uint64_t>(bmax, offsets[p] + lengths[p]);
            }
            if (bmax > byteCount) { rcs[i] = -static_cast<int>(hipErrorInvalidValue); return; }
            std::vector<uint64_t> off(hi - lo);
            for (size_t p = lo; p < hi; ++p) off[p - lo] = offsets[p] - bmin;
            rcs[i] = enet_hip_crc32_batch_host(contexts[i], bytes + bmin, bmax - bmin, off.data(), lengths + lo,
                                               hi - lo, out + lo);
        });
    }
    for (auto& t : th) t.join();
    for (int rc : rcs)
        if (rc) return rc;
    return 0;
}

int enet_hip_read_probe_device(enet_hip_context* ctx, const uint8_t* bytes, size_t byteCount, uint32_t* sink,
                               void* stream) {
    if (!ctx || !bytes || !sink || (reinterpret_cast<uintptr_t>(bytes) & 15u))
        return -static_cast<int>(hipErrorInvalidValue);
    ENH_CHECK(hipSetDevice(ctx->device));
    const uint64_t nvec = byteCount / 16;
    if (nvec == 0) return 0;
    const unsigned grid = static_cast<unsigned>(std::min<uint64_t>((nvec + kThreads - 1) / kThreads,
                                                                   static_cast<uint64_t>(ctx->num_cus) * 8));
    hipLaunchKernelGGL(read_probe_kernel, dim3(grid), dim3(kThreads), 0,
                       stream ? static_cast<hipStream_t>(stream) : ctx->stream, bytes, nvec, sink);
    return herr(hipGetLastError());
}

int enet_hip_device_alloc(enet_hip_context* ctx, size_t bytes, void** out) {
    if (!ctx || !out) return -static_cast<int>(hipErrorInvalidValue);
    ENH_CHECK(hipSetDevice(ctx->device));
    return herr(hipMalloc(out, bytes ? bytes : 1));
}
int enet_hip_device_free(enet_hip_context* ctx, void* ptr) {
    if (!ctx) return -static_cast<int>(hipErrorInvalidValue);
    ENH_CHECK(hipSetDevice(ctx->device));
    return herr(hipFree(ptr));
}
int enet_hip_host_alloc(size_t bytes, void** out) {
    if (!out) return -static_cast<int>(hipErrorInvalidValue);
    return herr(hipHostMalloc(out, bytes ? bytes : 1, hipHostMallocDefault));
}
int enet_hip_host_free(void* ptr) { return herr(hipHostFree(ptr)); }
int enet_hip_memcpy_h2d(enet_hip_context* ctx, void* dst, const void* src, size_t bytes) {
    if (!ctx) return -static_cast<int>(hipErrorInvalidValue);
    ENH_CHECK(hipSetDevice(ctx->device));
    return herr(hipMemcpy(dst, src, bytes, hipMemcpyHostToDevice));
}
int enet_hip_memcpy_d2h(enet_hip_context* ctx, void* dst, const void* src, size_t bytes) {
    if (!ctx) return -static_cast<int>(hipErrorInvalidValue);
    ENH_CHECK(hipSetDevice(ctx->device));
    return herr(hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost));
}
int enet_hip_synchronize(enet_hip_context* ctx) {
    if (!ctx) return -static_cast<int>(hipErrorInvalidValue);
    ENH_CHECK(hipSetDevice(ctx->device));
    ENH_CHECK(hipStreamSynchronize(ctx->stream));
    return herr(hipDeviceSynchronize());
}

}  // extern "C"
