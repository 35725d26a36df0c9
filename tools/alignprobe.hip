// alignprobe.hip -- measurement only: does gfx950 stream global_load_dwordx4 at
// addresses off a 16-byte boundary as fast as aligned ones?  (An end-aligned CRC
// window -- its last block ending on the packet's last byte, so no trailing zero
// bytes to undo -- reads every 16-B piece at the packet's end alignment.)
// Grid-stride over a resident buffer, 16 B per lane, 4 loads in flight per lane,
// the base shifted by `shift` bytes; every kernel XOR-reduces what it reads into a
// never-taken sink store.  Also the packet shape of the vring kernel (4 lanes per
// packet, lane k reading pieces 32 k and 32 k + 16 of each 128-B stage) with the
// windows 64-B aligned (as the kernel) or ending on packed packets' ends.
//   hipcc --offload-arch=gfx950 -O3 -o alignprobe tools/alignprobe.hip && ./alignprobe
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <vector>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ u32x4 ld16(const uint8_t* a) { return *reinterpret_cast<const u32x4*>(a); }

__global__ void __launch_bounds__(256) ap_stride(const uint8_t* p, uint64_t nvec, uint32_t shift, uint32_t* sink) {
    u32x4 acc = {0u, 0u, 0u, 0u};
    const uint64_t stride = static_cast<uint64_t>(gridDim.x) * 256u;
    uint64_t i = static_cast<uint64_t>(blockIdx.x) * 256u + threadIdx.x;
    const uint8_t* b = p + shift;
    for (; i + 3 * stride < nvec; i += 4 * stride) {
        const u32x4 v0 = ld16(b + 16 * i), v1 = ld16(b + 16 * (i + stride)), v2 = ld16(b + 16 * (i + 2 * stride)),
                    v3 = ld16(b + 16 * (i + 3 * stride));
        acc ^= v0 ^ v1 ^ v2 ^ v3;
    }
    const uint32_t x = acc.x ^ acc.y ^ acc.z ^ acc.w;
    if (x == 0x9E3779B9u) sink[0] = x;
}

// packets: starts s[j], window of nb blocks from w[j] (any alignment); 16 packets per
// wave (4 lanes each), a wave's group = 16 consecutive packets, stage t: lane k reads
// the two 16-B pieces of block k + 4 t
template <int P>
__global__ void __launch_bounds__(256) ap_packets(const uint8_t* p, const uint64_t* w, const uint32_t* nb,
                                                  uint64_t n, uint32_t* sink) {
    constexpr uint32_t kPk = 64 / P;
    u32x4 acc = {0u, 0u, 0u, 0u};
    const uint32_t lane = threadIdx.x & 63u, k = lane % P, pk = lane / P;
    const uint64_t waves = static_cast<uint64_t>(gridDim.x) * 4u;
    for (uint64_t g = static_cast<uint64_t>(blockIdx.x) * 4u + (threadIdx.x >> 6); g * kPk < n; g += waves) {
        const uint64_t j = g * kPk + pk;
        const bool live = j < n;
        const uint64_t ws = live ? w[j] : 0u;
        const uint32_t m = live ? nb[j] : 0u;
        uint32_t ms = m;                                  // the group's stage count: the max block count
        for (int o = P; o < 64; o <<= 1) ms = max(ms, static_cast<uint32_t>(__shfl_xor(static_cast<int>(ms), o)));
        const uint32_t st = (ms + P - 1u) / P;
        for (uint32_t t = 0; t < st; ++t) {
            const uint32_t blk = k + P * t;
            if (blk < m) acc ^= ld16(p + ws + 32u * blk) ^ ld16(p + ws + 32u * blk + 16u);
        }
    }
    const uint32_t x = acc.x ^ acc.y ^ acc.z ^ acc.w;
    if (x == 0x9E3779B9u) sink[0] = x;
}

int main(int argc, char** argv) {
    const uint64_t bytes = 768ull << 20;
    uint8_t* d;
    uint32_t* sink;
    hipMalloc(&d, bytes + 4096);
    hipMemset(d, 1, bytes + 4096);
    hipMalloc(&sink, 64);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    // packet launches read at d + region: consecutive launches rotate over `nreg` copies
    // of the packet span (set below), so a span smaller than the 256 MB MALL is read cold
    uint64_t region = 0, span = bytes, nreg = 1;
    auto timeit = [&](auto fn, double B, const char* what) {
        for (int r = 0; r < 3; ++r) fn();
        hipDeviceSynchronize();
        hipEventRecord(e0);
        const int reps = 20;
        for (int r = 0; r < reps; ++r) {
            region = (r % nreg) * span;
            fn();
        }
        region = 0;
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        printf("%-58s %7.3f TB/s (%.1f us per launch)\n", what, B * reps / (ms * 1e-3) / 1e12, ms * 1e3 / reps);
    };
    const uint64_t nvec = bytes / 16;
    for (uint32_t sh : {0u, 1u, 4u, 8u, 13u}) {
        char name[96];
        snprintf(name, sizeof name, "linear grid-stride, 16 B/lane, base + %u B", sh);
        timeit([&] { hipLaunchKernelGGL(ap_stride, dim3(256 * 8), dim3(256), 0, 0, d, nvec, sh, sink); },
               static_cast<double>(nvec) * 16, name);
    }
    // cfg3-like packed packets: lengths U[64, 1400], 1 M of them (~ 766 MB) unless argv[1] says
    const uint64_t n = argc > 1 ? strtoull(argv[1], nullptr, 10) : 1000000;   // cfg3: 262144
    std::vector<uint32_t> len(n);
    uint64_t s = 0x4C454E53ull;
    uint64_t tot = 0;
    for (uint64_t j = 0; j < n; ++j) {
        s = s * 6364136223846793005ull + 1442695040888963407ull;
        len[j] = 64u + static_cast<uint32_t>((s >> 33) % 1337u);
        tot += len[j];
    }
    if (tot + 256 > bytes) return 1;
    span = (tot + 256 + 4095) / 4096 * 4096;
    nreg = bytes / span;
    printf("%llu packets, %.1f MB, %llu rotating copies\n", static_cast<unsigned long long>(n), tot / 1e6,
           static_cast<unsigned long long>(nreg));
    std::vector<uint64_t> wa(n), we(n);
    std::vector<uint32_t> na(n), ne(n);
    uint64_t off = 64;
    for (uint64_t j = 0; j < n; ++j) {
        const uint64_t lz = off & 63u;                      // 64-B aligned window start (the vring kernel)
        wa[j] = off - lz;
        na[j] = static_cast<uint32_t>((lz + len[j] + 31u) / 32u);
        const uint32_t nbe = (len[j] + 31u) / 32u;          // end-aligned window: ends at the packet's end
        we[j] = off + len[j] - 32ull * nbe;
        ne[j] = nbe;
        off += len[j];
    }
    uint64_t *dw;
    uint32_t *dn;
    hipMalloc(&dw, 8 * n);
    hipMalloc(&dn, 4 * n);
    for (int v = 0; v < 2; ++v) {
        hipMemcpy(dw, v ? we.data() : wa.data(), 8 * n, hipMemcpyHostToDevice);
        hipMemcpy(dn, v ? ne.data() : na.data(), 4 * n, hipMemcpyHostToDevice);
        timeit([&] { hipLaunchKernelGGL(ap_packets<4>, dim3(256 * 4), dim3(256), 0, 0, d + region, dw, dn, n, sink); },
               static_cast<double>(tot),
               v ? "packets (4 lanes, 16/wave), windows ending on packet ends" : "packets (4 lanes, 16/wave), 64-B aligned windows");
    }
    // lanes per packet, 64-B aligned windows (packets in memory order: neighbours share lines)
    hipMemcpy(dw, wa.data(), 8 * n, hipMemcpyHostToDevice);
    hipMemcpy(dn, na.data(), 4 * n, hipMemcpyHostToDevice);
    timeit([&] { hipLaunchKernelGGL(ap_packets<1>, dim3(256 * 4), dim3(256), 0, 0, d + region, dw, dn, n, sink); },
           static_cast<double>(tot), "packets (1 lane, 64/wave), 64-B aligned windows");
    timeit([&] { hipLaunchKernelGGL(ap_packets<2>, dim3(256 * 4), dim3(256), 0, 0, d + region, dw, dn, n, sink); },
           static_cast<double>(tot), "packets (2 lanes, 32/wave), 64-B aligned windows");
    timeit([&] { hipLaunchKernelGGL(ap_packets<8>, dim3(256 * 4), dim3(256), 0, 0, d + region, dw, dn, n, sink); },
           static_cast<double>(tot), "packets (8 lanes, 8/wave), 64-B aligned windows");
    // the same in a shuffled packet order (binned records: neighbours in other groups)
    {
        std::vector<uint64_t> ws2(wa);
        std::vector<uint32_t> ns2(na);
        uint64_t r = 12345;
        for (uint64_t j = n - 1; j > 0; --j) {
            r = r * 6364136223846793005ull + 1442695040888963407ull;
            const uint64_t q = (r >> 33) % (j + 1);
            std::swap(ws2[j], ws2[q]);
            std::swap(ns2[j], ns2[q]);
        }
        hipMemcpy(dw, ws2.data(), 8 * n, hipMemcpyHostToDevice);
        hipMemcpy(dn, ns2.data(), 4 * n, hipMemcpyHostToDevice);
        timeit([&] { hipLaunchKernelGGL(ap_packets<2>, dim3(256 * 4), dim3(256), 0, 0, d + region, dw, dn, n, sink); },
               static_cast<double>(tot), "shuffled packets, 2 lanes");
        timeit([&] { hipLaunchKernelGGL(ap_packets<4>, dim3(256 * 4), dim3(256), 0, 0, d + region, dw, dn, n, sink); },
               static_cast<double>(tot), "shuffled packets, 4 lanes");
        timeit([&] { hipLaunchKernelGGL(ap_packets<8>, dim3(256 * 4), dim3(256), 0, 0, d + region, dw, dn, n, sink); },
               static_cast<double>(tot), "shuffled packets, 8 lanes");
    }
    // the binned records' order (crc32_lean.hip bin_tile_kernel): each tile of `tile`
    // packets sorted by window length (32-B bins, longest first, stable inside a bin),
    // group q of tile t placed at q * T + t (rank-interleaved) or left tile-local
    for (uint64_t tile : {1024ull, 512ull, 256ull, 128ull}) {
        for (int inter = 1; inter >= 0; --inter) {
            const uint64_t kpk = 16, T = n / tile;             // full tiles; the ragged rest stays in order
            std::vector<uint64_t> ws2(wa);
            std::vector<uint32_t> ns2(na);
            std::vector<uint64_t> idx(tile);
            for (uint64_t t = 0; t < T; ++t) {
                for (uint64_t i = 0; i < tile; ++i) idx[i] = t * tile + i;
                std::stable_sort(idx.begin(), idx.end(), [&](uint64_t a, uint64_t b) { return na[a] > na[b]; });
                for (uint64_t sr = 0; sr < tile; ++sr) {
                    const uint64_t dst = inter ? ((sr / kpk) * T + t) * kpk + sr % kpk : t * tile + sr;
                    ws2[dst] = wa[idx[sr]];
                    ns2[dst] = na[idx[sr]];
                }
            }
            hipMemcpy(dw, ws2.data(), 8 * n, hipMemcpyHostToDevice);
            hipMemcpy(dn, ns2.data(), 4 * n, hipMemcpyHostToDevice);
            char name[96];
            snprintf(name, sizeof name, "binned order, 4 lanes, tile %llu, %s", static_cast<unsigned long long>(tile),
                     inter ? "rank-interleaved" : "tile-local");
            timeit([&] { hipLaunchKernelGGL(ap_packets<4>, dim3(256 * 4), dim3(256), 0, 0, d + region, dw, dn, n, sink); },
                   static_cast<double>(tot), name);
        }
    }
    return 0;
}
