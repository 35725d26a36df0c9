// dealprobe.hip -- measurement only: how fast does the chip stream cfg3's packets
// (lengths U[64, 1400], packed) in the length-binned order under two deals?
//   global: the product's records order -- tiles of 1024 packets sorted by window
//           length, rank-interleaved (group q T + t), workgroup k's round r = groups
//           16 k' + w + 16 G r with k' = k, or G - 1 - k on odd rounds (crc32_vring.hip);
//   local:  workgroup k owns the packets [k n / G, (k + 1) n / G), sorted by window length
//           (one tile per workgroup, binned inside the records kernel's own launch);
//           wave w takes its tile's groups 16 r + w, reversed (16 r + 15 - w) on odd rounds.
// The kernel is the packet shape of the records instance (4 lanes per packet, 16
// packets a group, a stage = lane k's two 16-B pieces of block k + 4 t), 16-wave
// workgroups, one or two per CU; every wave reads its own group list from a schedule.
// Consecutive launches rotate over copies of the arena so every launch reads HBM.
//   hipcc --offload-arch=gfx950 -O3 -o tools/dealprobe tools/dealprobe.hip && tools/dealprobe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ u32x4 ld16(const uint8_t* a) { return *reinterpret_cast<const u32x4*>(a); }

// sched[(blk * 16 + wave) * R + r] = the group of the wave's round r (~0u: none)
__global__ void __launch_bounds__(1024) dp_sched(const uint8_t* p, const uint64_t* w, const uint32_t* nb, uint64_t n,
                                                 const uint32_t* sched, uint32_t R, uint32_t* sink) {
    constexpr uint32_t P = 4, kPk = 16;
    u32x4 acc = {0u, 0u, 0u, 0u};
    const uint32_t lane = threadIdx.x & 63u, k = lane % P, pk = lane / P;
    const uint32_t wave = threadIdx.x >> 6;
    const uint32_t* s = sched + (static_cast<uint64_t>(blockIdx.x) * 16u + wave) * R;
    for (uint32_t r = 0; r < R; ++r) {
        const uint32_t g = s[r];
        if (g == ~0u) break;
        const uint64_t j = static_cast<uint64_t>(g) * kPk + pk;
        const bool live = j < n;
        const uint64_t ws = live ? w[j] : 0u;
        const uint32_t m = live ? nb[j] : 0u;
        uint32_t ms = m;
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
    const uint64_t n = argc > 1 ? strtoull(argv[1], nullptr, 10) : 262144;   // cfg3
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    std::vector<uint32_t> len(n);
    uint64_t s = 0x4C454E53ull, tot = 0;
    for (uint64_t j = 0; j < n; ++j) {
        s = s * 6364136223846793005ull + 1442695040888963407ull;
        len[j] = 64u + static_cast<uint32_t>((s >> 33) % 1337u);
        tot += len[j];
    }
    const uint64_t span = (tot + 256 + 4095) / 4096 * 4096, ncopy = 5;
    uint8_t* d;
    uint32_t* sink;
    if (hipMalloc(&d, span * ncopy) != hipSuccess) return 1;
    hipMemset(d, 1, span * ncopy);
    hipMalloc(&sink, 64);
    std::vector<uint64_t> wa(n);
    std::vector<uint32_t> na(n);
    uint64_t off = 64;
    for (uint64_t j = 0; j < n; ++j) {
        const uint64_t lz = off & 63u;
        wa[j] = off - lz;
        na[j] = static_cast<uint32_t>((lz + len[j] + 31u) / 32u);
        off += len[j];
    }
    printf("%llu packets, %.1f MB, %llu rotating copies, %d CUs\n", static_cast<unsigned long long>(n), tot / 1e6,
           static_cast<unsigned long long>(ncopy), cus);
    uint64_t *dw;
    uint32_t *dn, *ds;
    hipMalloc(&dw, 8 * n);
    hipMalloc(&dn, 4 * n);
    hipMalloc(&ds, 4ull * 16 * 2 * cus * ((n + 15) / 16 + 64));
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    auto run = [&](const std::vector<uint64_t>& w2, const std::vector<uint32_t>& n2, const std::vector<uint32_t>& sch,
                   uint32_t G, uint32_t R, const char* what) {
        hipMemcpy(dw, w2.data(), 8 * n, hipMemcpyHostToDevice);
        hipMemcpy(dn, n2.data(), 4 * n, hipMemcpyHostToDevice);
        hipMemcpy(ds, sch.data(), 4 * sch.size(), hipMemcpyHostToDevice);
        for (int rep = 0; rep < 3; ++rep) {
            for (int r = 0; r < 3; ++r)
                hipLaunchKernelGGL(dp_sched, dim3(G), dim3(1024), 0, 0, d + (r % ncopy) * span, dw, dn, n, ds, R, sink);
            hipDeviceSynchronize();
            const int reps = 40;
            float best = 1e30f, sum = 0;
            for (int r = 0; r < reps; ++r) {          // each launch timed alone (serial, cold copy)
                hipEventRecord(e0);
                hipLaunchKernelGGL(dp_sched, dim3(G), dim3(1024), 0, 0, d + (r % ncopy) * span, dw, dn, n, ds, R, sink);
                hipEventRecord(e1);
                hipEventSynchronize(e1);
                float ms = 0;
                hipEventElapsedTime(&ms, e0, e1);
                best = std::min(best, ms);
                sum += ms;
            }
            printf("%-64s mean %6.1f us (%.3f TB/s), best %6.1f us\n", what, sum * 1e3 / reps,
                   tot / (sum / reps * 1e-3) / 1e12, best * 1e3);
        }
    };
    for (uint32_t per : {2u, 1u}) {                  // workgroups per CU
        const uint32_t G = per * cus;
        // global: tiles of 1024 sorted, rank-interleaved, snake deal over G workgroups
        {
            const uint64_t tile = 1024, kpk = 16, T = n / tile;
            std::vector<uint64_t> w2(wa);
            std::vector<uint32_t> n2(na);
            std::vector<uint64_t> idx(tile);
            for (uint64_t t = 0; t < T; ++t) {
                for (uint64_t i = 0; i < tile; ++i) idx[i] = t * tile + i;
                std::stable_sort(idx.begin(), idx.end(), [&](uint64_t a, uint64_t b) { return na[a] > na[b]; });
                for (uint64_t sr = 0; sr < tile; ++sr) {
                    const uint64_t dst = ((sr / kpk) * T + t) * kpk + sr % kpk;
                    w2[dst] = wa[idx[sr]];
                    n2[dst] = na[idx[sr]];
                }
            }
            const uint64_t groups = (n + 15) / 16, wt = 16ull * G;
            const uint32_t R = static_cast<uint32_t>((groups + wt - 1) / wt);
            std::vector<uint32_t> sch(static_cast<uint64_t>(G) * 16 * R, ~0u);
            for (uint32_t k = 0; k < G; ++k)
                for (uint32_t wv = 0; wv < 16; ++wv)
                    for (uint32_t r = 0; r < R; ++r) {
                        const uint64_t kk = (r & 1u) ? G - 1u - k : k;
                        const uint64_t g = kk * 16 + wv + r * wt;
                        sch[(static_cast<uint64_t>(k) * 16 + wv) * R + r] = g < groups ? static_cast<uint32_t>(g) : ~0u;
                    }
            char name[96];
            snprintf(name, sizeof name, "global: tiles of 1024, rank-interleaved, snake, %u WG/CU", per);
            run(w2, n2, sch, G, R, name);
        }
        // local: workgroup k sorts its own n / G packets; waves snake over its groups
        {
            const uint64_t per_wg = (n + G - 1) / G, gpw = (per_wg + 15) / 16;
            std::vector<uint64_t> w2(n, 0);
            std::vector<uint32_t> n2(n, 0);
            // record slots: workgroup k's records at [k gpw 16, ...), padding past its packets
            std::vector<uint64_t> w3(static_cast<uint64_t>(G) * gpw * 16, 0);
            std::vector<uint32_t> n3(static_cast<uint64_t>(G) * gpw * 16, 0);
            for (uint32_t k = 0; k < G; ++k) {
                const uint64_t a = k * per_wg, b = std::min<uint64_t>(n, a + per_wg);
                std::vector<uint64_t> idx;
                for (uint64_t i = a; i < b; ++i) idx.push_back(i);
                std::stable_sort(idx.begin(), idx.end(), [&](uint64_t x, uint64_t y) { return na[x] > na[y]; });
                for (uint64_t sr = 0; sr < idx.size(); ++sr) {
                    w3[k * gpw * 16 + sr] = wa[idx[sr]];
                    n3[k * gpw * 16 + sr] = na[idx[sr]];
                }
            }
            const uint32_t R = static_cast<uint32_t>((gpw + 15) / 16);
            std::vector<uint32_t> sch(static_cast<uint64_t>(G) * 16 * R, ~0u);
            for (uint32_t k = 0; k < G; ++k)
                for (uint32_t wv = 0; wv < 16; ++wv)
                    for (uint32_t r = 0; r < R; ++r) {
                        const uint64_t j = 16ull * r + ((r & 1u) ? 15u - wv : wv);
                        sch[(static_cast<uint64_t>(k) * 16 + wv) * R + r] =
                            j < gpw ? static_cast<uint32_t>(k * gpw + j) : ~0u;
                    }
            // (the probe's record arrays hold n entries: the local layout needs G gpw 16)
            if (w3.size() > n) {
                printf("local layout needs %zu records (> n): skipped\n", w3.size());
                continue;
            }
            std::copy(w3.begin(), w3.end(), w2.begin());
            std::copy(n3.begin(), n3.end(), n2.begin());
            char name[96];
            snprintf(name, sizeof name, "local: %llu packets per WG sorted, snake waves, %u WG/CU",
                     static_cast<unsigned long long>(per_wg), per);
            run(w2, n2, sch, G, R, name);
        }
    }
    return 0;
}
