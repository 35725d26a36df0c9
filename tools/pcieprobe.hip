// pcieprobe.hip -- measurement only: where a small in-place receive verify's
// kernel time goes.  Kernel durations by HIP events (median of 500 launches, each its own
// event pair) of:
//   empty      -- an empty kernel, one workgroup of 512 threads;
//   lds64k     -- the workgroup copies a 64 KiB table from device memory into LDS;
//   host_rd    -- 8 waves each read one 1200-B row of PINNED HOST memory (all loads at once)
//                 and write one byte back to pinned memory;
//   dev_rd     -- the same rows in device memory;
//   host_rd256 -- 256 rows (32 workgroups) of pinned host memory;
//   host_wr    -- only the byte writes to pinned memory.
//   hipcc --offload-arch=gfx950 -O2 -o tools/pcieprobe tools/pcieprobe.hip && tools/pcieprobe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__global__ void k_empty(uint32_t* out) {
    if (threadIdx.x == 1023u) out[0] = 1;
}

__global__ void k_lds(const u32x4* tab, uint32_t* out) {
    extern __shared__ u32x4 lds[];
    for (uint32_t q = threadIdx.x; q < 4096u; q += blockDim.x) lds[q] = tab[q];
    __syncthreads();
    if (threadIdx.x == 0) out[0] = lds[77].x;
}

// wave w of block b reads row (8 b + w): 1200 B = 75 granules, lanes 0..74 one each (two
// rounds of 64 lanes), then lane 0 writes the XOR of the wave's first dword to flag[row]
__global__ void k_rows(const uint8_t* rows, uint64_t stride, uint8_t* flag, uint32_t n, int write_only) {
    const uint32_t row = blockIdx.x * 8u + (threadIdx.x >> 6), lane = threadIdx.x & 63u;
    if (row >= n) return;
    uint32_t acc = 0;
    if (!write_only) {
        const u32x4* p = reinterpret_cast<const u32x4*>(rows + row * stride);
        const u32x4 a = p[lane];
        const u32x4 b = lane + 64u < 75u ? p[lane + 64u] : u32x4{0u, 0u, 0u, 0u};
        acc = a.x ^ a.y ^ b.z ^ b.w;
    }
    for (int o = 32; o > 0; o >>= 1) acc ^= __shfl_xor(acc, o);
    if (lane == 0) flag[row] = static_cast<uint8_t>(acc | 1u);
}

template <typename F>
static double median_us(hipStream_t st, F launch) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    std::vector<float> t;
    for (int r = 0; r < 560; ++r) {
        (void)hipEventRecord(e0, st);
        launch();
        (void)hipEventRecord(e1, st);
        (void)hipEventSynchronize(e1);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, e0, e1);
        if (r >= 60) t.push_back(ms * 1e3f);
    }
    std::sort(t.begin(), t.end());
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    return t[t.size() / 2];
}

int main() {
    hipStream_t st;
    if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) return 1;
    uint32_t* out = nullptr;
    u32x4* tab = nullptr;
    uint8_t *hrows = nullptr, *drows = nullptr, *hflag = nullptr, *dflag = nullptr;
    const uint64_t stride = 4096;
    if (hipMalloc(&out, 64) || hipMalloc(&tab, 65536) || hipMalloc(&drows, 256 * stride) ||
        hipHostMalloc(&hrows, 256 * stride, hipHostMallocDefault) || hipHostMalloc(&hflag, 4096, hipHostMallocDefault) ||
        hipMalloc(&dflag, 4096))
        return 1;
    (void)hipMemset(tab, 1, 65536);
    (void)hipMemset(drows, 2, 256 * stride);
    for (uint64_t i = 0; i < 256 * stride; ++i) hrows[i] = static_cast<uint8_t>(i * 7);
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(k_lds), hipFuncAttributeMaxDynamicSharedMemorySize, 65536);
    uint8_t* hf = nullptr;
    uint8_t* hr = nullptr;
    (void)hipHostGetDevicePointer(reinterpret_cast<void**>(&hf), hflag, 0);
    (void)hipHostGetDevicePointer(reinterpret_cast<void**>(&hr), hrows, 0);
    struct Case {
        const char* name;
        double us;
    };
    std::vector<Case> cs;
    cs.push_back({"empty (1 x 512 threads)", median_us(st, [&] { hipLaunchKernelGGL(k_empty, dim3(1), dim3(512), 0, st, out); })});
    cs.push_back({"lds64k (64 KiB device -> LDS)", median_us(st, [&] { hipLaunchKernelGGL(k_lds, dim3(1), dim3(512), 65536, st, tab, out); })});
    cs.push_back({"dev_rd 8 rows, flag in device memory", median_us(st, [&] { hipLaunchKernelGGL(k_rows, dim3(1), dim3(512), 0, st, drows, stride, dflag, 8u, 0); })});
    cs.push_back({"dev_rd 8 rows, flag in pinned host", median_us(st, [&] { hipLaunchKernelGGL(k_rows, dim3(1), dim3(512), 0, st, drows, stride, hf, 8u, 0); })});
    cs.push_back({"host_wr only: 8 flags to pinned host", median_us(st, [&] { hipLaunchKernelGGL(k_rows, dim3(1), dim3(512), 0, st, hr, stride, hf, 8u, 1); })});
    cs.push_back({"host_rd 8 rows (pinned), flag device", median_us(st, [&] { hipLaunchKernelGGL(k_rows, dim3(1), dim3(512), 0, st, hr, stride, dflag, 8u, 0); })});
    cs.push_back({"host_rd 8 rows (pinned), flag pinned", median_us(st, [&] { hipLaunchKernelGGL(k_rows, dim3(1), dim3(512), 0, st, hr, stride, hf, 8u, 0); })});
    cs.push_back({"host_rd 256 rows (pinned), flag pinned", median_us(st, [&] { hipLaunchKernelGGL(k_rows, dim3(32), dim3(512), 0, st, hr, stride, hf, 256u, 0); })});
    cs.push_back({"dev_rd 256 rows, flag device", median_us(st, [&] { hipLaunchKernelGGL(k_rows, dim3(32), dim3(512), 0, st, drows, stride, dflag, 256u, 0); })});
    for (const Case& c : cs) std::printf("{\"case\": \"%s\", \"median_us\": %.2f}\n", c.name, c.us);
    return 0;
}
