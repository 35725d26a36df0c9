// launchprobe.hip -- measurement only (the receive call's fixed cost): what a
// launch of an almost empty kernel costs the host (hipLaunchKernel) and a launch + stream
// sync round trip, against the size of its by-value kernel arguments (the vring kernels
// take a batch-list struct of about 2.3-3 KB).  One line per argument size.
//   hipcc --offload-arch=gfx950 -O2 -o tools/launchprobe tools/launchprobe.hip && tools/launchprobe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <vector>

template <int N>
struct Args {
    unsigned int v[N / 4];
};

template <int N>
__global__ void probe_kernel(Args<N> a, unsigned int* out) {
    if (threadIdx.x == 0 && blockIdx.x == 0) out[0] = a.v[0] + a.v[N / 4 - 1];
}

static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

template <int N>
static void run(hipStream_t st, unsigned int* out, int blocks) {
    Args<N> a{};
    for (int i = 0; i < N / 4; ++i) a.v[i] = i;
    std::vector<double> launch, trip;
    for (int r = 0; r < 2200; ++r) {
        const double t0 = now_us();
        hipLaunchKernelGGL(probe_kernel<N>, dim3(blocks), dim3(64), 0, st, a, out);
        const double t1 = now_us();
        (void)hipStreamSynchronize(st);
        const double t2 = now_us();
        if (r >= 200) {
            launch.push_back(t1 - t0);
            trip.push_back(t2 - t0);
        }
    }
    std::sort(launch.begin(), launch.end());
    std::sort(trip.begin(), trip.end());
    std::printf("{\"arg_bytes\": %d, \"blocks\": %d, \"launch_us_p50\": %.2f, \"launch_us_p10\": %.2f, "
                "\"launch_sync_us_p50\": %.2f, \"launch_sync_us_p10\": %.2f}\n",
                N, blocks, launch[launch.size() / 2], launch[launch.size() / 10], trip[trip.size() / 2],
                trip[trip.size() / 10]);
}

int main() {
    hipStream_t st;
    if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) return 1;
    unsigned int* out = nullptr;
    if (hipMalloc(&out, 64) != hipSuccess) return 1;
    for (int blocks : {1, 256}) {
        run<16>(st, out, blocks);
        run<256>(st, out, blocks);
        run<1024>(st, out, blocks);
        run<2304>(st, out, blocks);
        run<3072>(st, out, blocks);
    }
    (void)hipFree(out);
    (void)hipStreamDestroy(st);
    return 0;
}
