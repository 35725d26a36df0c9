// context.hpp -- the device context behind the opaque enet_hip_context* of the
// C-ABI (include/enet_hip.h), shared by the translation units that launch work:
// crc32_kernels.hip (device-resident entry points) and host_pipeline.hip (the
// host-memory and socket entry points).  Private: not installed, not in the ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include <atomic>
#include <mutex>

struct enet_hip_context {
    int device = 0;
    int num_cus = 256;
    hipStream_t stream = nullptr;
    uint32_t* d_image = nullptr;
    uint32_t* d_xn = nullptr;    // lo[65536] | hi[65536]
    uint32_t* d_init = nullptr;  // 32
    uint8_t* d_zero = nullptr;   // 256 zero bytes
    uint32_t* d_basis = nullptr; // lean-kernel table basis, kBasisDwords per image
    uint32_t* d_basis2 = nullptr; // vring-kernel table basis, kVrBasisDwords per image
    uint32_t* d_tz = nullptr;    // vring-kernel zero-byte multiplier tables (kTzTableDwords + kTzSmallDwords)
    int lanes_per_packet = 0;    // 0 = auto
    int wgs_per_cu = 0;          // 0 = auto (vring: 2; direct / gather kernels)
    int path = 0;                // enet_hip_set_kernel_path
    uint64_t* trace = nullptr;   // diagnostics library: per-wave timeline
    int ablation_prio = 0;       // diagnostics library: lean-kernel lagging-wave priority
    int ablation = 0;            // diagnostics library: ablations (wrong CRCs by design)
    int vr_abl = 0;              // diagnostics library: vring batch-list ablations
    // vring dynamic rounds: a ring of claim lines (kVrClaimLines x kVrClaimWords, zeroed
    // at creation), one per launch in turn, generation = the line's use count + 1;
    // vr_dynamic = use them (diagnostics library A/B; the static deal is the default)
    uint32_t* d_rounds = nullptr;
    std::atomic<uint64_t> rounds_next{0};
    bool vr_dynamic = false;
    // pair rounds (diagnostics A/B): a ring of kVrPairLines arrays of kVrPairWords words
    uint64_t* d_pairs = nullptr;
    std::atomic<uint64_t> pairs_next{0};
    bool vr_pair = false;
    int join_abl = 0;            // diagnostics library: gather-join ablations
    bool bin_identity = false;   // diagnostics library: binned records left in memory order (not sorted)
    int gather_small = -1;       // diagnostics library: the binned gather's short-segment bound (-1: default)
    // host-memory entry points (host_pipeline.hip): calls on one context serialize on mu
    std::mutex mu;
    hipStream_t pipe[2] = {nullptr, nullptr};   // double-buffered copy / compute streams
    uint8_t* d_pipe[2] = {nullptr, nullptr};    // per stream: chunk bytes | off | len | out (| ok)
    size_t d_pipe_cap[2] = {0, 0};
    uint8_t* h_pipe[2] = {nullptr, nullptr};    // per stream: pinned staging of the chunk's metadata
    size_t h_pipe_cap[2] = {0, 0};
    hipEvent_t pipe_ev[2] = {nullptr, nullptr}; // the staging of stream s has been copied
    uint8_t* h_out = nullptr;                   // pinned landing zone of the D2H result copies
    size_t h_out_cap = 0;
    // enet_hip_udp_receive_verify(_submit / _complete): slot s's batch in flight on its own
    // stream rx_st[s] with its own pinned / device staging (rx_h[s] / rx_d[s]), apart from
    // the pipe / h_pipe / d_pipe / h_out the send and batch host entries use, so those run
    // while a slot is in flight.  The caller's ok[], the DGRAM count, pending;
    // rx_busy[s]: the slot is reserved by a receive whose socket wait runs outside mu
    uint8_t* rx_ok[2] = {nullptr, nullptr};
    size_t rx_n[2] = {0, 0};
    bool rx_pending[2] = {false, false};
    bool rx_busy[2] = {false, false};
    hipStream_t rx_st[2] = {nullptr, nullptr};
    uint8_t* rx_h[2] = {nullptr, nullptr};
    size_t rx_h_cap[2] = {0, 0};
    uint8_t* rx_d[2] = {nullptr, nullptr};
    size_t rx_d_cap[2] = {0, 0};
    uint8_t* d_ws = nullptr;                    // gather / binned workspace
    size_t d_ws_cap = 0;
    // fragment reassembly claim words (all ~0 between calls)
    uint32_t* d_claim = nullptr;
    size_t d_claim_cap = 0;     // words of the FILLED layout (claim words + winner counts + flag)
    size_t d_claim_words = 0;   // claim words of the current layout (slots x bitmap bits)
    uint8_t* d_frag_desc = nullptr;   // copy descriptors, 28 B per command
    size_t d_frag_desc_cap = 0;
    uint8_t* d_rc_scratch = nullptr;  // range coder models, kRangeModelBytes per thread
    size_t d_rc_scratch_cap = 0;
};

namespace enethip {

inline int herr(hipError_t e) { return e == hipSuccess ? 0 : -static_cast<int>(e); }

#define ENH_CHECK(expr)                        \
    do {                                       \
        hipError_t e_ = (expr);                \
        if (e_ != hipSuccess) return enethip::herr(e_); \
    } while (0)

// Device buffer of at least `need` bytes (grown, never shrunk; contents not kept).
inline int ensure_device(uint8_t** p, size_t* cap, size_t need) {
    if (*cap >= need) return 0;
    if (*p) ENH_CHECK(hipFree(*p));
    *p = nullptr;
    *cap = 0;
    const size_t sz = need > (size_t(1) << 20) ? need : (size_t(1) << 20);
    ENH_CHECK(hipMalloc(reinterpret_cast<void**>(p), sz));
    *cap = sz;
    return 0;
}

// Pinned host buffer of at least `need` bytes (grown, never shrunk).
inline int ensure_pinned(uint8_t** p, size_t* cap, size_t need) {
    if (*cap >= need) return 0;
    if (*p) ENH_CHECK(hipHostFree(*p));
    *p = nullptr;
    *cap = 0;
    const size_t sz = need > (size_t(1) << 20) ? need : (size_t(1) << 20);
    ENH_CHECK(hipHostMalloc(reinterpret_cast<void**>(p), sz, hipHostMallocDefault));
    *cap = sz;
    return 0;
}

// The batched range coder (crc32_kernels.hip) for a caller that holds ctx->mu.
int range_coder_locked(enet_hip_context* ctx, bool decompress, const uint8_t* in, const uint64_t* inOffsets,
                       const uint32_t* inLengths, size_t count, uint8_t* out, const uint64_t* outOffsets,
                       const uint32_t* outLimits, uint32_t* outLengths, hipStream_t st);

// The host-memory pipeline's streams and events (created on first use).
int pipeline_init(enet_hip_context* ctx);
void pipeline_release(enet_hip_context* ctx);

}  // namespace enethip

// sendmmsg of gather lists given as segment pointers (host_io.cpp; the compressing
// send pipeline mixes the caller's arena with its compressed bytes)
int enethip_udp_send_ptrs(int fd, const uint8_t* const* segPtrs, const uint32_t* segLengths, const uint32_t* segFirst,
                          size_t dgramCount, uint32_t dstAddr, uint16_t dstPort, size_t* sent);
