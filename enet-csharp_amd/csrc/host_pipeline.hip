// host_pipeline.hip -- the host-memory entry points of libenethip: batches that
// start and end in host memory (a UDP socket buffer, BASELINE.json north_star) and
// cross PCIe around the device-resident kernels of crc32_kernels.hip.
//
//   * enet_hip_crc32_batch_host: double-buffered pipeline.  The batch is cut into
//     chunks of consecutive packets (about kChunkBytes of payload each); chunk k runs
//     on stream k % 2: H2D of its byte span and rebased metadata, the checksum kernel,
//     D2H of its CRCs.  So the copy of chunk k + 1 overlaps the kernel and the D2H of
//     chunk k, and PCIe (about 50 GB/s against the kernel's 5 TB/s) stays busy.
//   * enet_hip_crc32_gather_binned_host: the send side's gather lists (c/protocol.cs:
//     1690-1698) from host memory: arena and segment metadata H2D, the binned gather
//     CRC on the GPU, D2H.
//   * enet_hip_udp_receive_verify / enet_hip_udp_stamp_send: the socket harness of
//     host_io.cpp around the GPU -- recvmmsg into the arena, ENet's header stage,
//     receive verify (c/protocol.cs:1052-1068) in place on a pinned arena (or behind
//     one pitched H2D and a D2H of the keep mask for a pageable one); and the GPU stamp
//     (c/protocol.cs:1690-1698) of a send batch followed by sendmmsg.
//   * Pinned arenas of the context's device that are small or sparsely used are read in
//     place over PCIe by the batch and gather host entries too: no copies.
// Calls on one context serialize on its mutex; every call is synchronous except the
// two-slot receive's submit / complete halves.
#include <hip/hip_runtime.h>
#include <errno.h>
#include <string.h>

#include <algorithm>
#include <mutex>
#include <thread>
#include <vector>

#include "context.hpp"
#include "enet_hip.h"

namespace enethip {

constexpr size_t kChunkBytes = size_t(16) << 20;   // payload per pipeline chunk
constexpr size_t kChunkMaxPackets = size_t(1) << 18;
// the largest arena span the gather host entry reads in place (pinned arenas)
#ifndef ENET_HIP_GATHER_INPLACE_SPAN
#define ENET_HIP_GATHER_INPLACE_SPAN (size_t(4) << 20)
#endif
constexpr size_t kGatherInPlaceSpan = ENET_HIP_GATHER_INPLACE_SPAN;

int pipeline_init(enet_hip_context* ctx) {
    for (int s = 0; s < 2; ++s) {
        if (!ctx->pipe[s]) ENH_CHECK(hipStreamCreateWithFlags(&ctx->pipe[s], hipStreamNonBlocking));
        if (!ctx->rx_st[s]) ENH_CHECK(hipStreamCreateWithFlags(&ctx->rx_st[s], hipStreamNonBlocking));
        if (!ctx->pipe_ev[s]) ENH_CHECK(hipEventCreateWithFlags(&ctx->pipe_ev[s], hipEventDisableTiming));
    }
    return 0;
}

void pipeline_release(enet_hip_context* ctx) {
    for (int s = 0; s < 2; ++s) {
        if (ctx->rx_st[s]) {
            (void)hipStreamSynchronize(ctx->rx_st[s]);
            (void)hipStreamDestroy(ctx->rx_st[s]);
        }
        (void)hipFree(ctx->rx_d[s]);
        (void)hipHostFree(ctx->rx_h[s]);
        ctx->rx_st[s] = nullptr;
        ctx->rx_d[s] = nullptr;
        ctx->rx_h[s] = nullptr;
        ctx->rx_d_cap[s] = ctx->rx_h_cap[s] = 0;
        if (ctx->pipe[s]) (void)hipStreamSynchronize(ctx->pipe[s]);
        (void)hipFree(ctx->d_pipe[s]);
        (void)hipHostFree(ctx->h_pipe[s]);
        if (ctx->pipe_ev[s]) (void)hipEventDestroy(ctx->pipe_ev[s]);
        if (ctx->pipe[s]) (void)hipStreamDestroy(ctx->pipe[s]);
        ctx->d_pipe[s] = nullptr;
        ctx->h_pipe[s] = nullptr;
        ctx->pipe[s] = nullptr;
        ctx->pipe_ev[s] = nullptr;
    }
    (void)hipFree(ctx->d_ws);
    ctx->d_ws = nullptr;
    (void)hipHostFree(ctx->h_out);
    ctx->h_out = nullptr;
    ctx->h_out_cap = 0;
}

namespace {

inline size_t align16(size_t x) { return (x + 15u) & ~size_t(15); }

struct Chunk {
    size_t p0, p1;        // packets
    uint64_t b0, b1;      // byte span [b0, b1) of the arena
};

// Consecutive packets, about kChunkBytes of span each.  Offsets that are not
// ascending (spans overlapping or far apart) fall back to one chunk over the
// whole arena (every byte copied once either way).  So do plans of many small
// chunks -- packets alternating between distant regions make every chunk one
// packet long while the summed spans stay near byteCount, and a chunk is a launch,
// three copies and (from chunk 2 on) an event wait: more chunks than a plan of
// full chunks would need (2 ceil(byteCount / kChunkBytes) + 2, or an average under
// 64 packets per chunk) take the one-chunk plan.
std::vector<Chunk> plan_chunks(const uint64_t* off, const uint32_t* len, size_t n, size_t byteCount) {
    std::vector<Chunk> ch;
    uint64_t covered = 0;
    size_t p = 0;
    while (p < n) {
        Chunk c{p, p, off[p], off[p] + len[p]};
        while (c.p1 < n && c.p1 - c.p0 < kChunkMaxPackets) {
            const uint64_t lo = std::min<uint64_t>(c.b0, off[c.p1]), hi = std::max<uint64_t>(c.b1, off[c.p1] + len[c.p1]);
            if (c.p1 > c.p0 && hi - lo > kChunkBytes) break;
            c.b0 = lo;
            c.b1 = hi;
            ++c.p1;
        }
        covered += c.b1 - c.b0;
        ch.push_back(c);
        p = c.p1;
    }
    const size_t full = 2 * ((byteCount + kChunkBytes - 1) / kChunkBytes) + 2;
    if (covered > byteCount + byteCount / 8 + 4096 || (ch.size() > full && ch.size() * 64 > n))
        return {Chunk{0, n, 0, byteCount}};
    return ch;
}

constexpr uint32_t kHeaderFlagCompressed = 1u << 14, kHeaderFlagSentTime = 1u << 15;   // include/protocol.cs
constexpr uint32_t kRecvBuffer = 4096;                     // ENet's receive buffer (protocol.cs:1038-1044)

// Compressed DGRAM j of a receive batch (arena row rows[j], hsz[j] = header + slot
// bytes): the header copied in front of its decompressed body in plain row j, and row
// rows[j]'s offset / length in the verify batch -- length 0 (no slot: ok = 0) when the
// decompression failed or needed more than 4096 - hsz bytes (protocol.cs:1042-1043).
__global__ void rc_fix_kernel(uint8_t* d, const uint32_t* rows, const uint32_t* hsz, uint32_t k, uint64_t pitch,
                              uint64_t plain, const uint32_t* outLen, uint64_t* off, uint32_t* len) {
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= k) return;
    const uint32_t i = rows[j], h = hsz[j];
    const uint8_t* src = d + pitch * i;
    uint8_t* dst = d + plain + static_cast<uint64_t>(kRecvBuffer) * j;
    for (uint32_t b = 0; b < h; ++b) dst[b] = src[b];      // protocol.cs:1045 memcpy(packetData[1], header, headerSize)
    const uint32_t L = outLen[j];
    off[i] = plain + static_cast<uint64_t>(kRecvBuffer) * j;
    len[i] = (L > 0u && L <= kRecvBuffer - h) ? h + L : 0u;
}

}  // namespace
}  // namespace enethip

using namespace enethip;

extern "C" {

// The device address of pinned host memory (hipHostMalloc'd or registered) that was
// allocated under `device`, or null -- pageable memory, or pinned memory of another
// device's context, which that device's page tables may not map: the kernels of `device`
// can then read the memory in place over PCIe.
static uint8_t* pinned_device_view(void* host, int device) {
    hipPointerAttribute_t a{};
    if (hipPointerGetAttributes(&a, host) != hipSuccess) {
        (void)hipGetLastError();                         // (pageable memory: not an error here)
        return nullptr;
    }
    return a.type == hipMemoryTypeHost && a.device == device ? static_cast<uint8_t*>(a.devicePointer) : nullptr;
}

int enet_hip_crc32_batch_host(enet_hip_context* ctx, const uint8_t* bytes, size_t byteCount,
                              const uint64_t* offsets, const uint32_t* lengths, size_t count, uint32_t* out) {
    if (!ctx) return -static_cast<int>(hipErrorInvalidValue);
    if (count == 0) return 0;
    if (!bytes || !offsets || !lengths || !out) return -static_cast<int>(hipErrorInvalidValue);
    uint64_t lo = byteCount, hi = 0, used = 0;
    for (size_t i = 0; i < count; ++i) {  // host-side shape check before any launch
        if (offsets[i] > byteCount || lengths[i] > byteCount - offsets[i]) return -static_cast<int>(hipErrorInvalidValue);
        if (lengths[i]) {
            lo = std::min<uint64_t>(lo, offsets[i]);
            hi = std::max<uint64_t>(hi, offsets[i] + lengths[i]);
            used += lengths[i];
        }
    }
    std::lock_guard<std::mutex> lk(ctx->mu);
    ENH_CHECK(hipSetDevice(ctx->device));
    int rc;
    if ((rc = pipeline_init(ctx))) return rc;
    // a pinned arena, small or sparsely used: the kernel reads it in place (the gather
    // host entry's rule and measurements); offsets and lengths through
    // pinned staging, the CRCs into pinned memory
    const uint64_t span = hi > lo ? hi - lo : 0;
    if (span <= kGatherInPlaceSpan || 5u * used < 4u * span) {
        uint8_t* zb = pinned_device_view(const_cast<uint8_t*>(bytes), ctx->device);
        const size_t ho = align16(8 * count);
        if (zb) {
            if ((rc = ensure_pinned(&ctx->h_pipe[0], &ctx->h_pipe_cap[0], ho + 4 * count))) return rc;
            if ((rc = ensure_pinned(&ctx->h_out, &ctx->h_out_cap, 4 * count))) return rc;
        }
        uint8_t* zs = zb ? pinned_device_view(ctx->h_pipe[0], ctx->device) : nullptr;
        uint8_t* zo = zb ? pinned_device_view(ctx->h_out, ctx->device) : nullptr;
        if (zb && zs && zo) {
            memcpy(ctx->h_pipe[0], offsets, 8 * count);
            memcpy(ctx->h_pipe[0] + ho, lengths, 4 * count);
            hipStream_t st = ctx->pipe[0];
            if ((rc = enet_hip_crc32_batch_device(ctx, zb, reinterpret_cast<uint64_t*>(zs),
                                                  reinterpret_cast<uint32_t*>(zs + ho), count,
                                                  reinterpret_cast<uint32_t*>(zo), st))) {
                (void)hipStreamSynchronize(st);
                return rc;
            }
            ENH_CHECK(hipStreamSynchronize(st));
            memcpy(out, ctx->h_out, 4 * count);
            return 0;
        }
    }
    const std::vector<Chunk> plan = plan_chunks(offsets, lengths, count, byteCount);
    size_t span_max = 0, pk_max = 0;
    for (const Chunk& c : plan) {
        span_max = std::max<size_t>(span_max, c.b1 - c.b0);
        pk_max = std::max(pk_max, c.p1 - c.p0);
    }
    // per stream: device [bytes | off | len | out], pinned [off | len]
    const size_t dbytes = align16(span_max + 16) + align16(8 * pk_max) + 2 * align16(4 * pk_max);
    const size_t hbytes = align16(8 * pk_max) + align16(4 * pk_max);
    for (int s = 0; s < 2 && s < static_cast<int>(plan.size()); ++s) {
        if ((rc = ensure_device(&ctx->d_pipe[s], &ctx->d_pipe_cap[s], dbytes))) return rc;
        if ((rc = ensure_pinned(&ctx->h_pipe[s], &ctx->h_pipe_cap[s], hbytes))) return rc;
    }
    // The CRCs land in pinned memory: a D2H into the caller's (pageable) array would be
    // staged by the runtime, which holds the host thread until that chunk's kernel has
    // run -- the next chunk's H2D would no longer overlap it.
    if ((rc = ensure_pinned(&ctx->h_out, &ctx->h_out_cap, 4 * count))) return rc;
    uint32_t* h_out = reinterpret_cast<uint32_t*>(ctx->h_out);
    for (size_t k = 0; k < plan.size(); ++k) {
        const Chunk& c = plan[k];
        const int s = static_cast<int>(k & 1u);
        hipStream_t st = ctx->pipe[s];
        const size_t n = c.p1 - c.p0;
        uint8_t* d = ctx->d_pipe[s];
        uint8_t* d_bytes = d;
        uint64_t* d_off = reinterpret_cast<uint64_t*>(d + align16(span_max + 16));
        uint32_t* d_len = reinterpret_cast<uint32_t*>(reinterpret_cast<uint8_t*>(d_off) + align16(8 * pk_max));
        uint32_t* d_out = reinterpret_cast<uint32_t*>(reinterpret_cast<uint8_t*>(d_len) + align16(4 * pk_max));
        uint64_t* h_off = reinterpret_cast<uint64_t*>(ctx->h_pipe[s]);
        uint32_t* h_len = reinterpret_cast<uint32_t*>(ctx->h_pipe[s] + align16(8 * pk_max));
        // this stream's staging was last read by chunk k - 2's metadata copy
        if (k >= 2) ENH_CHECK(hipEventSynchronize(ctx->pipe_ev[s]));
        for (size_t i = 0; i < n; ++i) h_off[i] = offsets[c.p0 + i] - c.b0;   // rebased onto the span
        memcpy(h_len, lengths + c.p0, 4 * n);
        ENH_CHECK(hipMemcpyAsync(d_bytes, bytes + c.b0, c.b1 - c.b0, hipMemcpyHostToDevice, st));
        ENH_CHECK(hipMemcpyAsync(d_off, h_off, 8 * n, hipMemcpyHostToDevice, st));
        ENH_CHECK(hipMemcpyAsync(d_len, h_len, 4 * n, hipMemcpyHostToDevice, st));
        ENH_CHECK(hipEventRecord(ctx->pipe_ev[s], st));
        if ((rc = enet_hip_crc32_batch_device(ctx, d_bytes, d_off, d_len, n, d_out, st))) return rc;
        ENH_CHECK(hipMemcpyAsync(h_out + c.p0, d_out, 4 * n, hipMemcpyDeviceToHost, st));
    }
    ENH_CHECK(hipStreamSynchronize(ctx->pipe[0]));
    ENH_CHECK(hipStreamSynchronize(ctx->pipe[1]));
    memcpy(out, h_out, 4 * count);
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
            // the shard's packets go through the pipelined host entry of its device
            // (enet_hip_crc32_batch_host plans chunks over the shard's own byte spans)
            rcs[i] = enet_hip_crc32_batch_host(contexts[i], bytes, byteCount, offsets + lo, lengths + lo, hi - lo,
                                               out + lo);
        });
    }
    for (auto& t : th) t.join();
    for (int rc : rcs)
        if (rc) return rc;
    return 0;
}

int enet_hip_crc32_gather_binned_host(enet_hip_context* ctx, const uint8_t* bytes, size_t byteCount,
                                      const uint64_t* segOffsets, const uint32_t* segLengths, size_t segCount,
                                      const uint32_t* segFirst, size_t dgramCount, uint32_t* out) {
    if (!ctx) return -static_cast<int>(hipErrorInvalidValue);
    if (dgramCount == 0) return 0;
    if (!bytes || !segFirst || !out || (segCount && (!segOffsets || !segLengths)) || segCount > 0xFFFFFFFFull)
        return -static_cast<int>(hipErrorInvalidValue);
    // the DGRAMs use segments [s_lo, s_hi) (a send batch's slice of a longer list)
    const size_t s_lo = segFirst[0], s_hi = segFirst[dgramCount];
    if (s_hi > segCount) return -static_cast<int>(hipErrorInvalidValue);
    for (size_t d = 0; d < dgramCount; ++d)
        if (segFirst[d + 1] < segFirst[d]) return -static_cast<int>(hipErrorInvalidValue);
    for (size_t s = s_lo; s < s_hi; ++s)
        if (segOffsets[s] > byteCount || segLengths[s] > byteCount - segOffsets[s])
            return -static_cast<int>(hipErrorInvalidValue);
    const size_t ns = s_hi - s_lo;
    // only the arena span the used segments cover crosses PCIe ([lo, hi), 16-byte
    // aligned start so the device copy keeps the host's alignment mod 16); their
    // offsets are rebased onto it.  A send loop that stamps a long arena in slices
    // then copies each slice's bytes, not the whole arena per call.
    uint64_t lo = byteCount, hi = 0, used = 0;
    for (size_t s = s_lo; s < s_hi; ++s)
        if (segLengths[s]) {
            lo = std::min<uint64_t>(lo, segOffsets[s]);
            hi = std::max<uint64_t>(hi, segOffsets[s] + segLengths[s]);
            used += segLengths[s];
        }
    if (hi <= lo) lo = hi = 0;
    lo &= ~uint64_t(15);
    const size_t span = static_cast<size_t>(hi - lo);
    std::lock_guard<std::mutex> lk(ctx->mu);
    ENH_CHECK(hipSetDevice(ctx->device));
    int rc;
    if ((rc = pipeline_init(ctx))) return rc;
    // A pinned arena is read in place over PCIe when that moves fewer bytes or saves the
    // copies' fixed cost: a span up to kGatherInPlaceSpan, or segments covering under 4/5 of
    // their span (the kernels read about 38 GB/s of used bytes in place, the copy engines
    // 46 GB/s of the whole span: profiles/r05_rx_zero_copy/).  The segment tables go to
    // pinned staging (a host memcpy), the kernels read them there and write the CRCs into
    // pinned memory -- one stream, no copies (round 5)
    const bool in_place = span <= kGatherInPlaceSpan || 5u * used < 4u * static_cast<uint64_t>(span);
    uint8_t* zb = in_place ? pinned_device_view(const_cast<uint8_t*>(bytes), ctx->device) : nullptr;
    if (zb) {
        const size_t sf = align16(4 * (dgramCount + 1)), so = align16(8 * ns + 8), sl = align16(4 * ns + 4);
        if ((rc = ensure_pinned(&ctx->h_pipe[1], &ctx->h_pipe_cap[1], sf + so + sl))) return rc;
        if ((rc = ensure_pinned(&ctx->h_out, &ctx->h_out_cap, 4 * dgramCount))) return rc;
        const size_t wsb = enet_hip_gather_binned_workspace_size(ns);
        if ((rc = ensure_device(&ctx->d_ws, &ctx->d_ws_cap, wsb + 16))) return rc;
        uint8_t* zs = pinned_device_view(ctx->h_pipe[1], ctx->device);
        uint8_t* zo = pinned_device_view(ctx->h_out, ctx->device);
        if (zs && zo) {
            uint32_t* h_sf = reinterpret_cast<uint32_t*>(ctx->h_pipe[1]);
            uint64_t* h_so = reinterpret_cast<uint64_t*>(ctx->h_pipe[1] + sf);
            uint32_t* h_sl = reinterpret_cast<uint32_t*>(ctx->h_pipe[1] + sf + so);
            for (size_t d = 0; d <= dgramCount; ++d) h_sf[d] = static_cast<uint32_t>(segFirst[d] - s_lo);
            for (size_t s = 0; s < ns; ++s) {
                h_sl[s] = segLengths[s_lo + s];
                h_so[s] = h_sl[s] ? segOffsets[s_lo + s] : 0u;
            }
            hipStream_t s0 = ctx->pipe[0];
            if ((rc = enet_hip_crc32_gather_binned_device(
                     ctx, zb, ns ? reinterpret_cast<uint64_t*>(zs + sf) : nullptr,
                     ns ? reinterpret_cast<uint32_t*>(zs + sf + so) : nullptr, ns, reinterpret_cast<uint32_t*>(zs),
                     dgramCount, reinterpret_cast<uint32_t*>(zo), ctx->d_ws, ctx->d_ws_cap, s0))) {
                (void)hipStreamSynchronize(s0);
                return rc;
            }
            ENH_CHECK(hipStreamSynchronize(s0));
            memcpy(out, ctx->h_out, 4 * dgramCount);
            return 0;
        }
    }
    // device: [arena span | segOffsets | segLengths | segFirst | out], then the binned workspace
    const size_t a = align16(span + 16), so = align16(8 * ns + 8), sl = align16(4 * ns + 4);
    const size_t sf = align16(4 * (dgramCount + 1)), ob = align16(4 * dgramCount);
    if ((rc = ensure_device(&ctx->d_pipe[0], &ctx->d_pipe_cap[0], a + so + sl + sf + ob))) return rc;
    const size_t wsb = enet_hip_gather_binned_workspace_size(ns);
    if ((rc = ensure_device(&ctx->d_ws, &ctx->d_ws_cap, wsb + 16))) return rc;
    // pinned staging: segFirst rebased to s_lo, then the segment offsets rebased to lo
    if ((rc = ensure_pinned(&ctx->h_pipe[1], &ctx->h_pipe_cap[1], sf + so))) return rc;
    uint32_t* h_sf = reinterpret_cast<uint32_t*>(ctx->h_pipe[1]);
    uint64_t* h_so = reinterpret_cast<uint64_t*>(ctx->h_pipe[1] + sf);
    for (size_t d = 0; d <= dgramCount; ++d) h_sf[d] = static_cast<uint32_t>(segFirst[d] - s_lo);
    for (size_t s = 0; s < ns; ++s) h_so[s] = segLengths[s_lo + s] ? segOffsets[s_lo + s] - lo : 0u;
    uint8_t* d = ctx->d_pipe[0];
    uint64_t* d_so = reinterpret_cast<uint64_t*>(d + a);
    uint32_t* d_sl = reinterpret_cast<uint32_t*>(d + a + so);
    uint32_t* d_sf = reinterpret_cast<uint32_t*>(d + a + so + sl);
    uint32_t* d_out = reinterpret_cast<uint32_t*>(d + a + so + sl + sf);
    hipStream_t s0 = ctx->pipe[0], s1 = ctx->pipe[1];
    // the span in two halves on two streams (two copy engines), the metadata behind
    const size_t half = (span / 2 + 4095) & ~size_t(4095);
    if (span) ENH_CHECK(hipMemcpyAsync(d, bytes + lo, std::min(half, span), hipMemcpyHostToDevice, s0));
    if (span > half) ENH_CHECK(hipMemcpyAsync(d + half, bytes + lo + half, span - half, hipMemcpyHostToDevice, s1));
    if (ns) {
        ENH_CHECK(hipMemcpyAsync(d_so, h_so, 8 * ns, hipMemcpyHostToDevice, s1));
        ENH_CHECK(hipMemcpyAsync(d_sl, segLengths + s_lo, 4 * ns, hipMemcpyHostToDevice, s1));
    }
    ENH_CHECK(hipMemcpyAsync(d_sf, h_sf, 4 * (dgramCount + 1), hipMemcpyHostToDevice, s1));
    ENH_CHECK(hipEventRecord(ctx->pipe_ev[1], s1));
    ENH_CHECK(hipStreamWaitEvent(s0, ctx->pipe_ev[1], 0));
    if ((rc = enet_hip_crc32_gather_binned_device(ctx, d, ns ? d_so : nullptr, ns ? d_sl : nullptr, ns, d_sf,
                                                  dgramCount, d_out, ctx->d_ws, ctx->d_ws_cap, s0)))
        return rc;
    if ((rc = ensure_pinned(&ctx->h_out, &ctx->h_out_cap, 4 * dgramCount))) return rc;
    ENH_CHECK(hipMemcpyAsync(ctx->h_out, d_out, 4 * dgramCount, hipMemcpyDeviceToHost, s0));
    ENH_CHECK(hipStreamSynchronize(s0));
    memcpy(out, ctx->h_out, 4 * dgramCount);
    return 0;
}

// The receive batch of slot s (0 or 1), once the socket receive has returned its n
// DGRAMs: header stage, GPU verify and the keep mask into slot s's own pinned staging,
// all queued on its own stream rx_st[s]; the caller holds ctx->mu and waits with
// rx_complete.  A pinned arena (the usual case: enet_hip_host_alloc) is verified in
// place: the kernel reads the DGRAMs at their arena offsets and the metadata from the
// slot's pinned staging over PCIe, and writes the keep mask straight into it -- one
// launch and no copies, where the copy form queues a pitched H2D, a metadata H2D and a
// D2H around it (each several microseconds for a batch of a few dozen DGRAMs).  A
// pageable arena takes the copy form: only each DGRAM slot's first maxLen bytes cross.
static int rx_stage(enet_hip_context* ctx, int slot, uint8_t* arena, size_t stride, size_t n,
                    const uint32_t* peerConnectIds, size_t peerCount, uint32_t* lengths, uint8_t* ok) {
    ctx->rx_ok[slot] = ok;
    ctx->rx_n[slot] = n;
    if (n == 0) return 0;
    ENH_CHECK(hipSetDevice(ctx->device));
    int rc;
    if ((rc = pipeline_init(ctx))) return rc;
    // pinned staging: off u64 | len | slot | connect | verdict | ok (D2H)
    const size_t ho = align16(8 * n), hl = align16(4 * n), hv = align16(n);
    if ((rc = ensure_pinned(&ctx->rx_h[slot], &ctx->rx_h_cap[slot], ho + 3 * hl + 2 * hv))) return rc;
    uint64_t* h_off = reinterpret_cast<uint64_t*>(ctx->rx_h[slot]);
    uint32_t* h_len = reinterpret_cast<uint32_t*>(ctx->rx_h[slot] + ho);
    uint32_t* h_slot = reinterpret_cast<uint32_t*>(ctx->rx_h[slot] + ho + hl);
    uint32_t* h_conn = reinterpret_cast<uint32_t*>(ctx->rx_h[slot] + ho + 2 * hl);
    uint8_t* h_verdict = ctx->rx_h[slot] + ho + 3 * hl;
    uint8_t* h_ok = h_verdict + hv;
    if ((rc = enet_hip_parse_headers(arena, stride, lengths, n, peerConnectIds, peerCount, h_slot, h_conn, h_verdict)))
        return rc;
    hipStream_t st = ctx->rx_st[slot];
    uint8_t* zc = pinned_device_view(arena, ctx->device);
    uint8_t* zs = zc ? pinned_device_view(ctx->rx_h[slot], ctx->device) : nullptr;
    if (zc && zs) {
        for (size_t i = 0; i < n; ++i) {
            h_off[i] = i * stride;
            h_len[i] = h_verdict[i] == ENET_HIP_DGRAM_CHECKSUM ? lengths[i] : 0u;   // header-stage drops: no slot
        }
        if ((rc = enet_hip_verify_batch_device(ctx, zc, reinterpret_cast<uint64_t*>(zs), reinterpret_cast<uint32_t*>(zs + ho),
                                               reinterpret_cast<uint32_t*>(zs + ho + hl),
                                               reinterpret_cast<uint32_t*>(zs + ho + 2 * hl), n, zs + ho + 3 * hl + hv,
                                               nullptr, st)))
            return rc;
        ctx->rx_pending[slot] = true;
        return 0;
    }
    size_t maxLen = 16;
    for (size_t i = 0; i < n; ++i)
        if (h_verdict[i] == ENET_HIP_DGRAM_CHECKSUM) maxLen = std::max<size_t>(maxLen, lengths[i]);
    const size_t pitch = align16(maxLen);
    for (size_t i = 0; i < n; ++i) {
        h_off[i] = i * pitch;
        h_len[i] = h_verdict[i] == ENET_HIP_DGRAM_CHECKSUM ? lengths[i] : 0u;   // header-stage drops: no slot
    }
    // device: [DGRAMs at `pitch` | off | len | slot | connect | ok]
    const size_t db = align16(n * pitch + 16);
    if ((rc = ensure_device(&ctx->rx_d[slot], &ctx->rx_d_cap[slot], db + ho + 3 * hl + hv))) return rc;
    uint8_t* d = ctx->rx_d[slot];
    uint64_t* d_off = reinterpret_cast<uint64_t*>(d + db);
    uint32_t* d_len = reinterpret_cast<uint32_t*>(d + db + ho);
    uint32_t* d_slot = reinterpret_cast<uint32_t*>(d + db + ho + hl);
    uint32_t* d_conn = reinterpret_cast<uint32_t*>(d + db + ho + 2 * hl);
    uint8_t* d_ok = d + db + ho + 3 * hl;
    // only the first maxLen bytes of every stride-sized receive slot cross PCIe
    ENH_CHECK(hipMemcpy2DAsync(d, pitch, arena, stride, maxLen, n, hipMemcpyHostToDevice, st));
    ENH_CHECK(hipMemcpyAsync(d_off, h_off, ho + 3 * hl, hipMemcpyHostToDevice, st));   // off | len | slot | connect
    if ((rc = enet_hip_verify_batch_device(ctx, d, d_off, d_len, d_slot, d_conn, n, d_ok, nullptr, st))) return rc;
    ENH_CHECK(hipMemcpyAsync(h_ok, d_ok, n, hipMemcpyDeviceToHost, st));
    ctx->rx_pending[slot] = true;
    return 0;
}

// slot s's keep mask into the caller's ok[] once its stream is done (header-stage drops: 0)
static int rx_complete(enet_hip_context* ctx, int slot) {
    if (!ctx->rx_pending[slot]) return 0;                // (an empty batch: nothing queued)
    ctx->rx_pending[slot] = false;
    ENH_CHECK(hipSetDevice(ctx->device));
    ENH_CHECK(hipStreamSynchronize(ctx->rx_st[slot]));
    const size_t n = ctx->rx_n[slot];
    const size_t ho = align16(8 * n), hl = align16(4 * n), hv = align16(n);
    const uint8_t* h_verdict = ctx->rx_h[slot] + ho + 3 * hl;
    const uint8_t* h_ok = h_verdict + hv;
    for (size_t i = 0; i < n; ++i) ctx->rx_ok[slot][i] = h_verdict[i] == ENET_HIP_DGRAM_CHECKSUM ? h_ok[i] : 0u;
    return 0;
}

// A receive on slot s: the slot is reserved under ctx->mu (neither pending nor reserved
// by another receive), the socket wait -- up to timeoutMs, or forever when it is
// negative -- runs with mu released, so another thread's stamp_send, range coder or batch
// call on the same context is not held behind it, then the header stage and
// the launch run under mu again.  A failed staging drains what it queued.
static int rx_receive_submit(enet_hip_context* ctx, int slot, int fd, uint8_t* arena, size_t stride,
                             size_t maxDgrams, const uint32_t* peerConnectIds, size_t peerCount, int timeoutMs,
                             uint32_t* lengths, uint8_t* ok, size_t* received, std::unique_lock<std::mutex>& lk) {
    lk.lock();
    if (ctx->rx_pending[slot] || ctx->rx_busy[slot]) return -static_cast<int>(hipErrorInvalidValue);   // (complete it first)
    ctx->rx_busy[slot] = true;
    lk.unlock();
    size_t n = 0;
    const int rrc = enet_hip_udp_receive(fd, arena, stride, maxDgrams, lengths, nullptr, nullptr, timeoutMs, &n);
    lk.lock();
    ctx->rx_busy[slot] = false;
    if (rrc) return rrc;                                 // -errno
    *received = n;
    const int rc = rx_stage(ctx, slot, arena, stride, n, peerConnectIds, peerCount, lengths, ok);
    if (rc) {                                            // (whatever was queued before the failure: drained)
        if (ctx->rx_st[slot]) (void)hipStreamSynchronize(ctx->rx_st[slot]);
        ctx->rx_pending[slot] = false;
    }
    return rc;
}

int enet_hip_udp_receive_verify(enet_hip_context* ctx, int fd, uint8_t* arena, size_t stride, size_t maxDgrams,
                                const uint32_t* peerConnectIds, size_t peerCount, int timeoutMs, uint32_t* lengths,
                                uint8_t* ok, size_t* received) {
    if (received) *received = 0;
    if (!ctx || !received) return -static_cast<int>(hipErrorInvalidValue);
    if (!arena || !lengths || !ok || (peerCount && !peerConnectIds) || stride < 16)
        return -static_cast<int>(hipErrorInvalidValue);
    std::unique_lock<std::mutex> lk(ctx->mu, std::defer_lock);
    const int rc = rx_receive_submit(ctx, 0, fd, arena, stride, maxDgrams, peerConnectIds, peerCount, timeoutMs,
                                     lengths, ok, received, lk);
    if (rc) return rc;
    return rx_complete(ctx, 0);
}

int enet_hip_udp_receive_verify_submit(enet_hip_context* ctx, int fd, uint8_t* arena, size_t stride, size_t maxDgrams,
                                       const uint32_t* peerConnectIds, size_t peerCount, int timeoutMs,
                                       uint32_t* lengths, uint8_t* ok, size_t* received, int slot) {
    if (received) *received = 0;
    if (!ctx || !received) return -static_cast<int>(hipErrorInvalidValue);
    if (!arena || !lengths || !ok || (peerCount && !peerConnectIds) || stride < 16 || slot < 0 || slot > 1)
        return -static_cast<int>(hipErrorInvalidValue);
    std::unique_lock<std::mutex> lk(ctx->mu, std::defer_lock);
    return rx_receive_submit(ctx, slot, fd, arena, stride, maxDgrams, peerConnectIds, peerCount, timeoutMs, lengths,
                             ok, received, lk);
}

int enet_hip_udp_receive_verify_complete(enet_hip_context* ctx, int slot) {
    if (!ctx || slot < 0 || slot > 1) return -static_cast<int>(hipErrorInvalidValue);
    std::lock_guard<std::mutex> lk(ctx->mu);
    return rx_complete(ctx, slot);
}

int enet_hip_udp_receive_decompress_verify(enet_hip_context* ctx, int fd, uint8_t* arena, size_t stride,
                                           size_t maxDgrams, const uint32_t* peerConnectIds, size_t peerCount,
                                           int timeoutMs, uint32_t* lengths, uint8_t* ok, size_t* received) {
    if (received) *received = 0;
    if (!ctx || !received) return -static_cast<int>(hipErrorInvalidValue);
    if (!arena || !lengths || !ok || (peerCount && !peerConnectIds) || stride < kRecvBuffer)
        return -static_cast<int>(hipErrorInvalidValue);
    size_t n = 0;
    int rc = enet_hip_udp_receive(fd, arena, stride, maxDgrams, lengths, nullptr, nullptr, timeoutMs, &n);
    if (rc) return rc;                                   // -errno
    *received = n;
    if (n == 0) return 0;
    std::lock_guard<std::mutex> lk(ctx->mu);
    ENH_CHECK(hipSetDevice(ctx->device));
    if ((rc = pipeline_init(ctx))) return rc;
    // pinned staging: off u64 | len | slot | connect | verdict, then the compressed
    // DGRAMs' rows | hsz | inOff u64 | inLen | outOff u64 | outLim | outLen, then their
    // decompressed rows (D2H)
    const size_t ho = align16(8 * n), hl = align16(4 * n), hv = align16(n);
    const size_t base = ho + 3 * hl + hv, cmeta = 2 * ho + 5 * hl;
    if ((rc = ensure_pinned(&ctx->h_pipe[0], &ctx->h_pipe_cap[0], base + cmeta + n * kRecvBuffer))) return rc;
    uint8_t* hp = ctx->h_pipe[0];
    uint64_t* h_off = reinterpret_cast<uint64_t*>(hp);
    uint32_t* h_len = reinterpret_cast<uint32_t*>(hp + ho);
    uint32_t* h_slot = reinterpret_cast<uint32_t*>(hp + ho + hl);
    uint32_t* h_conn = reinterpret_cast<uint32_t*>(hp + ho + 2 * hl);
    uint8_t* h_verdict = hp + ho + 3 * hl;
    uint32_t* h_rows = reinterpret_cast<uint32_t*>(hp + base);
    uint32_t* h_hsz = reinterpret_cast<uint32_t*>(hp + base + hl);
    uint64_t* h_inoff = reinterpret_cast<uint64_t*>(hp + base + 2 * hl);
    uint32_t* h_inlen = reinterpret_cast<uint32_t*>(hp + base + 2 * hl + ho);
    uint64_t* h_outoff = reinterpret_cast<uint64_t*>(hp + base + 3 * hl + ho);
    uint32_t* h_outlim = reinterpret_cast<uint32_t*>(hp + base + 3 * hl + 2 * ho);
    uint32_t* h_outlen = reinterpret_cast<uint32_t*>(hp + base + 4 * hl + 2 * ho);
    uint8_t* h_plain = hp + base + cmeta;
    if ((rc = enet_hip_parse_headers(arena, stride, lengths, n, peerConnectIds, peerCount, h_slot, h_conn, h_verdict)))
        return rc;
    // the header stage's compressed DGRAMs go to the decompressor (protocol.cs:1033-1050)
    uint32_t k = 0;
    size_t maxLen = 16;
    for (size_t i = 0; i < n; ++i) {
        if (h_verdict[i] == ENET_HIP_DROP_COMPRESSED) {
            const uint8_t* dg = arena + i * stride;
            const uint32_t word = (static_cast<uint32_t>(dg[0]) << 8) | dg[1];
            const uint32_t peer = word & 0x0FFFu;
            const uint32_t hs = (word & kHeaderFlagSentTime) ? 4u : 2u;
            if (lengths[i] < hs + 4u) {                  // no room for the slot before the body
                h_verdict[i] = ENET_HIP_DROP_SHORT;
                continue;
            }
            h_slot[i] = hs;
            h_conn[i] = peer == 0x0FFFu ? 0u : peerConnectIds[peer];   // (peer < peerCount: checked before)
            h_rows[k] = static_cast<uint32_t>(i);
            h_hsz[k] = hs + 4u;
            ++k;
            maxLen = std::max<size_t>(maxLen, lengths[i]);
        } else if (h_verdict[i] == ENET_HIP_DGRAM_CHECKSUM) {
            maxLen = std::max<size_t>(maxLen, lengths[i]);
        }
    }
    const size_t pitch = align16(maxLen);
    for (size_t i = 0; i < n; ++i) {
        h_off[i] = i * pitch;
        h_len[i] = h_verdict[i] == ENET_HIP_DGRAM_CHECKSUM ? lengths[i] : 0u;   // compressed: set on the device
    }
    const uint64_t plain = align16(n * pitch + 16);        // decompressed rows after the received ones
    for (uint32_t j = 0; j < k; ++j) {
        h_inoff[j] = h_rows[j] * pitch + h_hsz[j];
        h_inlen[j] = lengths[h_rows[j]] - h_hsz[j];
        h_outoff[j] = plain + static_cast<uint64_t>(kRecvBuffer) * j + h_hsz[j];
        h_outlim[j] = kRecvBuffer - h_hsz[j];
    }
    // device: [DGRAMs at `pitch` | decompressed rows | off | len | slot | connect | ok | compressed metadata]
    const size_t db = plain + align16(static_cast<size_t>(k) * kRecvBuffer + 16);
    if ((rc = ensure_device(&ctx->d_pipe[0], &ctx->d_pipe_cap[0], db + base + cmeta))) return rc;
    uint8_t* d = ctx->d_pipe[0];
    uint64_t* d_off = reinterpret_cast<uint64_t*>(d + db);
    uint32_t* d_len = reinterpret_cast<uint32_t*>(d + db + ho);
    uint32_t* d_slot = reinterpret_cast<uint32_t*>(d + db + ho + hl);
    uint32_t* d_conn = reinterpret_cast<uint32_t*>(d + db + ho + 2 * hl);
    uint8_t* d_ok = d + db + ho + 3 * hl;
    uint8_t* dc = d + db + base;
    uint32_t* d_rows = reinterpret_cast<uint32_t*>(dc);
    uint32_t* d_hsz = reinterpret_cast<uint32_t*>(dc + hl);
    uint64_t* d_inoff = reinterpret_cast<uint64_t*>(dc + 2 * hl);
    uint32_t* d_inlen = reinterpret_cast<uint32_t*>(dc + 2 * hl + ho);
    uint64_t* d_outoff = reinterpret_cast<uint64_t*>(dc + 3 * hl + ho);
    uint32_t* d_outlim = reinterpret_cast<uint32_t*>(dc + 3 * hl + 2 * ho);
    uint32_t* d_outlen = reinterpret_cast<uint32_t*>(dc + 4 * hl + 2 * ho);
    hipStream_t st = ctx->pipe[0];
    ENH_CHECK(hipMemcpy2DAsync(d, pitch, arena, stride, maxLen, n, hipMemcpyHostToDevice, st));
    ENH_CHECK(hipMemcpyAsync(d_off, h_off, ho + 3 * hl, hipMemcpyHostToDevice, st));   // off | len | slot | connect
    if (k) {
        ENH_CHECK(hipMemcpyAsync(dc, hp + base, cmeta - hl, hipMemcpyHostToDevice, st));   // (all but outLen)
        if ((rc = range_coder_locked(ctx, true, d, d_inoff, d_inlen, k, d, d_outoff, d_outlim, d_outlen, st))) return rc;
        hipLaunchKernelGGL(rc_fix_kernel, dim3((k + 255) / 256), dim3(256), 0, st, d, d_rows, d_hsz, k,
                           static_cast<uint64_t>(pitch), plain, d_outlen, d_off, d_len);
        ENH_CHECK(hipGetLastError());
    }
    if ((rc = enet_hip_verify_batch_device(ctx, d, d_off, d_len, d_slot, d_conn, n, d_ok, nullptr, st))) return rc;
    ENH_CHECK(hipMemcpyAsync(ok, d_ok, n, hipMemcpyDeviceToHost, st));
    if (k) {
        ENH_CHECK(hipMemcpyAsync(h_outlen, d_outlen, 4 * k, hipMemcpyDeviceToHost, st));
        ENH_CHECK(hipMemcpyAsync(h_plain, d + plain, static_cast<size_t>(k) * kRecvBuffer, hipMemcpyDeviceToHost, st));
    }
    ENH_CHECK(hipStreamSynchronize(st));
    for (uint32_t j = 0; j < k; ++j) {                    // receivedData := the decompressed DGRAM
        const uint32_t L = h_outlen[j], h = h_hsz[j], i = h_rows[j];
        if (L == 0u || L > kRecvBuffer - h) continue;
        memcpy(arena + static_cast<size_t>(i) * stride, h_plain + static_cast<size_t>(j) * kRecvBuffer, h + L);
        lengths[i] = h + L;
        h_verdict[i] = ENET_HIP_DGRAM_CHECKSUM;
    }
    for (size_t i = 0; i < n; ++i)
        if (h_verdict[i] != ENET_HIP_DGRAM_CHECKSUM) ok[i] = 0;
    return 0;
}

int enet_hip_udp_compress_stamp_send(enet_hip_context* ctx, int fd, uint8_t* bytes, size_t byteCount,
                                     const uint64_t* segOffsets, const uint32_t* segLengths, size_t segCount,
                                     const uint32_t* segFirst, const uint32_t* slotOffsets, size_t dgramCount,
                                     uint32_t dstAddr, uint16_t dstPort, size_t* sent) {
    if (!sent) return -static_cast<int>(hipErrorInvalidValue);
    *sent = 0;
    if (!ctx) return -static_cast<int>(hipErrorInvalidValue);
    if (dgramCount == 0) return 0;
    if (!bytes || !segOffsets || !segLengths || !segFirst || !slotOffsets) return -static_cast<int>(hipErrorInvalidValue);
    for (size_t d = 0; d < dgramCount; ++d) {             // header + slot in the first buffer, at most 65 buffers
        const uint32_t s0 = segFirst[d];
        if (segFirst[d + 1] <= s0 || segFirst[d + 1] > segCount || segFirst[d + 1] - s0 > 65u ||
            static_cast<uint64_t>(slotOffsets[d]) + 4u > segLengths[s0] || segLengths[s0] < 2u)
            return -static_cast<int>(hipErrorInvalidValue);
    }
    for (size_t s = segFirst[0]; s < segFirst[dgramCount]; ++s)
        if (segOffsets[s] > byteCount || segLengths[s] > byteCount - segOffsets[s])
            return -static_cast<int>(hipErrorInvalidValue);
    const size_t n = dgramCount;
    // the commands of DGRAM d (its buffers after the first), concatenated: in[d]
    std::vector<uint64_t> in_off(n);
    std::vector<uint32_t> in_len(n), out_len(n);
    uint64_t total = 0;
    for (size_t d = 0; d < n; ++d) {
        uint64_t L = 0;
        for (uint32_t s = segFirst[d] + 1u; s < segFirst[d + 1]; ++s) L += segLengths[s];
        if (L > 0xFFFFFFFFull) return -static_cast<int>(hipErrorInvalidValue);
        in_off[d] = total;
        in_len[d] = static_cast<uint32_t>(L);
        total += L;
    }
    std::vector<uint8_t> comp(total + 16);
    int rc;
    {
        std::lock_guard<std::mutex> lk(ctx->mu);
        ENH_CHECK(hipSetDevice(ctx->device));
        if ((rc = pipeline_init(ctx))) return rc;
        const size_t ab = align16(total + 16), ho = align16(8 * n), hl = align16(4 * n);
        // pinned: commands | in_off | in_len | out_len, then the compressed bytes (D2H)
        if ((rc = ensure_pinned(&ctx->h_pipe[0], &ctx->h_pipe_cap[0], 2 * ab + ho + 2 * hl))) return rc;
        uint8_t* hp = ctx->h_pipe[0];
        for (size_t d = 0; d < n; ++d) {
            uint64_t o = in_off[d];
            for (uint32_t s = segFirst[d] + 1u; s < segFirst[d + 1]; ++s) {
                memcpy(hp + o, bytes + segOffsets[s], segLengths[s]);
                o += segLengths[s];
            }
        }
        memcpy(hp + ab, in_off.data(), 8 * n);
        memcpy(hp + ab + ho, in_len.data(), 4 * n);
        // device: commands | compressed | in_off | in_len | out_len (the output offsets and
        // limits are the input's: the reference's limit is the commands' own length)
        if ((rc = ensure_device(&ctx->d_pipe[0], &ctx->d_pipe_cap[0], 2 * ab + ho + 2 * hl))) return rc;
        uint8_t* d = ctx->d_pipe[0];
        uint64_t* d_off = reinterpret_cast<uint64_t*>(d + 2 * ab);
        uint32_t* d_len = reinterpret_cast<uint32_t*>(d + 2 * ab + ho);
        uint32_t* d_out = reinterpret_cast<uint32_t*>(d + 2 * ab + ho + hl);
        hipStream_t st = ctx->pipe[0];
        ENH_CHECK(hipMemcpyAsync(d, hp, total, hipMemcpyHostToDevice, st));
        ENH_CHECK(hipMemcpyAsync(d_off, hp + ab, ho + hl, hipMemcpyHostToDevice, st));
        if ((rc = range_coder_locked(ctx, false, d, d_off, d_len, n, d + ab, d_off, d_len, d_out, st))) return rc;
        ENH_CHECK(hipMemcpyAsync(hp + ab + ho + hl, d_out, 4 * n, hipMemcpyDeviceToHost, st));
        ENH_CHECK(hipMemcpyAsync(hp + ab + ho + 2 * hl, d + ab, total, hipMemcpyDeviceToHost, st));
        ENH_CHECK(hipStreamSynchronize(st));
        memcpy(out_len.data(), hp + ab + ho + hl, 4 * n);
        memcpy(comp.data(), hp + ab + ho + 2 * hl, total);
    }
    // protocol.cs:1670-1676: keep the compressed form only when it is shorter.  The
    // reference builds headerFlags fresh for every send, so the flag bit is SET for a kept
    // DGRAM and CLEARED for the others (a reused or retried arena may carry it from an
    // earlier send: sent uncompressed but flagged, the receiver would decompress plain
    // commands and drop it -- ADVICE r5).  It goes into the header before the CRC (it is
    // part of the checksummed bytes); a failed CRC call restores the caller's header bytes.
    constexpr uint8_t kFlagByte = static_cast<uint8_t>(kHeaderFlagCompressed >> 8);
    std::vector<uint8_t> keep(n), hdr0(n);
    for (size_t d = 0; d < n; ++d) {
        keep[d] = out_len[d] > 0u && out_len[d] < in_len[d];
        uint8_t& h = bytes[segOffsets[segFirst[d]]];
        hdr0[d] = h;
        h = keep[d] ? static_cast<uint8_t>(h | kFlagByte) : static_cast<uint8_t>(h & ~kFlagByte);
    }
    std::vector<uint32_t> crc(n);
    if ((rc = enet_hip_crc32_gather_binned_host(ctx, bytes, byteCount, segOffsets, segLengths, segCount, segFirst, n,
                                                crc.data()))) {
        for (size_t d = n; d-- > 0;) bytes[segOffsets[segFirst[d]]] = hdr0[d];   // (reverse: shared first buffers end as they began)
        return rc;
    }
    for (size_t d = 0; d < n; ++d)                        // protocol.cs:1697: the slot := the CRC
        memcpy(bytes + segOffsets[segFirst[d]] + slotOffsets[d], &crc[d], 4);
    // protocol.cs:1700-1705: the wire form -- the first buffer, then the compressed
    // bytes in place of the commands
    std::vector<const uint8_t*> ptrs;
    std::vector<uint32_t> lens, first(n + 1);
    for (size_t d = 0; d < n; ++d) {
        first[d] = static_cast<uint32_t>(ptrs.size());
        const uint32_t s0 = segFirst[d];
        ptrs.push_back(bytes + segOffsets[s0]);
        lens.push_back(segLengths[s0]);
        if (keep[d]) {
            ptrs.push_back(comp.data() + in_off[d]);
            lens.push_back(out_len[d]);
        } else {
            for (uint32_t s = s0 + 1u; s < segFirst[d + 1]; ++s) {
                ptrs.push_back(bytes + segOffsets[s]);
                lens.push_back(segLengths[s]);
            }
        }
    }
    first[n] = static_cast<uint32_t>(ptrs.size());
    return enethip_udp_send_ptrs(fd, ptrs.data(), lens.data(), first.data(), n, dstAddr, dstPort, sent);
}

int enet_hip_udp_stamp_send(enet_hip_context* ctx, int fd, uint8_t* bytes, size_t byteCount,
                            const uint64_t* segOffsets, const uint32_t* segLengths, size_t segCount,
                            const uint32_t* segFirst, const uint32_t* slotOffsets, size_t dgramCount, uint32_t dstAddr,
                            uint16_t dstPort, size_t* sent) {
    if (!sent) return -static_cast<int>(hipErrorInvalidValue);
    *sent = 0;
    if (!ctx) return -static_cast<int>(hipErrorInvalidValue);
    if (dgramCount == 0) return 0;
    if (!bytes || !segOffsets || !segLengths || !segFirst || !slotOffsets) return -static_cast<int>(hipErrorInvalidValue);
    for (size_t d = 0; d < dgramCount; ++d) {             // the slot lies in the DGRAM's first buffer
        const uint32_t s0 = segFirst[d];
        if (segFirst[d + 1] <= s0 || s0 >= segCount || static_cast<uint64_t>(slotOffsets[d]) + 4u > segLengths[s0])
            return -static_cast<int>(hipErrorInvalidValue);
    }
    std::vector<uint32_t> crc(dgramCount);
    int rc = enet_hip_crc32_gather_binned_host(ctx, bytes, byteCount, segOffsets, segLengths, segCount, segFirst,
                                               dgramCount, crc.data());
    if (rc) return rc;
    for (size_t d = 0; d < dgramCount; ++d)               // protocol.cs:1697: the slot := the CRC
        memcpy(bytes + segOffsets[segFirst[d]] + slotOffsets[d], &crc[d], 4);
    return enet_hip_udp_send(fd, bytes, segOffsets, segLengths, segFirst, dgramCount, dstAddr, dstPort, sent);
}

}  // extern "C"
