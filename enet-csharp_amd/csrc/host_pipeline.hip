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
//     host_io.cpp around the GPU -- recvmmsg into a pinned arena, ENet's header stage,
//     one pitched H2D (only each DGRAM slot's first maxLen bytes cross PCIe), receive
//     verify (c/protocol.cs:1052-1068) and D2H of the keep mask; and the GPU stamp
//     (c/protocol.cs:1690-1698) of a send batch followed by sendmmsg.
// Calls on one context serialize on its mutex; every call is synchronous.
#include <hip/hip_runtime.h>
#include <errno.h>
#include <string.h>

#include <algorithm>
#include <thread>
#include <vector>

#include "context.hpp"
#include "enet_hip.h"

namespace enethip {

constexpr size_t kChunkBytes = size_t(16) << 20;   // payload per pipeline chunk
constexpr size_t kChunkMaxPackets = size_t(1) << 18;

int pipeline_init(enet_hip_context* ctx) {
    for (int s = 0; s < 2; ++s) {
        if (!ctx->pipe[s]) ENH_CHECK(hipStreamCreateWithFlags(&ctx->pipe[s], hipStreamNonBlocking));
        if (!ctx->pipe_ev[s]) ENH_CHECK(hipEventCreateWithFlags(&ctx->pipe_ev[s], hipEventDisableTiming));
    }
    return 0;
}

void pipeline_release(enet_hip_context* ctx) {
    for (int s = 0; s < 2; ++s) {
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

}  // namespace
}  // namespace enethip

using namespace enethip;

extern "C" {

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
    if ((rc = pipeline_init(ctx))) return rc;
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
    uint64_t lo = byteCount, hi = 0;
    for (size_t s = s_lo; s < s_hi; ++s)
        if (segLengths[s]) {
            lo = std::min<uint64_t>(lo, segOffsets[s]);
            hi = std::max<uint64_t>(hi, segOffsets[s] + segLengths[s]);
        }
    if (hi <= lo) lo = hi = 0;
    lo &= ~uint64_t(15);
    const size_t span = static_cast<size_t>(hi - lo);
    std::lock_guard<std::mutex> lk(ctx->mu);
    ENH_CHECK(hipSetDevice(ctx->device));
    int rc;
    if ((rc = pipeline_init(ctx))) return rc;
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

int enet_hip_udp_receive_verify(enet_hip_context* ctx, int fd, uint8_t* arena, size_t stride, size_t maxDgrams,
                                const uint32_t* peerConnectIds, size_t peerCount, int timeoutMs, uint32_t* lengths,
                                uint8_t* ok, size_t* received) {
    if (!ctx || !received) return -static_cast<int>(hipErrorInvalidValue);
    *received = 0;
    if (!arena || !lengths || !ok || (peerCount && !peerConnectIds) || stride < 16)
        return -static_cast<int>(hipErrorInvalidValue);
    size_t n = 0;
    int rc = enet_hip_udp_receive(fd, arena, stride, maxDgrams, lengths, nullptr, nullptr, timeoutMs, &n);
    if (rc) return rc;                                   // -errno
    *received = n;
    if (n == 0) return 0;
    std::lock_guard<std::mutex> lk(ctx->mu);
    ENH_CHECK(hipSetDevice(ctx->device));
    if ((rc = pipeline_init(ctx))) return rc;
    // pinned staging: off u64 | len | slot | connect | verdict
    const size_t ho = align16(8 * n), hl = align16(4 * n), hv = align16(n);
    if ((rc = ensure_pinned(&ctx->h_pipe[0], &ctx->h_pipe_cap[0], ho + 3 * hl + hv))) return rc;
    uint64_t* h_off = reinterpret_cast<uint64_t*>(ctx->h_pipe[0]);
    uint32_t* h_len = reinterpret_cast<uint32_t*>(ctx->h_pipe[0] + ho);
    uint32_t* h_slot = reinterpret_cast<uint32_t*>(ctx->h_pipe[0] + ho + hl);
    uint32_t* h_conn = reinterpret_cast<uint32_t*>(ctx->h_pipe[0] + ho + 2 * hl);
    uint8_t* h_verdict = ctx->h_pipe[0] + ho + 3 * hl;
    if ((rc = enet_hip_parse_headers(arena, stride, lengths, n, peerConnectIds, peerCount, h_slot, h_conn, h_verdict)))
        return rc;
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
    if ((rc = ensure_device(&ctx->d_pipe[0], &ctx->d_pipe_cap[0], db + ho + 3 * hl + hv))) return rc;
    uint8_t* d = ctx->d_pipe[0];
    uint64_t* d_off = reinterpret_cast<uint64_t*>(d + db);
    uint32_t* d_len = reinterpret_cast<uint32_t*>(d + db + ho);
    uint32_t* d_slot = reinterpret_cast<uint32_t*>(d + db + ho + hl);
    uint32_t* d_conn = reinterpret_cast<uint32_t*>(d + db + ho + 2 * hl);
    uint8_t* d_ok = d + db + ho + 3 * hl;
    hipStream_t st = ctx->pipe[0];
    // only the first maxLen bytes of every stride-sized receive slot cross PCIe
    ENH_CHECK(hipMemcpy2DAsync(d, pitch, arena, stride, maxLen, n, hipMemcpyHostToDevice, st));
    ENH_CHECK(hipMemcpyAsync(d_off, h_off, ho + 3 * hl, hipMemcpyHostToDevice, st));   // off | len | slot | connect
    if ((rc = enet_hip_verify_batch_device(ctx, d, d_off, d_len, d_slot, d_conn, n, d_ok, nullptr, st))) return rc;
    ENH_CHECK(hipMemcpyAsync(ok, d_ok, n, hipMemcpyDeviceToHost, st));
    ENH_CHECK(hipStreamSynchronize(st));
    for (size_t i = 0; i < n; ++i)
        if (h_verdict[i] != ENET_HIP_DGRAM_CHECKSUM) ok[i] = 0;
    return 0;
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
