// host_io.cpp -- the host ends of the checksum path: DGRAMs arrive from a UDP
// socket buffer and leave through one (BASELINE.json north_star).  Linux, plain C++,
// no HIP: batched system calls, ENet's receive-header stage, and the per-DGRAM
// callback engine (the reference's own CPU path, batched) that the GPU pipelines of
// host_pipeline.hip are checked and timed against.
//
// Reference (paths under /root/reference/enet-csharp/ENet/):
//   receive: c/protocol.cs:1209-1240 enet_protocol_receive_incoming_commands -- up to
//            256 DGRAMs of <= 4096 B per service pass, one recvmsg each
//            (plugins/NativeSockets/Unix/Linux/c/LinuxSocketPal.cs:407-449
//            WSAReceiveFrom4: msg_flags != 0, i.e. a truncated DGRAM, returns -1);
//   header:  c/protocol.cs:1001-1030 (peerID / flags / headerSize; peerID 0xFFF = no
//            peer; peerID >= peerCount drops; compressed DGRAMs need the decompressor);
//   verify:  c/protocol.cs:1052-1068;  stamp: c/protocol.cs:1690-1698;
//   send:    LinuxSocketPal.cs:315-349 WSASendTo4 -- one sendmsg per DGRAM with the
//            gather list as the iovec array (<= ENET_BUFFER_MAXIMUM = 65 buffers).
#include <arpa/inet.h>
#include <errno.h>
#include <netinet/in.h>
#include <poll.h>
#include <stddef.h>
#include <stdint.h>
#include <string.h>
#include <sys/socket.h>
#include <sys/uio.h>

#include <algorithm>
#include <vector>

#include "enet_hip.h"

namespace {

constexpr size_t kMmsgBatch = 256;            // DGRAMs per recvmmsg / sendmmsg (ENet: 256 per pass)
constexpr size_t kMaxSegments = 65;           // ENET_BUFFER_MAXIMUM, include/enet.cs:417
constexpr uint32_t kHeaderFlagCompressed = 1u << 14, kHeaderFlagSentTime = 1u << 15;
constexpr uint32_t kHeaderFlagMask = kHeaderFlagCompressed | kHeaderFlagSentTime;
constexpr uint32_t kHeaderSessionMask = 3u << 12;
constexpr uint32_t kMaximumPeerId = 0xFFF;    // ENET_PROTOCOL_MAXIMUM_PEER_ID

// a failed system call: -(ENET_HIP_ERRNO_BASE + errno) (enet_hip_error_string names it)
int neg_errno() { return -(ENET_HIP_ERRNO_BASE + (errno ? errno : EIO)); }
constexpr int kBadArg = -1;                   // -hipErrorInvalidValue, as every entry point

// sendmmsg over DGRAM gather lists: DGRAM d = segments segFirst[d] .. segFirst[d+1]-1,
// segment s at seg(s) (a pointer), segLengths[s] bytes; 256 DGRAMs per call.
template <class Seg>
int send_lists(int fd, Seg seg, const uint32_t* segLengths, const uint32_t* segFirst, size_t dgramCount,
               uint32_t dstAddr, uint16_t dstPort, size_t* sent) {
    sockaddr_in to{};
    to.sin_family = AF_INET;
    to.sin_addr.s_addr = htonl(dstAddr);
    to.sin_port = htons(dstPort);
    std::vector<mmsghdr> msgs(kMmsgBatch);
    std::vector<iovec> iov(kMmsgBatch * kMaxSegments);
    size_t done = 0;
    while (done < dgramCount) {
        const size_t want = std::min(kMmsgBatch, dgramCount - done);
        for (size_t i = 0; i < want; ++i) {
            const size_t d = done + i;
            const uint32_t s0 = segFirst[d], s1 = segFirst[d + 1];
            if (s1 < s0 || s1 - s0 > kMaxSegments) return kBadArg;
            iovec* v = &iov[i * kMaxSegments];
            for (uint32_t s = s0; s < s1; ++s) {
                v[s - s0].iov_base = const_cast<uint8_t*>(seg(s));
                v[s - s0].iov_len = segLengths[s];
            }
            memset(&msgs[i].msg_hdr, 0, sizeof(msghdr));
            msgs[i].msg_hdr.msg_iov = v;
            msgs[i].msg_hdr.msg_iovlen = s1 - s0;
            msgs[i].msg_hdr.msg_name = &to;
            msgs[i].msg_hdr.msg_namelen = sizeof(to);
        }
        const int r = sendmmsg(fd, msgs.data(), static_cast<unsigned>(want), 0);
        if (r < 0) {
            if (errno == EINTR) continue;
            if (errno == EAGAIN || errno == EWOULDBLOCK || errno == ENOBUFS) break;   // socket buffer full
            *sent = done;
            return neg_errno();
        }
        done += static_cast<size_t>(r);
        if (r == 0) break;
    }
    *sent = done;
    return 0;
}

}  // namespace

// (host_io.hpp) the same with every segment given as a pointer: the compressing send
// pipeline (host_pipeline.hip) mixes the caller's arena and its compressed bytes
int enethip_udp_send_ptrs(int fd, const uint8_t* const* segPtrs, const uint32_t* segLengths, const uint32_t* segFirst,
                          size_t dgramCount, uint32_t dstAddr, uint16_t dstPort, size_t* sent) {
    if (!sent) return kBadArg;
    *sent = 0;
    if (dgramCount == 0) return 0;
    if (fd < 0 || !segFirst || (segFirst[dgramCount] > segFirst[0] && (!segPtrs || !segLengths))) return kBadArg;
    return send_lists(fd, [&](uint32_t s) { return segPtrs[s]; }, segLengths, segFirst, dgramCount, dstAddr, dstPort,
                      sent);
}

extern "C" {


int enet_hip_udp_receive(int fd, uint8_t* arena, size_t stride, size_t maxDgrams, uint32_t* lengths,
                         uint32_t* srcAddr, uint16_t* srcPort, int timeoutMs, size_t* received) {
    if (!received) return kBadArg;
    *received = 0;
    if (fd < 0 || !arena || !lengths || stride == 0 || stride > 0xFFFFFFFFu) return kBadArg;
    if (maxDgrams == 0) return 0;
    if (timeoutMs != 0) {                      // wait for the first DGRAM (enet_socket_wait's role)
        pollfd p{fd, POLLIN, 0};
        const int r = poll(&p, 1, timeoutMs < 0 ? -1 : timeoutMs);
        if (r < 0) return neg_errno();
        if (r == 0) return 0;
    }
    mmsghdr msgs[kMmsgBatch];
    iovec iov[kMmsgBatch];
    sockaddr_in from[kMmsgBatch];
    size_t got = 0;
    while (got < maxDgrams) {
        const size_t want = std::min(kMmsgBatch, maxDgrams - got);
        for (size_t i = 0; i < want; ++i) {
            iov[i].iov_base = arena + (got + i) * stride;
            iov[i].iov_len = stride;
            memset(&msgs[i].msg_hdr, 0, sizeof(msghdr));
            msgs[i].msg_hdr.msg_iov = &iov[i];
            msgs[i].msg_hdr.msg_iovlen = 1;
            msgs[i].msg_hdr.msg_name = &from[i];
            msgs[i].msg_hdr.msg_namelen = sizeof(sockaddr_in);
            msgs[i].msg_len = 0;
        }
        const int r = recvmmsg(fd, msgs, static_cast<unsigned>(want), MSG_DONTWAIT, nullptr);
        if (r < 0) {
            if (errno == EAGAIN || errno == EWOULDBLOCK || errno == EINTR) break;   // queue drained
            if (got) break;
            return neg_errno();
        }
        if (r == 0) break;
        for (int i = 0; i < r; ++i) {
            const size_t k = got + static_cast<size_t>(i);
            // MSG_TRUNC: the DGRAM did not fit (WSAReceiveFrom4 returns -1 on msg_flags)
            const bool trunc = (msgs[i].msg_hdr.msg_flags & MSG_TRUNC) != 0;
            lengths[k] = trunc ? ENET_HIP_DGRAM_TRUNCATED : msgs[i].msg_len;
            if (srcAddr) srcAddr[k] = ntohl(from[i].sin_addr.s_addr);
            if (srcPort) srcPort[k] = ntohs(from[i].sin_port);
        }
        got += static_cast<size_t>(r);
        if (static_cast<size_t>(r) < want) break;                // fewer queued than asked
    }
    *received = got;
    return 0;
}

int enet_hip_parse_headers(const uint8_t* arena, size_t stride, const uint32_t* lengths, size_t count,
                           const uint32_t* peerConnectIds, size_t peerCount, uint32_t* slotOffsets,
                           uint32_t* connectIds, uint8_t* verdict) {
    if (count == 0) return 0;
    if (!arena || !lengths || !slotOffsets || !connectIds || !verdict || (peerCount && !peerConnectIds))
        return kBadArg;
    for (size_t i = 0; i < count; ++i) {
        const uint8_t* d = arena + i * stride;
        const uint32_t L = lengths[i];
        slotOffsets[i] = 0;
        connectIds[i] = 0;
        if (L == ENET_HIP_DGRAM_TRUNCATED) { verdict[i] = ENET_HIP_DROP_TRUNCATED; continue; }
        if (L < 2) { verdict[i] = ENET_HIP_DROP_SHORT; continue; }            // protocol.cs:1001-1002
        const uint32_t word = (static_cast<uint32_t>(d[0]) << 8) | d[1];    // ENET_NET_TO_HOST_16(peerID)
        const uint32_t flags = word & kHeaderFlagMask;
        const uint32_t peerId = word & ~(kHeaderFlagMask | kHeaderSessionMask);
        const uint32_t headerSize = (flags & kHeaderFlagSentTime) ? 4u : 2u;   // + the 4-byte checksum slot
        if (peerId != kMaximumPeerId && peerId >= peerCount) { verdict[i] = ENET_HIP_DROP_PEER; continue; }
        if (flags & kHeaderFlagCompressed) { verdict[i] = ENET_HIP_DROP_COMPRESSED; continue; }
        // the slot at receivedData[headerSize - 4]; a DGRAM too short to hold it has
        // no slot bytes to compare (the reference reads past receivedDataLength)
        if (headerSize + 4u > L) { verdict[i] = ENET_HIP_DROP_SHORT; continue; }
        slotOffsets[i] = headerSize;
        connectIds[i] = peerId == kMaximumPeerId ? 0u : peerConnectIds[peerId];
        verdict[i] = ENET_HIP_DGRAM_CHECKSUM;
    }
    return 0;
}

int enet_hip_udp_send(int fd, const uint8_t* bytes, const uint64_t* segOffsets, const uint32_t* segLengths,
                      const uint32_t* segFirst, size_t dgramCount, uint32_t dstAddr, uint16_t dstPort, size_t* sent) {
    if (!sent) return kBadArg;
    *sent = 0;
    if (dgramCount == 0) return 0;
    if (fd < 0 || !bytes || !segFirst || (segFirst[dgramCount] > segFirst[0] && (!segOffsets || !segLengths)))
        return kBadArg;
    return send_lists(fd, [&](uint32_t s) { return bytes + segOffsets[s]; }, segLengths, segFirst, dgramCount,
                      dstAddr, dstPort, sent);
}

int enet_hip_stamp_callback(uint8_t* bytes, const uint64_t* segOffsets, const uint32_t* segLengths,
                            const uint32_t* segFirst, const uint32_t* slotOffsets, size_t dgramCount) {
    if (dgramCount == 0) return 0;
    if (!bytes || !segOffsets || !segLengths || !segFirst || !slotOffsets) return kBadArg;
    ENetBuffer bufs[kMaxSegments];
    for (size_t d = 0; d < dgramCount; ++d) {
        const uint32_t s0 = segFirst[d], s1 = segFirst[d + 1];
        if (s1 <= s0 || s1 - s0 > kMaxSegments || static_cast<uint64_t>(slotOffsets[d]) + 4u > segLengths[s0])
            return kBadArg;
        for (uint32_t s = s0; s < s1; ++s) {
            bufs[s - s0].dataLength = segLengths[s];
            bufs[s - s0].data = bytes + segOffsets[s];
        }
        // protocol.cs:1694-1697: the slot holds connectID (or 0) during the CRC, then the CRC
        const uint32_t crc = enet_hip_crc32(bufs, s1 - s0);
        memcpy(bytes + segOffsets[s0] + slotOffsets[d], &crc, 4);
    }
    return 0;
}

int enet_hip_verify_callback(uint8_t* arena, size_t stride, const uint32_t* lengths, const uint32_t* slotOffsets,
                             const uint32_t* connectIds, const uint8_t* verdict, size_t count, uint8_t* ok) {
    if (count == 0) return 0;
    if (!arena || !lengths || !slotOffsets || !connectIds || !ok) return kBadArg;
    for (size_t i = 0; i < count; ++i) {
        ok[i] = 0;
        if (verdict && verdict[i] != ENET_HIP_DGRAM_CHECKSUM) continue;
        const uint32_t L = lengths[i];
        if (L == ENET_HIP_DGRAM_TRUNCATED || static_cast<uint64_t>(slotOffsets[i]) + 4u > L) continue;
        uint8_t* d = arena + i * stride;
        // protocol.cs:1054-1067, in place as the reference does on receivedData
        uint32_t desired;
        memcpy(&desired, d + slotOffsets[i], 4);
        memcpy(d + slotOffsets[i], &connectIds[i], 4);
        ENetBuffer b{L, d};
        ok[i] = enet_hip_crc32(&b, 1) == desired ? 1 : 0;
    }
    return 0;
}

}  // extern "C"
