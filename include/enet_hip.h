/*
 * enet_hip.h -- C-ABI of libenethip.so, the MI355X (gfx950) CRC32 checksum engine
 * for enet-csharp (Molth/enet-csharp, a pure-C# ENet 1.3.18 translation).
 *
 * Only plain pointers, sizes and integers cross this boundary (no HIP or torch
 * types): a C# host binds it with [DllImport("enethip")], a C
 * or C++ host links it directly, Python uses ctypes.
 *
 * Reference interfaces replaced / extended (all paths under
 * /root/reference/enet-csharp/ENet/):
 *   ENetBuffer ............... include/win32.cs:25-29  { nuint dataLength; void* data; }
 *   enet_hip_crc32 ........... c/packet.cs:142-160      ENet.enet_crc32 (default checksum)
 *                              c/enet.cs:195-196        ENET_API.enet_crc32 facade
 *                              include/enet.cs:663-666  ENetHost.checksum callback field
 *   enet_hip_crc32_batch_* ... batched form of the per-DGRAM calls at
 *                              c/protocol.cs:1690-1698 (send stamp) and :1052-1068 (receive)
 *   enet_hip_verify_batch_* .. c/protocol.cs:1012-1014, 1052-1068 (slot substitution,
 *                              CRC over the whole DGRAM, drop on mismatch)
 *   enet_hip_crc32_gather_* .. c/protocol.cs:1546-1559, 1690-1698 (CRC over the
 *                              host->buffers gather list, <= ENET_BUFFER_MAXIMUM=65
 *                              buffers, include/enet.cs:417)
 *
 * Return values: the checksum functions return the CRC exactly as the reference
 * does (ENET_HOST_TO_NET_32(~crc), i.e. the 4 bytes to memcpy into the slot).
 * Every other function returns 0 on success or a negative number -hipError_t
 * (e.g. -1 = hipErrorInvalidValue for a bad argument, -2 = out of memory,
 * -100 = no device); enet_hip_error_string() names it.
 */
#ifndef ENET_HIP_H
#define ENET_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#if defined(_WIN32)
#define ENET_HIP_API __declspec(dllexport)
#else
#define ENET_HIP_API __attribute__((visibility("default")))
#endif

/* include/win32.cs:25-29 -- length FIRST (WSABUF order), also on Linux. */
typedef struct ENetBuffer {
    size_t dataLength;
    void* data;
} ENetBuffer;

/* Shape of ENetHost.checksum (include/enet.cs:666) for native hosts. */
typedef uint32_t (*ENetChecksumCallback)(const ENetBuffer* buffers, size_t bufferCount);

/* ---- callback path (CPU, synchronous, never fails, never touches the GPU) ---- */

/* Drop-in for ENet.enet_crc32 (c/packet.cs:142-160): CRC-32 over the
 * concatenation of the buffers, returned as ENET_HOST_TO_NET_32(~crc). */
ENET_HIP_API uint32_t enet_hip_crc32(const ENetBuffer* buffers, size_t bufferCount);

/* Register-level continuation: feeds `length` bytes into Sarwate register `reg`
 * (start with 0xFFFFFFFF; the callback value is bswap32(~reg)). */
ENET_HIP_API uint32_t enet_hip_crc32_update(uint32_t reg, const void* data, size_t length);

/* ---- device context ---- */

typedef struct enet_hip_context enet_hip_context;

ENET_HIP_API int enet_hip_device_count(int* count);
ENET_HIP_API int enet_hip_context_create(int device, enet_hip_context** out);
ENET_HIP_API int enet_hip_context_destroy(enet_hip_context* ctx);
ENET_HIP_API const char* enet_hip_error_string(int code);

/* Tuning knobs (0 = automatic).  lanes_per_packet: 4 or 8 lanes share one packet
 * (default 8, and 4 for the length-binned entries); libenethip_diag.so also takes
 * 1, 2, 16, 32 and 64 (the sweep-only direct and LDS-stream kernels), the product
 * returns -hipErrorInvalidValue for them.  workgroups_per_cu (0..8): resident
 * workgroups per CU.  The VGPR-ring kernel runs 1 or 2 (values above 2 mean 2
 * there; default 2 for a launch of several batches, 1 for a single checksum batch,
 * 2 for receive verify and for the binned gather's segment pass -- at 2 the
 * length-binned records run the compact records instance); the gather-join grid
 * uses the value as given. */
ENET_HIP_API int enet_hip_set_tuning(enet_hip_context* ctx, int lanes_per_packet, int workgroups_per_cu);

/* Kernel path for the packet batch entry points (0 = default): checksum batches
 * at 4 or 8 lanes per packet run the VGPR-ring kernel (crc32_vring.hip); so do
 * receive verify at 8 lanes (its verify instance) and the length-binned checksum
 * and gather entries (its records instance, 4 lanes by default).  The lean LDS-DMA
 * kernel (crc32_lean.hip) serves receive verify at 4 lanes and the length-binned
 * verify.  (Diagnostics library: 16 lanes run the LDS-ring stream kernel, other
 * lane counts the direct kernel.)
 * Every path gives the same (correct) checksums.  Built in every library: 13 = the
 * lean kernel, 17 = the vring kernel (for the length-binned entries: the bin
 * kernel and its records instance, the two-launch form at every batch size).  Tuning sweeps, libenethip_diag.so only (-1 elsewhere): 1 = direct
 * loads only, 2 + k = stream kernel geometry k (k < 11), 13 + g = lean kernel geometry g (g < 4), 18 = vring with nontemporal
 * stage loads, 19 / 20 = vring with each workgroup walking a contiguous range of
 * groups (plain / nontemporal loads), 21 = vring with the tail-first stage order
 * (each group's last stage first: less L2 refetch, more VALU; slower). */
ENET_HIP_API int enet_hip_set_kernel_path(enet_hip_context* ctx, int path);

/* 1 in libenethip_diag.so (built with -DENET_HIP_DIAG), 0 in libenethip.so. */
ENET_HIP_API int enet_hip_is_diagnostics_build(void);

/* ---- batched checksum, device-resident ----
 * Packet i is bytes[offsets[i] .. offsets[i]+lengths[i]).  All pointers are
 * device pointers on ctx's device; out[i] receives what enet_crc32 would return
 * for that packet as a single ENetBuffer.  Inputs are read-only; `out` is
 * caller-allocated.  `stream` is a hipStream_t (NULL = ctx's stream, a blocking
 * stream: ordered after work on the legacy null stream, not after other non-blocking
 * streams).  Async: returns after the launch.  Throughput comes from many packets
 * at once: each packet is folded by the 8 (or 4) lanes of one wave, so a packet far
 * longer than ENet's DGRAMs (ENET_PROTOCOL_MAXIMUM_MTU = 4096, include/protocol.cs:12)
 * streams at one wave's rate -- checksum a lone multi-megabyte buffer with
 * enet_hip_crc32 on the CPU instead. */
ENET_HIP_API int enet_hip_crc32_batch_device(enet_hip_context* ctx, const uint8_t* bytes,
                                             const uint64_t* offsets, const uint32_t* lengths,
                                             size_t count, uint32_t* out, void* stream);

/* ---- several batches in one launch ----
 * batches[0 .. batchCount) is a HOST array; each entry names one batch exactly as
 * enet_hip_crc32_batch_device's arguments do (device pointers).  Same results as
 * one enet_hip_crc32_batch_device call per batch, in one kernel launch per 48
 * batches: each batch is spread over the whole GPU in turn, with no barrier
 * between batches, so the per-launch start (table image, metadata) and end
 * (drain) are paid once per launch instead of once per batch.  Batches may not
 * share `out` ranges.  Async; graph-capturable (the descriptors are copied into
 * the kernel arguments at the call). */
typedef struct {
    const uint8_t* bytes;
    const uint64_t* offsets;
    const uint32_t* lengths;
    size_t count;
    uint32_t* out;
} ENetHipBatch;
ENET_HIP_API int enet_hip_crc32_batch_list_device(enet_hip_context* ctx, const ENetHipBatch* batches,
                                                  size_t batchCount, void* stream);

/* Same results as enet_hip_crc32_batch_device (enet_crc32, c/packet.cs:142-160,
 * per packet), for batches of mixed lengths (SURVEY cfg3): inside each tile of
 * packets the packet records are first ordered by window length (offset mod
 * 64 + length, 32-byte bins, longest first) on the GPU, so the packets the kernel
 * runs together need about the same number of stages; out[] stays in caller order.
 * Default path, count <= 1024 x CUs x workgroups per CU (two per CU unless
 * enet_hip_set_tuning sets one; cfg3 fits either): one
 * launch, workgroup k ordering its own tile of T <= 1024 packets in its prologue
 * (records [k T, (k + 1) T) of the workspace).  Larger batches, and kernel path 17:
 * a bin kernel over 1024-packet tiles, rank-interleaved, then the records instance
 * of the vring kernel.  `workspace` is caller-owned
 * device memory of at least enet_hip_binned_workspace_size(count) bytes (16 per
 * packet: the ordered {len, off_lo, off_hi, index} records), 16-byte aligned, not
 * shared with a call in flight on another stream; count < 2^32.  No state is
 * kept between calls; graph-capturable.  Runs 4 lanes per packet unless
 * enet_hip_set_tuning chose a count. */
ENET_HIP_API size_t enet_hip_binned_workspace_size(size_t count);
ENET_HIP_API int enet_hip_crc32_batch_device_binned(enet_hip_context* ctx, const uint8_t* bytes,
                                                    const uint64_t* offsets, const uint32_t* lengths,
                                                    size_t count, uint32_t* out, void* workspace,
                                                    size_t workspaceBytes, void* stream);

/* ---- batched checksum from/to host memory ----
 * Packets in host memory, CRCs back to host memory; synchronous.  Pipelined: the
 * batch is cut into chunks of consecutive packets (about 16 MiB of payload each)
 * on two streams -- H2D of a chunk's byte span and metadata, the checksum kernel,
 * D2H of its CRCs -- so one chunk's copy overlaps the previous chunk's kernel.
 * Host buffers allocated with enet_hip_host_alloc are pinned and give the full
 * PCIe rate.  A pinned `bytes` whose packets span at most 4 MiB, or cover under 4/5 of
 * their span, is read in place by the kernel over PCIe instead (no copies of the
 * bytes; 21-22 against 29-31 us for 8 packets). */
ENET_HIP_API int enet_hip_crc32_batch_host(enet_hip_context* ctx, const uint8_t* bytes, size_t byteCount,
                                           const uint64_t* offsets, const uint32_t* lengths,
                                           size_t count, uint32_t* out);

/* ---- batched receive verify (c/protocol.cs:1052-1068) ----
 * For DGRAM i: desired = the 4 bytes at slotOffsets[i] (memcpy, host order);
 * the slot is (virtually) replaced by connectIds[i] (pass 0 for "no peer"), the
 * CRC is taken over the whole DGRAM, ok[i] = (crc == desired).  The input bytes
 * are NOT modified.  computed may be NULL.  Device pointers, async. */
ENET_HIP_API int enet_hip_verify_batch_device(enet_hip_context* ctx, const uint8_t* bytes,
                                              const uint64_t* offsets, const uint32_t* lengths,
                                              const uint32_t* slotOffsets, const uint32_t* connectIds,
                                              size_t count, uint8_t* ok, uint32_t* computed, void* stream);

/* Receive verify over a list of batches (a receive batcher's DGRAM batches,
 * c/protocol.cs:1052-1068 per DGRAM): batches[0 .. batchCount) is a HOST array,
 * each entry names one batch exactly as enet_hip_verify_batch_device's arguments
 * do (device pointers; computed may be NULL).  Same ok[] / computed[] as one
 * enet_hip_verify_batch_device call per batch, in one kernel launch per 32
 * batches (8 lanes per packet, the default: the VGPR-ring kernel's verify
 * instance; 4 lanes: the lean kernel's list instance; other lane counts: one
 * launch per batch), so the per-launch start and drain are paid once per launch.  Batches may not share ok / computed ranges.  Async;
 * graph-capturable. */
typedef struct {
    const uint8_t* bytes;
    const uint64_t* offsets;
    const uint32_t* lengths;
    const uint32_t* slotOffsets;
    const uint32_t* connectIds;
    size_t count;
    uint8_t* ok;
    uint32_t* computed;
} ENetHipVerifyBatch;
ENET_HIP_API int enet_hip_verify_batch_list_device(enet_hip_context* ctx, const ENetHipVerifyBatch* batches,
                                                   size_t batchCount, void* stream);

/* enet_hip_verify_batch_device for batches of mixed lengths: the same per-tile
 * length ordering as enet_hip_crc32_batch_device_binned, with 32-byte records
 * {len, off_lo, off_hi, slotOffset, connectId, index, 0, 0} in `workspace`
 * (enet_hip_verify_binned_workspace_size(count) bytes, 16-byte aligned, not
 * shared with a call in flight on another stream); ok[] / computed[] stay in
 * caller order (c/protocol.cs:1012-1014, 1052-1068 per DGRAM). */
ENET_HIP_API size_t enet_hip_verify_binned_workspace_size(size_t count);
ENET_HIP_API int enet_hip_verify_batch_device_binned(enet_hip_context* ctx, const uint8_t* bytes,
                                                     const uint64_t* offsets, const uint32_t* lengths,
                                                     const uint32_t* slotOffsets, const uint32_t* connectIds,
                                                     size_t count, uint8_t* ok, uint32_t* computed,
                                                     void* workspace, size_t workspaceBytes, void* stream);

/* ---- batched gather-list checksum (send path, c/protocol.cs:1690-1698) ----
 * DGRAM d is the concatenation of segments segFirst[d] .. segFirst[d+1]-1;
 * segment s is bytes[segOffsets[s] .. +segLengths[s]).  segFirst has
 * dgramCount+1 entries.  Device pointers, async.  One lane per DGRAM: when the
 * host knows the segment count, enet_hip_crc32_gather_binned_device below gives
 * the same results 2.5x faster on cfg5 (60 against 152 us for 200 704 DGRAMs,
 * profiles/r06_close/gather_both.log). */
ENET_HIP_API int enet_hip_crc32_gather_device(enet_hip_context* ctx, const uint8_t* bytes,
                                              const uint64_t* segOffsets, const uint32_t* segLengths,
                                              const uint32_t* segFirst, size_t dgramCount, uint32_t* out,
                                              void* stream);

/* Same results as enet_hip_crc32_gather_device, with the segment count known on
 * the host (segCount = segFirst[dgramCount]).  Three passes on `stream`: segments
 * over 48 B (MTU payloads) sorted per tile of 1024 by length bin, their CRCs from
 * the vring kernel's records instance, then one thread per DGRAM folds the short
 * ones (headers, commands) itself and joins the long ones' CRCs with one GF(2)
 * multiply by x^(8 len) each.  `workspace`: caller-owned device memory of at least
 * enet_hip_gather_binned_workspace_size(segCount) bytes, 16-byte aligned, not
 * shared with a call in flight; segCount < 2^32.  Async; graph-capturable. */
ENET_HIP_API size_t enet_hip_gather_binned_workspace_size(size_t segCount);
ENET_HIP_API int enet_hip_crc32_gather_binned_device(enet_hip_context* ctx, const uint8_t* bytes,
                                                     const uint64_t* segOffsets, const uint32_t* segLengths,
                                                     size_t segCount, const uint32_t* segFirst, size_t dgramCount,
                                                     uint32_t* out, void* workspace, size_t workspaceBytes,
                                                     void* stream);

/* ---- batched fragment reassembly (receive side, c/protocol.cs:529-637) ----
 * The data movement of enet_protocol_handle_send_fragment for a batch of
 * SEND_FRAGMENT commands; replaces its per-command validation, bitmap update,
 * fragmentsRemaining countdown and memcpy (protocol.cs:546-552, 566-634).  The
 * caller keeps the channel / sequence-window search (protocol.cs:540-545,
 * 553-617) and passes the reassembly slot it matched for each command.
 *   command i : the 24-byte ENetProtocolSendFragment at bytes[cmdOffsets[i]]
 *               (network byte order, include/protocol.cs:156-165), followed by its
 *               data; cmdAvail[i] = bytes available after the command;
 *   slots[i]  : reassembly slot of command i, or -1 to skip it (status 0);
 *   slot s    : packet data msgBytes[msgOffsets[s] .. +msgLengths[s]) (totalLength
 *               bytes), fragmentCount msgFragCounts[s], received-fragment bitmap
 *               fragments[s*wordsPerMsg .. +wordsPerMsg), fragmentsRemaining
 *               remaining[s].
 * status[i] = -1 where the reference returns -1 (or the bitmap is shorter than
 * fragmentCount bits), 1 when the data was copied, 0 for a skipped command or a
 * duplicate: a fragment already in the bitmap, or one an earlier command of the
 * same batch carries (batch order = the reference's sequential order).  A message
 * is complete when remaining[s] reaches 0 (protocol.cs:632).  Device pointers,
 * async on `stream`; calls on one context must not overlap (shared scratch). */
ENET_HIP_API int enet_hip_fragment_reassemble_device(enet_hip_context* ctx, const uint8_t* bytes,
                                                     const uint64_t* cmdOffsets, const uint32_t* cmdAvail,
                                                     const int32_t* slots, size_t count,
                                                     uint32_t maximumPacketSize, uint8_t* msgBytes,
                                                     const uint64_t* msgOffsets, const uint32_t* msgLengths,
                                                     const uint32_t* msgFragCounts, uint32_t* fragments,
                                                     uint32_t wordsPerMsg, uint32_t* remaining,
                                                     size_t slotCount, int8_t* status, void* stream);

/* ---- batched range coder (c/compress.cs:69-943) ----
 * ENet's adaptive order-2 range coder (enet_host_compress_with_range_coder) over
 * a batch of DGRAMs, one independent model per DGRAM exactly as one
 * enet_range_coder_compress / _decompress call each.  DGRAM i is
 * in[inOffsets[i] .. +inLengths[i]) (the send path's buffer list, concatenated);
 * its result goes to out[outOffsets[i] .. +outLimits[i]) and outLengths[i]
 * receives the byte count, 0 where the reference returns 0 (empty input, output
 * over outLimit, or a corrupt compressed stream).  Device pointers, async on
 * `stream`; calls on one context must not overlap (shared model scratch). */
ENET_HIP_API int enet_hip_range_compress_device(enet_hip_context* ctx, const uint8_t* in, const uint64_t* inOffsets,
                                                const uint32_t* inLengths, size_t count, uint8_t* out,
                                                const uint64_t* outOffsets, const uint32_t* outLimits,
                                                uint32_t* outLengths, void* stream);
ENET_HIP_API int enet_hip_range_decompress_device(enet_hip_context* ctx, const uint8_t* in,
                                                  const uint64_t* inOffsets, const uint32_t* inLengths, size_t count,
                                                  uint8_t* out, const uint64_t* outOffsets, const uint32_t* outLimits,
                                                  uint32_t* outLengths, void* stream);

/* ---- host-memory gather lists (send side, c/protocol.cs:1690-1698) ----
 * enet_hip_crc32_gather_binned_device with HOST arrays: bytes[0 .. byteCount) and
 * the segment metadata are copied H2D (the arena in two halves on two streams),
 * the binned gather CRC runs on the GPU, out[] is copied back.  The DGRAMs use
 * segments segFirst[0] .. segFirst[dgramCount]-1 of the segCount given (a send
 * batch may be a slice of a longer list; checked).  Synchronous; pinned host
 * memory (enet_hip_host_alloc) gives the full PCIe rate.  A pinned arena whose used
 * segments span at most 4 MiB, or cover under 4/5 of their span, is read in place by
 * the kernels over PCIe instead (no copies of the arena). */
ENET_HIP_API int enet_hip_crc32_gather_binned_host(enet_hip_context* ctx, const uint8_t* bytes, size_t byteCount,
                                                   const uint64_t* segOffsets, const uint32_t* segLengths,
                                                   size_t segCount, const uint32_t* segFirst, size_t dgramCount,
                                                   uint32_t* out);

/* ---- UDP socket batching harness (Linux recvmmsg / sendmmsg) ----
 * The path's host ends: DGRAMs arrive from a UDP socket buffer and leave through
 * one.  These batch the system calls and the per-DGRAM steps ENet runs around
 * host->checksum:
 *   receive  c/protocol.cs:1209-1240 (up to 256 DGRAMs of <= 4096 B per service
 *            pass, one recvmsg each: plugins/NativeSockets/Unix/Linux/c/
 *            LinuxSocketPal.cs:407-449, a truncated DGRAM returns -1);
 *   header   c/protocol.cs:1001-1030;  verify c/protocol.cs:1052-1068;
 *   stamp    c/protocol.cs:1690-1698;  send LinuxSocketPal.cs:315-349 (sendmsg
 *            with the gather list as iovecs, <= 65 buffers).
 * fd is a bound IPv4 UDP socket; addresses and ports are in host order.  Socket
 * functions return 0, -1 for a bad argument, or -(ENET_HIP_ERRNO_BASE + errno) for
 * a failed system call; the GPU pipelines also -hipError_t. */
#define ENET_HIP_ERRNO_BASE 100000
#define ENET_HIP_DGRAM_TRUNCATED 0xFFFFFFFFu   /* lengths[i] of a DGRAM longer than the slot */
/* enet_hip_parse_headers verdicts: 0 = the DGRAM goes on to the checksum; else the
 * reason the reference returns before it (the DGRAM is dropped). */
#define ENET_HIP_DGRAM_CHECKSUM 0
#define ENET_HIP_DROP_SHORT 1       /* < 2 B (protocol.cs:1001), or no room for the slot */
#define ENET_HIP_DROP_PEER 2        /* peerID >= peerCount (protocol.cs:1017-1018) */
#define ENET_HIP_DROP_COMPRESSED 3  /* compressed, no decompressor here (protocol.cs:1033-1036) */
#define ENET_HIP_DROP_TRUNCATED 4   /* did not fit its receive slot (LinuxSocketPal.cs:425-426) */

/* Receive up to maxDgrams DGRAMs, DGRAM i into arena + i*stride (stride >= 4096 =
 * ENet's receive buffer), lengths[i] its length (ENET_HIP_DGRAM_TRUNCATED if it did
 * not fit).  Waits up to timeoutMs for the first DGRAM (0 = no wait, < 0 = forever),
 * then takes what is queued without blocking, 256 per recvmmsg.  srcAddr / srcPort
 * may be NULL.  *received = the count. */
ENET_HIP_API int enet_hip_udp_receive(int fd, uint8_t* arena, size_t stride, size_t maxDgrams, uint32_t* lengths,
                                      uint32_t* srcAddr, uint16_t* srcPort, int timeoutMs, size_t* received);

/* ENet's header stage for received DGRAMs (c/protocol.cs:1001-1030): from each
 * ENetProtocolHeader, slotOffsets[i] = the checksum slot's offset (2, or 4 with
 * ENET_PROTOCOL_HEADER_FLAG_SENT_TIME), connectIds[i] = peerConnectIds[peerID] (0
 * for peerID 0xFFF, "no peer"), verdict[i] = ENET_HIP_DGRAM_CHECKSUM or a drop
 * reason.  (Peer state, address and session checks are ENet's, out of scope.) */
ENET_HIP_API int enet_hip_parse_headers(const uint8_t* arena, size_t stride, const uint32_t* lengths, size_t count,
                                        const uint32_t* peerConnectIds, size_t peerCount, uint32_t* slotOffsets,
                                        uint32_t* connectIds, uint8_t* verdict);

/* Send DGRAM d = the gather list of segments segFirst[d] .. segFirst[d+1]-1
 * (bytes + segOffsets[s], segLengths[s]; at most 65) to dstAddr:dstPort, 256 per
 * sendmmsg.  *sent = the DGRAMs the socket accepted (a full socket buffer ends the
 * call early with 0). */
ENET_HIP_API int enet_hip_udp_send(int fd, const uint8_t* bytes, const uint64_t* segOffsets,
                                   const uint32_t* segLengths, const uint32_t* segFirst, size_t dgramCount,
                                   uint32_t dstAddr, uint16_t dstPort, size_t* sent);

/* The reference's per-DGRAM callback engine, batched, on the CPU (the path ENet
 * runs today, one enet_hip_crc32 call per DGRAM; the GPU pipelines below are
 * checked and timed against it).  stamp: the 4 bytes at slotOffsets[d] of DGRAM d's
 * first segment hold connectID (or 0) on entry and its CRC on return
 * (protocol.cs:1694-1697).  verify: ok[i] as protocol.cs:1054-1067 decides, with
 * the slot replaced by connectIds[i] IN PLACE in the arena as the reference does;
 * DGRAMs whose verdict (may be NULL) is not ENET_HIP_DGRAM_CHECKSUM get ok = 0. */
ENET_HIP_API int enet_hip_stamp_callback(uint8_t* bytes, const uint64_t* segOffsets, const uint32_t* segLengths,
                                         const uint32_t* segFirst, const uint32_t* slotOffsets, size_t dgramCount);
ENET_HIP_API int enet_hip_verify_callback(uint8_t* arena, size_t stride, const uint32_t* lengths,
                                          const uint32_t* slotOffsets, const uint32_t* connectIds,
                                          const uint8_t* verdict, size_t count, uint8_t* ok);

/* Receive side on the GPU, socket to keep mask: enet_hip_udp_receive into `arena`,
 * the header stage, receive verify of the whole batch (enet_hip_verify_batch_device):
 * ok[i] = 1 where ENet keeps DGRAM i.  A pinned arena (enet_hip_host_alloc, or host
 * memory registered with HIP) is verified in place: the kernel reads the DGRAMs and the
 * metadata over PCIe and writes the keep mask into pinned staging, with no copies.  A
 * pageable arena takes one pitched H2D (only each slot's first maxLen bytes cross PCIe)
 * and a D2H of the keep mask.  The arena is not modified.  Synchronous.  Runs as slot 0
 * of the two-slot form below (-hipErrorInvalidValue while slot 0 is in flight).  The
 * socket wait (up to timeoutMs; forever when negative) holds no lock of the context:
 * another thread's send or batch call on the same context runs meanwhile. */
ENET_HIP_API int enet_hip_udp_receive_verify(enet_hip_context* ctx, int fd, uint8_t* arena, size_t stride,
                                             size_t maxDgrams, const uint32_t* peerConnectIds, size_t peerCount,
                                             int timeoutMs, uint32_t* lengths, uint8_t* ok, size_t* received);

/* enet_hip_udp_receive_verify in two halves, so that the GPU work of one batch
 * overlaps the socket receive of the next.  A host keeps two receive arenas (pinned:
 * enet_hip_host_alloc) and uses them in turn as slot 0 and slot 1:
 *   submit(slot 0, arena A); loop { submit(slot 1, arena B); complete(slot 0) ->
 *   process A; submit(slot 0, arena A); complete(slot 1) -> process B; }
 * _submit receives and runs the header stage like enet_hip_udp_receive_verify
 * (lengths[] and *received are set when it returns), queues the GPU verify (in place
 * on a pinned arena; else with the pitched H2D and the keep mask's D2H) on the
 * slot's own stream, and returns without waiting; _complete(slot) waits for that batch
 * and writes ok[] (the header stage's drops 0).  arena, lengths and ok of a slot stay
 * the caller's until its _complete.  -hipErrorInvalidValue for a slot already in
 * flight (or still receiving on another thread).  Each slot has its own stream and
 * staging, apart from the other host-memory entry points' (round 6): a host sends
 * (enet_hip_udp_stamp_send, _compress_stamp_send) and runs batch calls on the same
 * context while slots are in flight, and a receive's socket wait holds no lock. */
ENET_HIP_API int enet_hip_udp_receive_verify_submit(enet_hip_context* ctx, int fd, uint8_t* arena, size_t stride,
                                                    size_t maxDgrams, const uint32_t* peerConnectIds,
                                                    size_t peerCount, int timeoutMs, uint32_t* lengths, uint8_t* ok,
                                                    size_t* received, int slot);
ENET_HIP_API int enet_hip_udp_receive_verify_complete(enet_hip_context* ctx, int slot);

/* Send side on the GPU: every DGRAM's CRC over its gather list
 * (enet_hip_crc32_gather_binned_host), written into its slot as protocol.cs:1697
 * does (slot bytes hold connectID or 0 on entry; `bytes` is modified), then
 * enet_hip_udp_send.  Synchronous. */
ENET_HIP_API int enet_hip_udp_stamp_send(enet_hip_context* ctx, int fd, uint8_t* bytes, size_t byteCount,
                                         const uint64_t* segOffsets, const uint32_t* segLengths, size_t segCount,
                                         const uint32_t* segFirst, const uint32_t* slotOffsets, size_t dgramCount,
                                         uint32_t dstAddr, uint16_t dstPort, size_t* sent);

/* The same two pipelines for hosts that set ENet's range coder as their compressor
 * (enet_host_compress_with_range_coder, c/compress.cs:69-943) beside the checksum.
 *
 * Receive (c/protocol.cs:1033-1068): a DGRAM whose header carries
 * ENET_PROTOCOL_HEADER_FLAG_COMPRESSED is decompressed on the GPU
 * (enet_hip_range_decompress_device) -- the body after the header and checksum slot,
 * to at most 4096 - headerSize bytes; a result of 0 or over that limit drops the
 * DGRAM -- the header copied in front, and the CRC verified over the DGRAM so
 * decompressed, as the reference does on packetData[1].  Each decompressed DGRAM
 * replaces the received one in its arena slot (stride >= 4096) and lengths[i] becomes
 * its length (receivedData / receivedDataLength).  Uncompressed DGRAMs go as in
 * enet_hip_udp_receive_verify.
 *
 * Send (c/protocol.cs:1665-1705): each DGRAM's commands (the segments after its first,
 * which holds the header and the slot) are compressed on the GPU
 * (enet_hip_range_compress_device, limit = their length); where the result is
 * shorter, the header's peerID word gets ENET_PROTOCOL_HEADER_FLAG_COMPRESSED (in
 * `bytes`), the CRC is taken over the UNCOMPRESSED gather list on the GPU and
 * written into the slot, and the DGRAM goes out as its first segment followed by
 * the compressed bytes.  Synchronous, both. */
ENET_HIP_API int enet_hip_udp_receive_decompress_verify(enet_hip_context* ctx, int fd, uint8_t* arena, size_t stride,
                                                        size_t maxDgrams, const uint32_t* peerConnectIds,
                                                        size_t peerCount, int timeoutMs, uint32_t* lengths, uint8_t* ok,
                                                        size_t* received);
ENET_HIP_API int enet_hip_udp_compress_stamp_send(enet_hip_context* ctx, int fd, uint8_t* bytes, size_t byteCount,
                                                  const uint64_t* segOffsets, const uint32_t* segLengths,
                                                  size_t segCount, const uint32_t* segFirst,
                                                  const uint32_t* slotOffsets, size_t dgramCount, uint32_t dstAddr,
                                                  uint16_t dstPort, size_t* sent);

/* ---- multi-GPU: independent contiguous shards, no collective ----
 * Packets [i*count/k, (i+1)*count/k) go to contexts[i], each through the pipelined
 * enet_hip_crc32_batch_host of its device (its own streams, PCIe link and HBM), the
 * CRCs into out[].  Synchronous; one host thread per device. */
ENET_HIP_API int enet_hip_crc32_batch_multi(enet_hip_context* const* contexts, int contextCount,
                                            const uint8_t* bytes, size_t byteCount, const uint64_t* offsets,
                                            const uint32_t* lengths, size_t count, uint32_t* out);

/* ---- diagnostics: HBM read-roofline probe ----
 * Streams bytes[0 .. byteCount) once with 16-byte coalesced loads (no table
 * work) and XOR-folds it into *sink (device pointer, 16 bytes); the bench times
 * it beside the checksum kernel as the "achievable read bandwidth" line. */
ENET_HIP_API int enet_hip_read_probe_device(enet_hip_context* ctx, const uint8_t* bytes, size_t byteCount,
                                            uint32_t* sink, void* stream);

#ifdef ENET_HIP_DIAG
/* ==== diagnostics: exported by libenethip_diag.so only ==== */

/* ---- diagnostics: roofline ablation of the stream kernel ----
 * 0 = normal; 1 = skip the table lookups (memory path alone); 2 = skip the
 * LDS-DMA (compute path alone).  Modes 1 and 2 produce WRONG checksums by
 * design and exist only to price the two halves of the kernel (tools/).
 * Bits 2048 / 4096 price parts of the VGPR-ring kernel in batch-list launches
 * at 4 lanes (2048: no head/tail masking, 4096: no table lookups), also WRONG
 * checksums by design; 8192 (alone or with 4096): no load in flight during a
 * fold (correct checksums); 16384 (alone, 8 lanes): 128-byte windows and
 * line-shaped stage loads (WRONG checksums: the memory side alone);
 * 2048 + 4096 + 32768 (4 lanes): no masks, lookups or end-of-packet
 * corrections (WRONG checksums: the kernel's memory and control skeleton);
 * 65536 (4 lanes, correct checksums): the stage loads with the sc1 (path 17)
 * or sc0 sc1 (path 18) cache policy; at 8 lanes on path 17 (correct checksums): each
 * stage's loads issued at s_setprio 3; 262144: the vring's end-record trace
 * instance (with enet_hip_diag_trace).  Also on the linear-stream paths 22 / 23:
 * 2048 = no boundary passes, 2048 + 4096 = no fold lookups either (WRONG
 * checksums).  524288 (correct checksums): the vring's dynamic rounds (rounds
 * past the third claimed chip-wide from a per-launch claim line) instead of the
 * static deal; 8388608 (correct checksums): pair rounds (workgroups k and k + G/2
 * share a claim word).  1048576 x j, j = 1..7: the gather join without its
 * short-segment fold (bit 0 of j), its multiplies (bit 1), its short-segment loads
 * (bit 2) -- WRONG checksums.  16777216 x (1 + b), b < 48 (correct checksums): the
 * binned gather folds segments of at most b bytes in the join (default 48).  The
 * length-binned entry's records instance (4 lanes) takes 4096 (no lookups), 38912 (the
 * skeleton) and 131072 (CRCs stored in record order, alone or with 38912) -- WRONG
 * checksums; 2^30 (correct checksums): the binned entry leaves its records in memory
 * order (no sort). */
ENET_HIP_API int enet_hip_diag_ablation(enet_hip_context* ctx, int mode);

/* ---- diagnostics: per-wave timeline of the lean stream kernel ----
 * With a non-null device buffer of 8 x uint64 per wave (waves = grid x waves per
 * workgroup), every lean launch records per wave (s_memrealtime, 100 MHz):
 * start, metadata landed, table landed, after the table barrier, first stage
 * landed, end, HW_ID | XCC_ID << 32, groups.  NULL turns it off.  Checksums are
 * unaffected. */
ENET_HIP_API int enet_hip_diag_trace(enet_hip_context* ctx, uint64_t* deviceBuffer);
#endif /* ENET_HIP_DIAG */

/* ---- small memory helpers (so C#/ctypes hosts need no HIP binding) ---- */
ENET_HIP_API int enet_hip_device_alloc(enet_hip_context* ctx, size_t bytes, void** out);
ENET_HIP_API int enet_hip_device_free(enet_hip_context* ctx, void* ptr);
ENET_HIP_API int enet_hip_host_alloc(size_t bytes, void** out); /* pinned */
ENET_HIP_API int enet_hip_host_free(void* ptr);
ENET_HIP_API int enet_hip_memcpy_h2d(enet_hip_context* ctx, void* dst, const void* src, size_t bytes);
ENET_HIP_API int enet_hip_memcpy_d2h(enet_hip_context* ctx, void* dst, const void* src, size_t bytes);
ENET_HIP_API int enet_hip_synchronize(enet_hip_context* ctx);

#ifdef __cplusplus
}
#endif
#endif /* ENET_HIP_H */
