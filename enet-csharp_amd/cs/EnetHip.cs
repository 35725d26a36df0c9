// EnetHip.cs -- C# side of libenethip (the MI355X CRC32 checksum engine) for
// enet-csharp.  Drop this file into the ENet project (namespace enet) and ship
// libenethip.so next to the application.  See INTEGRATION.md.
//
// Binds include/enet_hip.h.  Reference interfaces (enet-csharp/ENet/):
//   ENetHost.checksum ........ include/enet.cs:663-666  (delegate* managed<ENetBuffer*, nuint, uint>)
//   ENet.enet_crc32 .......... c/packet.cs:142-160       (the default checksum)
//   ENetBuffer ............... include/win32.cs:25-29    ({ nuint dataLength; void* data; }, length first)
//
// The callback field holds a *managed* function pointer, so the native export is
// wrapped by EnetHip.Checksum, which has exactly the reference signature:
//     host->checksum = &EnetHip.Checksum;
// The batch API (device-resident or host-memory batches, receive verify, gather
// lists, multi-GPU shards) returns 0 or -hipError_t; the wrappers below turn a
// negative code into EnetHipException.  The callback itself never fails and never
// touches the GPU.
//
// No .NET toolchain exists in the build image, so this file is shipped as source
// and is not compiled by the repository's build; its declarations mirror the
// C header one to one (tests/test_library_cpu.py checks the header against the
// exported symbols).

using System;
using System.Runtime.CompilerServices;
using System.Runtime.InteropServices;
using System.Security;

namespace enet
{
    public sealed class EnetHipException : Exception
    {
        public int Code { get; }

        public EnetHipException(string call, int code)
            : base($"{call} failed: {code} ({Marshal.PtrToStringAnsi(EnetHipNative.enet_hip_error_string(code))})")
        {
            Code = code;
        }
    }

    /// <summary>One batch of a batch-list call (include/enet_hip.h ENetHipBatch; device pointers).</summary>
    [StructLayout(LayoutKind.Sequential)]
    public unsafe struct ENetHipBatch
    {
        public byte* bytes;
        public ulong* offsets;
        public uint* lengths;
        public nuint count;
        public uint* output;
    }

    /// <summary>One batch of a receive-verify list call (include/enet_hip.h ENetHipVerifyBatch; device pointers).</summary>
    [StructLayout(LayoutKind.Sequential)]
    public unsafe struct ENetHipVerifyBatch
    {
        public byte* bytes;
        public ulong* offsets;
        public uint* lengths;
        public uint* slotOffsets;
        public uint* connectIds;
        public nuint count;
        public byte* ok;
        public uint* computed;
    }

    [SuppressUnmanagedCodeSecurity]
    public static unsafe class EnetHipNative
    {
        private const string LIB = "enethip";

        // ---- callback path (CPU) ----
        [DllImport(LIB, CallingConvention = CallingConvention.Cdecl)]
        public static extern uint enet_hip_crc32(ENetBuffer* buffers, nuint bufferCount);

        [DllImport(LIB, CallingConvention = CallingConvention.Cdecl)]
        public static extern uint enet_hip_crc32_update(uint reg, void* data, nuint length);

        // ---- context ----
        [DllImport(LIB, CallingConvention = CallingConvention.Cdecl)]
        public static extern int enet_hip_device_count(int* count);

        [DllImport(LIB, CallingConvention = CallingConvention.Cdecl)]
        public static extern int enet_hip_context_create(int device, IntPtr* ctx);

        [DllImport(LIB, CallingConvention = CallingConvention.Cdecl)]
        public static extern int enet_hip_context_destroy(IntPtr ctx);

        [DllImport(LIB, CallingConvention = CallingConvention.Cdecl)]
        public static extern IntPtr enet_hip_error_string(int code);

        [DllImport(LIB, CallingConvention = CallingConvention.Cdecl)]
        public static extern int enet_hip_set_tuning(IntPtr ctx, int lanesPerPacket, int workgroupsPerCu);

        [DllImport(LIB, CallingConvention = CallingConvention.Cdecl)]
        public static extern int enet_hip_set_kernel_path(IntPtr ctx, int path);

        // ---- batches ----
        [DllImport(LIB, CallingConvention = CallingConvention.Cdecl)]
        public static extern int enet_hip_crc32_batch_device(IntPtr ctx, byte* bytes, ulong* offsets, uint* lengths,
                                                             nuint count, uint* output, IntPtr stream);

        [DllImport(LIB, CallingConvention = CallingConvention.Cdecl)]
        public static extern int enet_hip_crc32_batch_list_device(IntPtr ctx, ENetHipBatch* batches, nuint batchCount,
                                                                  IntPtr stream);

        [DllImport(LIB, CallingConvention = CallingConvention.Cdecl)]
        public static extern nuint enet_hip_binned_workspace_size(nuint count);

        [DllImport(LIB, CallingConvention = CallingConvention.Cdecl)]
        public static extern int enet_hip_crc32_batch_device_binned(IntPtr ctx, byte* bytes, ulong* offsets, uint* lengths,
                                                                    nuint count, uint* output, void* workspace,
                                                                    nuint workspaceBytes, IntPtr stream);

        [DllImport(LIB, CallingConvention = CallingConvention.Cdecl)]
        public static extern nuint enet_hip_verify_binned_workspace_size(nuint count);

        [DllImport(LIB, CallingConvention = CallingConvention.Cdecl)]
        public static extern int enet_hip_verify_batch_device_binned(IntPtr ctx, byte* bytes, ulong* offsets, uint* lengths,
                                                                     uint* slotOffsets, uint* connectIds, nuint count,
                                                                     byte* ok, uint* computed, void* workspace,
                                                                     nuint workspaceBytes, IntPtr stream);

        [DllImport(LIB, CallingConvention = CallingConvention.Cdecl)]
        public static extern int enet_hip_crc32_batch_host(IntPtr ctx, byte* bytes, nuint byteCount, ulong* offsets,
                                                           uint* lengths, nuint count, uint* output);

        [DllImport(LIB, CallingConvention = CallingConvention.Cdecl)]
        public static extern int enet_hip_verify_batch_device(IntPtr ctx, byte* bytes, ulong* offsets, uint* lengths,
                                                              uint* slotOffsets, uint* connectIds, nuint count,
                                                              byte* ok, uint* computed, IntPtr stream);

        [DllImport(LIB, CallingConvention = CallingConvention.Cdecl)]
        public static extern int enet_hip_verify_batch_list_device(IntPtr ctx, ENetHipVerifyBatch* batches,
                                                                   nuint batchCount, IntPtr stream);

        [DllImport(LIB, CallingConvention = CallingConvention.Cdecl)]
        public static extern int enet_hip_crc32_gather_device(IntPtr ctx, byte* bytes, ulong* segOffsets,
                                                              uint* segLengths, uint* segFirst, nuint dgramCount,
                                                              uint* output, IntPtr stream);

        [DllImport(LIB, CallingConvention = CallingConvention.Cdecl)]
        public static extern nuint enet_hip_gather_binned_workspace_size(nuint segCount);

        [DllImport(LIB, CallingConvention = CallingConvention.Cdecl)]
        public static extern int enet_hip_crc32_gather_binned_device(IntPtr ctx, byte* bytes, ulong* segOffsets,
                                                                     uint* segLengths, nuint segCount, uint* segFirst,
                                                                     nuint dgramCount, uint* output, void* workspace,
                                                                     nuint workspaceBytes, IntPtr stream);

        // batched range coder, c/compress.cs:69-943
        [DllImport(LIB, CallingConvention = CallingConvention.Cdecl)]
        public static extern int enet_hip_range_compress_device(IntPtr ctx, byte* input, ulong* inOffsets,
                                                                uint* inLengths, nuint count, byte* output,
                                                                ulong* outOffsets, uint* outLimits,
                                                                uint* outLengths, IntPtr stream);

        [DllImport(LIB, CallingConvention = CallingConvention.Cdecl)]
        public static extern int enet_hip_range_decompress_device(IntPtr ctx, byte* input, ulong* inOffsets,
                                                                  uint* inLengths, nuint count, byte* output,
                                                                  ulong* outOffsets, uint* outLimits,
                                                                  uint* outLengths, IntPtr stream);

        // receive-side fragment reassembly, c/protocol.cs:529-637
        [DllImport(LIB, CallingConvention = CallingConvention.Cdecl)]
        public static extern int enet_hip_fragment_reassemble_device(IntPtr ctx, byte* bytes, ulong* cmdOffsets,
                                                                     uint* cmdAvail, int* slots, nuint count,
                                                                     uint maximumPacketSize, byte* msgBytes,
                                                                     ulong* msgOffsets, uint* msgLengths,
                                                                     uint* msgFragCounts, uint* fragments,
                                                                     uint wordsPerMsg, uint* remaining,
                                                                     nuint slotCount, sbyte* status, IntPtr stream);

        [DllImport(LIB, CallingConvention = CallingConvention.Cdecl)]
        public static extern int enet_hip_crc32_batch_multi(IntPtr* contexts, int contextCount, byte* bytes,
                                                            nuint byteCount, ulong* offsets, uint* lengths,
                                                            nuint count, uint* output);

        [DllImport(LIB, CallingConvention = CallingConvention.Cdecl)]
        public static extern int enet_hip_crc32_gather_binned_host(IntPtr ctx, byte* bytes, nuint byteCount,
            ulong* segOffsets, uint* segLengths, nuint segCount, uint* segFirst, nuint dgramCount, uint* output);

        // ---- UDP socket batching harness (Linux recvmmsg / sendmmsg; include/enet_hip.h) ----
        // fd: a bound IPv4 UDP socket (Socket.Handle); addresses and ports in host order.
        // Return 0, -1 (bad argument) or -(ENET_HIP_ERRNO_BASE + errno).
        public const int ENET_HIP_ERRNO_BASE = 100000;
        public const uint ENET_HIP_DGRAM_TRUNCATED = 0xFFFFFFFFu;
        public const byte ENET_HIP_DGRAM_CHECKSUM = 0, ENET_HIP_DROP_SHORT = 1, ENET_HIP_DROP_PEER = 2,
                          ENET_HIP_DROP_COMPRESSED = 3, ENET_HIP_DROP_TRUNCATED = 4;

        [DllImport(LIB, CallingConvention = CallingConvention.Cdecl)]
        public static extern int enet_hip_udp_receive(int fd, byte* arena, nuint stride, nuint maxDgrams, uint* lengths,
            uint* srcAddr, ushort* srcPort, int timeoutMs, nuint* received);

        [DllImport(LIB, CallingConvention = CallingConvention.Cdecl)]
        public static extern int enet_hip_parse_headers(byte* arena, nuint stride, uint* lengths, nuint count,
            uint* peerConnectIds, nuint peerCount, uint* slotOffsets, uint* connectIds, byte* verdict);

        [DllImport(LIB, CallingConvention = CallingConvention.Cdecl)]
        public static extern int enet_hip_udp_send(int fd, byte* bytes, ulong* segOffsets, uint* segLengths,
            uint* segFirst, nuint dgramCount, uint dstAddr, ushort dstPort, nuint* sent);

        [DllImport(LIB, CallingConvention = CallingConvention.Cdecl)]
        public static extern int enet_hip_stamp_callback(byte* bytes, ulong* segOffsets, uint* segLengths,
            uint* segFirst, uint* slotOffsets, nuint dgramCount);

        [DllImport(LIB, CallingConvention = CallingConvention.Cdecl)]
        public static extern int enet_hip_verify_callback(byte* arena, nuint stride, uint* lengths, uint* slotOffsets,
            uint* connectIds, byte* verdict, nuint count, byte* ok);

        [DllImport(LIB, CallingConvention = CallingConvention.Cdecl)]
        public static extern int enet_hip_udp_receive_verify(IntPtr ctx, int fd, byte* arena, nuint stride,
            nuint maxDgrams, uint* peerConnectIds, nuint peerCount, int timeoutMs, uint* lengths, byte* ok,
            nuint* received);

        [DllImport(LIB, CallingConvention = CallingConvention.Cdecl)]
        public static extern int enet_hip_udp_stamp_send(IntPtr ctx, int fd, byte* bytes, nuint byteCount,
            ulong* segOffsets, uint* segLengths, nuint segCount, uint* segFirst, uint* slotOffsets, nuint dgramCount,
            uint dstAddr, ushort dstPort, nuint* sent);

        [DllImport(LIB, CallingConvention = CallingConvention.Cdecl)]
        public static extern int enet_hip_udp_receive_verify_submit(IntPtr ctx, int fd, byte* arena, nuint stride,
            nuint maxDgrams, uint* peerConnectIds, nuint peerCount, int timeoutMs, uint* lengths, byte* ok,
            nuint* received, int slot);

        [DllImport(LIB, CallingConvention = CallingConvention.Cdecl)]
        public static extern int enet_hip_udp_receive_verify_complete(IntPtr ctx, int slot);

        [DllImport(LIB, CallingConvention = CallingConvention.Cdecl)]
        public static extern int enet_hip_udp_receive_decompress_verify(IntPtr ctx, int fd, byte* arena,
            nuint stride, nuint maxDgrams, uint* peerConnectIds, nuint peerCount, int timeoutMs, uint* lengths,
            byte* ok, nuint* received);

        [DllImport(LIB, CallingConvention = CallingConvention.Cdecl)]
        public static extern int enet_hip_udp_compress_stamp_send(IntPtr ctx, int fd, byte* bytes, nuint byteCount,
            ulong* segOffsets, uint* segLengths, nuint segCount, uint* segFirst, uint* slotOffsets, nuint dgramCount,
            uint dstAddr, ushort dstPort, nuint* sent);

        [DllImport(LIB, CallingConvention = CallingConvention.Cdecl)]
        public static extern int enet_hip_read_probe_device(IntPtr ctx, byte* bytes, nuint byteCount, uint* sink,
            void* stream);

        [DllImport(LIB, CallingConvention = CallingConvention.Cdecl)]
        public static extern int enet_hip_is_diagnostics_build();

        // ---- memory helpers ----
        [DllImport(LIB, CallingConvention = CallingConvention.Cdecl)]
        public static extern int enet_hip_device_alloc(IntPtr ctx, nuint bytes, void** output);

        [DllImport(LIB, CallingConvention = CallingConvention.Cdecl)]
        public static extern int enet_hip_device_free(IntPtr ctx, void* ptr);

        [DllImport(LIB, CallingConvention = CallingConvention.Cdecl)]
        public static extern int enet_hip_host_alloc(nuint bytes, void** output);

        [DllImport(LIB, CallingConvention = CallingConvention.Cdecl)]
        public static extern int enet_hip_host_free(void* ptr);

        [DllImport(LIB, CallingConvention = CallingConvention.Cdecl)]
        public static extern int enet_hip_memcpy_h2d(IntPtr ctx, void* dst, void* src, nuint bytes);

        [DllImport(LIB, CallingConvention = CallingConvention.Cdecl)]
        public static extern int enet_hip_memcpy_d2h(IntPtr ctx, void* dst, void* src, nuint bytes);

        [DllImport(LIB, CallingConvention = CallingConvention.Cdecl)]
        public static extern int enet_hip_synchronize(IntPtr ctx);
    }

    public static unsafe class EnetHip
    {
        /// <summary>
        ///     Drop-in for ENet.enet_crc32 (c/packet.cs:142-160): <c>host->checksum = &amp;EnetHip.Checksum;</c>
        ///     CPU, synchronous, bit-exact, never fails.
        /// </summary>
        [MethodImpl(MethodImplOptions.AggressiveInlining)]
        public static uint Checksum(ENetBuffer* buffers, nuint bufferCount) => EnetHipNative.enet_hip_crc32(buffers, bufferCount);

        internal static void Check(string call, int rc)
        {
            if (rc != 0)
                throw new EnetHipException(call, rc);
        }
    }

    /// <summary>One GPU: owns the library context (tables, stream, staging).</summary>
    public sealed unsafe class EnetHipContext : IDisposable
    {
        public IntPtr Handle { get; private set; }

        public EnetHipContext(int device = 0, int lanesPerPacket = 0)
        {
            IntPtr h;
            EnetHip.Check("enet_hip_context_create", EnetHipNative.enet_hip_context_create(device, &h));
            Handle = h;
            if (lanesPerPacket != 0)
                EnetHip.Check("enet_hip_set_tuning", EnetHipNative.enet_hip_set_tuning(h, lanesPerPacket, 0));
        }

        /// <summary>
        ///     CRCs of packets bytes[offsets[i] .. +lengths[i]) from host memory (H2D, kernel, D2H; synchronous).
        ///     Buffers from <see cref="PinnedBuffer{T}" /> run at full PCIe rate.
        /// </summary>
        public void BatchHost(ReadOnlySpan<byte> bytes, ReadOnlySpan<ulong> offsets, ReadOnlySpan<uint> lengths,
                              Span<uint> output)
        {
            if (offsets.Length != lengths.Length || output.Length < offsets.Length)
                throw new ArgumentException("offsets, lengths and output must have the same length");
            fixed (byte* b = bytes)
            fixed (ulong* o = offsets)
            fixed (uint* l = lengths)
            fixed (uint* r = output)
                EnetHip.Check("enet_hip_crc32_batch_host",
                    EnetHipNative.enet_hip_crc32_batch_host(Handle, b, (nuint)bytes.Length, o, l, (nuint)offsets.Length, r));
        }

        /// <summary>Device-resident batch (device pointers, async on <paramref name="stream" />).</summary>
        public void BatchDevice(byte* bytes, ulong* offsets, uint* lengths, nuint count, uint* output, IntPtr stream = default)
            => EnetHip.Check("enet_hip_crc32_batch_device",
                EnetHipNative.enet_hip_crc32_batch_device(Handle, bytes, offsets, lengths, count, output, stream));

        /// <summary>Several device-resident batches in one launch per 48 (same results as one
        /// BatchDevice call each; the launch's start and drain are paid once for the list).</summary>
        public void BatchListDevice(ENetHipBatch* batches, nuint batchCount, IntPtr stream = default)
            => EnetHip.Check("enet_hip_crc32_batch_list_device",
                EnetHipNative.enet_hip_crc32_batch_list_device(Handle, batches, batchCount, stream));

        /// <summary>Device-resident batch of mixed lengths: records ordered by length per 1024-packet
        /// tile in <paramref name="workspace" /> (EnetHipNative.enet_hip_binned_workspace_size bytes),
        /// CRCs in caller order.</summary>
        public void BatchDeviceBinned(byte* bytes, ulong* offsets, uint* lengths, nuint count, uint* output,
                                      void* workspace, nuint workspaceBytes, IntPtr stream = default)
            => EnetHip.Check("enet_hip_crc32_batch_device_binned",
                EnetHipNative.enet_hip_crc32_batch_device_binned(Handle, bytes, offsets, lengths, count, output,
                                                                 workspace, workspaceBytes, stream));

        /// <summary>Batched receive verify for DGRAMs of mixed lengths (records ordered by length per
        /// 1024-DGRAM tile in <paramref name="workspace" />, EnetHipNative.enet_hip_verify_binned_workspace_size
        /// bytes); ok[i] / computed[i] in caller order.</summary>
        public void VerifyDeviceBinned(byte* bytes, ulong* offsets, uint* lengths, uint* slotOffsets, uint* connectIds,
                                       nuint count, byte* ok, void* workspace, nuint workspaceBytes,
                                       uint* computed = null, IntPtr stream = default)
            => EnetHip.Check("enet_hip_verify_batch_device_binned",
                EnetHipNative.enet_hip_verify_batch_device_binned(Handle, bytes, offsets, lengths, slotOffsets,
                                                                  connectIds, count, ok, computed, workspace,
                                                                  workspaceBytes, stream));

        /// <summary>Batched receive verify (c/protocol.cs:1052-1068); ok[i] = 1 keeps DGRAM i.</summary>
        public void VerifyDevice(byte* bytes, ulong* offsets, uint* lengths, uint* slotOffsets, uint* connectIds,
                                 nuint count, byte* ok, uint* computed = null, IntPtr stream = default)
            => EnetHip.Check("enet_hip_verify_batch_device",
                EnetHipNative.enet_hip_verify_batch_device(Handle, bytes, offsets, lengths, slotOffsets, connectIds,
                    count, ok, computed, stream));

        /// <summary>Send-side gather-list CRCs (c/protocol.cs:1690-1698), segment count known on the host:
        /// a length-binned pass over the segments, then a join per DGRAM.</summary>
        public void GatherDeviceBinned(byte* bytes, ulong* segOffsets, uint* segLengths, nuint segCount, uint* segFirst,
                                       nuint dgramCount, uint* output, void* workspace, nuint workspaceBytes,
                                       IntPtr stream = default)
            => EnetHip.Check("enet_hip_crc32_gather_binned_device",
                EnetHipNative.enet_hip_crc32_gather_binned_device(Handle, bytes, segOffsets, segLengths, segCount,
                    segFirst, dgramCount, output, workspace, workspaceBytes, stream));

        /// <summary>Receive verify over a list of batches, one launch per 32 (same ok[] / computed[] as VerifyDevice per batch).</summary>
        public void VerifyListDevice(ENetHipVerifyBatch* batches, nuint batchCount, IntPtr stream = default)
            => EnetHip.Check("enet_hip_verify_batch_list_device",
                EnetHipNative.enet_hip_verify_batch_list_device(Handle, batches, batchCount, stream));

        public void FragmentReassembleDevice(byte* bytes, ulong* cmdOffsets, uint* cmdAvail, int* slots, nuint count,
                                             uint maximumPacketSize, byte* msgBytes, ulong* msgOffsets,
                                             uint* msgLengths, uint* msgFragCounts, uint* fragments, uint wordsPerMsg,
                                             uint* remaining, nuint slotCount, sbyte* status,
                                             IntPtr stream = default)
            => EnetHip.Check("enet_hip_fragment_reassemble_device",
                EnetHipNative.enet_hip_fragment_reassemble_device(Handle, bytes, cmdOffsets, cmdAvail, slots, count,
                    maximumPacketSize, msgBytes, msgOffsets, msgLengths, msgFragCounts, fragments, wordsPerMsg,
                    remaining, slotCount, status, stream));

        public void RangeCompressDevice(byte* input, ulong* inOffsets, uint* inLengths, nuint count, byte* output,
                                        ulong* outOffsets, uint* outLimits, uint* outLengths, IntPtr stream = default)
            => EnetHip.Check("enet_hip_range_compress_device",
                EnetHipNative.enet_hip_range_compress_device(Handle, input, inOffsets, inLengths, count, output,
                    outOffsets, outLimits, outLengths, stream));

        public void RangeDecompressDevice(byte* input, ulong* inOffsets, uint* inLengths, nuint count, byte* output,
                                          ulong* outOffsets, uint* outLimits, uint* outLengths,
                                          IntPtr stream = default)
            => EnetHip.Check("enet_hip_range_decompress_device",
                EnetHipNative.enet_hip_range_decompress_device(Handle, input, inOffsets, inLengths, count, output,
                    outOffsets, outLimits, outLengths, stream));

        public void Synchronize() => EnetHip.Check("enet_hip_synchronize", EnetHipNative.enet_hip_synchronize(Handle));

        public void Dispose()
        {
            if (Handle != IntPtr.Zero)
            {
                EnetHipNative.enet_hip_context_destroy(Handle);
                Handle = IntPtr.Zero;
            }
        }
    }

    /// <summary>Page-locked host memory for full-rate H2D/D2H.</summary>
    public sealed unsafe class PinnedBuffer<T> : IDisposable where T : unmanaged
    {
        public T* Pointer { get; private set; }
        public int Length { get; }

        public PinnedBuffer(int length)
        {
            void* p;
            EnetHip.Check("enet_hip_host_alloc", EnetHipNative.enet_hip_host_alloc((nuint)(length * sizeof(T)), &p));
            Pointer = (T*)p;
            Length = length;
        }

        public Span<T> Span => new Span<T>(Pointer, Length);

        public void Dispose()
        {
            if (Pointer != null)
            {
                EnetHipNative.enet_hip_host_free(Pointer);
                Pointer = null;
            }
        }
    }
}
