// rx_small.hpp -- receive verify of a small batch read in place over PCIe (round 6,
// csrc/rx_small.hip): the socket pipeline's kernel for batches of at most kRxSmallMax
// DGRAMs of at most 4096 bytes.  Private: not in the ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace enethip {

constexpr int kRxSmallMax = 256;     // DGRAMs per launch: their metadata rides in the kernel arguments
constexpr uint32_t kRxSmallMaxLen = 4096;   // one wave of 64 lanes x 64 bytes per DGRAM (ENet's MTU ceiling)
// the chunk-advance tables in the P = 1 image: free column kRxAdvCol + 4 j + b (j < 6, b < 4),
// row v = (v << 8 b) advanced over 64 * 2^j zero bytes (HostTables, crc32_kernels.hip);
// the P = 1 image uses no correction column (corr_col, P > 1 only)
constexpr uint32_t kRxAdvCol = 0;
constexpr int kRxAdvLevels = 6;

// Receive verify (c/protocol.cs:1052-1068) of DGRAM i = arena + i * stride, length
// len[i] (0: dropped by the header stage, ok = 0), checksum slot at slotOff[i] replaced by
// connectId[i]: ok[i] = 1 when the CRC of the DGRAM so modified equals the slot's bytes;
// computed[i] (may be null) = that CRC, 0 where there is no slot.  image1 is the
// context's P = 1 table image (its free columns hold the chunk-advance tables).  Returns
// 1 without launching when the batch does not fit the kernel (count > kRxSmallMax, a
// DGRAM longer than min(stride, kRxSmallMaxLen), stride not a multiple of 16): the
// caller then takes the general verify.  Async on `st`.
int rx_small_verify(hipStream_t st, const uint8_t* arena, uint64_t stride, const uint32_t* len,
                    const uint32_t* slotOff, const uint32_t* connectId, size_t count, uint8_t* ok, uint32_t* computed,
                    const uint32_t* image1);
int rx_small_setup();

}  // namespace enethip
