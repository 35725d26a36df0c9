// crc32_vring.hpp -- host-side entry of the VGPR-ring CRC32 kernel
// (crc32_vring.hip), the default batched checksum path of libenethip.
#pragma once
#include <hip/hip_runtime.h>

#include "crc32_stream_common.hpp"

namespace enethip {

// Table basis of the vring kernel, per image: rows 0..7 = image rows 2^b of the
// GF(2)-linear columns (INIT / CINV dwords zero), row 8 = INIT[0..63],
// row 9 = CINV[0..63].
constexpr int kVrBasisRows = 10;
constexpr int kVrBasisDwords = kVrBasisRows * 64;

// Set the dynamic-LDS attribute of every vring kernel instance (once per context).
int vring_setup();


// Launch the vring kernel: checksum mode, lanes per packet 2^lg (lg = 2 or 3),
// one 16-wave workgroup per CU.  basis2 = kVrBasisDwords per image (images for
// P = 1, 4, 8, 16 in that order).  Returns 0 or -hipError_t.
int vring_launch(int lg, int num_cus, hipStream_t st, const PacketArgs& pa, const KernelTables& tb,
                 const uint32_t* basis2);

}  // namespace enethip
