// crc32_lin.hpp -- host-side entry of the linear-stream CRC32 kernel (crc32_lin.hip):
// each wave streams the contiguous byte span of 62 consecutive packets through LDS
// tiles by line-shaped LDS-DMA, folds fixed 128-byte super-blocks packet-blind, and
// turns the super-blocks' chain states into per-packet CRCs in short per-lane passes
// (tests/kernel_model.py lin_unit).
// Reference: ENet.enet_crc32, /root/reference/enet-csharp/ENet/c/packet.cs:142-160.
#pragma once
#include <hip/hip_runtime.h>

#include "crc32_vring.hpp"

namespace enethip {

// packets per unit (one lane each; lane 62 holds the unit's end boundary)
constexpr uint32_t kLnPk = 62;
// the linear kernel's 64 KiB LDS image: slicing tables T_0..T_31 (P = 1 layout) plus
// byte-indexed tables in the free columns (crc32_lin.hip), built on the host
int lin_image(uint32_t* img /* kImageDwords */);

// Set the dynamic-LDS attribute of the built instances (once per context).
int lin_setup();

// One launch over a list of batches (bl.count <= kVrMaxBatches); bl.b[i].g0 is
// ignored (the units are numbered here).  image = the lin image on the device,
// zero = 16 zero bytes (the DMA source of pieces outside a unit's packets).
// abl (diagnostics library only, WRONG CRCs by design): 1 = no boundary / join
// passes (the stream and fold alone), 2 = no fold lookups either.  nt = the tile
// DMA's nontemporal policy.  Returns 0 or -hipError_t.
int lin_launch_list(int max_wgs, hipStream_t st, const VrBatches& bl, const uint32_t* image, const uint8_t* zero,
                    int abl = 0, bool nt = true);

}  // namespace enethip
