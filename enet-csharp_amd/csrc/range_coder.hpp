// range_coder.hpp -- host-side entry of the batched range coder (range_coder.hip),
// called by enet_hip_range_compress_device / enet_hip_range_decompress_device.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace enethip {

constexpr uint32_t kRangeSymbols = 4096;                 // ENetSymbols (include/compress.cs:23-24)
constexpr uint64_t kRangeModelBytes = 16ull * kRangeSymbols;

struct RangeArgs {
    const uint8_t* in;           // DGRAM i: in[in_off[i] .. +in_len[i])
    const uint64_t* in_off;
    const uint32_t* in_len;
    uint64_t n;
    uint8_t* out;                // result i: out[out_off[i] .. +out_limit[i])
    const uint64_t* out_off;
    const uint32_t* out_limit;
    uint32_t* out_len;           // bytes written, 0 = did not fit / corrupt input
    uint8_t* scratch;            // kRangeModelBytes per thread
    uint32_t interleave = 0;     // 1: a wave's models symbol-major (symbol i of its lanes adjacent)
};

// threads = DGRAM lanes launched (each needs kRangeModelBytes of scratch), `lanes` of
// them per 64-wide wave (1..64: fewer active lanes per wave, less divergence)
int range_coder_launch(bool decompress, const RangeArgs& a, uint64_t threads, uint32_t lanes, hipStream_t st);

}  // namespace enethip
