// crc32_lean.hpp -- host-side entry of the lean streamed CRC32 kernel
// (crc32_lean.hip), called by the C-ABI launch dispatch in crc32_kernels.hip.
#pragma once
#include <hip/hip_runtime.h>

#include "crc32_stream_common.hpp"
#include "gather_join.hpp"
#include "enet_hip.h"

namespace enethip {

constexpr int kLeanGeoms = 4;

// Batch lists (lean_launch_list): one launch over up to kLeanMaxBatches batches,
// batch b's groups numbered from g0 in one concatenated group space.
struct LeanListBatch {
    const uint8_t* bytes;
    const uint64_t* off;
    const uint32_t* len;
    uint32_t* out;
    uint64_t n;
    uint64_t g0;
};
constexpr int kLeanMaxBatches = 48;
struct LeanList {
    uint32_t count;
    uint32_t pad;
    uint64_t groups;   // all batches' groups
    LeanListBatch b[kLeanMaxBatches];
};
static_assert(sizeof(LeanList) <= 3072, "kernel arguments");   // 0: 16 waves x 2 stages, 1: 12 waves x 3 stages; sweeps: 2: 14 x 3, 3: 10 x 4

// Receive-verify batch lists (lean_launch_vlist): the same, with each batch's
// slot offsets, connectIDs and ok[] (out = the computed CRCs, may be null).
struct LeanVListBatch {
    const uint8_t* bytes;
    const uint64_t* off;
    const uint32_t* len;
    const uint32_t* slot_off;
    const uint32_t* connect;
    uint8_t* ok;
    uint32_t* out;
    uint64_t n;
    uint64_t g0;
};
constexpr int kLeanMaxVBatches = 32;
struct LeanVList {
    uint32_t count;
    uint32_t pad;
    uint64_t groups;
    LeanVListBatch b[kLeanMaxVBatches];
};
static_assert(sizeof(LeanVList) <= 3072, "kernel arguments");

// Set the dynamic-LDS attribute of every lean kernel instance (once per context).
int lean_setup();

// Launch the lean kernel for lanes-per-packet 2^lg (lg = 2 or 3) and MODE 0 (crc)
// or 1 (receive verify); abl != 0 selects a diagnostic ablation (geometry 0, crc
// only; wrong checksums by design).  Returns 0 or -hipError_t.
int lean_launch(int mode, int lg, int geom, int abl, int num_cus, hipStream_t st, const PacketArgs& pa,
                const KernelTables& tb);

// Checksum a list of batches (count <= kLeanMaxBatches) in one launch at lanes
// per packet 2^lg (lg = 2 or 3).  Returns 0 or -hipError_t.
int lean_launch_list(int lg, int num_cus, hipStream_t st, const ENetHipBatch* batches, size_t count,
                     const KernelTables& tb);

// Receive-verify a list of batches (count <= kLeanMaxVBatches) in one launch at
// lanes per packet 2^lg (lg = 2 or 3).  Returns 0 or -hipError_t.
int lean_launch_vlist(int lg, int num_cus, hipStream_t st, const ENetHipVerifyBatch* batches, size_t count,
                      const KernelTables& tb);

// Order the packet records of each 1024-packet tile by length bin, longest first,
// and interleave the tiles' groups of kpk records rank by rank (see
// crc32_lean.hip).  workspace (length_bin_workspace(n, verify) bytes, 16-B
// aligned) = n x {len, off_lo, off_hi, index} records, or with slot_off and
// connect (receive verify) n x {len, off_lo, off_hi, slot_off, connect, index, 0, 0}.
// Stream-ordered; n < 2^32.  Returns 0 or -hipError_t.
size_t length_bin_workspace(uint64_t n, bool verify);
int length_bin(const uint32_t* len, const uint64_t* off, const uint32_t* slot_off, const uint32_t* connect, uint64_t n,
               uint32_t kpk, void* workspace, hipStream_t st, bool identity = false);
// The binned gather's records: per 1024-segment tile (T = ceil(n / 1024), the
// ragged last one included), the records {len, off_lo, off_hi, index} of the
// segments longer than `small`, sorted longest first, then empty records {0, 0, 0,
// n} up to 1024, rank-interleaved as length_bin's full tiles (group q T + t =
// tile t's records [q kpk, (q + 1) kpk)); counts[t] = tile t's kept records.
// records: 16 x 1024 T bytes; counts: 4 T bytes.  No global atomics.
int length_bin_compact(const uint32_t* len, const uint64_t* off, uint64_t n, uint32_t kpk, uint32_t small,
                       void* records, uint32_t* counts, hipStream_t st);
// (diagnostics) length_bin_compact over ga's segments (ga.segs of them) and, in the same launch
// (prejoin_blocks more workgroups), the split join's pre-join over ga's DGRAMs
// (gather_join.hpp): out[d] = finalize(A_d), info[q] for the long segments.
int gather_bin_prejoin(const GatherArgs& ga, uint2* info, const KernelTables& tb, uint32_t small, uint32_t kpk,
                       void* records, uint32_t* counts, unsigned prejoin_blocks, hipStream_t st);

}  // namespace enethip
