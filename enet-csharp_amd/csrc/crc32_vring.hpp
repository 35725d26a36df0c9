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

// One batch of a batch-list launch (device pointers; packet i of the batch is
// bytes[off[i] .. off[i] + len[i]), its CRC goes to out[i]).
struct VrBatch {
    const uint8_t* bytes;
    const uint64_t* off;
    const uint32_t* len;
    uint32_t* out;
    uint64_t n;
    // set by vring_launch_list: the batch's first group in the launch's concatenated
    // group space (its G = ceil(n / packets per group) groups follow)
    uint64_t g0;
};
// Kernel-argument block (<= 4 KiB): up to kVrMaxBatches batches per launch.
constexpr int kVrMaxBatches = 48;
struct VrBatches {
    uint32_t count;
    // BIN with tile_counts: the number of 1024-record tiles (see tile_counts)
    uint32_t tiles;
    uint64_t groups;    // all batches' groups (set by vring_launch_list)
    // BIN only (one batch), or null: the binned gather's records, length_bin_tiles's
    // layout -- tile t's kept records sorted and padded with empty records to 1024,
    // rank-interleaved (group q T + t holds tile t's records [q kpk, (q + 1) kpk)) --
    // and tile_counts[t] = tile t's kept records.  The kernel runs the groups of the
    // ranks q < ceil(max_t tile_counts[t] / kpk): a count the host does not know.
    const uint32_t* tile_counts;
    // dynamic rounds (VrVariant::claim): the launch's claim word, or null for the
    // static deal, and the launch's generation of it
    uint64_t* claim;
    uint32_t claim_gen;
    // the local-tile records instance (vring_launch_local): packets per workgroup, and
    // the records it writes (16 B per packet, workgroup k's at [k tile_local, ...))
    uint32_t tile_local;
    void* local_rec;
    // ... and the shortest packet it keeps (shorter ones get no record and no CRC: the
    // binned gather's short segments, folded by its join); 0 = every packet
    uint32_t local_keep_min;
    uint32_t local_pad;
    VrBatch b[kVrMaxBatches];
};
static_assert(sizeof(VrBatches) <= 3072, "kernel arguments");

// One batch of a receive-verify list (c/protocol.cs:1052-1068 per DGRAM): the
// checksum fields (out = computed[], may be null) plus each DGRAM's slot offset and
// connectID and the keep mask ok[].
struct VrVBatch {
    const uint8_t* bytes;
    const uint64_t* off;
    const uint32_t* len;
    uint32_t* out;
    uint64_t n;
    uint64_t g0;
    const uint32_t* slot_off;
    const uint32_t* connect;
    uint8_t* ok;
};
constexpr int kVrMaxVBatches = 32;
struct VrVBatches {
    uint32_t count;
    uint32_t claim_gen;  // as VrBatches::claim_gen
    uint64_t groups;
    uint64_t* claim;     // as VrBatches::claim
    VrVBatch b[kVrMaxVBatches];
};
static_assert(sizeof(VrVBatches) <= 3072, "kernel arguments");

// Kernel variants.  The product library builds the default alone (all fields at
// their defaults); the diagnostics library (ENET_HIP_DIAG) also builds the sweep
// variants: nt = nontemporal stage loads, abl = ablations (crc32_vring.hip; most
// give wrong CRCs by design), walk = each workgroup takes a contiguous range of the
// launch's groups in order, tail_first = the tail-first stage order (crc32_vring.hip).
struct VrVariant {
    bool nt = false;
    int abl = 0;
    bool walk = false;
    bool tail_first = false;
    // dynamic rounds: the launch's claim word {generation, round counter} (64 bits, in
    // a line no launch in flight shares) and generation -- larger than any generation
    // the word has seen -- or null = the static deal
    uint64_t* claim = nullptr;
    uint32_t claim_gen = 0;
    // 1: one claim word for the launch (chip-wide rounds); 2 (diagnostics library):
    // claim points at an array of words, one per pair of workgroups k and k + G / 2
    // (the pair's rounds balance between its two workgroups; G made even)
    int claim_mode = 1;
    // length-binned records: the compact instance (no x^(-8 c) tables, two workgroups per CU)
    bool compact = false;
};
constexpr int kVrClaimWords = 16;     // 32-bit words: one 64-byte line per launch
constexpr int kVrPairWords = 512;     // pair rounds: 64-bit words per launch (grids up to 1024)

// Set the dynamic-LDS attribute of every vring kernel instance built (once per context).
int vring_setup();

// Launch over a list of batches (bl.count <= kVrMaxBatches): one launch, each batch
// spread over the whole chip in turn, at most max_wgs 16-wave workgroups (the CU
// count: one per CU; twice that: two).  trace = per-wave timestamps (diagnostics
// library) or null.  bin = the batches' metadata are length-binned records {len,
// off_lo, off_hi, index} (VrBatch::off points at them, len unused): results go to
// out[index].  70.5 KiB of LDS either way: one or two workgroups per CU.  Returns 0
// or -hipError_t (-hipErrorInvalidValue for a variant this library does not build).
int vring_launch_list(int lg, int max_wgs, const VrVariant& v, hipStream_t st, const VrBatches& bl,
                      const KernelTables& tb, const uint32_t* basis2, uint64_t* trace, bool bin = false);

// Receive verify over a list of batches (bl.count <= kVrMaxVBatches), 8 lanes per
// packet (lg = 3): the slot is substituted by connectID in the registers of the lane
// folding it, the CRC compared, ok[] and (if set) computed[] written.  Same
// workgroups, LDS and variants as vring_launch_list (trace: end records only).
int vring_launch_vlist(int max_wgs, const VrVariant& v, hipStream_t st, const VrVBatches& bl, const KernelTables& tb,
                       const uint32_t* basis2, uint64_t* trace);

// The length-binned checksum in ONE launch (enet_hip_crc32_batch_device_binned and
// the binned gather's segment pass when n <= kVrLocalTile x max_wgs): workgroup k
// takes the packets [k T, (k + 1) T) of the batch (T <= kVrLocalTile, a multiple of
// the packets per group), orders the records of those of at least keep_min bytes by
// window length in its own prologue -- a counting sort in LDS, the records written to
// `records` from 16 k T on (16 B per packet) -- and checksums them longest first,
// CRCs to out[index] (shorter packets: none).  No bin kernel, no dependent launch.
// Returns 0 or -hipError_t (-hipErrorInvalidValue when the batch is too large for one
// tile per workgroup).
constexpr uint32_t kVrLocalTile = 2048;
int vring_launch_local(int lg, int max_wgs, hipStream_t st, const PacketArgs& pa, void* records,
                       const KernelTables& tb, const uint32_t* basis2, uint32_t keep_min = 0);

// Launch the vring kernel over one batch: checksum mode, lanes per packet 2^lg
// (lg = 2 or 3), at most max_wgs workgroups; pa.meta4 set = binned records.
// basis2 = kVrBasisDwords per image (images for P = 1, 4, 8, 16 in that order).
int vring_launch(int lg, int max_wgs, const VrVariant& v, hipStream_t st, const PacketArgs& pa, const KernelTables& tb,
                 const uint32_t* basis2);

}  // namespace enethip
