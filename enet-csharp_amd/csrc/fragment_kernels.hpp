// fragment_kernels.hpp -- host-side entry of the batched fragment reassembly
// kernels (fragment_kernels.hip), called by enet_hip_fragment_reassemble_device.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace enethip {

struct FragArgs {
    const uint8_t* bytes;        // received DGRAM arena
    const uint64_t* cmd_off;     // command i: 24-byte ENetProtocolSendFragment at bytes + cmd_off[i]
    const uint32_t* cmd_avail;   // bytes available after the command (its data must fit)
    const int32_t* slots;        // reassembly slot of command i, or -1 (skipped)
    uint64_t n;
    uint32_t max_packet;         // host->maximumPacketSize
    uint8_t* msg_bytes;          // reassembly buffers
    const uint64_t* msg_off;     // slot s: packet data at msg_bytes + msg_off[s]
    const uint32_t* msg_len;     //   its totalLength
    const uint32_t* msg_count;   //   its fragmentCount
    uint32_t* fragments;         //   received-fragment bitmap, `words` uint32 per slot
    uint32_t words;
    uint32_t* remaining;         //   fragmentsRemaining
    uint64_t slot_count;
    int8_t* status;              // per command: -1 rejected, 0 skipped / duplicate, 1 copied
                                 // (2 = deferred to the serial pass, internal only)
    uint32_t* claim;             // scratch, slot_count * words * 32 words, all ~0 between calls
    uint32_t* wcount;            // scratch, slot_count words: winners per slot (atomic decide), 0 between calls
    uint32_t* deferred;          // scratch word: some winner was deferred, 0 between calls
    uint64_t* copy_src;          // scratch, n each: copy descriptors (decide -> copy kernel)
    uint64_t* copy_dst;
    uint32_t* copy_len;
    uint64_t* copy_claim;
    // scratch, claim space (slot_count * words * 32 each), the slots decide path only:
    // the copy descriptor of fragment number f of slot s at s * words * 32 + f
    // (len 0 = nothing to copy), written coalesced and copied in message order
    uint64_t* q_src;
    uint64_t* q_dst;
    uint32_t* q_len;
};

// the slots decide path (claim space descriptors) serves a batch whose claim space
// (slots x bitmap bits) is at most this many words
inline bool frag_slots_path(uint64_t claim_space, uint64_t n) { return claim_space <= 8u * n + 65536u; }

int fragment_reassemble_launch(const FragArgs& a, int num_cus, hipStream_t st);

}  // namespace enethip
