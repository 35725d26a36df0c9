// fragment_kernels.hip -- batched fragment reassembly for gfx950 (MI355X): the
// data movement of ENet's receive-side fragment handler for a whole batch of
// SEND_FRAGMENT commands.
// Reference: /root/reference/enet-csharp/ENet/c/protocol.cs:529-637
// (enet_protocol_handle_send_fragment); the send-side split that produces the
// fragments is c/peer.cs:130-196; the command layout include/protocol.cs:156-165.
//
// What stays with the caller: the channel / sequence-window search that finds
// (or creates) the reassembly command (protocol.cs:540-545, 553-617).  The caller
// passes, per command, the reassembly slot it matched.  What runs here, per
// command, in the reference's order:
//   * the -1 checks of protocol.cs:546-552 and 571-577, and the startCommand
//     consistency check of 598-601 (totalLength / fragmentCount vs the slot);
//   * duplicate suppression by the slot's fragment bitmap (619-623), first
//     command in batch order wins, exactly as the sequential reference;
//   * fragmentsRemaining countdown (621) and the memcpy of the fragment data to
//     packet->data + fragmentOffset, length clamped as at 625-626.
// Memory: HBM-bound byte copy, 1 byte read + 1 byte written per fragment byte.
//
// Launches on one stream:
//   1. frag_claim_kernel (thread per command): parse, validate, atomicMin of the
//      command index into the claim word of its (slot, fragmentNumber), and leave
//      the parsed command in the copy-descriptor slots;
//   2. the decide step, one of two kernels (fragment_reassemble_launch picks
//      frag_decide_slots_kernel when the claim space, slots x bitmap bits, is at
//      most 8 n + 65536 words, else frag_decide_kernel): the claim winner (first
//      command of the batch for its fragment) tests-and-sets the bitmap bit (a bit
//      set by an earlier batch = duplicate), decrements remaining and gets a copy
//      descriptor.  Winners whose byte ranges may overlap another winner of the
//      same slot are DEFERRED (status 2): the slot kernel checks, per slot, that
//      the winners' ranges are disjoint and ascending in fragment-number order;
//      on the atomic path frag_clash_kernel runs the same check after the decide
//      kernel, for the slots with two or more winners (round 6);
//   3. the copy, 4 descriptors per wave as one flat space of 16-byte chunks:
//      frag_copy_claims_kernel on the slots path (descriptors slot-major in claim
//      space, written coalesced by the decide kernel: on a shuffled batch the
//      command-indexed stores cost the decide kernel 19.1 against 10.3 us,
//      profiles/r04_frag_copy/), frag_copy_kernel (by command) on the atomic path;
//      the non-deferred winners' copies, and the claim words back to ~0;
//   4. frag_serial_kernel (one wave; returns at once unless something was
//      deferred): the deferred winners in batch order, each command's stores
//      drained before the next, so where a batch's fragments overlap the later
//      command's bytes win as in the sequential reference (protocol.cs:628).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "fragment_kernels.hpp"

namespace enethip {

namespace {

constexpr uint32_t kMaxFragmentCount = 1024u * 1024u;   // ENET_PROTOCOL_MAXIMUM_FRAGMENT_COUNT, include/protocol.cs:19
constexpr uint32_t kCmdBytes = 24u;                      // sizeof(ENetProtocolSendFragment)

typedef uint32_t u32x4v __attribute__((ext_vector_type(4)));

struct Frag {
    uint32_t len, count, number, total, offset;
    int32_t slot;
    bool valid;
};

// Parse + validate command i (the -1 paths of protocol.cs:546-552, 571-577, 598-601).
__device__ __forceinline__ Frag parse(const FragArgs& a, uint64_t i) {
    Frag f{};
    f.slot = a.slots[i];
    f.valid = false;
    if (f.slot < 0 || static_cast<uint64_t>(f.slot) >= a.slot_count) return f;
    // the 24-byte command as two overlapping unaligned 16-byte loads (bytes 0-15, 8-23)
    const uint8_t* c = a.bytes + a.cmd_off[i];
    u32x4v h0, h1;
    __builtin_memcpy(&h0, c, 16);
    __builtin_memcpy(&h1, c + 8, 16);
    f.len = __builtin_bswap32(h0.y) & 0xFFFFu;            // sendFragment.dataLength, bytes 6-7
    f.count = __builtin_bswap32(h1.x);                    // bytes 8-11
    f.number = __builtin_bswap32(h1.y);
    f.total = __builtin_bswap32(h1.z);
    f.offset = __builtin_bswap32(h1.w);
    if (f.len == 0 || f.len > a.max_packet || f.len > a.cmd_avail[i]) return f;                 // 546-552
    if (f.count > kMaxFragmentCount || f.number >= f.count || f.total > a.max_packet || f.total < f.count ||
        f.offset >= f.total || f.len > f.total - f.offset)
        return f;                                                                              // 571-577
    if (f.total != a.msg_len[f.slot] || f.count != a.msg_count[f.slot]) return f;              // 598-601
    if (f.count > 32u * a.words) return f;               // bitmap smaller than fragmentCount bits: rejected
    f.valid = true;
    return f;
}

__device__ __forceinline__ uint64_t claim_index(const FragArgs& a, const Frag& f) {
    return (static_cast<uint64_t>(f.slot) * a.words << 5) + f.number;
}

__global__ void __launch_bounds__(256) frag_claim_kernel(FragArgs a) {
    const uint64_t stride = static_cast<uint64_t>(gridDim.x) * blockDim.x;
    for (uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < a.n; i += stride) {
        const Frag f = parse(a, i);
        const uint64_t cidx = f.valid ? claim_index(a, f) : ~0ull;
        if (f.valid) atomicMin(a.claim + cidx, static_cast<uint32_t>(i));
        a.status[i] = f.valid ? 0 : (f.slot < 0 ? 0 : -1);
        // the parsed command for the decide kernel (its copy descriptor slots, overwritten there)
        a.copy_claim[i] = cidx;
        a.copy_src[i] = f.len;
        a.copy_dst[i] = static_cast<uint64_t>(f.offset) | (static_cast<uint64_t>(static_cast<uint32_t>(f.slot)) << 32);
        a.copy_len[i] = 0;                                   // nothing to copy unless a decide kernel says so
    }
}

// Thread per command: the claim winner tests-and-sets the bitmap bit (a bit set
// by an earlier batch = duplicate) and counts itself into its slot's winners
// (frag_clash_kernel decrements remaining by that count); every command gets a
// copy descriptor (len 0 = nothing to copy) for the copy kernel.
// Reads the command as the claim kernel parsed it (no second parse of the arena).
__global__ void __launch_bounds__(256) frag_decide_kernel(FragArgs a) {
    const uint64_t stride = static_cast<uint64_t>(gridDim.x) * blockDim.x;
    for (uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < a.n; i += stride) {
        const uint64_t cidx = a.copy_claim[i];
        uint32_t len = 0;
        uint64_t src = 0, dst = 0;
        if (cidx != ~0ull && a.claim[cidx] == static_cast<uint32_t>(i)) {   // first command of the batch for it
            const uint64_t packed = a.copy_dst[i];
            const uint32_t slot = static_cast<uint32_t>(packed >> 32), offset = static_cast<uint32_t>(packed);
            const uint32_t number = static_cast<uint32_t>(cidx - (static_cast<uint64_t>(slot) * a.words << 5));
            const uint32_t bit = 1u << (number & 31u);
            const uint32_t old =
                atomicOr(a.fragments + static_cast<uint64_t>(slot) * a.words + (number >> 5), bit);   // 619, 623
            if (!(old & bit)) {
                // winners per slot: frag_clash_kernel takes them off fragmentsRemaining (621)
                // with one subtraction per slot (a second contended atomic per winner cost
                // more than the whole overlap check)
                atomicAdd(a.wcount + slot, 1u);
                a.status[i] = 1;
                len = min(static_cast<uint32_t>(a.copy_src[i]), a.msg_len[slot] - offset);   // clamp (625-626)
                src = a.cmd_off[i] + kCmdBytes;
                dst = a.msg_off[slot] + offset;
            }
        }
        a.copy_src[i] = src;
        a.copy_dst[i] = dst;
        a.copy_len[i] = len;
    }
}

// Same decisions without atomics: one wave owns a slot and walks its claim words
// 64 fragment numbers at a time; the winner (first command of the batch) of a
// fragment whose bitmap bit is clear sets it, counts it off fragmentsRemaining and
// gets its copy descriptor.  Used when the claim space (slots x bitmap bits) is
// not much larger than the batch.
__global__ void __launch_bounds__(256) frag_decide_slots_kernel(FragArgs a) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t waves = static_cast<uint64_t>(gridDim.x) * (blockDim.x >> 6);
    const uint32_t bits = a.words << 5;
    for (uint64_t sl = static_cast<uint64_t>(blockIdx.x) * (blockDim.x >> 6) + (threadIdx.x >> 6); sl < a.slot_count;
         sl += waves) {
        uint32_t* bm = a.fragments + sl * a.words;
        uint32_t removed = 0;
        uint32_t mx = 0;                                   // largest end of the slot's winners so far
        bool clash = false;                                // a winner starts before an earlier one ends
        for (uint32_t f0 = 0; f0 < bits; f0 += 64u) {
            const uint32_t f = f0 + lane;
            const uint32_t w = f < bits ? a.claim[sl * bits + f] : ~0u;
            bool take = false;
            if (w != ~0u) take = ((bm[f >> 5] >> (f & 31u)) & 1u) == 0u;               // 619-620
            const uint64_t m = __ballot(take);
            if (lane == 0u && static_cast<uint32_t>(m)) bm[f0 >> 5] |= static_cast<uint32_t>(m);        // 623
            if (lane == 32u && (m >> 32) && (f0 >> 5) + 1u < a.words) bm[(f0 >> 5) + 1u] |= static_cast<uint32_t>(m >> 32);
            removed += static_cast<uint32_t>(__builtin_popcountll(m));
            uint32_t offset = 0, end = 0;
            const uint64_t q = sl * bits + f;             // the claim-space descriptor (coalesced)
            if (f < bits) {
                uint32_t len = 0;
                if (take) {
                    const uint64_t packed = a.copy_dst[w];
                    offset = static_cast<uint32_t>(packed);
                    len = min(static_cast<uint32_t>(a.copy_src[w]), a.msg_len[sl] - offset);   // 625-626
                    end = offset + len;
                    a.status[w] = 1;
                    a.q_src[q] = a.cmd_off[w] + kCmdBytes;
                    a.q_dst[q] = a.msg_off[sl] + offset;
                }
                a.q_len[q] = len;                          // (every number: 0 = nothing to copy)
            }
            if (m) {
                // exclusive prefix max of the winners' ends in fragment-number (lane) order
                uint32_t pm = end;
#pragma unroll
                for (int d = 1; d < 64; d <<= 1) {
                    const uint32_t o = static_cast<uint32_t>(__shfl_up(static_cast<int>(pm), d));
                    if (lane >= static_cast<uint32_t>(d)) pm = max(pm, o);
                }
                uint32_t before = static_cast<uint32_t>(__shfl_up(static_cast<int>(pm), 1));
                before = lane ? max(before, mx) : mx;
                if (__ballot(take && offset < before)) clash = true;
                mx = max(mx, static_cast<uint32_t>(__shfl(static_cast<int>(pm), 63)));
            }
        }
        if (lane == 0u && removed) a.remaining[sl] -= removed;                     // 621
        if (clash) {                                       // defer the slot's winners to the serial pass
            for (uint32_t f0 = 0; f0 < bits; f0 += 64u) {
                const uint32_t f = f0 + lane;
                const uint64_t q = sl * bits + f;
                const uint32_t w = f < bits ? a.claim[q] : ~0u;
                if (w != ~0u && a.status[w] == 1) {        // (this lane wrote q's descriptor above)
                    a.status[w] = 2;
                    a.copy_len[w] = a.q_len[q];            // the serial pass copies by command
                    a.copy_src[w] = a.q_src[q];
                    a.copy_dst[w] = a.q_dst[q];
                    a.q_len[q] = 0u;                       // not in the claim-space copy
                }
            }
            if (lane == 0u) *a.deferred = 1u;
        }
    }
}

// The atomic decide path's overlap check (round 6).  Before, the atomic path deferred
// every slot with two or more winners to the one-wave serial pass: a batch of ordinary
// multi-fragment messages against a large claim space (a host that sizes its bitmaps
// for its largest message) was copied one command at a time -- cfg5 with 64 bitmap
// words per slot took 282 ms per call, against 0.15 ms on the slots path
// (profiles/r06_frag/).  Now one wave per slot with two or more winners walks the
// slot's claim words in fragment-number order, as frag_decide_slots_kernel does, but
// only up to min(bits, fragmentCount) -- no command of a slot carries a number past its
// fragmentCount (parse) -- and defers the slot's winners (status 2) only when their
// byte ranges are not disjoint and ascending in number order.  The walk reads one
// claim word per number, so a slot of more than 1024 numbers and over 64 per winner
// (a few fragments of a huge message) is not walked: its winner count becomes
// kDeferSlot and frag_copy_kernel defers its winners as before (the serial pass puts
// the count back to 0).  Every other slot's winner count goes back to 0 here.
constexpr uint32_t kClashWalkPerWinner = 64u;    // numbers walked per winner before deferring instead
constexpr uint32_t kClashWalkFree = 1024u;       // numbers always walked
constexpr uint32_t kDeferSlot = ~0u;             // winner count of a slot whose winners all go serial
__global__ void __launch_bounds__(256) frag_clash_kernel(FragArgs a) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t waves = static_cast<uint64_t>(gridDim.x) * (blockDim.x >> 6);
    const uint32_t bits = a.words << 5;
    for (uint64_t sl = static_cast<uint64_t>(blockIdx.x) * (blockDim.x >> 6) + (threadIdx.x >> 6); sl < a.slot_count;
         sl += waves) {
        const uint32_t wc = a.wcount[sl];
        if (wc == 0u) continue;
        if (lane == 0u) a.remaining[sl] -= wc;             // --fragmentsRemaining per winner (621)
        if (wc >= 2u) {
            const uint32_t nb = min(bits, a.msg_count[sl]);
            const uint64_t mo = a.msg_off[sl];
            if (nb > max(kClashWalkFree, kClashWalkPerWinner * wc)) {   // too sparse to walk: defer them all
                if (lane == 0u) a.wcount[sl] = kDeferSlot;
                continue;
            }
            bool clash = false;
            uint32_t mx = 0;                               // largest end of the slot's winners so far
            for (uint32_t f0 = 0; f0 < nb && !clash; f0 += 64u) {
                const uint32_t f = f0 + lane;
                const uint32_t w = f < nb ? a.claim[sl * bits + f] : ~0u;
                const bool take = w != ~0u && a.status[w] == 1;
                if (!__ballot(take)) continue;
                uint32_t offset = 0, end = 0;
                if (take) {
                    offset = static_cast<uint32_t>(a.copy_dst[w] - mo);
                    end = offset + a.copy_len[w];
                }
                // exclusive prefix max of the winners' ends in fragment-number (lane) order
                uint32_t pm = end;
#pragma unroll
                for (int d = 1; d < 64; d <<= 1) {
                    const uint32_t o = static_cast<uint32_t>(__shfl_up(static_cast<int>(pm), d));
                    if (lane >= static_cast<uint32_t>(d)) pm = max(pm, o);
                }
                uint32_t before = static_cast<uint32_t>(__shfl_up(static_cast<int>(pm), 1));
                before = lane ? max(before, mx) : mx;
                if (__ballot(take && offset < before)) clash = true;
                mx = max(mx, static_cast<uint32_t>(__shfl(static_cast<int>(pm), 63)));
            }
            if (clash) {                                   // the slot's winners to the serial pass, in batch order
                for (uint32_t f0 = 0; f0 < nb; f0 += 64u) {
                    const uint32_t f = f0 + lane;
                    const uint32_t w = f < nb ? a.claim[sl * bits + f] : ~0u;
                    if (w != ~0u && a.status[w] == 1) a.status[w] = 2;
                }
                if (lane == 0u) *a.deferred = 1u;
            }
        }
        if (lane == 0u) a.wcount[sl] = 0u;                 // for the next batch
    }
}

// Unaligned 16-byte access (gfx950 unaligned mode), both ways with the nontemporal
// policy: every fragment byte is read once and written once, so neither side is worth
// keeping in L2 (cfg5 151.1 against 159.7 us with the default policy,
// profiles/r05_frag_nt/)
typedef uint32_t u32x4u __attribute__((ext_vector_type(4), aligned(1)));
__device__ __forceinline__ u32x4v load16(const uint8_t* p) {
    return __builtin_nontemporal_load(reinterpret_cast<const u32x4u*>(p));
}
__device__ __forceinline__ void store16(uint8_t* p, u32x4v v) {
    __builtin_nontemporal_store(static_cast<u32x4u>(v), reinterpret_cast<u32x4u*>(p));
}

__device__ __forceinline__ void copy_span(const uint8_t* src, uint8_t* dst, uint32_t L, uint32_t x) {
    if (x + 16u <= L) {
        store16(dst + x, load16(src + x));
    } else {
        for (uint32_t b = x; b < L; ++b) dst[b] = src[b];
    }
}

// One wave copies kCopyCmds commands at a time as one flat space of 16-byte chunks
// (chunk k of the wave belongs to the command whose prefix range holds it), so a
// 1360-byte fragment no longer leaves a third of the lanes idle in its second pass.
// Every write stays inside [dst, dst + len) of its own command.
constexpr uint32_t kCopyCmds = 4;

__global__ void __launch_bounds__(256) frag_copy_kernel(FragArgs a) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t waves = static_cast<uint64_t>(gridDim.x) * (blockDim.x >> 6);
    const uint64_t w = static_cast<uint64_t>(blockIdx.x) * (blockDim.x >> 6) + (threadIdx.x >> 6);
    for (uint64_t base = w * kCopyCmds; base < a.n; base += waves * kCopyCmds) {
        uint32_t L[kCopyCmds], pre[kCopyCmds + 1];
        uint64_t src[kCopyCmds], dst[kCopyCmds];
        pre[0] = 0;
#pragma unroll
        for (uint32_t c = 0; c < kCopyCmds; ++c) {
            const uint64_t i = base + c;
            const bool h = i < a.n;
            L[c] = h ? a.copy_len[i] : 0u;
            const uint64_t ci = h ? a.copy_claim[i] : ~0ull;
            bool defer = false;
            if (L[c]) {
                const int8_t st = a.status[i];
                const uint64_t slot = ci / (static_cast<uint64_t>(a.words) << 5);
                // deferred by frag_clash_kernel: its own status, or its whole slot
                defer = st == 2 || a.wcount[slot] == kDeferSlot;
                if (lane == c) {
                    if (defer && st != 2) {
                        a.status[i] = 2;
                        *a.deferred = 1u;
                    }
                }
            }
            if (defer) L[c] = 0u;                          // copied by frag_serial_kernel, in batch order
            src[c] = h ? a.copy_src[i] : 0u;
            dst[c] = h ? a.copy_dst[i] : 0u;
            pre[c + 1] = pre[c] + ((L[c] + 15u) >> 4);
            if (h && lane == c && ci != ~0ull) a.claim[ci] = ~0u;   // claim words back to ~0 for the next batch
        }
        // chunk k's command, its byte x and its end
        auto chunk = [&](uint32_t k, uint32_t& Lc, uint64_t& sc, uint64_t& dc, uint32_t& x) __attribute__((always_inline)) {
            uint32_t c = 0;
#pragma unroll
            for (uint32_t q = 1; q < kCopyCmds; ++q) c += k >= pre[q] ? 1u : 0u;
            uint32_t pc = pre[0];
            Lc = L[0];
            sc = src[0];
            dc = dst[0];
#pragma unroll
            for (uint32_t q = 1; q < kCopyCmds; ++q)
                if (c == q) {
                    Lc = L[q];
                    pc = pre[q];
                    sc = src[q];
                    dc = dst[q];
                }
            x = (k - pc) << 4;
        };
        // two chunks per lane per turn: both whole-chunk loads issued before either store
        const uint32_t nk = pre[kCopyCmds];
        for (uint32_t k = lane; k < nk; k += 128u) {
            uint32_t L0, L1, x0, x1;
            uint64_t s0, d0, s1, d1;
            chunk(k, L0, s0, d0, x0);
            const bool two = k + 64u < nk;
            chunk(two ? k + 64u : k, L1, s1, d1, x1);
            const bool f0 = x0 + 16u <= L0, f1 = two && x1 + 16u <= L1;
            u32x4v v0 = {0u, 0u, 0u, 0u}, v1 = {0u, 0u, 0u, 0u};
            if (f0) v0 = load16(a.bytes + s0 + x0);
            if (f1) v1 = load16(a.bytes + s1 + x1);
            if (f0) store16(a.msg_bytes + d0 + x0, v0);
            else copy_span(a.bytes + s0, a.msg_bytes + d0, L0, x0);
            if (f1) store16(a.msg_bytes + d1 + x1, v1);
            else if (two) copy_span(a.bytes + s1, a.msg_bytes + d1, L1, x1);
        }
    }
}

// The slots decide path's copy: one wave takes kCopyCmds fragment numbers of the
// claim space at a time (a slot's fragments in number order, so the message is
// written front to back), as one flat space of 16-byte chunks, and puts every claim
// word back to ~0 for the next batch.
__global__ void __launch_bounds__(256) frag_copy_claims_kernel(FragArgs a, uint64_t claims) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t waves = static_cast<uint64_t>(gridDim.x) * (blockDim.x >> 6);
    const uint64_t w = static_cast<uint64_t>(blockIdx.x) * (blockDim.x >> 6) + (threadIdx.x >> 6);
    for (uint64_t base = w * kCopyCmds; base < claims; base += waves * kCopyCmds) {
        uint32_t L[kCopyCmds], pre[kCopyCmds + 1];
        uint64_t src[kCopyCmds], dst[kCopyCmds];
        pre[0] = 0;
#pragma unroll
        for (uint32_t c = 0; c < kCopyCmds; ++c) {
            const uint64_t q = base + c;
            const bool h = q < claims;
            L[c] = h ? a.q_len[q] : 0u;
            src[c] = L[c] ? a.q_src[q] : 0u;
            dst[c] = L[c] ? a.q_dst[q] : 0u;
            pre[c + 1] = pre[c] + ((L[c] + 15u) >> 4);
            if (h && lane == c) a.claim[q] = ~0u;
        }
        const uint32_t nk = pre[kCopyCmds];
        for (uint32_t k = lane; k < nk; k += 64u) {
            uint32_t c = 0;
#pragma unroll
            for (uint32_t q = 1; q < kCopyCmds; ++q) c += k >= pre[q] ? 1u : 0u;
            uint32_t Lc = L[0], pc = pre[0];
            uint64_t sc = src[0], dc = dst[0];
#pragma unroll
            for (uint32_t q = 1; q < kCopyCmds; ++q)
                if (c == q) {
                    Lc = L[q];
                    pc = pre[q];
                    sc = src[q];
                    dc = dst[q];
                }
            copy_span(a.bytes + sc, a.msg_bytes + dc, Lc, (k - pc) << 4);
        }
    }
}

// One wave: the deferred winners (status 2) in batch order.  A command's stores
// are drained (vmcnt counts stores on gfx950) before the next command's begin, so
// overlapping bytes end up with the later command's data (protocol.cs:628 copies
// in arrival order).  Resets the deferred flag and the slots' winner counts.
__global__ void __launch_bounds__(64) frag_serial_kernel(FragArgs a) {
    if (*a.deferred == 0u) return;
    const uint32_t lane = threadIdx.x & 63u;
    for (uint64_t i0 = 0; i0 < a.n; i0 += 64u) {
        const uint64_t i = i0 + lane;
        const bool mine = i < a.n && a.status[i] == 2;
        uint64_t m = __ballot(mine);
        while (m) {
            const uint32_t c = static_cast<uint32_t>(__builtin_ctzll(m));
            m &= m - 1u;
            const uint64_t j = i0 + c;
            const uint32_t L = a.copy_len[j];
            const uint64_t src = a.copy_src[j], dst = a.copy_dst[j];
            for (uint32_t x = lane << 4; x < L; x += 64u << 4) copy_span(a.bytes + src, a.msg_bytes + dst, L, x);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this command's stores done before the next's
            if (lane == 0u) {
                a.status[j] = 1;
                const uint64_t ci = a.copy_claim[j];
                a.wcount[ci / (static_cast<uint64_t>(a.words) << 5)] = 0u;
            }
        }
    }
    if (lane == 0u) *a.deferred = 0u;
}

}  // namespace

int fragment_reassemble_launch(const FragArgs& a, int num_cus, hipStream_t st) {
    if (a.n == 0) return 0;
    const uint64_t cap = static_cast<uint64_t>(num_cus) * 8u;
    const unsigned g_thr = static_cast<unsigned>(std::max<uint64_t>(1, std::min<uint64_t>((a.n + 255) / 256, cap)));
    const unsigned g_wave = static_cast<unsigned>(
        std::max<uint64_t>(1, std::min<uint64_t>((a.n + 4 * kCopyCmds - 1) / (4 * kCopyCmds), cap)));
    hipLaunchKernelGGL(frag_claim_kernel, dim3(g_thr), dim3(256), 0, st, a);
    const uint64_t claim_space = a.slot_count * (static_cast<uint64_t>(a.words) << 5);
    if (frag_slots_path(claim_space, a.n)) {
        if (!a.q_src || !a.q_dst || !a.q_len) return -static_cast<int>(hipErrorInvalidValue);
        const unsigned g_slot = static_cast<unsigned>(std::max<uint64_t>(1, std::min<uint64_t>((a.slot_count + 3) / 4, cap)));
        hipLaunchKernelGGL(frag_decide_slots_kernel, dim3(g_slot), dim3(256), 0, st, a);
        // (slot-major descriptors: the claims' copy, message by message)
        const unsigned g_q = static_cast<unsigned>(
            std::max<uint64_t>(1, std::min<uint64_t>((claim_space + 4 * kCopyCmds - 1) / (4 * kCopyCmds), cap)));
        hipLaunchKernelGGL(frag_copy_claims_kernel, dim3(g_q), dim3(256), 0, st, a, claim_space);
    } else {
        hipLaunchKernelGGL(frag_decide_kernel, dim3(g_thr), dim3(256), 0, st, a);
        const unsigned g_clash = static_cast<unsigned>(std::max<uint64_t>(1, std::min<uint64_t>((a.slot_count + 3) / 4, cap)));
        hipLaunchKernelGGL(frag_clash_kernel, dim3(g_clash), dim3(256), 0, st, a);
        hipLaunchKernelGGL(frag_copy_kernel, dim3(g_wave), dim3(256), 0, st, a);
    }
    hipLaunchKernelGGL(frag_serial_kernel, dim3(1), dim3(64), 0, st, a);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : -static_cast<int>(e);
}

}  // namespace enethip
