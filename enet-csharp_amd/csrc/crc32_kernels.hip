// crc32_kernels.hip -- gfx950 (MI355X, CDNA4) kernels of libenethip and the
// C-ABI entry points that launch them.  See DESIGN.md for the derivation.
//
// Path replaced: ENet.enet_crc32 (/root/reference/enet-csharp/ENet/c/packet.cs:142-160)
// applied to a whole batch of DGRAMs at once.  Bit-exact with the reference: the
// kernels compute the same Sarwate register (packet.cs:153) by a different but
// algebraically identical route.
//
// Kernels:
//   * crc32_lean_kernel (crc32_lean.hip) -- the hot path for 4 and 8 lanes per
//     packet: persistent, LDS-DMA streamed, strided lanes, table rebuilt in LDS;
//   * crc32_stream_kernel -- the same arithmetic with per-lane-run staging: 16
//     lanes per packet and the sweep geometries (enet_hip_set_kernel_path).
//   * crc32_direct_kernel -- general fallback (any lanes per packet): blocks
//     loaded into VGPRs, contiguous segments joined by the carry-combine.
//   * crc32_gather_kernel -- one lane per DGRAM over an ENetBuffer gather list.
// All fold 32-byte blocks with slicing-by-32 from a conflict-free 64 KiB LDS
// image (crc32_device.hpp); every identity used is modelled and checked against
// the oracle on CPU in tests/kernel_model.py.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <thread>
#include <tuple>
#include <vector>

#include "crc32_device.hpp"
#include "crc32_math.hpp"
#include "crc32_lean.hpp"
#include "crc32_vring.hpp"
#include "crc32_stream_common.hpp"
#include "context.hpp"
#include "enet_hip.h"
#include "fragment_kernels.hpp"
#include "gather_join.hpp"
#include "range_coder.hpp"

namespace enethip {

constexpr int kThreads = 512;                     // direct / gather kernels: 8 waves

template <int NT>
__device__ __forceinline__ void fill_table(uint8_t* lds, const uint32_t* image) {
    const u32x4* src = reinterpret_cast<const u32x4*>(image);
    u32x4* dst = reinterpret_cast<u32x4*>(lds);
#pragma unroll
    for (int i = threadIdx.x; i < kLdsTableBytes / 16; i += NT) dst[i] = src[i];
    __syncthreads();
}

#ifdef ENET_HIP_DIAG   // the LDS-stream and direct kernels: 16 / 1, 2, 32, 64 lanes (diagnostics only since round 5)
// ============================================================ stream kernel
//
// One persistent workgroup of W waves per CU.  A wave owns groups g = wv,
// wv + W*grid, ...; a group is 64 consecutive tasks = 64/P packets, P = 2^lg
// (4, 8 or 16) lanes per packet.  Per packet (crc32 of bytes [a, a+L)):
//   * window: NB whole 32-byte blocks ending at the 16-byte granule boundary at
//     or after the packet end (tz < 16 zero bytes behind, lz < 32 in front).  A
//     16-byte piece wholly in front of the packet is read from a zero buffer
//     (memory-safe at page ends, no masking); only partial head/tail pieces of
//     unaligned packets get byte masks;
//   * lane k folds the window blocks w with (w + r) % P == k, r = (-NB) % P,
//     using the ADVANCING tables T'_t = T_{t+32(P-1)} of this P: each fold also
//     skips the P-1 blocks the other lanes own, so the P lanes of a packet walk
//     it front to back together and one stage of a packet is ONE contiguous
//     P*SB*32-byte chunk.  The rotation r makes lane k end exactly 32k bytes
//     past the window end; the block-0 lane (k == r) starts at INIT[lz];
//   * finish: lane k undoes its 32k-byte overshoot by x^(-256k) = four byte-
//     indexed lookups in the image's correction columns, the P registers are
//     XORed (DPP), then x^(-8 tz) for packets whose end is not 16-byte aligned.
// No x^(8n) gathers and no alignment precondition.  Verify mode substitutes the
// slot bytes by connectID inside the block that holds them (protocol.cs:1052-1068)
// and collects the original bytes as `desired`.  tests/kernel_model.py restates
// all of it and checks it against the oracle.
//
// Memory: everything a wave reads from HBM arrives by LDS-DMA
// (global_load_lds): its share of the table image, the per-group packet
// metadata and the packet bytes.  A wave streams its groups through a ring of
// NB stage buffers (a stage = SB blocks of every lane) with NB-1 stages in flight
// while one is folded, ACROSS group boundaries: the next group's metadata is
// fetched one group ahead and its first stages are issued while the current
// group is still being folded.  The wave's own counted s_waitcnt vmcnt(N) orders
// DMA and ds_read (N = VMEM operations issued after the awaited one; stores are
// not counted, which only over-waits).  The loop is unrolled NB times so every
// ring address is an immediate.
template <int W, int SB, int NB>
struct StreamGeom {
    static constexpr int kWaves = W, kSB = SB, kNB = NB;
    static constexpr int kThreads = 64 * W;
    static constexpr uint32_t kRun = 32u * SB;               // bytes per lane per stage
    static constexpr uint32_t kStage = 64u * kRun;           // bytes per wave per stage
    static constexpr int kDma = static_cast<int>(kStage / 1024u);
    static constexpr uint32_t kPieces = kRun / 16u;          // 16-byte pieces per run
    static constexpr uint32_t kRunsPerDma = 1024u / kRun;
    static constexpr uint32_t kLsb = SB == 1 ? 0u : SB == 2 ? 1u : 2u;
    static constexpr uint32_t kMetaAhead = 2;                // metadata fetched this many groups ahead
    static constexpr uint32_t kMetaSlots = NB + kMetaAhead;
    static constexpr uint32_t kMetaSlot = 512u;
    static constexpr uint32_t kWaveLds = NB * kStage + kMetaSlots * kMetaSlot;
    static constexpr int kLds = kLdsTableBytes + W * static_cast<int>(kWaveLds);
    static constexpr int kTableRounds = (kImageDwords / 4 + 64 * W - 1) / (64 * W);
    static_assert(kLds <= 160 * 1024, "LDS budget");
    static_assert(NB >= 2 && NB <= 4 && (SB == 1 || SB == 2 || SB == 4), "geometry");
};


// Lane c's run sits at buf + kRun*c, its 16-byte piece p in slot p ^ swz(c):
// swz(c) = ((c >> log2(16/R)) & (R-1)) ^ ((c >> 4) & 1), R = pieces per run,
// keeps every 16-lane ds_read_b128 group on 16 distinct slots (the (c >> 4) term
// undoes the lane's half swap).
template <class G>
__device__ __forceinline__ uint32_t run_swz(uint32_t c) {
    constexpr uint32_t R = G::kPieces;
    constexpr uint32_t sh = R == 2 ? 3u : R == 4 ? 2u : R == 8 ? 1u : 0u;
    return ((c >> sh) & (R - 1u)) ^ ((c >> 4) & 1u);
}

// Metadata of one group into a meta slot: field f of packet j lands at
// slot + 4*(f*Gp + j); f = 0 len, 1/2 offset lo/hi, 3 slot offset, 4 connectID.
template <int MODE>
__device__ __forceinline__ void issue_meta(const PacketArgs& pa, uint64_t pk0, uint32_t lg, uint32_t nmeta,
                                           uint32_t slot, uint32_t lane) {
    const uint32_t gsh = 6u - lg;                     // log2(packets per group)
    for (uint32_t r = 0; r < nmeta; ++r) {
        const uint32_t idx = 64u * r + lane;
        const uint32_t f = idx >> gsh;
        const uint64_t pk = min(pk0 + (idx & ((1u << gsh) - 1u)), pa.n - 1);
        const uint32_t* src = pa.len + pk;
        if (f == 1u || f == 2u) src = reinterpret_cast<const uint32_t*>(pa.off) + 2u * pk + (f - 1u);
        if (MODE && f == 3u) src = pa.slot_off + pk;
        if (MODE && f == 4u) src = pa.connect + pk;
        dma4(src, slot + 256u * r);
    }
}

__device__ __forceinline__ uint32_t meta_field(uint32_t slot, uint32_t lg, uint32_t f, uint32_t j) {
    return lds_load(slot + 4u * ((f << (6u - lg)) + j));
}

__device__ __forceinline__ Window packet_window(const PacketArgs& pa, uint32_t slot, uint32_t lg, uint64_t pk0,
                                                uint32_t j) {
    Window w;
    w.active = pk0 + j < pa.n;
    w.L = w.active ? meta_field(slot, lg, 0, j) : 0u;
    const uint64_t off = static_cast<uint64_t>(meta_field(slot, lg, 1, j)) |
                         (static_cast<uint64_t>(meta_field(slot, lg, 2, j)) << 32);
    const uint64_t a = reinterpret_cast<uint64_t>(pa.bytes) + off, e = a + w.L;
    // the window ends at the granule boundary at or after the packet end
    w.tz = w.L ? static_cast<uint32_t>((0u - e) & 15u) : 0u;
    w.nb = w.L ? (w.L + w.tz + 31u) >> 5 : 0u;
    w.lz = 32u * w.nb - w.tz - w.L;
    w.ws = e + w.tz - 32ull * w.nb;
    w.r = (0u - w.nb) & ((1u << lg) - 1u);
    return w;
}

// Producer side of a group: per DMA slot i, the address of this lane's 16-byte
// piece at the group's next stage and how many stages it holds packet bytes;
// past that, and for a head piece lying wholly in front of the packet, the
// piece is read from the zero buffer (so whole-piece head/tail zeroing is free).
template <class G>
struct Producer {
    uint64_t cur[G::kDma];
    uint32_t nval[G::kDma];
    uint32_t head;       // bit i: piece i is a wholly-outside head piece at stage 0
    uint32_t stages;
};

template <class G>
__device__ __forceinline__ void producer_setup(Producer<G>& pr, const PacketArgs& pa, uint32_t slot, uint32_t lg,
                                               uint64_t pk0, uint32_t lane) {
    const uint32_t P = 1u << lg;
    uint32_t most = 0;
    pr.head = 0;
#pragma unroll
    for (int i = 0; i < G::kDma; ++i) {
        const uint32_t c = G::kRunsPerDma * i + lane / G::kPieces;    // run (task lane) of this piece
        const uint32_t p = (lane % G::kPieces) ^ run_swz<G>(c);        // piece index in the run
        const uint32_t b = p >> 1, h = p & 1u;
        const Window w = packet_window(pa, slot, lg, pk0, c >> lg);
        const uint32_t w0 = ((c - w.r) & (P - 1u)) + P * b;            // block of this piece at stage 0
        (void)h;
        pr.nval[i] = w0 < w.nb ? ((w.nb - 1u - w0) >> (lg + G::kLsb)) + 1u : 0u;
        if (w0 == 0 && h == 0 && w.lz >= 16u) pr.head |= 1u << i;
        pr.cur[i] = w.ws + 32ull * w0 + 16u * h;
        most = max(most, pr.nval[i]);
    }
    pr.stages = max(1u, wave_max_u(most));        // a group of empty packets: one stage of zero lines
}

template <int MODE>
__device__ __forceinline__ Task consumer_setup(const PacketArgs& pa, uint32_t slot, uint32_t lg, uint64_t pk0,
                                               uint32_t lane) {
    const uint32_t P = 1u << lg;
    Task t;
    const uint32_t j = lane >> lg;
    const Window w = packet_window(pa, slot, lg, pk0, j);
    t.pk = pk0 + j;
    t.active = w.active;
    t.k = lane & (P - 1u);
    t.w0 = (t.k - w.r) & (P - 1u);
    t.nb = w.nb;
    t.lz = w.lz;
    t.tz = w.tz;
    t.cnt = t.w0 < w.nb ? ((w.nb - 1u - t.w0) >> lg) + 1u : 0u;
    t.reg = t.k == w.r ? lds_load(init_addr(w.lz)) : 0u;
    // partial head / tail pieces need byte masks (whole ones come from the zero buffer)
    t.e0 = ((w.lz & 15u) && t.w0 == 0 && w.nb) ? 0u : ~0u;
    t.e1 = (w.tz && t.cnt && t.w0 + P * (t.cnt - 1u) == w.nb - 1u) ? t.cnt - 1u : ~0u;
    t.e2 = t.e3 = ~0u;
    t.ps = -4096;
    t.connect = 0;
    t.slot_ok = false;
    if (MODE) {
        const uint32_t so = meta_field(slot, lg, 3, j);
        t.connect = meta_field(slot, lg, 4, j);
        t.slot_ok = w.L >= 4u && so <= w.L - 4u;
        if (t.slot_ok) {
            t.ps = static_cast<int32_t>(w.lz + so);
            const uint32_t ws_ = static_cast<uint32_t>(t.ps) >> 5, we_ = static_cast<uint32_t>(t.ps + 3) >> 5;
            if (((ws_ + w.r) & (P - 1u)) == t.k) t.e2 = ws_ >> lg;
            if (we_ != ws_ && ((we_ + w.r) & (P - 1u)) == t.k) t.e3 = we_ >> lg;
        }
    }
    return t;
}

template <class G>
__device__ __forceinline__ uint32_t next_edge_stage(const Task& t, uint32_t from) {
    return next_edge_stage_l<G::kLsb>(t, from);
}

// ABL (diagnostics only): 0 = real, 1 = no table lookups, 2 = no packet DMA.
template <int MODE, class G, int ABL = 0>
__global__ void __launch_bounds__(G::kThreads) crc32_stream_kernel(PacketArgs pa, KernelTables tb) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t lg = pa.lg, P = 1u << lg;
    const uint32_t gsh = 6u - lg;                                       // log2(packets per group)
    constexpr uint32_t F = MODE ? 5u : 3u;
    const uint32_t nmeta = (F << gsh) > 64u ? 2u : 1u;                  // F * 64/P <= 80 dwords
    const uint64_t ngroups = (pa.n + (1u << gsh) - 1u) >> gsh;
    const uint64_t wv = static_cast<uint64_t>(blockIdx.x) * G::kWaves + wave;
    const uint64_t wt = static_cast<uint64_t>(gridDim.x) * G::kWaves;
    const uint32_t J = wv < ngroups ? static_cast<uint32_t>((ngroups - 1u - wv) / wt) + 1u : 0u;
    const uint32_t ring = kLdsTableBytes + wave * G::kWaveLds;
    const uint32_t meta = ring + G::kNB * G::kStage;
    const uint64_t zero = reinterpret_cast<uint64_t>(tb.zero);
    const uint64_t stepB = 32ull * P * G::kSB;                          // bytes per stage per piece
    auto group_pk0 = [&](uint32_t j) __attribute__((always_inline)) -> uint64_t { return (wv + static_cast<uint64_t>(j) * wt) << gsh; };
    auto meta_slot = [&](uint32_t j) __attribute__((always_inline)) -> uint32_t { return meta + (j % G::kMetaSlots) * G::kMetaSlot; };

    uint32_t ops = 0;                    // counted VMEM operations issued by this wave
    // 1. metadata of the first group, then this wave's share of the table image
    if (J) {
        issue_meta<MODE>(pa, group_pk0(0), lg, nmeta, meta_slot(0), lane);
        ops += nmeta;
    }
    const uint32_t m_first = ops;
    {
        const uint32_t img = lg == 2 ? 1u : lg == 3 ? 2u : 3u;
        const uint32_t* src = tb.image + static_cast<size_t>(img) * kImageDwords;
#pragma unroll
        for (int r = 0; r < G::kTableRounds; ++r) {
            const uint32_t piece0 = min((static_cast<uint32_t>(r) * G::kWaves + wave) * 64u,
                                        static_cast<uint32_t>(kImageDwords / 4 - 64));
            dma16(src + 4u * (piece0 + lane), 16u * piece0);
        }
        ops += G::kTableRounds;
    }
    const uint32_t m_table = ops;

    // producer state
    Producer<G> pr;
    uint32_t pj = 0, pst = 0;
    bool pdone = J == 0;
    // metadata marks of the groups after pj (ops count mod 2^16 after each issue)
    uint64_t mmarks = 0;
    uint32_t nmm = 0;
    auto fetch_meta = [&](uint32_t j) __attribute__((always_inline)) {
        if (j < J) {
            issue_meta<MODE>(pa, group_pk0(j), lg, nmeta, meta_slot(j), lane);
            ops += nmeta;
        }
        mmarks |= static_cast<uint64_t>(ops & 0xFFFFu) << (16u * nmm);
        ++nmm;
    };
    // marks: ops count (mod 2^16) right after each in-flight stage, oldest in the
    // low 16 bits -- one scalar, no indexed array
    uint64_t marks = 0;
    uint32_t nfl = 0;

    auto produce = [&](uint32_t slotc) __attribute__((always_inline)) {
        const uint32_t buf = ring + slotc * G::kStage;
        const uint32_t skip = pst == 0 ? pr.head : 0u;                   // wave-uniform
        static_for<0, G::kDma>([&](auto ic) __attribute__((always_inline)) {
            constexpr int i = decltype(ic)::value;
            const bool in = pst < pr.nval[i] && !((skip >> i) & 1u);
            const uint64_t g = in ? pr.cur[i] : zero;
            if (ABL != 2) dma16(reinterpret_cast<const void*>(g), buf + 1024u * i);
            pr.cur[i] += stepB;
        });
        if (ABL != 2) ops += G::kDma;
        marks |= static_cast<uint64_t>(ops & 0xFFFFu) << (16u * nfl);
        ++nfl;
        if (++pst == pr.stages) {
            pst = 0;
            if (++pj < J) {
                wait_vm((ops - static_cast<uint32_t>(mmarks)) & 0xFFFFu);   // metadata of group pj
                mmarks >>= 16;
                --nmm;
                producer_setup<G>(pr, pa, meta_slot(pj), lg, group_pk0(pj), lane);
                fetch_meta(pj + G::kMetaAhead);
            } else {
                pdone = true;
            }
        }
    };

    if (J) {
        wait_vm(ops - m_first);
        producer_setup<G>(pr, pa, meta_slot(0), lg, group_pk0(0), lane);
#pragma unroll
        for (uint32_t d = 1; d <= G::kMetaAhead; ++d) fetch_meta(d);
        unroll_slots<G::kNB - 1>([&](auto sc) __attribute__((always_inline)) {
            if (!pdone) produce(decltype(sc)::value);
        });
    }
    // 2. the table must be complete (all waves' shares) before any lookup
    wait_vm(ops - m_table);
    __builtin_amdgcn_s_barrier();
    if (!J) return;

    const LaneSched s = make_sched(lane);
    const uint32_t swz = run_swz<G>(lane);
    const uint32_t hsb = s.hs & 1u;
    // LDS address of this lane's half-blocks in ring slot 0 (others: + slot*kStage)
    uint32_t offA[G::kSB], offB[G::kSB];
#pragma unroll
    for (int b = 0; b < G::kSB; ++b) {
        offA[b] = ring + G::kRun * lane + 16u * ((2u * b + hsb) ^ swz);
        offB[b] = ring + G::kRun * lane + 16u * ((2u * b + (hsb ^ 1u)) ^ swz);
    }

    uint32_t cj = 0, cst = 0;
    Task t = consumer_setup<MODE>(pa, meta_slot(0), lg, group_pk0(0), lane);
    uint32_t cstages = max(1u, wave_max_u((t.cnt + G::kSB - 1u) >> G::kLsb));   // (as pr.stages)
    uint32_t nedge = next_edge_stage<G>(t, 0);
    uint32_t reg = t.reg, desired = 0;
    bool done = false;

    auto stage = [&](auto sc) __attribute__((always_inline)) {
        constexpr uint32_t S = decltype(sc)::value;
        if (done) return;
        if (!pdone) {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");          // WAR on the buffer being refilled
            produce((S + G::kNB - 1) % G::kNB);
        }
        wait_vm((ops - static_cast<uint32_t>(marks)) & 0xFFFFu);        // this stage has landed
        const bool edges = cst == nedge;
#pragma unroll
        for (int b = 0; b < G::kSB; ++b) {
            const uint32_t jb = G::kSB * cst + b;                       // this lane's block ordinal
            u32x4 A = lds_load16(offA[b] + S * G::kStage);
            u32x4 B = lds_load16(offB[b] + S * G::kStage);
            const bool valid = jb < t.cnt;
            if (edges) {
                const bool fix = valid && (jb == t.e0 || jb == t.e1 || (MODE && (jb == t.e2 || jb == t.e3)));
                if (fix) edge_fix<MODE>(A, B, s.hs, t, t.w0 + P * jb, desired);
            }
            const uint32_t nr = ABL == 1 ? xor3(reg ^ A.x ^ A.y, A.z ^ A.w ^ B.x, B.y ^ B.z ^ B.w)
                                         : fold_block_lane(reg, A, B, s);
            reg = valid ? nr : reg;
        }
        if (edges) nedge = next_edge_stage<G>(t, cst + 1);
        marks >>= 16;
        --nfl;
        if (++cst == cstages) {
            reg = finish_packet(lg, t.k, t.tz, lane, reg);
            if (MODE) desired = xor_lanes<0>(lg, desired);
            if (t.active && t.k == 0) {
                if (MODE == 0) {
                    pa.out[t.pk] = finalize(reg);                        // packet.cs:159
                } else {
                    const uint32_t comp = t.slot_ok ? finalize(reg) : 0u;
                    pa.ok[t.pk] = (t.slot_ok && comp == desired) ? 1 : 0;
                    if (pa.out) pa.out[t.pk] = comp;
                }
            }
            if (++cj == J) {
                done = true;
                return;
            }
            t = consumer_setup<MODE>(pa, meta_slot(cj), lg, group_pk0(cj), lane);
            cstages = max(1u, wave_max_u((t.cnt + G::kSB - 1u) >> G::kLsb));
            nedge = next_edge_stage<G>(t, 0);
            reg = t.reg;
            desired = 0;
            cst = 0;
        }
    };
    while (!done) unroll_slots<G::kNB>(stage);
}

#endif  // ENET_HIP_DIAG

#ifdef ENET_HIP_DIAG
// ============================================================ register-stream kernel
// (diagnostics library only: a comparison point kept for the sweeps)
//
// Same per-packet arithmetic as crc32_stream_kernel (strided lanes, advancing
// tables, rotation, table-driven finish), but each lane loads its own blocks
// straight into a ring of R VGPR block slots with plain 16-byte loads: the P
// lanes of a packet read one contiguous P*32-byte chunk per step, every lane
// keeps R blocks in flight (16 waves x R x 2 KiB per CU) and the compiler's own
// counted vmcnt waits order the loads.  A LOAD cursor runs R steps ahead of the
// FOLD cursor across group boundaries.  Packet metadata never uses VGPR loads
// inside the loop (their waits would drain the ring): each wave stages the
// metadata of a window of 2H groups in LDS and refills one half at a time.  A
// piece wholly in front of a packet is read from the zero buffer; lanes past
// their last block read zeros, so every load is unconditional and the ring stays
// regular; a step whose load side had nothing to issue is a bubble.
template <int W, int R, int H>
struct VGeom {
    static constexpr int kWaves = W, kR = R;
    static constexpr int kThreads = 64 * W;
    // metadata window half (groups): H for send; verify stages 5 fields per lane,
    // so its half shrinks to what the LDS holds
    static constexpr int kHalf(int mode) {
        return mode ? ((160 * 1024 - kLdsTableBytes) / (W * 2 * 1280) < H ? (160 * 1024 - kLdsTableBytes) / (W * 2 * 1280) : H)
                    : H;
    }
    static constexpr uint32_t kSlot(int mode) { return (mode ? 5u : 3u) * 256u; }   // metadata per group
    static constexpr int kLds(int mode) { return kLdsTableBytes + W * 2 * kHalf(mode) * static_cast<int>(kSlot(mode)); }
    static_assert(kLdsTableBytes + W * 2 * H * 3 * 256 <= 160 * 1024 && kHalf(1) >= 1, "LDS budget");
};

struct Meta {
    uint32_t len, lo, hi, so, cid;
};

__device__ __forceinline__ Window window_of(const PacketArgs& pa, const Meta& m, bool active, uint32_t lg) {
    Window w;
    w.active = active;
    w.L = active ? m.len : 0u;
    const uint64_t off = static_cast<uint64_t>(m.lo) | (static_cast<uint64_t>(m.hi) << 32);
    const uint64_t a = reinterpret_cast<uint64_t>(pa.bytes) + off, e = a + w.L;
    w.tz = w.L ? static_cast<uint32_t>((0u - e) & 15u) : 0u;
    w.nb = w.L ? (w.L + w.tz + 31u) >> 5 : 0u;
    w.lz = 32u * w.nb - w.tz - w.L;
    w.ws = e + w.tz - 32ull * w.nb;
    w.r = (0u - w.nb) & ((1u << lg) - 1u);
    return w;
}

// Load side of this lane for one group: cursors of its next block's two halves
// in LANE order (first = original bytes 0-15 unless the lane swaps halves).
struct LSide {
    uint64_t cur0, cur1;
    uint32_t cnt;
    uint32_t hz;        // first block's original bytes 0-15 wholly in front of the packet
};

__device__ __forceinline__ LSide lside_of(const Window& w, uint32_t k, uint32_t lg, uint32_t hsb) {
    LSide l;
    const uint32_t P = 1u << lg;
    const uint32_t w0 = (k - w.r) & (P - 1u);
    l.cnt = w0 < w.nb ? ((w.nb - 1u - w0) >> lg) + 1u : 0u;
    const uint64_t base = w.ws + 32ull * w0;
    l.cur0 = base + 16u * hsb;
    l.cur1 = base + 16u * (hsb ^ 1u);
    l.hz = (w0 == 0 && w.nb && w.lz >= 16u) ? 1u : 0u;
    return l;
}

template <int MODE>
__device__ __forceinline__ Task task_of(const Window& w, const Meta& m, uint64_t pk, uint32_t k, uint32_t lg,
                                        uint32_t init_reg_lane) {
    const uint32_t P = 1u << lg;
    Task t;
    t.pk = pk;
    t.active = w.active;
    t.k = k;
    t.w0 = (k - w.r) & (P - 1u);
    t.nb = w.nb;
    t.lz = w.lz;
    t.tz = w.tz;
    t.cnt = t.w0 < w.nb ? ((w.nb - 1u - t.w0) >> lg) + 1u : 0u;
    t.reg = init_reg_lane;
    t.e0 = ((w.lz & 15u) && t.w0 == 0 && w.nb) ? 0u : ~0u;
    t.e1 = (w.tz && t.cnt && t.w0 + P * (t.cnt - 1u) == w.nb - 1u) ? t.cnt - 1u : ~0u;
    t.e2 = t.e3 = ~0u;
    t.ps = -4096;
    t.connect = 0;
    t.slot_ok = false;
    if (MODE) {
        t.connect = m.cid;
        t.slot_ok = w.L >= 4u && m.so <= w.L - 4u;
        if (t.slot_ok) {
            t.ps = static_cast<int32_t>(w.lz + m.so);
            const uint32_t ws_ = static_cast<uint32_t>(t.ps) >> 5, we_ = static_cast<uint32_t>(t.ps + 3) >> 5;
            if (((ws_ + w.r) & (P - 1u)) == k) t.e2 = ws_ >> lg;
            if (we_ != ws_ && ((we_ + w.r) & (P - 1u)) == k) t.e3 = we_ >> lg;
        }
    }
    return t;
}

template <int MODE, class G, int ABL = 0>
__global__ void __launch_bounds__(G::kThreads) crc32_vstream_kernel(PacketArgs pa, KernelTables tb) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    constexpr uint32_t F = MODE ? 5u : 3u;
    constexpr uint32_t kSlot = F * 256u;
    constexpr int kH = G::kHalf(MODE);
    constexpr uint32_t kWin = 2u * kH;                     // groups staged per wave
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t lg = pa.lg, P = 1u << lg;
    const uint32_t gsh = 6u - lg;
    const uint64_t ngroups = (pa.n + (1u << gsh) - 1u) >> gsh;
    const uint64_t wv = static_cast<uint64_t>(blockIdx.x) * G::kWaves + wave;
    const uint64_t wt = static_cast<uint64_t>(gridDim.x) * G::kWaves;
    const uint32_t J = wv < ngroups ? static_cast<uint32_t>((ngroups - 1u - wv) / wt) + 1u : 0u;
    const uint64_t zero = reinterpret_cast<uint64_t>(tb.zero);
    const uint64_t step = 32ull * P;
    const uint32_t k = lane & (P - 1u);
    const uint32_t hsb = (lane >> 4) & 1u;                 // the lane's half swap (LaneSched::hs)
    const uint32_t mbase = kLdsTableBytes + wave * kWin * kSlot;
    auto pk_of = [&](uint32_t j) __attribute__((always_inline)) -> uint64_t {
        return ((wv + static_cast<uint64_t>(j) * wt) << gsh) + (lane >> lg);
    };
    // metadata staging: group j -> LDS slot j % 2H, field f of lane l at +256f + 4l
    auto stage_meta = [&](uint32_t j0, uint32_t cnt) __attribute__((always_inline)) {
        uint32_t v[kH][F];
#pragma unroll
        for (int q = 0; q < kH; ++q) {
            if (static_cast<uint32_t>(q) < cnt) {
                const uint64_t pk = min(pk_of(j0 + q), pa.n - 1);
                v[q][0] = pa.len[pk];
                const uint32_t* o = reinterpret_cast<const uint32_t*>(pa.off) + 2 * pk;
                v[q][1] = o[0];
                v[q][2] = o[1];
                if (MODE) {
                    v[q][3] = pa.slot_off[pk];
                    v[q][4] = pa.connect[pk];
                }
            }
        }
#pragma unroll
        for (int q = 0; q < kH; ++q) {
            if (static_cast<uint32_t>(q) < cnt) {
                const uint32_t slot = mbase + ((j0 + q) % kWin) * kSlot + 4u * lane;
#pragma unroll
                for (uint32_t f = 0; f < F; ++f)
                    *reinterpret_cast<__attribute__((address_space(3))) uint32_t*>(
                        static_cast<uintptr_t>(slot + 256u * f)) = v[q][f];
            }
        }
    };
    auto read_meta = [&](uint32_t j) __attribute__((always_inline)) -> Meta {
        const uint32_t slot = mbase + (j % kWin) * kSlot + 4u * lane;
        Meta m;
        m.len = lds_load(slot);
        m.lo = lds_load(slot + 256u);
        m.hi = lds_load(slot + 512u);
        m.so = MODE ? lds_load(slot + 768u) : 0u;
        m.cid = MODE ? lds_load(slot + 1024u) : 0u;
        return m;
    };

    // prologue: table image and the first window of metadata (one drain, here only)
    const uint32_t img = lg == 2 ? 1u : lg == 3 ? 2u : 3u;
    fill_table<G::kThreads>(lds, tb.image + static_cast<size_t>(img) * kImageDwords);
    uint32_t staged = min(J, kWin);                          // groups [0, staged) are in LDS
    stage_meta(0, min(staged, static_cast<uint32_t>(kH)));
    if (staged > static_cast<uint32_t>(kH)) stage_meta(kH, staged - kH);
    __syncthreads();
    if (!J) return;

    // load side
    u32x4 ra[G::kR], rb[G::kR];
    uint32_t jl = 0, bl = 0, sl = 0, cminl = 0;
    bool ldone = false;
    LSide ls = lside_of(window_of(pa, read_meta(0), pk_of(0) < pa.n, lg), k, lg, hsb);
    sl = wave_max_u(ls.cnt);
    cminl = wave_min_u(ls.cnt);
    uint32_t bubbles = 0;                                     // bit i: ring slot i holds no block
    auto issue = [&](u32x4& x0, u32x4& x1, uint32_t slotbit) __attribute__((always_inline)) {
        while (!ldone && bl == sl) {                          // next group of the load side
            if (jl + 1 == J) {
                ldone = true;
                break;
            }
            if (jl + 1 >= staged) break;                      // metadata not staged yet: bubble
            ++jl;
            ls = lside_of(window_of(pa, read_meta(jl), pk_of(jl) < pa.n, lg), k, lg, hsb);
            sl = wave_max_u(ls.cnt);
            cminl = wave_min_u(ls.cnt);
            bl = 0;
        }
        uint64_t a0 = zero, a1 = zero;
        const bool live = !ldone && bl < sl;
        if (live) {
            if (bl < cminl) {
                a0 = ls.cur0;
                a1 = ls.cur1;
            } else {
                const bool v = bl < ls.cnt;
                a0 = v ? ls.cur0 : a0;
                a1 = v ? ls.cur1 : a1;
            }
            if (bl == 0 && ls.hz) {                           // head piece wholly in front
                if (hsb) a1 = zero;
                else a0 = zero;
            }
            ls.cur0 += step;
            ls.cur1 += step;
            ++bl;
            bubbles &= ~slotbit;
        } else {
            bubbles |= slotbit;
        }
        if (ABL == 2) {
            a0 = zero;
            a1 = zero;
        }
        x0 = ldg16_addr(a0);
        x1 = ldg16_addr(a1);
    };
    static_for<0, G::kR>([&](auto ic) __attribute__((always_inline)) {
        constexpr int i = decltype(ic)::value;
        issue(ra[i], rb[i], 1u << i);
        __builtin_amdgcn_sched_barrier(0);                    // keep slot order = issue order
    });

    const LaneSched s = make_sched(lane);
    // fold side
    uint32_t jf = 0, bf = 0;
    Task t{};
    uint32_t sf = 0, cminf = 0, nedge = ~0u, reg = 0, desired = 0;
    bool done = false;
    auto begin_group = [&]() __attribute__((always_inline)) {
        const Meta m = read_meta(jf);
        const Window w = window_of(pa, m, pk_of(jf) < pa.n, lg);
        const uint32_t init = lds_load(init_addr(w.lz));
        t = task_of<MODE>(w, m, pk_of(jf), k, lg, k == w.r ? init : 0u);
        sf = wave_max_u(t.cnt);
        cminf = wave_min_u(t.cnt);
        nedge = next_edge_stage_l<0>(t, 0);
        reg = t.reg;
        desired = 0;
        bf = 0;
    };
    // finish the current fold group, then set up the next one with blocks (groups
    // whose packets are all empty finish at once, as the load side skips them);
    // refill a half of the metadata window when the fold side has left it
    auto end_group = [&]() __attribute__((always_inline)) {
        for (;;) {
            reg = finish_packet(lg, t.k, t.tz, lane, reg);
            if (MODE) desired = xor_lanes<0>(lg, desired);
            if (t.active && t.k == 0) {
                if (MODE == 0) {
                    pa.out[t.pk] = finalize(reg);                // packet.cs:159
                } else {
                    const uint32_t comp = t.slot_ok ? finalize(reg) : 0u;
                    pa.ok[t.pk] = (t.slot_ok && comp == desired) ? 1 : 0;
                    if (pa.out) pa.out[t.pk] = comp;
                }
            }
            if (++jf == J) {
                done = true;
                return;
            }
            if (jf % kH == 0 && staged < J && jf >= static_cast<uint32_t>(kH)) {   // the fold left a half
                const uint32_t c = min(J - staged, static_cast<uint32_t>(kH));
                stage_meta(staged, c);
                staged += c;
            }
            begin_group();
            if (sf) return;
        }
    };
    begin_group();
    if (!sf) end_group();

    // A step folds its ring slot (if work remains and it holds a block) and ALWAYS
    // refills it, so every path back to the loop header has issued the R slots in
    // order and the compiler's counted vmcnt waits stay at 2R-2 instead of draining.
    auto step_fn = [&](auto ic) __attribute__((always_inline)) {
        constexpr int i = decltype(ic)::value;
        if (!done && !((bubbles >> i) & 1u)) {
            u32x4 A = ra[i], B = rb[i];
            if (bf == nedge) {
                const bool valid = bf < t.cnt;
                const bool fix = valid && (bf == t.e0 || bf == t.e1 || (MODE && (bf == t.e2 || bf == t.e3)));
                if (fix) edge_fix<MODE>(A, B, s.hs, t, t.w0 + P * bf, desired);
                nedge = next_edge_stage_l<0>(t, bf + 1);
            }
            const uint32_t nr = ABL == 1 ? xor3(reg ^ A.x ^ A.y, A.z ^ A.w ^ B.x, B.y ^ B.z ^ B.w)
                                         : fold_block_lane(reg, A, B, s);
            if (bf < cminf) reg = nr;
            else reg = bf < t.cnt ? nr : reg;
            if (++bf == sf) end_group();
        }
        issue(ra[i], rb[i], 1u << i);                         // refill this slot R steps ahead
        __builtin_amdgcn_sched_barrier(0);
    };
    if (!done) {
        for (;;) {
            static_for<0, G::kR>(step_fn);
            if (done) break;
        }
    }
}

#endif  // ENET_HIP_DIAG

#ifdef ENET_HIP_DIAG
// ============================================================ direct kernel
//
// General direct-load path (every block loaded straight into VGPRs, any P):
// packet split into P CONTIGUOUS segments cut at 128-byte-aligned absolute
// addresses, each an END-aligned window started at INIT[rp], joined by the
// carry-combine reg(A||B) = reg(A) x^(8|B|) ^ reg(B).  Runs for lanes-per-packet
// values the stream kernel does not take, and as the comparison point.
struct DTask {
    const uint8_t* a;   // packet start
    const uint8_t* sp;  // segment start
    uint64_t pk;
    uint32_t L, len, nb, rp, after, k;
    bool active;
};

__device__ __forceinline__ DTask make_dtask(const PacketArgs& pa, uint64_t t, uint64_t total) {
    DTask tk;
    const uint32_t P = 1u << pa.lg;
    tk.active = t < total;
    tk.pk = t >> pa.lg;
    tk.k = static_cast<uint32_t>(t) & (P - 1u);
    tk.L = 0;
    tk.a = pa.bytes;
    if (tk.active) {
        tk.L = pa.len[tk.pk];
        tk.a = pa.bytes + pa.off[tk.pk];
    }
    const uint64_t A = reinterpret_cast<uint64_t>(tk.a), E = A + tk.L;
    auto cut = [&](uint32_t k) -> uint64_t {
        if (k == 0) return A;
        if (k >= P) return E;
        const uint64_t r = (A + ((static_cast<uint64_t>(tk.L) * k) >> pa.lg) + 64u) & ~static_cast<uint64_t>(127);
        return min(max(r, A), E);
    };
    const uint64_t s0 = cut(tk.k), s1 = cut(tk.k + 1);
    tk.sp = reinterpret_cast<const uint8_t*>(s0);
    tk.len = static_cast<uint32_t>(s1 - s0);
    tk.nb = (tk.len + 31u) >> 5;
    tk.rp = (tk.nb << 5) - tk.len;
    tk.after = static_cast<uint32_t>(E - s1);
    return tk;
}

template <int MODE>
__device__ __forceinline__ void finish_dtask(const PacketArgs& pa, const DTask& tk, uint32_t reg,
                                             const KernelTables& tb) {
    if (tk.after) reg = mulmod(reg, x8n_dev(tk.after, tb));    // reg(A||B) = reg(A) x^(8|B|) ^ reg(B)
    for (uint32_t m = 1; m < (1u << pa.lg); m <<= 1) reg ^= __shfl_xor(reg, static_cast<int>(m));
    if (!tk.active || tk.k != 0) return;
    if (MODE == 0) {
        pa.out[tk.pk] = finalize(reg);                            // packet.cs:159
    } else {
        // protocol.cs:1052-1068: desired = slot; slot := connectID; crc over the
        // DGRAM; keep iff equal.  By linearity the substitution adds
        // (slot ^ connectID) fed at byte offset so, followed by L-so zero bytes.
        const uint32_t so = pa.slot_off[tk.pk];
        uint32_t comp = 0;
        uint8_t okv = 0;
        if (so <= tk.L && tk.L - so >= 4u) {
            uint32_t desired;
            __builtin_memcpy(&desired, tk.a + so, 4);
            const uint32_t delta = desired ^ pa.connect[tk.pk];
            const uint32_t fixed = reg ^ mulmod(delta, x8n_dev(tk.L - so, tb));
            comp = finalize(fixed);
            okv = (comp == desired) ? 1 : 0;
        }
        pa.ok[tk.pk] = okv;
        if (pa.out) pa.out[tk.pk] = comp;
    }
}

template <int MODE>
__global__ void __launch_bounds__(kThreads) crc32_direct_kernel(PacketArgs pa, KernelTables tb) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    fill_table<kThreads>(lds, tb.image);
    const LaneSched s = make_sched(threadIdx.x & 63u);
    const uint64_t total = pa.n << pa.lg;
    const uint64_t stride = static_cast<uint64_t>(gridDim.x) * kThreads;
    const uint8_t* safe = reinterpret_cast<const uint8_t*>(tb.xn_lo);
    for (uint64_t base = static_cast<uint64_t>(blockIdx.x) * kThreads + (threadIdx.x & ~63u); base < total;
         base += stride) {
        const DTask tk = make_dtask(pa, base + (threadIdx.x & 63u), total);
        uint32_t reg = (tk.k == 0) ? tb.init[tk.rp] : 0u;
        reg = fold_window(reg, tk.sp, tk.len, s, safe);
        finish_dtask<MODE>(pa, tk, reg, tb);
    }
}
#endif  // ENET_HIP_DIAG

// One lane per DGRAM; segments folded in order and joined by the carry-combine.
__global__ void __launch_bounds__(kThreads) crc32_gather_kernel(GatherArgs ga, KernelTables tb) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    fill_table<kThreads>(lds, tb.image);
    const LaneSched s = make_sched(threadIdx.x & 63u);
    const uint64_t stride = static_cast<uint64_t>(gridDim.x) * kThreads;
    for (uint64_t d = static_cast<uint64_t>(blockIdx.x) * kThreads + threadIdx.x; d < ga.n; d += stride) {
        const uint32_t s0 = ga.seg_first[d], s1 = ga.seg_first[d + 1];
        uint32_t reg = 0xFFFFFFFFu;
        bool first = true;
        for (uint32_t q = s0; q < s1; ++q) {
            const uint32_t L = ga.seg_len[q];
            if (L == 0) continue;
            const uint8_t* a = ga.bytes + ga.seg_off[q];
            const uint32_t nb = (L + 31u) >> 5;
            const uint32_t rp = (nb << 5) - L;
            if (first) {
                reg = fold_window(tb.init[rp], a, L, s, reinterpret_cast<const uint8_t*>(tb.xn_lo));
                first = false;
            } else {
                const uint32_t part = fold_window(0u, a, L, s, reinterpret_cast<const uint8_t*>(tb.xn_lo));
                reg = mulmod(reg, x8n_dev(L, tb)) ^ part;
            }
        }
        ga.out[d] = finalize(reg);
    }
}

// The join of enet_hip_crc32_gather_binned_device: thread per DGRAM.  seg_crc[q] =
// finalize(reg(0xFFFFFFFF, segment q)) from the length-binned checksum pass over the
// segments.  reg(s, A||B) = adv_|B|(reg(s, A)) ^ reg(0, B) and reg(0, B) =
// reg(0xFFFFFFFF, B) ^ adv_|B|(0xFFFFFFFF), so one multiply per segment:
// reg' = (reg ^ 0xFFFFFFFF) x^(8|B|) ^ reg(0xFFFFFFFF, B), from reg = 0xFFFFFFFF
// (packet.cs:144-159 over the concatenated buffers, as enet_crc32 walks them).
// Segments of at most `small` (<= kGatherSmall) bytes -- an ENet DGRAM's protocol
// header and command headers: 4-8 and 4-48 B -- had no checksum pass: the thread
// folds them into reg itself (packet.cs:150-155).  Latency first: a thread takes its
// DGRAM's segments four at a time and issues every load of the four -- lengths and
// offsets, then the short segments' aligned dwords (never past the dword holding a
// segment's last byte), the long ones' CRCs and x^(8 len) -- before folding any.  A
// short segment's 4-byte steps are slicing-by-4 on the dword v_alignbyte cuts at its
// offset, its last L mod 4 bytes Sarwate steps (T_3 .. T_0 = columns 6, 4, 2, 0 of
// the P = 1 image, 4 KiB in LDS).  (fold_small, gather_join.hpp.)

// JV (diagnostics, wrong CRCs by design): bit 0 = no short-segment fold (its dwords
// XORed in), bit 1 = no multiply (XOR), bit 2 = no short-segment loads
template <int JV = 0>
__global__ void __launch_bounds__(kThreads) crc32_gather_join_kernel(GatherArgs ga, const uint32_t* seg_crc,
                                                                     KernelTables tb, uint32_t small) {
    constexpr int kQ = 4;                                    // segments in flight per thread
    __shared__ uint32_t t4[4][256];
    if (small) {
        for (uint32_t i = threadIdx.x; i < 1024u; i += kThreads) t4[i >> 8][i & 255u] = tb.image[64u * (i & 255u) + 2u * (i >> 8)];
        __syncthreads();
    }
    const uint64_t stride = static_cast<uint64_t>(gridDim.x) * kThreads;
    for (uint64_t d = static_cast<uint64_t>(blockIdx.x) * kThreads + threadIdx.x; d < ga.n; d += stride) {
        // segFirst lives in device memory, so the host cannot check segFirst[n] ==
        // segCount: clamp to the segments the binned pass filled (a short segCount
        // then gives wrong CRCs for the DGRAMs past it, never a read past seg_crc)
        const uint32_t s1 = static_cast<uint32_t>(umin64(ga.seg_first[d + 1], ga.segs));
        const uint32_t s0 = min(ga.seg_first[d], s1);
        uint32_t reg = 0xFFFFFFFFu;
        for (uint32_t q0 = s0; q0 < s1; q0 += kQ) {
            uint32_t L[kQ];
            const uint8_t* A[kQ];
#pragma unroll
            for (int i = 0; i < kQ; ++i) {
                const bool in = q0 + i < s1;
                L[i] = in ? ga.seg_len[q0 + i] : 0u;
                A[i] = ga.bytes + (in ? ga.seg_off[q0 + i] : 0u);
            }
            uint32_t D[kQ][kSmallDwords + 1], C[kQ], X[kQ];
#pragma unroll
            for (int i = 0; i < kQ; ++i) {
                const bool sm = L[i] != 0u && L[i] <= small && !(JV & 4);
                if (sm) load_small(A[i], L[i], D[i]);   // (global loads: see load_small)
                else
#pragma unroll
                    for (int k = 0; k <= kSmallDwords; ++k) D[i][k] = 0u;
                C[i] = L[i] > small ? seg_crc[q0 + i] : 0u;
                X[i] = L[i] > small ? tb.xn_lo[L[i] & 0xFFFFu] : 0u;
            }
#pragma unroll
            for (int i = 0; i < kQ; ++i) {
                if (L[i] == 0u) continue;
                if (L[i] <= small) {
                    if constexpr (JV & 1) {
#pragma unroll
                        for (int k = 0; k <= kSmallDwords; ++k) reg ^= D[i][k];
                    } else {
                        reg = fold_small(reg, static_cast<uint32_t>(reinterpret_cast<uintptr_t>(A[i])) & 3u, L[i], D[i], t4);
                    }
                } else if constexpr (JV & 2) {
                    reg ^= X[i] ^ ~bswap32(C[i]);
                } else {
                    const uint32_t x = (L[i] >> 16) ? mulmod(X[i], tb.xn_hi[L[i] >> 16]) : X[i];
                    reg = (reg == 0xFFFFFFFFu ? 0u : mulmod(reg ^ 0xFFFFFFFFu, x)) ^ ~bswap32(C[i]);
                }
            }
        }
        ga.out[d] = finalize(reg);
    }
}


#ifdef ENET_HIP_DIAG
// The post-join of the split join (gather_join.hpp): one thread per segment, after
// the records pass.  A long segment q of DGRAM d = info[q].x adds
// bswap(R_q x^(8 after_q)) to out[d] (R_q = ~bswap(seg_crc[q])), ~seg_crc[q] when
// nothing follows it.  Only segFirst[0] <= q < segFirst[n] (clamped to the binned
// segments) belong to a DGRAM; d < n bounds the atomic whatever the arrays hold.
__global__ void __launch_bounds__(256) crc32_gather_post_kernel(const uint32_t* seg_len, const uint32_t* seg_crc,
                                                                const uint2* info, const uint32_t* seg_first,
                                                                uint64_t n, uint64_t segs, uint32_t small,
                                                                uint32_t* out) {
    constexpr uint32_t kPer = 2;                             // segments per thread, loads issued together
    const uint64_t hi = umin64(seg_first[n], segs), lo = seg_first[0];
    const uint64_t stride = static_cast<uint64_t>(gridDim.x) * 256u * kPer;
    for (uint64_t c = lo + static_cast<uint64_t>(blockIdx.x) * 256u * kPer + threadIdx.x; c < hi; c += stride) {
        uint32_t L[kPer], C[kPer];
        uint2 in[kPer];
#pragma unroll
        for (uint32_t i = 0; i < kPer; ++i) {
            const uint64_t q = c + 256u * i;
            const bool h = q < hi;
            L[i] = h ? seg_len[q] : 0u;
            in[i] = h ? info[q] : make_uint2(~0u, 0u);
            C[i] = h ? seg_crc[q] : 0u;
        }
#pragma unroll
        for (uint32_t i = 0; i < kPer; ++i) {
            if (L[i] <= small || in[i].x >= n) continue;
            const uint32_t add = in[i].y == kOneReflected ? ~C[i] : bswap32(mulmod(~bswap32(C[i]), in[i].y));
            atomicXor(out + in[i].x, add);
        }
    }
}
#endif  // ENET_HIP_DIAG

// Read-roofline probe: every byte loaded once by 16-byte coalesced loads,
// 4 loads in flight per lane, XOR-folded so nothing is dead code.
__global__ void __launch_bounds__(kThreads) read_probe_kernel(const uint8_t* bytes, uint64_t nvec, uint32_t* sink) {
    const u32x4* p = reinterpret_cast<const u32x4*>(bytes);
    u32x4 acc = {0u, 0u, 0u, 0u};
    const uint64_t stride = static_cast<uint64_t>(gridDim.x) * kThreads;
    uint64_t i = static_cast<uint64_t>(blockIdx.x) * kThreads + threadIdx.x;
    for (; i + 3 * stride < nvec; i += 4 * stride) {
        const u32x4 a = p[i], b = p[i + stride], c = p[i + 2 * stride], d = p[i + 3 * stride];
        acc ^= a ^ b ^ c ^ d;
    }
    for (; i < nvec; i += stride) acc ^= p[i];
    const uint32_t x = acc.x ^ acc.y ^ acc.z ^ acc.w;
    if (x == 0x9E3779B9u) sink[0] = x;  // practically never taken; keeps the loads live
}

}  // namespace enethip

// =================================================================== host side

using namespace enethip;

namespace {

// x^-1 mod p = (p(x) + 1) / x in the reflected representation (bit 31-i <-> x^i).
constexpr uint32_t x_inverse() {
    uint32_t v = 1u;                                   // x^32 / x = x^31
    for (int i = 1; i < 32; ++i)
        if ((kPoly >> (31 - i)) & 1u) v |= 1u << (31 - (i - 1));
    return v;
}
static_assert(gf2_mulmod(x_inverse(), kOneReflected >> 1) == kOneReflected, "x * x^-1 = 1");

constexpr int kImages = 4;                             // P = 1, 4, 8, 16
constexpr int kImageP[kImages] = {1, 4, 8, 16};

struct HostTables {
    std::vector<uint32_t> image, xn, init, basis, basis2, tz;
    bool basis_ok = true;   // the bases rebuild every image dword the lean / vring kernels read
    HostTables()
        : image(static_cast<size_t>(kImages) * kImageDwords), xn(2 * kXnEntries), init(64),
          basis(static_cast<size_t>(kImages) * kBasisDwords), basis2(static_cast<size_t>(kImages) * kVrBasisDwords),
          tz(kTzTableDwords + kTzSmallDwords) {
        init[0] = 0xFFFFFFFFu;
        for (int r = 1; r < 64; ++r) init[r] = unstep_zero(init[r - 1]);
        std::vector<uint32_t> cinv(kCinvEntries);
        uint32_t xinv8 = kOneReflected;
        for (int i = 0; i < 8; ++i) xinv8 = gf2_mulmod(xinv8, x_inverse());
        cinv[0] = kOneReflected;
        for (int i = 1; i < kCinvEntries; ++i) cinv[i] = gf2_mulmod(cinv[i - 1], xinv8);
        for (uint32_t k = 0; k < static_cast<uint32_t>(kTzTables); ++k)       // x^(-128), x^(-64) by byte
            for (uint32_t b = 0; b < 4; ++b)
                for (uint32_t v = 0; v < 256; ++v)
                    tz[tz_addr(k, b, v) / 4] = gf2_mulmod(v << (8 * b), cinv[k ? 8 : 16]);
        for (uint32_t c = 1; c <= static_cast<uint32_t>(kTzSmallTables); ++c)     // x^(-8 c), c < 8
            for (uint32_t b = 0; b < 4; ++b)
                for (uint32_t v = 0; v < 256; ++v)
                    tz[kTzTableDwords + tz_small_addr(c, b, v) / 4] = gf2_mulmod(v << (8 * b), cinv[c]);
        // image of P: dword 64j + 2t + (t>>4) = T_{t+32(P-1)}[j] (byte j followed by
        // t + 32(P-1) zero bytes); the free dwords hold INIT[] and CINV[]
        for (int im = 0; im < kImages; ++im) {
            uint32_t* img = image.data() + static_cast<size_t>(im) * kImageDwords;
            std::vector<uint32_t> row(256);
            for (uint32_t j = 0; j < 256; ++j) {
                uint32_t r = crc_table_entry(j);
                for (int z = 0; z < 32 * (kImageP[im] - 1); ++z) r = sarwate_step(r, 0);
                row[j] = r;
            }
            for (uint32_t t = 0; t < 32; ++t) {
                for (uint32_t j = 0; j < 256; ++j) img[(j * 256 + col_byte(t)) / 4] = row[j];
                for (uint32_t j = 0; j < 256; ++j) row[j] = sarwate_step(row[j], 0);
            }
            for (uint32_t k = 1; k < std::min<uint32_t>(kImageP[im], kCorrLanes); ++k)
                for (uint32_t b = 0; b < 4; ++b)
                    for (uint32_t v = 0; v < 256; ++v)
                        img[(256u * v + corr_col(k, b)) / 4] = gf2_mulmod(v << (8 * b), cinv[32 * k]);
            for (uint32_t b = 0; b < 256; ++b) {                // U: reg x^(-8) = (reg << 8) ^ U[reg >> 24]
                const uint32_t t = crc_table_entry(b);
                img[unstep_addr(t >> 24) / 4] = (t << 8) | b;
            }
            for (uint32_t r = 0; r < 64; ++r) img[init_addr(r) / 4] = init[r];
            for (uint32_t i = 0; i < static_cast<uint32_t>(kCinvEntries); ++i) img[cinv_addr(i) / 4] = cinv[i];
            // lean-kernel basis: image rows 2^b of the linear columns, then INIT | CINV
            uint32_t* bs = basis.data() + static_cast<size_t>(im) * kBasisDwords;
            auto nonlinear = [](uint32_t d) { return d == kInitDword || d == kCinvDword || d == kCinvDword + 2u; };
            for (uint32_t b = 0; b < 8; ++b)
                for (uint32_t d = 0; d < 64; ++d) bs[64 * b + d] = nonlinear(d) ? 0u : img[64u * (1u << b) + d];
            for (uint32_t r = 0; r < 32; ++r) {
                bs[512 + r] = init[r];
                bs[544 + r] = cinv[r];
            }
            // vring-kernel basis: the same linear rows, then INIT[0..63], CINV[0..63]
            uint32_t* b2 = basis2.data() + static_cast<size_t>(im) * kVrBasisDwords;
            for (uint32_t d = 0; d < 512; ++d) b2[d] = bs[d];
            for (uint32_t r = 0; r < 64; ++r) {
                b2[512 + r] = init[r];
                b2[576 + r] = cinv[r];
            }
            // what crc32_lean.hip rebuilds must equal the image wherever that kernel
            // looks (INIT rows < 32, CINV rows < 16; CINV n >= 256 never); the same
            // for crc32_vring.hip with INIT / CINV rows < 64
            for (uint32_t j = 0; j < 256; ++j)
                for (uint32_t d = 0; d < 64; ++d) {
                    if (d == kCinvDword + 2u || ((d == kInitDword || d == kCinvDword) && j >= 32)) continue;
                    uint32_t v = 0;
                    for (uint32_t b = 0; b < 8; ++b)
                        if ((j >> b) & 1u) v ^= bs[64 * b + d];
                    if (d == kInitDword) v = bs[512 + j];
                    if (d == kCinvDword) v = bs[544 + j];
                    if (v != img[64 * j + d]) basis_ok = false;
                }
            for (uint32_t j = 0; j < 256; ++j)
                for (uint32_t d = 0; d < 64; ++d) {
                    if (d == kCinvDword + 2u || ((d == kInitDword || d == kCinvDword) && j >= 64)) continue;
                    uint32_t v = 0;
                    for (uint32_t b = 0; b < 8; ++b)
                        if ((j >> b) & 1u) v ^= b2[64 * b + d];
                    if (d == kInitDword) v = b2[512 + j];
                    if (d == kCinvDword) v = b2[576 + j];
                    if (v != img[64 * j + d]) basis_ok = false;
                }
        }
        // x^(8n) for n < 65536: one zero-byte step per n
        xn[0] = kOneReflected;
        for (int n = 1; n < kXnEntries; ++n) xn[n] = sarwate_step(xn[n - 1], 0);
        const uint32_t x64k = sarwate_step(xn[kXnEntries - 1], 0);  // x^(8*65536)
        xn[kXnEntries] = kOneReflected;
        for (int q = 1; q < kXnEntries; ++q) xn[kXnEntries + q] = gf2_mulmod(xn[kXnEntries + q - 1], x64k);
    }
};

const HostTables& host_tables() {
    static const HostTables t;
    return t;
}

// Default lanes per packet: 8 for checksum batches and for receive verify.  The
// vring kernel with its lane constants kept live runs cfg2 at 5.26-5.34 TB/s in the
// serial 5-batch region at 8 lanes against 5.14-5.26 at 4, with the same bench value
// (three interleaved repeats on one box, profiles/r02e_lanes_4_vs_8/); before that, 4
// lanes had led (profiles/r02_*).  The length-binned entries keep their own default (4).
int auto_lanes(const enet_hip_context* ctx, int mode = 0) {
    (void)mode;
    return ctx->lanes_per_packet > 0 ? ctx->lanes_per_packet : 8;
}

int log2i(int v) {
    int l = 0;
    while ((1 << l) < v) ++l;
    return l;
}

KernelTables tables_of(const enet_hip_context* ctx) {
    return KernelTables{ctx->d_image, ctx->d_xn, ctx->d_xn + kXnEntries, ctx->d_init, ctx->d_zero, ctx->d_basis,
                        ctx->d_tz};
}

unsigned grid_for(const enet_hip_context* ctx, uint64_t tasks) {
    const int per_cu = ctx->wgs_per_cu > 0 ? ctx->wgs_per_cu : 2;
    const uint64_t cap = static_cast<uint64_t>(ctx->num_cus) * per_cu;
    const uint64_t need = (tasks + kThreads - 1) / kThreads;
    return static_cast<unsigned>(std::max<uint64_t>(1, std::min(need, cap)));
}

#ifdef ENET_HIP_DIAG
// Stream geometries (waves per CU, blocks per stage, stage buffers).
// kStreamDefault is what path 0 runs; the others are reachable through
// enet_hip_set_kernel_path (2 + index) for tuning sweeps.
template <class G>
struct StreamVariant {
    static void launch(int mode, int abl, unsigned grid, hipStream_t st, const PacketArgs& pa,
                       const KernelTables& tb) {
        if (mode == 1)
            hipLaunchKernelGGL((crc32_stream_kernel<1, G>), dim3(grid), dim3(G::kThreads), G::kLds, st, pa, tb);
#ifdef ENET_HIP_DIAG
        else if (abl == 1)
            hipLaunchKernelGGL((crc32_stream_kernel<0, G, 1>), dim3(grid), dim3(G::kThreads), G::kLds, st, pa, tb);
        else if (abl == 2)
            hipLaunchKernelGGL((crc32_stream_kernel<0, G, 2>), dim3(grid), dim3(G::kThreads), G::kLds, st, pa, tb);
#endif
        else
            hipLaunchKernelGGL((crc32_stream_kernel<0, G, 0>), dim3(grid), dim3(G::kThreads), G::kLds, st, pa, tb);
        (void)abl;
    }
    static int setup() {
        const void* fns[] = {reinterpret_cast<const void*>(crc32_stream_kernel<0, G, 0>),
#ifdef ENET_HIP_DIAG
                             reinterpret_cast<const void*>(crc32_stream_kernel<0, G, 1>),
                             reinterpret_cast<const void*>(crc32_stream_kernel<0, G, 2>),
#endif
                             reinterpret_cast<const void*>(crc32_stream_kernel<1, G, 0>)};
        for (const void* f : fns) {
            const hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, G::kLds);
            if (e != hipSuccess) return herr(e);
        }
        return 0;
    }
};
#endif  // ENET_HIP_DIAG

// Kernel paths (enet_hip_set_kernel_path): 1 = direct, 2 + k = stream geometry k (k <
// 6), then 5 register-stream geometries, 4 lean geometries, the vring variants.  The
// product library builds the default (0), lean geometry 0 and the vring path; the rest,
// with the lane counts other than 4 and 8 they served, are sweep-only (ENET_HIP_DIAG,
// since round 5).
constexpr int kStreamPaths = 6, kVStreamPaths = 5;
#ifdef ENET_HIP_DIAG
using StreamGeoms = std::tuple<StreamGeom<16, 1, 2>, StreamGeom<11, 1, 3>, StreamGeom<8, 1, 4>,
                               StreamGeom<8, 2, 2>, StreamGeom<6, 2, 3>, StreamGeom<10, 1, 3>>;
#endif
constexpr int kNumStreamGeoms = kStreamPaths;
#ifdef ENET_HIP_DIAG
constexpr int kStreamDefault = 0;
#endif

#ifdef ENET_HIP_DIAG
template <class G>
struct VStreamVariant {
    static void launch(int mode, int abl, unsigned grid, hipStream_t st, const PacketArgs& pa,
                       const KernelTables& tb) {
        if (mode == 1)
            hipLaunchKernelGGL((crc32_vstream_kernel<1, G>), dim3(grid), dim3(G::kThreads), G::kLds(1), st, pa, tb);
        else if (abl == 1)
            hipLaunchKernelGGL((crc32_vstream_kernel<0, G, 1>), dim3(grid), dim3(G::kThreads), G::kLds(0), st, pa, tb);
        else if (abl == 2)
            hipLaunchKernelGGL((crc32_vstream_kernel<0, G, 2>), dim3(grid), dim3(G::kThreads), G::kLds(0), st, pa, tb);
        else
            hipLaunchKernelGGL((crc32_vstream_kernel<0, G, 0>), dim3(grid), dim3(G::kThreads), G::kLds(0), st, pa, tb);
    }
    static int setup() {
        const void* fns[] = {reinterpret_cast<const void*>(crc32_vstream_kernel<0, G, 0>),
                             reinterpret_cast<const void*>(crc32_vstream_kernel<0, G, 1>),
                             reinterpret_cast<const void*>(crc32_vstream_kernel<0, G, 2>),
                             reinterpret_cast<const void*>(crc32_vstream_kernel<1, G, 0>)};
        for (int i = 0; i < 4; ++i) {
            const hipError_t e = hipFuncSetAttribute(fns[i], hipFuncAttributeMaxDynamicSharedMemorySize,
                                                     G::kLds(i == 3 ? 1 : 0));
            if (e != hipSuccess) return herr(e);
        }
        return 0;
    }
};

// register-stream geometries: paths 2 + kNumStreamGeoms + index
using VStreamGeoms = std::tuple<VGeom<16, 3, 3>, VGeom<16, 2, 3>, VGeom<16, 4, 4>, VGeom<8, 4, 4>, VGeom<8, 6, 6>>;
static_assert(std::tuple_size<VStreamGeoms>::value == kVStreamPaths, "path numbering");
static_assert(std::tuple_size<StreamGeoms>::value == kStreamPaths, "path numbering");
#endif  // ENET_HIP_DIAG
constexpr int kNumVStreamGeoms = kVStreamPaths;
// lean kernel geometries (crc32_lean.hip): paths kLeanPath0 + geom; path 0 runs geom 0
constexpr int kLeanPath0 = 2 + kNumStreamGeoms + kNumVStreamGeoms;
constexpr int kVringPath = kLeanPath0 + kLeanGeoms;     // crc32_vring.hip (path 0 for checksum batches)
constexpr int kVringAltPath = kVringPath + 1;           // the same with nontemporal stage loads
constexpr int kVringWalkPath = kVringAltPath + 1;       // vring, workgroups walking contiguous group ranges
constexpr int kVringWalkAltPath = kVringWalkPath + 1;   // the same with nontemporal stage loads
constexpr int kVringTailFirstPath = kVringWalkAltPath + 1;   // vring, the tail-first stage order
// (paths 22 / 23, round 4's linear-stream kernel, were removed in round 6: closed by its
// gate)
#ifdef ENET_HIP_DIAG
constexpr int kMaxPath = kVringTailFirstPath;
#endif

// Paths this library builds: all in the diagnostics library; in the product one
// the default (0), lean geometry 0 and vring.
bool path_built(int path) {
#ifdef ENET_HIP_DIAG
    return path >= 0 && path <= kMaxPath;
#else
    return path == 0 || path == kLeanPath0 || path == kVringPath;
#endif
}
// the binned gather's short-segment bound (segments of at most this many bytes are
// folded by the join, not binned): kGatherSmall, or (diagnostics A/B) a smaller one
uint32_t gather_small(const enet_hip_context* ctx) {
    return ctx->gather_small >= 0 && static_cast<uint32_t>(ctx->gather_small) < kGatherSmall
               ? static_cast<uint32_t>(ctx->gather_small) : kGatherSmall;
}

#ifdef ENET_HIP_DIAG
template <size_t I = 0>
void launch_stream(int geom, int mode, int abl, int num_cus, uint64_t groups, hipStream_t st,
                   const PacketArgs& pa, const KernelTables& tb) {
    if constexpr (I < std::tuple_size<StreamGeoms>::value) {
        using G = std::tuple_element_t<I, StreamGeoms>;
        if (geom == static_cast<int>(I)) {
            const unsigned grid = static_cast<unsigned>(std::max<uint64_t>(
                1, std::min<uint64_t>((groups + G::kWaves - 1) / G::kWaves, static_cast<uint64_t>(num_cus))));
            StreamVariant<G>::launch(mode, abl, grid, st, pa, tb);
        } else {
            launch_stream<I + 1>(geom, mode, abl, num_cus, groups, st, pa, tb);
        }
    }
}

#endif  // ENET_HIP_DIAG
#ifdef ENET_HIP_DIAG
template <size_t I = 0>
void launch_vstream(int geom, int mode, int abl, int num_cus, uint64_t groups, hipStream_t st,
                    const PacketArgs& pa, const KernelTables& tb) {
    if constexpr (I < std::tuple_size<VStreamGeoms>::value) {
        using G = std::tuple_element_t<I, VStreamGeoms>;
        if (geom == static_cast<int>(I)) {
            const unsigned grid = static_cast<unsigned>(std::max<uint64_t>(
                1, std::min<uint64_t>((groups + G::kWaves - 1) / G::kWaves, static_cast<uint64_t>(num_cus))));
            VStreamVariant<G>::launch(mode, abl, grid, st, pa, tb);
        } else {
            launch_vstream<I + 1>(geom, mode, abl, num_cus, groups, st, pa, tb);
        }
    }
}

template <size_t I = 0>
int setup_vstream() {
    if constexpr (I < std::tuple_size<VStreamGeoms>::value) {
        const int rc = VStreamVariant<std::tuple_element_t<I, VStreamGeoms>>::setup();
        return rc ? rc : setup_vstream<I + 1>();
    }
    return 0;
}
#endif  // ENET_HIP_DIAG

#ifdef ENET_HIP_DIAG
template <size_t I = 0>
int setup_stream() {
    if constexpr (I < std::tuple_size<StreamGeoms>::value) {
        const int rc = StreamVariant<std::tuple_element_t<I, StreamGeoms>>::setup();
        return rc ? rc : setup_stream<I + 1>();
    }
    return 0;
}
#endif  // ENET_HIP_DIAG

// vring workgroups per CU of one launch (enet_hip_set_tuning's workgroups_per_cu,
// clamped to 2: the LDS and 64-VGPR budget of two 16-wave workgroups; values 3..8
// are for the direct and gather grids and mean 2 here, as they did before round 3).
// Default (0): two for a launch of several batches, one for a single batch.  Measured
// on one box (profiles/r03_wgs_ab/): 5-batch lists 5270-5360 GiB/s at two against
// 5153-5213 at one; single-batch launches 5183 at one against 4301-4918 at two.
int vring_wgs(const enet_hip_context* ctx, size_t batches) {
    if (ctx->wgs_per_cu >= 1) return std::min(ctx->wgs_per_cu, 2);
    return batches > 1 ? 2 : 1;
}
bool vring_path(const enet_hip_context* ctx) {
    return ctx->path == 0 || (ctx->path >= kVringPath && ctx->path <= kVringTailFirstPath);
}
// The claim line of the next vring launch (dynamic rounds) and its generation, or
// null (static deal).  Lines are handed out in turn: a line is reused kVrClaimLines
// launches later, when the launch that used it has ended (the context's launches run
// on at most a few streams at once), with a generation one larger, so the kernel
// needs no reset of it (crc32_vring.hip vr_claim_next).  After 2^32 - 2 uses of a
// line (2^40 launches) the context falls back to the static deal.
// Contract of the dynamic modes (diagnostics A/B only; the product never sets them):
// a launch must have ended before 255 later launches of the context have started
// (kVrClaimLines - 1; a launch held back behind an event while 256 others run would
// find its line at a newer generation and skip its dynamic chunks), and a launch
// being captured into a graph takes the static deal -- a replay would reuse the
// captured {line, generation} and find the word already counted up.
constexpr uint32_t kVrClaimLines = 256;
constexpr uint32_t kVrPairLines = 64;
VrVariant with_claim(enet_hip_context* ctx, VrVariant v, hipStream_t st) {
    if (ctx->vr_pair || ctx->vr_dynamic) {
        hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
        if (hipStreamIsCapturing(st, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) return v;
    }
    if (!v.walk && ctx->vr_pair && ctx->d_pairs) {           // pair rounds (diagnostics)
        const uint64_t seq = ctx->pairs_next.fetch_add(1u);
        const uint64_t gen = seq / kVrPairLines + 1u;
        if (gen >= 0xFFFFFFFFull) return v;
        v.claim = ctx->d_pairs + static_cast<size_t>(kVrPairWords) * (seq % kVrPairLines);
        v.claim_gen = static_cast<uint32_t>(gen);
        v.claim_mode = 2;
        return v;
    }
    if (v.walk || !ctx->vr_dynamic || !ctx->d_rounds) return v;
    const uint64_t seq = ctx->rounds_next.fetch_add(1u);
    const uint64_t gen = seq / kVrClaimLines + 1u;
    if (gen >= 0xFFFFFFFFull) return v;
    v.claim = reinterpret_cast<uint64_t*>(ctx->d_rounds + static_cast<size_t>(kVrClaimWords) * (seq % kVrClaimLines));
    v.claim_gen = static_cast<uint32_t>(gen);
    return v;
}
VrVariant vring_variant(const enet_hip_context* ctx, bool lists) {
    VrVariant v;
    v.nt = ctx->path == kVringAltPath || ctx->path == kVringWalkAltPath;
    v.walk = (ctx->path == kVringWalkPath || ctx->path == kVringWalkAltPath) && !ctx->trace;
    v.tail_first = ctx->path == kVringTailFirstPath;
    v.abl = (lists || ctx->vr_abl == 128) ? ctx->vr_abl : 0;   // (128: the end-record trace instance)
    return v;
}

// the records instance: plain, or (diagnostics) its no-lookup / skeleton ablations
VrVariant bin_variant(const enet_hip_context* ctx) {
    VrVariant v;
    const int a = ctx->vr_abl;
    v.abl = (a == 2 || a == 19 || a == 64 || a == 83) ? a : 0;
    v.compact = vring_wgs(ctx, 1) >= 2;                      // (two workgroups per CU: the compact instance)
    return v;
}

// Receive verify on the vring kernel (8 lanes per packet, VF instance): the default
// (path 0) and the vring paths 17 / 21; the lean kernel serves 4 lanes, the binned
// records and path 13.
bool verify_on_vring(const enet_hip_context* ctx, int lg) {
    return lg == 3 && ctx->ablation == 0 &&
           (ctx->path == 0 || ctx->path == kVringPath || ctx->path == kVringTailFirstPath);
}

int verify_vring_list(enet_hip_context* ctx, const ENetHipVerifyBatch* batches, size_t count, hipStream_t st) {
    const KernelTables tb = tables_of(ctx);
    VrVariant v;
    v.tail_first = ctx->path == kVringTailFirstPath;
    v.abl = ctx->vr_abl == 128 ? 128 : 0;
    for (size_t b0 = 0; b0 < count; b0 += kVrMaxVBatches) {
        VrVBatches bl{};
        for (size_t b = b0; b < std::min(count, b0 + kVrMaxVBatches); ++b) {
            const ENetHipVerifyBatch& e = batches[b];
            bl.b[bl.count++] = VrVBatch{e.bytes, e.offsets, e.lengths, e.computed, static_cast<uint64_t>(e.count), 0u,
                                        e.slotOffsets, e.connectIds, e.ok};
        }
        // two workgroups per CU by default, single batches too: one cfg2 batch 20.4-20.5 us
        // against 22.1 at one (profiles/r04_verify_wgs/; the checksum instance is the
        // other way round, 18.9 against 18.2-18.4)
        const int wgs = ctx->wgs_per_cu >= 1 ? std::min(ctx->wgs_per_cu, 2) : 2;
        const int rc = vring_launch_vlist(ctx->num_cus * wgs, with_claim(ctx, v, st), st, bl, tb, ctx->d_basis2,
                                          v.abl ? ctx->trace : nullptr);
        if (rc) return rc;
    }
    return 0;
}

int launch_packets(enet_hip_context* ctx, int mode, const PacketArgs& pa, hipStream_t st) {
    if (pa.n == 0) return 0;
    const KernelTables tb = tables_of(ctx);
    const_cast<PacketArgs&>(pa).trace = ctx->trace;
    const_cast<PacketArgs&>(pa).prio = static_cast<uint32_t>(ctx->ablation_prio);
    // the stream kernel takes 4, 8 or 16 lanes per packet; anything else runs direct
    // default (path 0) checksum batches at 4 or 8 lanes: the VGPR-ring kernel, also for
    // length-binned records (its records instance: cfg3 at 4 lanes 59.4 us against the
    // lean kernel's 63.3 since the in-place edge masks, profiles/r03_cfg3_binned/;
    // the lean kernel on paths 13-16)
    if (mode == 0 && (pa.lg == 2 || pa.lg == 3) && ctx->ablation == 0 && vring_path(ctx))
        return vring_launch(pa.lg, ctx->num_cus * vring_wgs(ctx, 1),
                            with_claim(ctx, pa.meta4 ? bin_variant(ctx) : vring_variant(ctx, false), st), st, pa, tb,
                            ctx->d_basis2);
    if (ctx->path != 1 && pa.lg >= 2 && pa.lg <= 4) {
        const bool lean_path = (ctx->path >= kLeanPath0 && ctx->path < kVringPath) || (ctx->path == 0 && ctx->ablation == 0);
        if (lean_path && pa.lg <= 3)
            return lean_launch(mode, pa.lg, ctx->path == 0 ? 0 : ctx->path - kLeanPath0, ctx->ablation,
                               ctx->num_cus, st, pa, tb);
#ifndef ENET_HIP_DIAG
    }
    return -static_cast<int>(hipErrorInvalidValue);          // (the product takes 4 or 8 lanes: set_tuning)
#else
        const uint64_t groups = (pa.n + (64u >> pa.lg) - 1) >> (6 - pa.lg);
        const int geom = (ctx->path == 0 || ctx->path >= kLeanPath0) ? kStreamDefault : ctx->path - 2;
        if (geom < kNumStreamGeoms)
            launch_stream(geom, mode, ctx->ablation, ctx->num_cus, groups, st, pa, tb);
#ifdef ENET_HIP_DIAG
        else
            launch_vstream(geom - kNumStreamGeoms, mode, ctx->ablation, ctx->num_cus, groups, st, pa, tb);
#endif
    } else {
        const uint64_t tasks = pa.n << pa.lg;
        const unsigned grid = grid_for(ctx, tasks);
        if (mode == 0)
            hipLaunchKernelGGL(crc32_direct_kernel<0>, dim3(grid), dim3(kThreads), kLdsTableBytes, st, pa, tb);
        else
            hipLaunchKernelGGL(crc32_direct_kernel<1>, dim3(grid), dim3(kThreads), kLdsTableBytes, st, pa, tb);
    }
    return herr(hipGetLastError());
#endif
}

int ensure(uint8_t** p, size_t* cap, size_t need) { return ensure_device(p, cap, need); }

// The binned gather's workspace: records (1024 per tile of segments, length_bin_compact's
// layout; the binned entry's records fit too) | seg_crc[segCount + 1] (the last: the
// padding records' CRCs, never read) | tile counts | info[segCount] (the split join)
size_t gather_tiles(size_t segCount) { return (segCount + 1023u) / 1024u; }
size_t gather_records_bytes(size_t segCount) { return 16u * 1024u * gather_tiles(segCount); }
size_t gather_crc_bytes(size_t segCount) { return (4u * (segCount + 1u) + 15u) & ~static_cast<size_t>(15u); }

}  // namespace

extern "C" {

int enet_hip_device_count(int* count) {
    if (!count) return -static_cast<int>(hipErrorInvalidValue);
    int c = 0;
    hipError_t e = hipGetDeviceCount(&c);
    *count = (e == hipSuccess) ? c : 0;
    return herr(e);
}

const char* enet_hip_error_string(int code) {
    if (code == 0) return "success";
    if (code > 0) return "unknown";
    if (-code >= ENET_HIP_ERRNO_BASE) return strerror(-code - ENET_HIP_ERRNO_BASE);   // a failed system call
    return hipGetErrorString(static_cast<hipError_t>(-code));
}

int enet_hip_context_create(int device, enet_hip_context** out) {
    if (!out) return -static_cast<int>(hipErrorInvalidValue);
    *out = nullptr;
    int ndev = 0;
    ENH_CHECK(hipGetDeviceCount(&ndev));
    if (device < 0 || device >= ndev) return -static_cast<int>(hipErrorInvalidDevice);
    ENH_CHECK(hipSetDevice(device));
    auto* ctx = new enet_hip_context();
    ctx->device = device;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) == hipSuccess && prop.multiProcessorCount > 0)
        ctx->num_cus = prop.multiProcessorCount;
    const HostTables& ht = host_tables();
    int rc = 0;
    do {
        // the stream a NULL `stream` argument selects: a BLOCKING stream, so work on it
        // is ordered after work on the legacy null stream (hipStreamNonBlocking let a
        // caller's fill of out[] on the null stream run concurrently with the kernel
        // that writes it: the intermittent "unwritten" CRCs of tools/dbg/stress.py)
        if ((rc = herr(hipStreamCreateWithFlags(&ctx->stream, hipStreamDefault)))) break;
        if ((rc = herr(hipMalloc(reinterpret_cast<void**>(&ctx->d_image), ht.image.size() * 4)))) break;
        if ((rc = herr(hipMalloc(reinterpret_cast<void**>(&ctx->d_xn), ht.xn.size() * 4)))) break;
        if ((rc = herr(hipMalloc(reinterpret_cast<void**>(&ctx->d_init), ht.init.size() * 4)))) break;
        if ((rc = herr(hipMalloc(reinterpret_cast<void**>(&ctx->d_zero), 256)))) break;
        if ((rc = herr(hipMemset(ctx->d_zero, 0, 256)))) break;
        if ((rc = herr(hipMemcpy(ctx->d_image, ht.image.data(), ht.image.size() * 4, hipMemcpyHostToDevice)))) break;
        if ((rc = herr(hipMemcpy(ctx->d_xn, ht.xn.data(), ht.xn.size() * 4, hipMemcpyHostToDevice)))) break;
        if ((rc = herr(hipMemcpy(ctx->d_init, ht.init.data(), ht.init.size() * 4, hipMemcpyHostToDevice)))) break;
        if (!ht.basis_ok) {
            rc = -static_cast<int>(hipErrorInvalidImage);
            break;
        }
        if ((rc = herr(hipMalloc(reinterpret_cast<void**>(&ctx->d_basis), ht.basis.size() * 4)))) break;
        if ((rc = herr(hipMemcpy(ctx->d_basis, ht.basis.data(), ht.basis.size() * 4, hipMemcpyHostToDevice)))) break;
        if ((rc = herr(hipMalloc(reinterpret_cast<void**>(&ctx->d_tz), ht.tz.size() * 4)))) break;
        if ((rc = herr(hipMemcpy(ctx->d_tz, ht.tz.data(), ht.tz.size() * 4, hipMemcpyHostToDevice)))) break;
        if ((rc = herr(hipMalloc(reinterpret_cast<void**>(&ctx->d_basis2), ht.basis2.size() * 4)))) break;
        if ((rc = herr(hipMemcpy(ctx->d_basis2, ht.basis2.data(), ht.basis2.size() * 4, hipMemcpyHostToDevice)))) break;
#ifdef ENET_HIP_DIAG
        // the dynamic-round claim words: diagnostics paths only (the product library
        // builds no dynamic-round kernel -- ADVICE r4)
        const size_t claim_bytes = static_cast<size_t>(kVrClaimLines) * kVrClaimWords * 4;
        if ((rc = herr(hipMalloc(reinterpret_cast<void**>(&ctx->d_rounds), claim_bytes)))) break;
        if ((rc = herr(hipMemset(ctx->d_rounds, 0, claim_bytes)))) break;
        const size_t pair_bytes = static_cast<size_t>(kVrPairLines) * kVrPairWords * 8;
        if ((rc = herr(hipMalloc(reinterpret_cast<void**>(&ctx->d_pairs), pair_bytes)))) break;
        if ((rc = herr(hipMemset(ctx->d_pairs, 0, pair_bytes)))) break;
#endif
        if ((rc = vring_setup())) break;
#ifdef ENET_HIP_DIAG
        if ((rc = setup_stream())) break;
        if ((rc = setup_vstream())) break;
        if ((rc = herr(hipFuncSetAttribute(reinterpret_cast<const void*>(crc32_direct_kernel<0>),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, kLdsTableBytes)))) break;
        if ((rc = herr(hipFuncSetAttribute(reinterpret_cast<const void*>(crc32_direct_kernel<1>),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, kLdsTableBytes)))) break;
#endif
        if ((rc = lean_setup())) break;
        if ((rc = herr(hipFuncSetAttribute(reinterpret_cast<const void*>(crc32_gather_kernel),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, kLdsTableBytes)))) break;
    } while (0);
    if (rc) {
        enet_hip_context_destroy(ctx);
        return rc;
    }
    *out = ctx;
    return 0;
}

int enet_hip_context_destroy(enet_hip_context* ctx) {
    if (!ctx) return 0;
    (void)hipSetDevice(ctx->device);
    if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
    (void)hipFree(ctx->d_image);
    (void)hipFree(ctx->d_xn);
    (void)hipFree(ctx->d_init);
    (void)hipFree(ctx->d_zero);
    (void)hipFree(ctx->d_basis);
    (void)hipFree(ctx->d_basis2);
    (void)hipFree(ctx->d_tz);
    (void)hipFree(ctx->d_rounds);
    (void)hipFree(ctx->d_pairs);
    pipeline_release(ctx);
    (void)hipFree(ctx->d_claim);
    (void)hipFree(ctx->d_frag_desc);
    (void)hipFree(ctx->d_rc_scratch);
    if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
    delete ctx;
    return 0;
}

int enet_hip_set_tuning(enet_hip_context* ctx, int lanes_per_packet, int workgroups_per_cu) {
    if (!ctx) return -static_cast<int>(hipErrorInvalidValue);
#ifdef ENET_HIP_DIAG
    if (lanes_per_packet < 0 || lanes_per_packet > 64 || (lanes_per_packet & (lanes_per_packet - 1)))
        return -static_cast<int>(hipErrorInvalidValue);
#else
    if (lanes_per_packet != 0 && lanes_per_packet != 4 && lanes_per_packet != 8)   // (the vring / lean lane counts)
        return -static_cast<int>(hipErrorInvalidValue);
#endif
    if (workgroups_per_cu < 0 || workgroups_per_cu > 8) return -static_cast<int>(hipErrorInvalidValue);
    ctx->lanes_per_packet = lanes_per_packet;
    ctx->wgs_per_cu = workgroups_per_cu;
    return 0;
}

#ifdef ENET_HIP_DIAG
int enet_hip_diag_ablation(enet_hip_context* ctx, int mode) {
    if (!ctx || mode < 0) return -static_cast<int>(hipErrorInvalidValue);
    ctx->bin_identity = (mode >> 30) & 1;                    // 2^30: binned records left in memory order
    ctx->vr_pair = (mode >> 23) & 1;                         // 8388608: vring pair rounds
    ctx->join_abl = (mode >> 20) & 7;                        // 1048576 x (1, 2, 3, 5, 7): gather-join ablations; 4194304: the split join
    // 16777216 x (1 + b), b < 63: the binned gather's short-segment bound b bytes (0: 48)
    ctx->gather_small = (mode >> 24) ? ((mode >> 24) & 63) - 1 : -1;
    ctx->vr_dynamic = (mode >> 19) & 1;                      // 524288: vring dynamic rounds
    const int prio = (mode & 1024) ? 2 : (mode >> 3) & 1;    // 8: static / 1024: progress priority
    ctx->vr_abl = (mode >> 11) & 255;                        // 2048 ... 262144: vring ablations / end records
    mode &= 511;
    ctx->ablation = mode & ~8;
    ctx->ablation_prio = prio;
    return 0;
}

int enet_hip_diag_trace(enet_hip_context* ctx, uint64_t* deviceBuffer) {
    if (!ctx) return -static_cast<int>(hipErrorInvalidValue);
    ctx->trace = deviceBuffer;
    return 0;
}

#endif  // ENET_HIP_DIAG

int enet_hip_set_kernel_path(enet_hip_context* ctx, int path) {
    if (!ctx || !path_built(path)) return -static_cast<int>(hipErrorInvalidValue);
    ctx->path = path;
    return 0;
}

int enet_hip_is_diagnostics_build(void) {
#ifdef ENET_HIP_DIAG
    return 1;
#else
    return 0;
#endif
}

int enet_hip_crc32_batch_device(enet_hip_context* ctx, const uint8_t* bytes, const uint64_t* offsets,
                                const uint32_t* lengths, size_t count, uint32_t* out, void* stream) {
    if (!ctx) return -static_cast<int>(hipErrorInvalidValue);
    if (count == 0) return 0;
    if (!bytes || !offsets || !lengths || !out) return -static_cast<int>(hipErrorInvalidValue);
    ENH_CHECK(hipSetDevice(ctx->device));
    PacketArgs pa{};
    pa.bytes = bytes;
    pa.off = offsets;
    pa.len = lengths;
    pa.n = count;
    pa.lg = static_cast<uint32_t>(log2i(auto_lanes(ctx)));
    pa.out = out;
    return launch_packets(ctx, 0, pa, stream ? static_cast<hipStream_t>(stream) : ctx->stream);
}

int enet_hip_crc32_batch_list_device(enet_hip_context* ctx, const ENetHipBatch* batches, size_t batchCount,
                                     void* stream) {
    if (!ctx) return -static_cast<int>(hipErrorInvalidValue);
    if (batchCount == 0) return 0;
    if (!batches) return -static_cast<int>(hipErrorInvalidValue);
    for (size_t b = 0; b < batchCount; ++b) {
        const ENetHipBatch& e = batches[b];
        if (e.count && (!e.bytes || !e.offsets || !e.lengths || !e.out)) return -static_cast<int>(hipErrorInvalidValue);
    }
    ENH_CHECK(hipSetDevice(ctx->device));
    hipStream_t st = stream ? static_cast<hipStream_t>(stream) : ctx->stream;
    // path 13 (kLeanPath0): the lean kernel over the list, 8 lanes per packet unless
    // set -- the faster one on long serial lists (20 batches: 5.43 vs 5.10 TB/s), the
    // slower one when lists of 4-5 batches overlap on streams (bench driver form:
    // 4548-4784 vs 5011-5186 GiB/s; its one 160-KiB workgroup per CU leaves no room
    // for the next launch's), profiles/r02d_lists_*; default (path 0) and 17 / 18: vring
    if (ctx->path == kLeanPath0 && ctx->ablation == 0 && ctx->vr_abl == 0 &&
        (ctx->lanes_per_packet == 0 || ctx->lanes_per_packet == 4 || ctx->lanes_per_packet == 8)) {
        const int llg = ctx->lanes_per_packet == 4 ? 2 : 3;
        const KernelTables tb = tables_of(ctx);
        for (size_t b0 = 0; b0 < batchCount; b0 += kLeanMaxBatches) {
            const int rc = lean_launch_list(llg, ctx->num_cus, st, batches + b0,
                                            std::min<size_t>(batchCount - b0, kLeanMaxBatches), tb);
            if (rc) return rc;
        }
        return 0;
    }
    const int lg = log2i(auto_lanes(ctx));
    if ((lg == 2 || lg == 3) && ctx->ablation == 0 && vring_path(ctx)) {
        const KernelTables tb = tables_of(ctx);
        for (size_t b0 = 0; b0 < batchCount; b0 += kVrMaxBatches) {
            VrBatches bl{};
            for (size_t b = b0; b < std::min(batchCount, b0 + kVrMaxBatches); ++b)
                bl.b[bl.count++] = VrBatch{batches[b].bytes, batches[b].offsets, batches[b].lengths, batches[b].out,
                                           static_cast<uint64_t>(batches[b].count), 0u};
            const int rc = vring_launch_list(lg, ctx->num_cus * vring_wgs(ctx, bl.count),
                                             with_claim(ctx, vring_variant(ctx, true), st), st, bl, tb, ctx->d_basis2,
                                             ctx->trace);
            if (rc) return rc;
        }
        return 0;
    }
    // other lane counts / paths: one launch per batch on the path they select
    for (size_t b = 0; b < batchCount; ++b) {
        const ENetHipBatch& e = batches[b];
        const int rc = enet_hip_crc32_batch_device(ctx, e.bytes, e.offsets, e.lengths, e.count, e.out, st);
        if (rc) return rc;
    }
    return 0;
}

size_t enet_hip_binned_workspace_size(size_t count) { return length_bin_workspace(count, false); }

size_t enet_hip_verify_binned_workspace_size(size_t count) { return length_bin_workspace(count, true); }

int enet_hip_crc32_batch_device_binned(enet_hip_context* ctx, const uint8_t* bytes, const uint64_t* offsets,
                                       const uint32_t* lengths, size_t count, uint32_t* out, void* workspace,
                                       size_t workspaceBytes, void* stream) {
    if (!ctx) return -static_cast<int>(hipErrorInvalidValue);
    if (count == 0) return 0;
    if (!bytes || !offsets || !lengths || !out || !workspace || count > 0xFFFFFFFFull ||
        workspaceBytes < enet_hip_binned_workspace_size(count) || (reinterpret_cast<uintptr_t>(workspace) & 15u))
        return -static_cast<int>(hipErrorInvalidValue);
    ENH_CHECK(hipSetDevice(ctx->device));
    hipStream_t st = stream ? static_cast<hipStream_t>(stream) : ctx->stream;
    PacketArgs pa{};
    pa.bytes = bytes;
    pa.off = offsets;
    pa.len = lengths;
    pa.n = count;
    // mixed lengths (mean well under the 1200-B MTU payload): 4 lanes per packet unless set
    // (cfg3: 3160-3217 GiB/s at 4 lanes against 2495 at 8, profiles/r01e_*, r01f_*)
    pa.lg = static_cast<uint32_t>(log2i(ctx->lanes_per_packet > 0 ? ctx->lanes_per_packet : 4));
    pa.out = out;
    // default path: one launch -- each workgroup orders its own tile of at most 1024
    // packets in its prologue (vring_launch_local) -- when the batch fits one tile per
    // workgroup (cfg3: 262144 packets); larger batches, path 17 and the diagnostics
    // ablations: the bin kernel, then the records instance
    // (two workgroups per CU unless set: cfg3 49.5-49.9 us against 50.7-51.0 at one, and
    // against 51.3-51.5 for the two-launch form at two, one box, profiles/r06_local/)
    const int wgs = ctx->wgs_per_cu >= 1 ? std::min(ctx->wgs_per_cu, 2) : 2;
    if (ctx->path == 0 && (pa.lg == 2 || pa.lg == 3) && ctx->ablation == 0 && ctx->vr_abl == 0 &&
        !ctx->bin_identity && !ctx->vr_dynamic &&
        count <= static_cast<uint64_t>(kVrLocalTile) * static_cast<uint64_t>(ctx->num_cus * wgs)) {
        pa.trace = ctx->trace;
        return vring_launch_local(pa.lg, ctx->num_cus * wgs, st, pa, workspace, tables_of(ctx), ctx->d_basis2);
    }
    // the ordered records pay on the vring (path 0) and lean kernels; every other path
    // reads len/off itself
    const bool lean = ctx->path != 1 && (pa.lg == 2 || pa.lg == 3) && ctx->ablation == 0 &&
                      ((ctx->path >= kLeanPath0 && ctx->path < kVringPath) || vring_path(ctx));
    if (lean) {
        int rc;
        if ((rc = length_bin(lengths, offsets, nullptr, nullptr, count, 64u >> pa.lg, workspace, st, ctx->bin_identity)))
            return rc;
        pa.meta4 = static_cast<const uint32_t*>(workspace);
    }
    return launch_packets(ctx, 0, pa, st);
}

int enet_hip_verify_batch_device(enet_hip_context* ctx, const uint8_t* bytes, const uint64_t* offsets,
                                 const uint32_t* lengths, const uint32_t* slotOffsets, const uint32_t* connectIds,
                                 size_t count, uint8_t* ok, uint32_t* computed, void* stream) {
    if (!ctx) return -static_cast<int>(hipErrorInvalidValue);
    if (count == 0) return 0;
    if (!bytes || !offsets || !lengths || !slotOffsets || !connectIds || !ok)
        return -static_cast<int>(hipErrorInvalidValue);
    ENH_CHECK(hipSetDevice(ctx->device));
    PacketArgs pa{};
    pa.bytes = bytes;
    pa.off = offsets;
    pa.len = lengths;
    pa.n = count;
    pa.lg = static_cast<uint32_t>(log2i(auto_lanes(ctx, 1)));
    pa.out = computed;
    pa.slot_off = slotOffsets;
    pa.connect = connectIds;
    pa.ok = ok;
    hipStream_t st = stream ? static_cast<hipStream_t>(stream) : ctx->stream;
    if (verify_on_vring(ctx, static_cast<int>(pa.lg))) {
        const ENetHipVerifyBatch b{bytes, offsets, lengths, slotOffsets, connectIds, count, ok, computed};
        return verify_vring_list(ctx, &b, 1, st);
    }
    return launch_packets(ctx, 1, pa, st);
}

int enet_hip_verify_batch_list_device(enet_hip_context* ctx, const ENetHipVerifyBatch* batches, size_t batchCount,
                                      void* stream) {
    if (!ctx) return -static_cast<int>(hipErrorInvalidValue);
    if (batchCount == 0) return 0;
    if (!batches) return -static_cast<int>(hipErrorInvalidValue);
    for (size_t b = 0; b < batchCount; ++b) {
        const ENetHipVerifyBatch& e = batches[b];
        if (e.count && (!e.bytes || !e.offsets || !e.lengths || !e.slotOffsets || !e.connectIds || !e.ok))
            return -static_cast<int>(hipErrorInvalidValue);
    }
    ENH_CHECK(hipSetDevice(ctx->device));
    hipStream_t st = stream ? static_cast<hipStream_t>(stream) : ctx->stream;
    const int lg = log2i(auto_lanes(ctx, 1));
    if (verify_on_vring(ctx, lg)) return verify_vring_list(ctx, batches, batchCount, st);
    // the lean kernel's verify-list instance (geometry 0) on the paths where single
    // verify batches run the lean kernel (launch_packets, mode 1)
    if ((lg == 2 || lg == 3) && ctx->ablation == 0 && ctx->vr_abl == 0 &&
        (ctx->path == 0 || (ctx->path >= kLeanPath0 && ctx->path < kVringPath))) {
        const KernelTables tb = tables_of(ctx);
        for (size_t b0 = 0; b0 < batchCount; b0 += kLeanMaxVBatches) {
            const int rc = lean_launch_vlist(lg, ctx->num_cus, st, batches + b0,
                                             std::min<size_t>(batchCount - b0, kLeanMaxVBatches), tb);
            if (rc) return rc;
        }
        return 0;
    }
    for (size_t b = 0; b < batchCount; ++b) {                // other lane counts / paths: one launch per batch
        const ENetHipVerifyBatch& e = batches[b];
        const int rc = enet_hip_verify_batch_device(ctx, e.bytes, e.offsets, e.lengths, e.slotOffsets, e.connectIds,
                                                    e.count, e.ok, e.computed, st);
        if (rc) return rc;
    }
    return 0;
}

int enet_hip_verify_batch_device_binned(enet_hip_context* ctx, const uint8_t* bytes, const uint64_t* offsets,
                                        const uint32_t* lengths, const uint32_t* slotOffsets,
                                        const uint32_t* connectIds, size_t count, uint8_t* ok, uint32_t* computed,
                                        void* workspace, size_t workspaceBytes, void* stream) {
    if (!ctx) return -static_cast<int>(hipErrorInvalidValue);
    if (count == 0) return 0;
    if (!bytes || !offsets || !lengths || !slotOffsets || !connectIds || !ok || !workspace ||
        count > 0xFFFFFFFFull || workspaceBytes < enet_hip_verify_binned_workspace_size(count) ||
        (reinterpret_cast<uintptr_t>(workspace) & 15u))
        return -static_cast<int>(hipErrorInvalidValue);
    ENH_CHECK(hipSetDevice(ctx->device));
    hipStream_t st = stream ? static_cast<hipStream_t>(stream) : ctx->stream;
    PacketArgs pa{};
    pa.bytes = bytes;
    pa.off = offsets;
    pa.len = lengths;
    pa.n = count;
    pa.lg = static_cast<uint32_t>(log2i(auto_lanes(ctx, 1)));
    pa.out = computed;
    pa.slot_off = slotOffsets;
    pa.connect = connectIds;
    pa.ok = ok;
    const bool lean = ctx->path != 1 && (pa.lg == 2 || pa.lg == 3) &&
                      ((ctx->path >= kLeanPath0 && ctx->path < kVringPath) || (ctx->path == 0 && ctx->ablation == 0));
    if (lean) {
        int rc;
        if ((rc = length_bin(lengths, offsets, slotOffsets, connectIds, count, 64u >> pa.lg, workspace, st))) return rc;
        pa.meta4 = static_cast<const uint32_t*>(workspace);
    }
    return launch_packets(ctx, 1, pa, st);
}

int enet_hip_crc32_gather_device(enet_hip_context* ctx, const uint8_t* bytes, const uint64_t* segOffsets,
                                 const uint32_t* segLengths, const uint32_t* segFirst, size_t dgramCount,
                                 uint32_t* out, void* stream) {
    if (!ctx) return -static_cast<int>(hipErrorInvalidValue);
    if (dgramCount == 0) return 0;
    if (!bytes || !segOffsets || !segLengths || !segFirst || !out) return -static_cast<int>(hipErrorInvalidValue);
    ENH_CHECK(hipSetDevice(ctx->device));
    GatherArgs ga{bytes, segOffsets, segLengths, segFirst, dgramCount, out, ~0ull};
    const unsigned grid = grid_for(ctx, dgramCount);
    hipLaunchKernelGGL(crc32_gather_kernel, dim3(grid), dim3(kThreads), kLdsTableBytes,
                       stream ? static_cast<hipStream_t>(stream) : ctx->stream, ga, tables_of(ctx));
    return herr(hipGetLastError());
}

// records | seg_crc | tile counts (| diagnostics: the split join's info[], 8 B per segment)
static size_t gather_counts_bytes(size_t segCount) { return (4u * gather_tiles(segCount) + 15u) & ~static_cast<size_t>(15u); }

size_t enet_hip_gather_binned_workspace_size(size_t segCount) {
#ifdef ENET_HIP_DIAG
    return gather_records_bytes(segCount) + gather_crc_bytes(segCount) + gather_counts_bytes(segCount) +
           8u * segCount + 16u;
#else
    return gather_records_bytes(segCount) + gather_crc_bytes(segCount) + gather_counts_bytes(segCount) + 16u;
#endif
}

int enet_hip_crc32_gather_binned_device(enet_hip_context* ctx, const uint8_t* bytes, const uint64_t* segOffsets,
                                        const uint32_t* segLengths, size_t segCount, const uint32_t* segFirst,
                                        size_t dgramCount, uint32_t* out, void* workspace, size_t workspaceBytes,
                                        void* stream) {
    if (!ctx) return -static_cast<int>(hipErrorInvalidValue);
    if (dgramCount == 0) return 0;
    if (!bytes || !segFirst || !out || (segCount && (!segOffsets || !segLengths || !workspace)) ||
        segCount > 0xFFFFFFFFull || workspaceBytes < enet_hip_gather_binned_workspace_size(segCount) ||
        (reinterpret_cast<uintptr_t>(workspace) & 15u))
        return -static_cast<int>(hipErrorInvalidValue);
    ENH_CHECK(hipSetDevice(ctx->device));
    hipStream_t st = stream ? static_cast<hipStream_t>(stream) : ctx->stream;
    const size_t bws = gather_records_bytes(segCount);
    uint32_t* seg_crc = reinterpret_cast<uint32_t*>(static_cast<uint8_t*>(workspace) + bws);
    uint32_t* counts = reinterpret_cast<uint32_t*>(static_cast<uint8_t*>(workspace) + bws + gather_crc_bytes(segCount));
    const int lanes = ctx->lanes_per_packet > 0 ? ctx->lanes_per_packet : 8;
    // The default (vring paths, 4 or 8 lanes): segments of at most kGatherSmall bytes
    // are folded by the join, the rest sorted per tile into records (padded, tile
    // counts on the device: VrBatches::tile_counts) and checksummed by the vring's
    // records instance.  Other paths: every segment through the binned entry.
    const bool split = vring_path(ctx) && ctx->ablation == 0 && (lanes == 4 || lanes == 8);
    GatherArgs ga{bytes, segOffsets, segLengths, segFirst, dgramCount, out, segCount};
#ifdef ENET_HIP_DIAG
    if (split && ctx->join_abl == 4) {
        // (diagnostics 4194304) the split join (gather_join.hpp): pre-join beside the
        // binning tiles, records, post-join per segment.  Bit-exact, and slower than the
        // one-pass join below: 70.3-72.4 against 68.3-70.4 us on cfg5 (DESIGN 4.4,
        // profiles/r05_split_join/)
        const KernelTables tb = tables_of(ctx);
        const uint32_t kpk = lanes == 4 ? 16u : 8u;
        uint2* info = reinterpret_cast<uint2*>(reinterpret_cast<uint8_t*>(counts) + gather_counts_bytes(segCount));
        const uint32_t small = gather_small(ctx);
        const unsigned pj = static_cast<unsigned>(std::min<uint64_t>((dgramCount + 255u) / 256u, 8u * ctx->num_cus));
        int rc;
        if ((rc = gather_bin_prejoin(ga, info, tb, small, kpk, workspace, counts, pj, st))) return rc;
        if (!segCount) return 0;
        VrBatches bl{};
        bl.count = 1;
        bl.tiles = static_cast<uint32_t>(gather_tiles(segCount));
        bl.tile_counts = counts;
        bl.b[0] = VrBatch{bytes, static_cast<const uint64_t*>(workspace), nullptr, seg_crc, 1024ull * bl.tiles, 0u};
        const int gw = ctx->wgs_per_cu >= 1 ? std::min(ctx->wgs_per_cu, 2) : 2;
        VrVariant gv = bin_variant(ctx);
        gv.compact = gw >= 2;
        if ((rc = vring_launch_list(lanes == 4 ? 2 : 3, ctx->num_cus * gw, with_claim(ctx, gv, st), st, bl, tb,
                                    ctx->d_basis2, nullptr, true)))
            return rc;
        const unsigned pg = static_cast<unsigned>(std::min<uint64_t>((segCount + 511u) / 512u, 8u * ctx->num_cus));
        hipLaunchKernelGGL(crc32_gather_post_kernel, dim3(pg), dim3(256), 0, st, segLengths, seg_crc, info, segFirst,
                           static_cast<uint64_t>(dgramCount), static_cast<uint64_t>(segCount), small, out);
        return herr(hipGetLastError());
    }
#endif
    // default path, up to 2048 segments per workgroup (cfg5: 602112 at two per CU): one
    // launch -- each workgroup sorts its own tile's segments longer than the short bound
    // and checksums them (vring_launch_local) -- then the join
    const int lgw = ctx->wgs_per_cu >= 1 ? std::min(ctx->wgs_per_cu, 2) : 2;
    if (segCount && split && ctx->path == 0 && ctx->vr_abl == 0 && !ctx->vr_dynamic &&
        segCount <= static_cast<uint64_t>(kVrLocalTile) * static_cast<uint64_t>(ctx->num_cus * lgw)) {
        PacketArgs pa{};
        pa.bytes = bytes;
        pa.off = segOffsets;
        pa.len = segLengths;
        pa.n = segCount;
        pa.out = seg_crc;
        const int rc = vring_launch_local(lanes == 4 ? 2 : 3, ctx->num_cus * lgw, st, pa, workspace, tables_of(ctx),
                                          ctx->d_basis2, gather_small(ctx) + 1u);
        if (rc) return rc;
    } else if (segCount && split) {
        const KernelTables tb = tables_of(ctx);
        const uint32_t kpk = lanes == 4 ? 16u : 8u;
        int rc;
        if ((rc = length_bin_compact(segLengths, segOffsets, segCount, kpk, gather_small(ctx), workspace, counts, st)))
            return rc;
        VrBatches bl{};
        bl.count = 1;
        bl.tiles = static_cast<uint32_t>(gather_tiles(segCount));
        bl.tile_counts = counts;
        bl.b[0] = VrBatch{bytes, static_cast<const uint64_t*>(workspace), nullptr, seg_crc, 1024ull * bl.tiles, 0u};
        // two workgroups per CU unless set: the compact records instance (cfg5 67.8-68.3 against
        // 69.9-70.0 us at one, profiles/r04_compact/)
        const int gw = ctx->wgs_per_cu >= 1 ? std::min(ctx->wgs_per_cu, 2) : 2;
        VrVariant gv = bin_variant(ctx);
        gv.compact = gw >= 2;
        if ((rc = vring_launch_list(lanes == 4 ? 2 : 3, ctx->num_cus * gw, with_claim(ctx, gv, st), st, bl, tb,
                                    ctx->d_basis2, nullptr, true)))
            return rc;
    } else if (segCount) {                                   // every segment's CRC, mixed lengths: length-binned
        const int rc = enet_hip_crc32_batch_device_binned(ctx, bytes, segOffsets, segLengths, segCount, seg_crc,
                                                          workspace, bws, st);
        if (rc) return rc;
    }
    const unsigned grid = grid_for(ctx, dgramCount);
    const uint32_t small = split ? gather_small(ctx) : 0u;
#ifdef ENET_HIP_DIAG
    switch (ctx->join_abl) {
        case 1: hipLaunchKernelGGL(crc32_gather_join_kernel<1>, dim3(grid), dim3(kThreads), 0, st, ga, seg_crc, tables_of(ctx), small); break;
        case 2: hipLaunchKernelGGL(crc32_gather_join_kernel<2>, dim3(grid), dim3(kThreads), 0, st, ga, seg_crc, tables_of(ctx), small); break;
        case 3: hipLaunchKernelGGL(crc32_gather_join_kernel<3>, dim3(grid), dim3(kThreads), 0, st, ga, seg_crc, tables_of(ctx), small); break;
        case 5: hipLaunchKernelGGL(crc32_gather_join_kernel<5>, dim3(grid), dim3(kThreads), 0, st, ga, seg_crc, tables_of(ctx), small); break;
        case 7: hipLaunchKernelGGL(crc32_gather_join_kernel<7>, dim3(grid), dim3(kThreads), 0, st, ga, seg_crc, tables_of(ctx), small); break;
        default: hipLaunchKernelGGL(crc32_gather_join_kernel<0>, dim3(grid), dim3(kThreads), 0, st, ga, seg_crc, tables_of(ctx), small);
    }
#else
    hipLaunchKernelGGL(crc32_gather_join_kernel<0>, dim3(grid), dim3(kThreads), 0, st, ga, seg_crc, tables_of(ctx), small);
#endif
    return herr(hipGetLastError());
}

int enet_hip_fragment_reassemble_device(enet_hip_context* ctx, const uint8_t* bytes, const uint64_t* cmdOffsets,
                                        const uint32_t* cmdAvail, const int32_t* slots, size_t count,
                                        uint32_t maximumPacketSize, uint8_t* msgBytes, const uint64_t* msgOffsets,
                                        const uint32_t* msgLengths, const uint32_t* msgFragCounts, uint32_t* fragments,
                                        uint32_t wordsPerMsg, uint32_t* remaining, size_t slotCount, int8_t* status,
                                        void* stream) {
    if (!ctx) return -static_cast<int>(hipErrorInvalidValue);
    if (count == 0) return 0;
    if (!bytes || !cmdOffsets || !cmdAvail || !slots || !status || (slotCount && (!msgBytes || !msgOffsets ||
        !msgLengths || !msgFragCounts || !fragments || !remaining || wordsPerMsg == 0)))
        return -static_cast<int>(hipErrorInvalidValue);
    if (slotCount > (static_cast<size_t>(1) << 31) || wordsPerMsg > (1u << 15)) return -static_cast<int>(hipErrorInvalidValue);
    // claim words hold command indices as uint32 with 0xFFFFFFFF = unclaimed
    if (count >= 0xFFFFFFFFull) return -static_cast<int>(hipErrorInvalidValue);
    std::lock_guard<std::mutex> lk(ctx->mu);
    ENH_CHECK(hipSetDevice(ctx->device));
    hipStream_t st = stream ? static_cast<hipStream_t>(stream) : ctx->stream;
    // scratch: claim words (~0 between calls, restored by frag_copy_kernel or
    // frag_copy_claims_kernel), then the per-slot winner counts and the deferred flag
    // (0 between calls, restored by frag_copy_kernel / frag_serial_kernel)
    const size_t claims = std::max<size_t>(1, slotCount * wordsPerMsg * 32u);
    const size_t need = claims + slotCount + 1;
    // Refill on any layout change that could expose words not in the filled state.
    // d_claim_cap is the END OF THE FILLED LAYOUT (set to `need` at each fill, not
    // the allocation size): with the same claim-word count, a call whose winner
    // counts and flag fit in [claims, d_claim_cap) reads words the last fill zeroed
    // and every call since restored to zero; a larger slotCount refills
    // (tests/test_gpu_fragments.py test_fragments_scratch_layout_changes).
    if (need > ctx->d_claim_cap || claims != ctx->d_claim_words) {
        ENH_CHECK(hipStreamSynchronize(st));
        if (need > ctx->d_claim_cap) {
            (void)hipFree(ctx->d_claim);
            ctx->d_claim = nullptr;
            ctx->d_claim_cap = 0;
            ENH_CHECK(hipMalloc(reinterpret_cast<void**>(&ctx->d_claim), need * 4));
        }
        ctx->d_claim_cap = 0;                  // valid only once both fills are queued
        ENH_CHECK(hipMemsetAsync(ctx->d_claim, 0xFF, claims * 4, st));
        ENH_CHECK(hipMemsetAsync(ctx->d_claim + claims, 0, (need - claims) * 4, st));
        ctx->d_claim_cap = need;
        ctx->d_claim_words = claims;
    }
    int rc;
    // copy descriptors: by command (n each), and on the slots decide path also by claim
    // word (slot-major, `claims` each; fragment_kernels.hpp frag_slots_path)
    const size_t qn = frag_slots_path(static_cast<uint64_t>(slotCount) * wordsPerMsg * 32u, count) ? claims : 0;
    if ((rc = ensure(&ctx->d_frag_desc, &ctx->d_frag_desc_cap, count * 28 + qn * 20 + 64))) return rc;
    uint64_t* d_src = reinterpret_cast<uint64_t*>(ctx->d_frag_desc);
    uint64_t* d_dst = d_src + count;
    uint64_t* d_cl = d_dst + count;
    uint64_t* q_src = d_cl + count;
    uint64_t* q_dst = q_src + qn;
    uint32_t* d_len = reinterpret_cast<uint32_t*>(q_dst + qn);
    uint32_t* q_len = d_len + count;
    FragArgs a{bytes, cmdOffsets, cmdAvail, slots, count, maximumPacketSize, msgBytes, msgOffsets, msgLengths,
               msgFragCounts, fragments, wordsPerMsg, remaining, slotCount, status, ctx->d_claim,
               ctx->d_claim + claims, ctx->d_claim + claims + slotCount, d_src, d_dst, d_len, d_cl,
               qn ? q_src : nullptr, qn ? q_dst : nullptr, qn ? q_len : nullptr};
    rc = fragment_reassemble_launch(a, ctx->num_cus, st);
    // a failed launch may leave claim words set: the next call starts from fresh fills
    if (rc) ctx->d_claim_cap = 0;
    return rc;
}

}  // extern "C"

// The batched range coder with the context's lock already held (the public entries
// below, and the UDP pipelines of host_pipeline.hip that decompress / compress inside
// their own locked call).
int enethip::range_coder_locked(enet_hip_context* ctx, bool decompress, const uint8_t* in, const uint64_t* inOffsets,
                                const uint32_t* inLengths, size_t count, uint8_t* out, const uint64_t* outOffsets,
                                const uint32_t* outLimits, uint32_t* outLengths, hipStream_t st) {
    if (count == 0) return 0;
    ENH_CHECK(hipSetDevice(ctx->device));
    // one lane per DGRAM, 16 per wave, at most 16 waves per CU: 65 536 DGRAMs in flight,
    // as many as 4 full waves per CU had, with a quarter of the stragglers per wave
    // (1.30-1.36 against 1.05 GB/s on tools/rc_bench.py, profiles/r04_range_coder/);
    // the models are HBM scratch, kRangeModelBytes per lane
    uint32_t lanes = 16, waves = 16;
#ifdef ENET_HIP_DIAG
    if (const char* e = getenv("ENET_HIP_RC_LANES")) lanes = static_cast<uint32_t>(atoi(e));
    if (const char* e = getenv("ENET_HIP_RC_WAVES")) waves = static_cast<uint32_t>(atoi(e));
    if (lanes == 0 || lanes > 64 || waves == 0 || waves > 32) return -static_cast<int>(hipErrorInvalidValue);
    const char* il = getenv("ENET_HIP_RC_INTERLEAVE");
    const uint32_t interleave = il ? static_cast<uint32_t>(atoi(il) != 0) : 0u;
#else
    const uint32_t interleave = 0;
#endif
    const uint64_t threads = std::min<uint64_t>(count, static_cast<uint64_t>(ctx->num_cus) * waves * lanes);
    const size_t need = ((threads + lanes - 1) / lanes) * lanes * kRangeModelBytes;
    if (need > ctx->d_rc_scratch_cap) {
        ENH_CHECK(hipStreamSynchronize(st));
        int rc;
        if ((rc = ensure(&ctx->d_rc_scratch, &ctx->d_rc_scratch_cap, need))) return rc;
    }
    RangeArgs a{in, inOffsets, inLengths, count, out, outOffsets, outLimits, outLengths, ctx->d_rc_scratch, interleave};
    return range_coder_launch(decompress, a, threads, lanes, st);
}

extern "C" {

static int range_coder_call(enet_hip_context* ctx, bool decompress, const uint8_t* in, const uint64_t* inOffsets,
                            const uint32_t* inLengths, size_t count, uint8_t* out, const uint64_t* outOffsets,
                            const uint32_t* outLimits, uint32_t* outLengths, void* stream) {
    if (!ctx) return -static_cast<int>(hipErrorInvalidValue);
    if (count == 0) return 0;
    if (!in || !inOffsets || !inLengths || !out || !outOffsets || !outLimits || !outLengths)
        return -static_cast<int>(hipErrorInvalidValue);
    std::lock_guard<std::mutex> lk(ctx->mu);
    return range_coder_locked(ctx, decompress, in, inOffsets, inLengths, count, out, outOffsets, outLimits, outLengths,
                              stream ? static_cast<hipStream_t>(stream) : ctx->stream);
}

int enet_hip_range_compress_device(enet_hip_context* ctx, const uint8_t* in, const uint64_t* inOffsets,
                                   const uint32_t* inLengths, size_t count, uint8_t* out, const uint64_t* outOffsets,
                                   const uint32_t* outLimits, uint32_t* outLengths, void* stream) {
    return range_coder_call(ctx, false, in, inOffsets, inLengths, count, out, outOffsets, outLimits, outLengths,
                            stream);
}

int enet_hip_range_decompress_device(enet_hip_context* ctx, const uint8_t* in, const uint64_t* inOffsets,
                                     const uint32_t* inLengths, size_t count, uint8_t* out,
                                     const uint64_t* outOffsets, const uint32_t* outLimits, uint32_t* outLengths,
                                     void* stream) {
    return range_coder_call(ctx, true, in, inOffsets, inLengths, count, out, outOffsets, outLimits, outLengths,
                            stream);
}

int enet_hip_read_probe_device(enet_hip_context* ctx, const uint8_t* bytes, size_t byteCount, uint32_t* sink,
                               void* stream) {
    if (!ctx || !bytes || !sink || (reinterpret_cast<uintptr_t>(bytes) & 15u))
        return -static_cast<int>(hipErrorInvalidValue);
    ENH_CHECK(hipSetDevice(ctx->device));
    const uint64_t nvec = byteCount / 16;
    if (nvec == 0) return 0;
    const unsigned grid = static_cast<unsigned>(std::min<uint64_t>((nvec + kThreads - 1) / kThreads,
                                                                   static_cast<uint64_t>(ctx->num_cus) * 8));
    hipLaunchKernelGGL(read_probe_kernel, dim3(grid), dim3(kThreads), 0,
                       stream ? static_cast<hipStream_t>(stream) : ctx->stream, bytes, nvec, sink);
    return herr(hipGetLastError());
}

int enet_hip_device_alloc(enet_hip_context* ctx, size_t bytes, void** out) {
    if (!ctx || !out) return -static_cast<int>(hipErrorInvalidValue);
    ENH_CHECK(hipSetDevice(ctx->device));
    return herr(hipMalloc(out, bytes ? bytes : 1));
}
int enet_hip_device_free(enet_hip_context* ctx, void* ptr) {
    if (!ctx) return -static_cast<int>(hipErrorInvalidValue);
    ENH_CHECK(hipSetDevice(ctx->device));
    return herr(hipFree(ptr));
}
int enet_hip_host_alloc(size_t bytes, void** out) {
    if (!out) return -static_cast<int>(hipErrorInvalidValue);
    return herr(hipHostMalloc(out, bytes ? bytes : 1, hipHostMallocDefault));
}
int enet_hip_host_free(void* ptr) { return herr(hipHostFree(ptr)); }
int enet_hip_memcpy_h2d(enet_hip_context* ctx, void* dst, const void* src, size_t bytes) {
    if (!ctx) return -static_cast<int>(hipErrorInvalidValue);
    ENH_CHECK(hipSetDevice(ctx->device));
    return herr(hipMemcpy(dst, src, bytes, hipMemcpyHostToDevice));
}
int enet_hip_memcpy_d2h(enet_hip_context* ctx, void* dst, const void* src, size_t bytes) {
    if (!ctx) return -static_cast<int>(hipErrorInvalidValue);
    ENH_CHECK(hipSetDevice(ctx->device));
    return herr(hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost));
}
int enet_hip_synchronize(enet_hip_context* ctx) {
    if (!ctx) return -static_cast<int>(hipErrorInvalidValue);
    ENH_CHECK(hipSetDevice(ctx->device));
    ENH_CHECK(hipStreamSynchronize(ctx->stream));
    return herr(hipDeviceSynchronize());
}

}  // extern "C"
