// crc32_lean.hip -- the lean streamed CRC32 kernel for gfx950 (MI355X): the hot
// path of libenethip.  Path replaced: ENet.enet_crc32
// (/root/reference/enet-csharp/ENet/c/packet.cs:142-160) over a whole batch of
// DGRAMs, and the receive verify around it (c/protocol.cs:1052-1068).
//
// Arithmetic = crc32_stream_kernel's (tests/kernel_model.py):
// P = 2^LG lanes per packet walk its 32-byte window blocks strided (lane k folds
// blocks w with (w + r) % P == k) with the advancing slicing-by-32 tables of the
// P image, lane k's 32k-byte overshoot is undone by four correction lookups and
// the P registers are XORed.  What differs is the schedule, cut down to what the
// memory stream needs (tools/dmabench.hip: this loop shape alone streams 75 MiB
// in 12.6-13.3 us):
//   * a stage of a packet is one contiguous P*32-byte chunk (2P pieces of 16 B);
//     lane k of the packet DMAs pieces k and P + k, so each of the two
//     global_load_lds_dwordx4 per stage reads P*16 contiguous bytes per packet and
//     a lane's producer needs only its own packet's window.  Lane k's block (chunk
//     block w0) then sits as 32 contiguous LDS bytes in instruction 2w0/P's area;
//   * every stage issues exactly two data DMAs (a lane past its blocks, or a
//     wave past its groups, reads the zero buffer), so the wait for a stage is
//     the constant vmcnt(2(NB-1)) -- plus the metadata DMAs of a chunk in the
//     one or two stages after one is issued, picked by a scalar count;
//   * packet metadata (len, offset; slot offset and connectID for verify) is
//     DMA'd per chunk of JM groups into one of two LDS halves, a chunk ahead;
//   * the 8 data dwords are read with eight ds_read_b32 whose per-lane addresses
//     already apply the lane's dword permutation D(l) (conflict-free: see
//     LeanSched), so the fold is 8 reg-injection bitop3 + 32 v_perm + 32
//     ds_read_b32 + 16 xor3 (the b128 form needs 18 bitop3 for the permutation);
//   * lanes per packet is a template parameter;
//   * the 64 KiB table image is not copied into every CU: waves 0..8 DMA one
//     256-byte row each of a 2.3 KiB basis (KernelTables::basis) and every wave
//     rebuilds 256/W rows from it between two raw barriers, while its first
//     stages are already in flight.
// Blocks holding a partial head/tail piece (or, in verify, the checksum slot) are
// read in original order and go through edge_fix + fold_block, as before.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "crc32_lean.hpp"
#include "gather_join.hpp"

namespace enethip {

// Lane schedule: lane l looks up byte m = i ^ pi(l) at step i, pi(l) = 4 D(l) + b(l),
// D(l) the dword permutation, b(l) the byte permutation inside a dword.  pi is a
// bit permutation of l & 31, so the 32 lanes of a half-wave read 32 different
// tables in every lookup.  The data read of register r (original
// dword r ^ D) of lane (packet j, lane k) hits bank 4jP + 8 (w0 mod P/2) + (r ^ D)
// mod 32; it is conflict-free for every r and every rotation when D holds the two
// low packet bits and the lane bit that separates w0 from w0 + P/2:
//   P = 8 (l = 8j + k): D = l3 | l4 << 1 | l2 << 2, b = l0 | l1 << 1
//   P = 4 (l = 4j + k): D = l3 | l4 << 1 | l1 << 2, b = l0 | l2 << 1
// (tests/test_kernel_model.py checks both).
struct LeanSched {
    LaneSched a;        // col/sel for the lookups; m1/m2/hs realise D for fold_block
    uint32_t dq[8];     // byte offset in the lane's 32-byte block of data register r
    uint32_t dm[8];     // all-ones in the register that holds original dword 0
};

template <int LG>
__device__ __forceinline__ LeanSched make_lean_sched(uint32_t lane) {
    LeanSched s;
    const uint32_t l5 = lane & 31u;
    const uint32_t sb = LG == 3 ? 2u : 1u;                  // lane bit giving D's bit 2
    const uint32_t ob = LG == 3 ? 1u : 2u;                  // lane bit giving b's bit 1
    const uint32_t D = ((l5 >> 3) & 3u) | (((l5 >> sb) & 1u) << 2);
    const uint32_t b = (l5 & 1u) | (((l5 >> ob) & 1u) << 1);
    const uint32_t pi = 4u * D + b;
#pragma unroll
    for (int g = 0; g < 8; ++g) {
        uint32_t r = 0;
#pragma unroll
        for (int h = 0; h < 4; ++h) r |= col_byte(31u - ((4u * g + h) ^ pi)) << (8 * h);
        s.a.col[g] = r;
    }
#pragma unroll
    for (int h = 0; h < 4; ++h) s.a.sel[h] = static_cast<uint32_t>(h) | ((4u + (h ^ b)) << 8) | 0x0C0C0000u;
    s.a.m1 = 0u - (D & 1u);
    s.a.m2 = 0u - ((D >> 1) & 1u);
    s.a.hs = 0u - ((D >> 2) & 1u);
#pragma unroll
    for (int r = 0; r < 8; ++r) {
        s.dq[r] = 4u * (static_cast<uint32_t>(r) ^ D);
        s.dm[r] = static_cast<uint32_t>(r) == D ? 0xFFFFFFFFu : 0u;
    }
    return s;
}

// One block (32 Sarwate steps, packet.cs:153) from the lane-permuted dwords x.
__device__ __forceinline__ uint32_t fold_perm(uint32_t reg, const uint32_t (&x)[8], const LeanSched& s) {
    uint32_t d[8];
#pragma unroll
    for (int r = 0; r < 8; ++r) d[r] = __builtin_amdgcn_bitop3_b32(x[r], reg, s.dm[r], 0x78);   // x ^ (reg & dm)
    uint32_t v[32];
#pragma unroll
    for (int i = 0; i < 32; ++i) v[i] = lds_load(__builtin_amdgcn_perm(d[i >> 2], s.a.col[i >> 2], s.a.sel[i & 3]));
    uint32_t acc = xor3(v[0], v[1], v[2]);
#pragma unroll
    for (int i = 3; i + 1 < 32; i += 2) acc = xor3(acc, v[i], v[i + 1]);
    return acc ^ v[31];
}

constexpr uint32_t floor_pow2(uint32_t v) { return v < 2u ? v : 2u * floor_pow2(v / 2u); }

template <int MODE, int LG, int W, int NB>
struct LeanGeom {
    static constexpr uint32_t P = 1u << LG, kPk = 64u >> LG;           // lanes / packets per group
    static constexpr uint32_t kF = MODE ? 8u : 4u;                      // metadata dwords per packet (padded)
    static constexpr uint32_t kGroupMeta = kF * kPk;                    // metadata dwords per group
    static constexpr uint32_t kRing = NB * 2048u;                       // NB stages of 64 lanes x 32 B
    static constexpr uint32_t kWaveLds = (160u * 1024u - kLdsTableBytes) / W / 256u * 256u;
    static constexpr uint32_t kHalf = (kWaveLds - kRing) / 2u / 256u * 256u;
    static constexpr uint32_t JM = floor_pow2(kHalf / (4u * kGroupMeta));   // groups per metadata chunk
    static constexpr uint32_t kMetaOps = JM * kGroupMeta / 64u;
    static constexpr int kThreads = 64 * W;
    static constexpr int kLds = kLdsTableBytes + W * static_cast<int>(kRing + 2u * kHalf);
    static_assert(JM >= 2 && (JM & (JM - 1)) == 0 && (JM * kGroupMeta) % 64u == 0, "metadata chunk");
    static_assert(JM + 2 > NB, "the prologue stages (pj <= NB-2) stay in chunk 0: chunk 1 is issued after barrier B");
    static_assert(W >= kBasisRows && kHalf >= 256u, "waves 0..8 each stage one basis row in their half 1");
    static_assert(kLds <= 160 * 1024, "LDS budget");
};

template <int N>
__device__ __forceinline__ void wait_vm_n() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// vmcnt(Base + c * K) for a wave-uniform c in [0, NB-1]
template <int Base, int K, int C>
__device__ __forceinline__ void wait_vm_sel(uint32_t c) {
    if constexpr (C == 0) {
        wait_vm_n<Base>();
    } else {
        if (c == static_cast<uint32_t>(C)) wait_vm_n<(Base + C * K > 63 ? 63 : Base + C * K)>();
        else wait_vm_sel<Base, K, C - 1>(c);
    }
}

// ABL (diagnostics, wrong checksums by design): 1 = no table lookups (the fold is
// an XOR of the data), 2 = packet DMA from an L2-resident 2 KiB slice of the table
// images per wave (no HBM traffic), 4 = no table image load (with 1 only),
// 16 = synthetic metadata (1200-byte packets packed from offset 0, nothing read);
// 32 (tuning, correct checksums) = each wave takes a contiguous range of groups;
// 64 (tuning, correct checksums) = s_setprio 1 for the later-dispatched half of the waves;
// 256 (tuning, correct checksums) = nt cache policy on the packet-data DMAs;
// 128 (product, correct checksums) = metadata from the length-ordered records of the
// *_binned entry points (PacketArgs::meta4): a separate instance, so the plain path
// carries no per-op test for it.

// a wave-uniform 64-bit value as such (both halves through readfirstlane)
__device__ __forceinline__ uint64_t uni64(uint64_t v) {
    const uint32_t lo = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(v));
    const uint32_t hi = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(v >> 32));
    return static_cast<uint64_t>(lo) | (static_cast<uint64_t>(hi) << 32);
}                     // (the one-batch instances never read it)

// LIST = 1 (no ablation): the batches of a LeanList (checksum, MODE 0) or a
// LeanVList (receive verify, MODE 1: also each batch's slot offsets, connectIDs and
// ok[]), their groups concatenated (batch b's groups are global groups g0_b ..) and
// dealt over the waves as one batch's are; pa is unused.  A wave's groups ascend, so each of its
// three walkers (metadata, producer, consumer) finds a group's batch with a cursor
// that only moves forward.
// The list lives in the kernel-argument segment and is read there (llp, scalar
// loads): a reference to the by-value argument made hipcc copy all 2.3 KiB of it
// into scratch.
using LeanListPtr = const __attribute__((address_space(4))) LeanList*;
// receive-verify lists (MODE 1): LeanVList, the same walkers
using LeanVListPtr = const __attribute__((address_space(4))) LeanVList*;

template <int MODE, int LG, int W, int NB, int ABL, int LIST, typename LLP = LeanListPtr>
__device__ __forceinline__ void lean_body(const PacketArgs& pa, const KernelTables& tb, LLP llp) {
    using G = LeanGeom<MODE, LG, W, NB>;
    constexpr uint32_t P = G::P, kPk = G::kPk, JM = G::JM;
    static_assert(!LIST || ABL == 0, "batch lists: product instances");
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t ngroups = LIST ? llp->groups : (pa.n + kPk - 1u) >> (6 - LG);
    // the batch of global group gg, from cursor b on (LIST)
    auto locate = [&](uint64_t gg, uint32_t& b) __attribute__((always_inline)) {
        while (b + 1u < llp->count && gg >= llp->b[b + 1u].g0) ++b;
    };
    uint32_t mb = 0, pb = 0, cb = 0;                         // metadata / producer / consumer cursors (LIST)
    const uint64_t wv = static_cast<uint64_t>(blockIdx.x) * W + wave;
    const uint64_t wt = static_cast<uint64_t>(gridDim.x) * W;
    // groups of this wave: wv, wv + wt, ... (default) or, with ABL & 32, a contiguous range
    constexpr bool kContig = (ABL & 32) != 0;
    constexpr bool kBin = (ABL & 128) != 0;
    const uint64_t g0 = kContig ? wv * ngroups / wt : wv;
    const uint32_t J = kContig ? static_cast<uint32_t>((wv + 1u) * ngroups / wt - g0)
                               : (wv < ngroups ? static_cast<uint32_t>((ngroups - 1u - wv) / wt) + 1u : 0u);
    auto group_of = [&](uint32_t j) __attribute__((always_inline)) -> uint64_t {
        return kContig ? g0 + j : wv + static_cast<uint64_t>(j) * wt;
    };
    const uint32_t ring = kLdsTableBytes + wave * (G::kRing + 2u * G::kHalf);
    const uint32_t meta0 = ring + G::kRing;
    const uint64_t zero = reinterpret_cast<uint64_t>(tb.zero);
    const uint32_t k = lane & (P - 1u), pj_lane = lane >> LG;
    // diagnostics (enet_hip_diag_trace): per-wave timestamps, 8 x u64 per wave
    uint64_t tmark[5] = {0, 0, 0, 0, 0};
    auto mark = [&](int i) __attribute__((always_inline)) {
        if (pa.trace) tmark[i] = __builtin_amdgcn_s_memrealtime();
    };
    mark(0);
    if constexpr ((ABL & 64) != 0) {
        if (wave >= W / 2) __builtin_amdgcn_s_setprio(1);   // tuning: the later-dispatched half first
    }
    auto trace_end = [&]() __attribute__((always_inline)) {
        if (pa.trace && lane == 0u) {
            uint64_t* tr = pa.trace + 8u * wv;
            tr[5] = __builtin_amdgcn_s_memrealtime();
#pragma unroll
            for (int i = 0; i < 5; ++i) tr[i] = tmark[i];
            const uint32_t hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);      // HW_ID
            const uint32_t xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20);    // XCC_ID
            tr[6] = hw | (static_cast<uint64_t>(xcc) << 32);
            tr[7] = J;
        }
    };

    // ---- metadata chunks: chunk c = this wave's groups [c JM, (c+1) JM) in half c & 1
    auto issue_meta = [&](uint32_t c) __attribute__((always_inline)) {
        const uint32_t half = meta0 + (c & 1u) * G::kHalf;
#pragma unroll
        for (uint32_t o = 0; o < G::kMetaOps; ++o) {
            const uint32_t x = 64u * o + lane;
            const uint32_t q = x / G::kGroupMeta, f = (x / kPk) % G::kF, p = x % kPk;
            const uint32_t j = min(c * JM + q, J - 1u);
            if constexpr (LIST) {
                // an op covers the groups of its first and last lane (1 or 2 groups): their
                // batches from the metadata cursor, then each lane takes its own
                const uint32_t qa = 64u * o / G::kGroupMeta, qb = (64u * o + 63u) / G::kGroupMeta;
                const uint64_t ga = group_of(min(c * JM + qa, J - 1u)), gb = group_of(min(c * JM + qb, J - 1u));
                locate(ga, mb);
                const uint32_t ba = mb;
                locate(gb, mb);
                // (each field read as a wave-uniform value first: a select of two kernel-argument
                // addresses would be a divergent index into the argument block, i.e. a scratch copy)
                const bool ia = q == qa;
                const uint64_t g0 = ia ? uni64(llp->b[ba].g0) : uni64(llp->b[mb].g0);
                const uint64_t n = ia ? uni64(llp->b[ba].n) : uni64(llp->b[mb].n);
                const uint64_t pk = min((group_of(j) - g0) * kPk + p, n - 1u);
                const uint32_t* lp = reinterpret_cast<const uint32_t*>(
                    ia ? uni64(reinterpret_cast<uint64_t>(llp->b[ba].len)) : uni64(reinterpret_cast<uint64_t>(llp->b[mb].len)));
                const uint32_t* op = reinterpret_cast<const uint32_t*>(
                    ia ? uni64(reinterpret_cast<uint64_t>(llp->b[ba].off)) : uni64(reinterpret_cast<uint64_t>(llp->b[mb].off)));
                const uint32_t* src = (f == 1u || f == 2u) ? op + 2u * pk + (f - 1u) : lp + pk;
                if constexpr (MODE) {                        // receive verify: slot offset, connectID
                    const uint32_t* sp = reinterpret_cast<const uint32_t*>(
                        ia ? uni64(reinterpret_cast<uint64_t>(llp->b[ba].slot_off))
                           : uni64(reinterpret_cast<uint64_t>(llp->b[mb].slot_off)));
                    const uint32_t* cp = reinterpret_cast<const uint32_t*>(
                        ia ? uni64(reinterpret_cast<uint64_t>(llp->b[ba].connect))
                           : uni64(reinterpret_cast<uint64_t>(llp->b[mb].connect)));
                    if (f == 3u) src = sp + pk;
                    if (f == 4u) src = cp + pk;
                }
                dma4(src, half + 256u * o);
                continue;
            }
            const uint64_t pk = min(group_of(j) * kPk + p, pa.n - 1u);
            const uint32_t* src = pa.len + pk;
            if (f == 1u || f == 2u) src = reinterpret_cast<const uint32_t*>(pa.off) + 2u * pk + (f - 1u);
            if (MODE && f == 3u) src = pa.slot_off + pk;
            if (MODE && f == 4u) src = pa.connect + pk;
            if constexpr (kBin) src = pa.meta4 + G::kF * pk + f;    // binned: the record in field order
            dma4(src, half + 256u * o);
        }
    };
    auto meta_at = [&](uint32_t j, uint32_t f) __attribute__((always_inline)) -> uint32_t {
        return lds_load(meta0 + ((j / JM) & 1u) * G::kHalf + 4u * (((j % JM) * G::kF + f) * kPk + pj_lane));
    };
    // (LIST: b = the group's batch)
    auto window_of = [&](uint32_t j, uint32_t b) __attribute__((always_inline)) -> Window {
        Window w;
        const uint64_t pkw = (group_of(j) - (LIST ? llp->b[b].g0 : 0u)) * kPk + pj_lane;
        w.active = pkw < (LIST ? llp->b[b].n : pa.n);
        w.L = w.active ? ((ABL & 16) ? 1200u : meta_at(j, 0)) : 0u;
        const uint64_t off = (ABL & 16) ? 1200u * pkw
                                        : static_cast<uint64_t>(meta_at(j, 1)) | (static_cast<uint64_t>(meta_at(j, 2)) << 32);
        const uint64_t a = reinterpret_cast<uint64_t>(LIST ? llp->b[b].bytes : pa.bytes) + off, e = a + w.L;
        w.tz = w.L ? static_cast<uint32_t>((0u - e) & 15u) : 0u;       // window ends at the granule after the end
        w.nb = w.L ? (w.L + w.tz + 31u) >> 5 : 0u;
        w.lz = 32u * w.nb - w.tz - w.L;
        w.ws = e + w.tz - 32ull * w.nb;
        w.r = (0u - w.nb) & (P - 1u);
        return w;
    };

    // ---- prologue: basis row `wave` of the table (waves < kBasisRows) into this
    // wave's metadata half 1 -- chunk 1 goes there only after barrier B below --
    // and metadata chunk 0
    auto basis_row = [&](uint32_t b) __attribute__((always_inline)) -> uint32_t {
        return kLdsTableBytes + b * (G::kRing + 2u * G::kHalf) + G::kRing + G::kHalf;
    };
    if (!(ABL & 4) && wave < static_cast<uint32_t>(kBasisRows))
        dma4(tb.basis + static_cast<size_t>(LG == 2 ? 1 : 2) * kBasisDwords + 64u * wave + lane, basis_row(wave));
    uint32_t issued = 0;                                     // metadata chunks issued so far
    const uint32_t nchunks = (J + JM - 1u) / JM;
    if (J && !(ABL & 16)) {
        issue_meta(0);
        issued = 1;
    }
    wait_vm_n<0>();                                          // basis row and metadata chunk 0 have landed
    mark(1);

    // ---- producer: this lane's block of its packet, one stage ahead per slot
    uint64_t pcur = 0;                                       // piece k of the packet's next chunk
    uint32_t pv0 = 0, pv1 = 0, pst = 0, pstages = 0, pj = 0; // stages holding pieces k / P + k
    bool phz = false, pdone = J == 0;
    uint32_t it = 0;                                         // loop iteration (stage) counter
    uint32_t meta_guard = 0;                                 // from this iteration on chunk `issued - 1` has landed
    uint32_t mbits = 0;                                      // bit u: iteration it-1-u issued a metadata chunk
    auto producer_setup = [&](uint32_t j) __attribute__((always_inline)) {
        if constexpr (LIST) locate(group_of(j), pb);
        const Window w = window_of(j, pb);
        const uint32_t w0 = (k - w.r) & (P - 1u);
        const uint32_t cnt = w0 < w.nb ? ((w.nb - 1u - w0) >> LG) + 1u : 0u;
        const uint32_t np = 2u * w.nb;                       // window pieces
        pv0 = np > k ? (np - k + 2u * P - 1u) >> (LG + 1) : 0u;
        pv1 = np > P + k ? (np - P - k + 2u * P - 1u) >> (LG + 1) : 0u;
        pcur = w.ws + 16u * k;
        phz = k == 0u && w.lz >= 16u;                        // piece 0 lies wholly in front
        pstages = max(1u, wave_max_u(cnt));
        pst = 0;
    };
    auto produce = [&](uint32_t slot) __attribute__((always_inline)) {
        if (!pdone && pst == pstages) {
            if (++pj < J) {
                if (!(ABL & 16) && pj % JM == 0u) {          // entering chunk pj / JM
                    const uint32_t c = pj / JM;
                    if (c >= issued) {                        // the consumer has not prefetched it yet
                        issue_meta(c);
                        issued = c + 1u;
                        wait_vm_n<0>();
                    } else if (c + 1u == issued && it < meta_guard) {
                        wait_vm_n<0>();                       // prefetched, landing not yet guaranteed
                    }
                }
                producer_setup(pj);
            } else {
                pdone = true;
            }
        }
        const bool v0 = !pdone && pst < pv0 && !(pst == 0u && phz);
        const bool v1 = !pdone && pst < pv1;
        uint64_t a0 = v0 ? pcur : zero, a1 = v1 ? pcur + 16u * P : zero;
        if (ABL & 2) {
            const uint64_t l2 = reinterpret_cast<uint64_t>(tb.image) + (wv % 128u) * 2048u + 16u * lane;
            a0 = l2;
            a1 = l2 + 1024u;
        }
        constexpr int kAux = (ABL & 256) ? 2 : 0;           // 256 (tuning): nt data loads
        dma16_pol<kAux>(reinterpret_cast<const void*>(a0), ring + 2048u * slot);
        dma16_pol<kAux>(reinterpret_cast<const void*>(a1), ring + 2048u * slot + 1024u);
        pcur += 32u * P;
        ++pst;
    };

    if (J) {
        producer_setup(0);
        unroll_slots<NB - 1>([&](auto sc) __attribute__((always_inline)) { produce(decltype(sc)::value); });
    }

    // ---- the table image, rebuilt in LDS while the first stages are in flight.
    // Wave w writes rows w, w + W, ...: row j = XOR of the basis rows b with bit b
    // of j set, except the INIT and CINV dwords (not linear in j), whose rows < 32
    // come from basis row 8.  Raw s_barrier: the stage DMAs stay in flight.
    __builtin_amdgcn_s_barrier();                            // (A) every basis row has landed
    if (!(ABL & 4)) {
        uint32_t bb[8];
#pragma unroll
        for (int b = 0; b < 8; ++b) bb[b] = lds_load(basis_row(b) + 4u * lane);
        const bool nonlin = lane == kInitDword || lane == kCinvDword;
        const uint32_t row8 = basis_row(8) + (lane == kInitDword ? 0u : 128u);
        if constexpr (W == 16) {
            // rows wave + 16 i with i in Gray-code order: one XOR per row (the VALU
            // cost of the generic loop below, ~1 us per CU, sat on the startup path)
            uint32_t v = 0;
#pragma unroll
            for (int b = 0; b < 4; ++b) v ^= ((wave >> b) & 1u) ? bb[b] : 0u;
#pragma unroll
            for (uint32_t q = 0; q < 16u; ++q) {
                const uint32_t i = q ^ (q >> 1);
                if (q) v ^= bb[4 + __builtin_ctz(q)];
                uint32_t x = v;
                if (i < 2u) {                                // rows < 32: INIT / CINV
                    const uint32_t e = lds_load(row8 + 4u * (wave + 16u * i));
                    x = nonlin ? e : x;
                }
                lds_store(256u * (wave + 16u * i) + 4u * lane, x);
            }
        } else {
            for (uint32_t j = wave; j < 256u; j += W) {
                uint32_t v = 0;
#pragma unroll
                for (int b = 0; b < 8; ++b) v ^= ((j >> b) & 1u) ? bb[b] : 0u;
                if (j < 32u) {
                    const uint32_t e = lds_load(row8 + 4u * j);
                    v = nonlin ? e : v;
                }
                lds_store(256u * j + 4u * lane, v);
            }
        }
    }
    mark(2);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();                            // (B) the image is complete, the basis rows read
    mark(3);
    if (!J) {                                                // no groups: this wave only helped build the table
        trace_end();
        return;
    }
    if (!(ABL & 16) && nchunks > 1u) {                       // chunk 1 into half 1, now free
        issue_meta(1);
        issued = 2;
        meta_guard = NB;                                     // issued before data(0): covered by wait(NB - 1)
        mbits = 1u;                                          // counted by the waits of iterations 0 .. NB-2
    }

    const LeanSched s = make_lean_sched<LG>(lane);
    uint32_t rb = 0;                                         // LDS address (ring slot 0) of the lane's block
    uint32_t ra[8];                                          // ... and of its permuted data registers

    // ---- consumer
    uint32_t cj = 0, cst = 0, cstages = 0, nedge = ~0u, reg = 0, desired = 0;
    Task t{};
    uint32_t* cout = pa.out;                                 // (LIST: the consumer's batch's)
    uint8_t* cok = pa.ok;                                    // (MODE 1)
    auto consumer_setup = [&](uint32_t j) __attribute__((always_inline)) {
        if constexpr (LIST) {
            locate(group_of(j), cb);
            cout = llp->b[cb].out;
            if constexpr (MODE) cok = llp->b[cb].ok;
        }
        const Window w = window_of(j, cb);
        t.pk = (group_of(j) - (LIST ? llp->b[cb].g0 : 0u)) * kPk + pj_lane;
        if constexpr (kBin) if (w.active) t.pk = meta_at(j, MODE ? 5u : 3u);   // binned: the packet's caller index
        t.active = w.active;
        t.k = k;
        t.w0 = (k - w.r) & (P - 1u);
        t.nb = w.nb;
        t.lz = w.lz;
        t.tz = w.tz;
        t.cnt = t.w0 < w.nb ? ((w.nb - 1u - t.w0) >> LG) + 1u : 0u;
        const uint32_t init = lds_load(init_addr(w.lz));
        t.reg = k == w.r ? init : 0u;
        t.e0 = ((w.lz & 15u) && t.w0 == 0u && w.nb) ? 0u : ~0u;
        t.e1 = (w.tz && t.cnt && t.w0 + P * (t.cnt - 1u) == w.nb - 1u) ? t.cnt - 1u : ~0u;
        t.e2 = t.e3 = ~0u;
        t.ps = -4096;
        t.connect = 0;
        t.slot_ok = false;
        if (MODE) {
            const uint32_t so = meta_at(j, 3);
            t.connect = meta_at(j, 4);
            t.slot_ok = w.L >= 4u && so <= w.L - 4u;
            if (t.slot_ok) {
                t.ps = static_cast<int32_t>(w.lz + so);
                const uint32_t ws_ = static_cast<uint32_t>(t.ps) >> 5, we_ = static_cast<uint32_t>(t.ps + 3) >> 5;
                if (((ws_ + w.r) & (P - 1u)) == k) t.e2 = ws_ >> LG;
                if (we_ != ws_ && ((we_ + w.r) & (P - 1u)) == k) t.e3 = we_ >> LG;
            }
        }
        rb = ring + 1024u * ((2u * t.w0) >> LG) + 16u * (pj_lane * P + ((2u * t.w0) & (P - 1u)));
#pragma unroll
        for (int r = 0; r < 8; ++r) ra[r] = rb + s.dq[r];
        cstages = max(1u, wave_max_u(t.cnt));
        nedge = next_edge_stage_l<0>(t, 0);
        reg = t.reg;
        desired = 0;
        cst = 0;
    };

    consumer_setup(0);                                       // reads INIT[] from the finished image
    mark(4);
    bool done = false;
    auto iteration = [&](auto sc) __attribute__((always_inline)) {
        constexpr uint32_t S = decltype(sc)::value;          // ring slot consumed by this iteration
        if (done) return;
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // WAR: the slot refilled below was read last iteration
        produce((S + NB - 1) % NB);
        wait_vm_sel<2 * (NB - 1), static_cast<int>(G::kMetaOps), NB - 1>(
            __builtin_popcount(mbits & ((1u << (NB - 1)) - 1u)));   // stage S has landed
        mbits <<= 1;
        if (pa.prio) {
            // tail fairness: a wave with more stages left than its CU neighbours is
            // issued first (s_setprio: 0..3), so lagging waves catch up
            const uint32_t rem = (J - 1u - cj) * cstages + (cstages - cst);
            if (rem >= 8u) __builtin_amdgcn_s_setprio(3);
            else if (rem >= 5u) __builtin_amdgcn_s_setprio(2);
            else if (rem >= 3u) __builtin_amdgcn_s_setprio(1);
            else __builtin_amdgcn_s_setprio(0);
        }
        uint32_t nr;
        if (cst == nedge) {                                  // head/tail/slot fix-ups: original dword order
            u32x4 A = lds_load16(rb + 2048u * S), B = lds_load16(rb + 2048u * S + 16u);
            const bool fix = cst < t.cnt && (cst == t.e0 || cst == t.e1 || (MODE && (cst == t.e2 || cst == t.e3)));
            if (fix) edge_fix<MODE>(A, B, 0u, t, t.w0 + P * cst, desired);
            nr = fold_block(reg, A, B, s.a);
            nedge = next_edge_stage_l<0>(t, cst + 1u);
        } else {
            uint32_t x[8];
#pragma unroll
            for (int r = 0; r < 8; ++r) x[r] = lds_load(ra[r] + 2048u * S);
            nr = (ABL & 1) ? xor3(reg ^ x[0] ^ x[1], x[2] ^ x[3] ^ x[4], x[5] ^ x[6] ^ x[7]) : fold_perm(reg, x, s);
        }
        reg = cst < t.cnt ? nr : reg;
        if (++cst == cstages) {
            reg = finish_packet(LG, t.k, t.tz, lane, reg);
            if (MODE) desired = xor_lanes<0>(LG, desired);
            if (t.active && t.k == 0u) {
                if (MODE == 0) {
                    cout[t.pk] = finalize(reg);              // packet.cs:159
                } else {
                    const uint32_t comp = t.slot_ok ? finalize(reg) : 0u;
                    cok[t.pk] = (t.slot_ok && comp == desired) ? 1 : 0;     // protocol.cs:1066-1068
                    if (cout) cout[t.pk] = comp;
                }
            }
            if (++cj == J) {
                done = true;
                return;
            }
            if (!(ABL & 16) && cj % JM == 0u) {             // the consumer left chunk cj/JM - 1: prefetch the next
                const uint32_t c = cj / JM + 1u;
                if (c < nchunks && c >= issued) {
                    issue_meta(c);
                    issued = c + 1u;
                    meta_guard = it + NB + 1u;               // issued after data(it): landed by wait(it + NB)
                    mbits |= 1u;
                }
            }
            consumer_setup(cj);
        }
        ++it;
    };
    while (!done) unroll_slots<NB>(iteration);
    wait_vm_n<0>();                                          // no LDS-DMA may outlive the wave
    trace_end();
}

template <int MODE, int LG, int W, int NB, int ABL = 0>
__global__ void __launch_bounds__(64 * W) crc32_lean_kernel(PacketArgs pa, KernelTables tb) {
    lean_body<MODE, LG, W, NB, ABL, 0>(pa, tb, static_cast<LeanListPtr>(nullptr));
}

// batch lists (enet_hip_crc32_batch_list_device): checksum mode
template <int LG, int W, int NB>
__global__ void __launch_bounds__(64 * W) crc32_lean_list_kernel(LeanList ll, KernelTables tb) {
    PacketArgs pa{};
    (void)ll;
    // the first kernel argument sits at the start of the segment
    lean_body<0, LG, W, NB, 0, 1>(pa, tb, (LeanListPtr)(__builtin_amdgcn_kernarg_segment_ptr()));
}

// receive-verify lists (enet_hip_verify_batch_list_device): MODE 1
template <int LG, int W, int NB>
__global__ void __launch_bounds__(64 * W) crc32_lean_vlist_kernel(LeanVList ll, KernelTables tb) {
    PacketArgs pa{};
    (void)ll;
    lean_body<1, LG, W, NB, 0, 1, LeanVListPtr>(pa, tb, (LeanVListPtr)(__builtin_amdgcn_kernarg_segment_ptr()));
}

// ---------------------------------------------------------------- host side

template <int W, int NB>
struct LeanVariant {
    template <int MODE, int LG, int ABL = 0>
    static const void* fn() {
        return reinterpret_cast<const void*>(crc32_lean_kernel<MODE, LG, W, NB, ABL>);
    }
    static int setup() {
        const void* fns[12] = {fn<0, 2>(), fn<0, 3>(), fn<1, 2>(), fn<1, 3>(),
                               fn<0, 2, 128>(), fn<0, 3, 128>(), fn<1, 2, 128>(), fn<1, 3, 128>(),
                               reinterpret_cast<const void*>(crc32_lean_list_kernel<2, W, NB>),
                               reinterpret_cast<const void*>(crc32_lean_list_kernel<3, W, NB>),
                               reinterpret_cast<const void*>(crc32_lean_vlist_kernel<2, W, NB>),
                               reinterpret_cast<const void*>(crc32_lean_vlist_kernel<3, W, NB>)};
        const int lds[12] = {LeanGeom<0, 2, W, NB>::kLds, LeanGeom<0, 3, W, NB>::kLds, LeanGeom<1, 2, W, NB>::kLds,
                             LeanGeom<1, 3, W, NB>::kLds, LeanGeom<0, 2, W, NB>::kLds, LeanGeom<0, 3, W, NB>::kLds,
                             LeanGeom<1, 2, W, NB>::kLds, LeanGeom<1, 3, W, NB>::kLds, LeanGeom<0, 2, W, NB>::kLds,
                             LeanGeom<0, 3, W, NB>::kLds, LeanGeom<1, 2, W, NB>::kLds, LeanGeom<1, 3, W, NB>::kLds};
        for (int i = 0; i < 12; ++i) {
            const hipError_t e = hipFuncSetAttribute(fns[i], hipFuncAttributeMaxDynamicSharedMemorySize, lds[i]);
            if (e != hipSuccess) return -static_cast<int>(e);
        }
        return 0;
    }
    template <int MODE, int LG>
    static void go(int num_cus, hipStream_t st, const PacketArgs& pa, const KernelTables& tb) {
        using G = LeanGeom<MODE, LG, W, NB>;
        const uint64_t groups = (pa.n + G::kPk - 1u) / G::kPk;
        const unsigned grid = static_cast<unsigned>(
            std::max<uint64_t>(1, std::min<uint64_t>((groups + W - 1) / W, static_cast<uint64_t>(num_cus))));
        if (pa.meta4)
            hipLaunchKernelGGL((crc32_lean_kernel<MODE, LG, W, NB, 128>), dim3(grid), dim3(G::kThreads), G::kLds, st,
                               pa, tb);
        else
            hipLaunchKernelGGL((crc32_lean_kernel<MODE, LG, W, NB>), dim3(grid), dim3(G::kThreads), G::kLds, st, pa,
                               tb);
    }
    template <int LG, int ABL>
    static void go_abl(int num_cus, hipStream_t st, const PacketArgs& pa, const KernelTables& tb) {
        using G = LeanGeom<0, LG, W, NB>;
        static bool set = false;
        if (!set) {
            (void)hipFuncSetAttribute(reinterpret_cast<const void*>(crc32_lean_kernel<0, LG, W, NB, ABL>),
                                      hipFuncAttributeMaxDynamicSharedMemorySize, G::kLds);
            set = true;
        }
        const uint64_t groups = (pa.n + G::kPk - 1u) / G::kPk;
        const unsigned grid = static_cast<unsigned>(
            std::max<uint64_t>(1, std::min<uint64_t>((groups + W - 1) / W, static_cast<uint64_t>(num_cus))));
        hipLaunchKernelGGL((crc32_lean_kernel<0, LG, W, NB, ABL>), dim3(grid), dim3(G::kThreads), G::kLds, st, pa,
                           tb);
    }
    static void launch(int mode, int lg, int abl, int num_cus, hipStream_t st, const PacketArgs& pa,
                       const KernelTables& tb) {
#ifdef ENET_HIP_DIAG
        if (mode == 0 && abl) {
            switch (abl) {                                   // diagnostics: 8-lane packets only
                case 1: go_abl<3, 1>(num_cus, st, pa, tb); break;
                case 2: go_abl<3, 2>(num_cus, st, pa, tb); break;
                case 3: go_abl<3, 3>(num_cus, st, pa, tb); break;
                case 5: go_abl<3, 5>(num_cus, st, pa, tb); break;
                case 17: go_abl<3, 17>(num_cus, st, pa, tb); break;
                case 21: go_abl<3, 21>(num_cus, st, pa, tb); break;
                case 16: go_abl<3, 16>(num_cus, st, pa, tb); break;
                case 32: go_abl<3, 32>(num_cus, st, pa, tb); break;
                case 64: go_abl<3, 64>(num_cus, st, pa, tb); break;
                case 256: go_abl<3, 256>(num_cus, st, pa, tb); break;
                default: break;
            }
            return;
        }
#endif
        (void)abl;
        if (mode == 0) {
            if (lg == 2) go<0, 2>(num_cus, st, pa, tb);
            else go<0, 3>(num_cus, st, pa, tb);
        } else {
            if (lg == 2) go<1, 2>(num_cus, st, pa, tb);
            else go<1, 3>(num_cus, st, pa, tb);
        }
    }
};

// A batch list in one launch: the batches' groups concatenated (empty batches
// dropped) and dealt over one 16-wave workgroup per CU (geometry 0).
int lean_launch_list(int lg, int num_cus, hipStream_t st, const ENetHipBatch* batches, size_t count,
                     const KernelTables& tb) {
    if ((lg != 2 && lg != 3) || count > static_cast<size_t>(kLeanMaxBatches)) return -static_cast<int>(hipErrorInvalidValue);
    LeanList ll{};
    const uint64_t kpk = 64u >> lg;
    for (size_t i = 0; i < count; ++i) {
        if (!batches[i].count) continue;
        LeanListBatch& b = ll.b[ll.count++];
        b = LeanListBatch{batches[i].bytes, batches[i].offsets, batches[i].lengths, batches[i].out,
                          static_cast<uint64_t>(batches[i].count), ll.groups};
        ll.groups += (b.n + kpk - 1u) / kpk;
    }
    if (ll.count == 0) return 0;
    const unsigned grid = static_cast<unsigned>(
        std::max<uint64_t>(1, std::min<uint64_t>((ll.groups + 15u) / 16u, static_cast<uint64_t>(num_cus))));
    constexpr int lds2 = LeanGeom<0, 2, 16, 2>::kLds, lds3 = LeanGeom<0, 3, 16, 2>::kLds;
    if (lg == 2)
        hipLaunchKernelGGL((crc32_lean_list_kernel<2, 16, 2>), dim3(grid), dim3(64 * 16), lds2, st, ll, tb);
    else
        hipLaunchKernelGGL((crc32_lean_list_kernel<3, 16, 2>), dim3(grid), dim3(64 * 16), lds3, st, ll, tb);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : -static_cast<int>(e);
}

// A receive-verify list: the same deal as lean_launch_list (MODE 1 metadata, 8
// dwords per packet), one 16-wave workgroup per CU.
int lean_launch_vlist(int lg, int num_cus, hipStream_t st, const ENetHipVerifyBatch* batches, size_t count,
                      const KernelTables& tb) {
    if ((lg != 2 && lg != 3) || count > static_cast<size_t>(kLeanMaxVBatches))
        return -static_cast<int>(hipErrorInvalidValue);
    LeanVList ll{};
    const uint64_t kpk = 64u >> lg;
    for (size_t i = 0; i < count; ++i) {
        if (!batches[i].count) continue;
        LeanVListBatch& b = ll.b[ll.count++];
        b = LeanVListBatch{batches[i].bytes, batches[i].offsets, batches[i].lengths, batches[i].slotOffsets,
                           batches[i].connectIds, batches[i].ok, batches[i].computed,
                           static_cast<uint64_t>(batches[i].count), ll.groups};
        ll.groups += (b.n + kpk - 1u) / kpk;
    }
    if (ll.count == 0) return 0;
    const unsigned grid = static_cast<unsigned>(
        std::max<uint64_t>(1, std::min<uint64_t>((ll.groups + 15u) / 16u, static_cast<uint64_t>(num_cus))));
    constexpr int lds2 = LeanGeom<1, 2, 16, 2>::kLds, lds3 = LeanGeom<1, 3, 16, 2>::kLds;
    if (lg == 2)
        hipLaunchKernelGGL((crc32_lean_vlist_kernel<2, 16, 2>), dim3(grid), dim3(64 * 16), lds2, st, ll, tb);
    else
        hipLaunchKernelGGL((crc32_lean_vlist_kernel<3, 16, 2>), dim3(grid), dim3(64 * 16), lds3, st, ll, tb);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : -static_cast<int>(e);
}

int lean_setup() {
    int rc = LeanVariant<16, 2>::setup();
#ifdef ENET_HIP_DIAG
    if (!rc) rc = LeanVariant<12, 3>::setup();
#endif
    return rc;
}

int lean_launch(int mode, int lg, int geom, int abl, int num_cus, hipStream_t st, const PacketArgs& pa,
                const KernelTables& tb) {
    if (lg != 2 && lg != 3) return -static_cast<int>(hipErrorInvalidValue);
#ifdef ENET_HIP_DIAG
    // geoms 2, 3 (tuning sweeps): checksum mode, 8 lanes per packet only
    if (geom == 2 && mode == 0 && lg == 3) LeanVariant<14, 3>::go_abl<3, 0>(num_cus, st, pa, tb);
    else if (geom == 3 && mode == 0 && lg == 3) LeanVariant<10, 4>::go_abl<3, 0>(num_cus, st, pa, tb);
    else if (geom == 1) LeanVariant<12, 3>::launch(mode, lg, 0, num_cus, st, pa, tb);
    else
#endif
        LeanVariant<16, 2>::launch(mode, lg, abl, num_cus, st, pa, tb);
    (void)geom;
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : -static_cast<int>(e);
}

// ---------------------------------------------------------------- length bins
// Mixed-length batches (cfg3): a group's stage count is the longest of its
// packets, so a group of short and long packets idles most of its lanes.
// enet_hip_crc32_batch_device_binned first orders the packet records of each
// tile of 1024 packets by length bin (32-byte bins, longest first): one launch,
// one workgroup per tile, a counting sort in LDS, no global atomics and nothing
// carried between calls.  Sorted group q of full tile t (kpk records) is written
// as global group q * T + t (T = full tiles): the groups of rank q from every
// tile sit side by side, so the lean kernel's rounds (consecutive groups across
// all waves) see about one length each and run longest first, close to a
// global sort at the cost of a local one.  A ragged last tile stays in place.
// The lean kernel reads the ordered records (PacketArgs::meta4) and writes each
// CRC to its caller index.  The order inside a tile's bin is
// scheduling-dependent; the CRCs are not (each is its own packet's).

constexpr uint32_t kBins = 256, kBinThreads = 256, kBinItems = 4, kBinTile = kBinThreads * kBinItems;

// the bin of a record: its vring window length, lz + L (the window starts at the
// 64-byte boundary at or before the packet), in 32-byte bins, longest first.  Keyed
// by the window rather than L, a group's packets need about the same stage count
// whatever their alignment.
__device__ __forceinline__ uint32_t bin_of(uint32_t len, uint64_t off) {
    return kBins - 1u - min((len + (static_cast<uint32_t>(off) & 63u)) >> 5, kBins - 1u);
}

// VERIFY: 32-byte records {len, off_lo, off_hi, slot_off, connect, index, 0, 0}
// (the lean kernel's MODE 1 metadata fields), else 16-byte {len, off_lo, off_hi, index}.
// COMPACT (the binned gather): records of length <= small are left out (the join
// folds those segments itself); each tile, the ragged last one included, writes
// its kept records sorted and then empty records {0, 0, 0, pad_index} up to 1024,
// all rank-interleaved (group q T + t, T = every tile), and count[t] = its kept
// records.  No global atomics: the vring's records instance reads the counts.
// IDENT (diagnostics): every record left at its own position (memory order), to price
// the binned order against the records machinery.
template <bool VERIFY, bool COMPACT = false, bool IDENT = false>
__device__ __forceinline__ void bin_tile_body(uint32_t blk, uint32_t ntiles, const uint32_t* len, const uint64_t* off,
                                              uint64_t n, uint32_t kpk, const uint32_t* slot_off,
                                              const uint32_t* connect, uint4* rec, uint32_t small, uint32_t* count) {
    __shared__ uint32_t h[kBins], wsum[kBinThreads / 64];
    const uint32_t tid = threadIdx.x;
    h[tid] = 0;
    __syncthreads();
    const uint64_t base = static_cast<uint64_t>(blk) * kBinTile;
    uint32_t L[kBinItems], slot[kBinItems];
    uint64_t o[kBinItems];
#pragma unroll
    for (uint32_t r = 0; r < kBinItems; ++r) {
        const uint64_t i = base + r * kBinThreads + tid;
        L[r] = i < n ? len[i] : 0u;
        o[r] = i < n ? off[i] : 0u;
    }
    auto kept = [&](uint32_t r) { return base + r * kBinThreads + tid < n && (!COMPACT || L[r] > small); };
#pragma unroll
    for (uint32_t r = 0; r < kBinItems; ++r)
        slot[r] = kept(r) ? atomicAdd(&h[bin_of(L[r], o[r])], 1u) : 0u;
    __syncthreads();
    // exclusive scan over the bins (thread tid = bin tid): an inclusive scan inside
    // each wave (ds_bpermute shifts, no barrier), then the waves' totals -- two
    // barriers instead of the sixteen of a block-wide Hillis-Steele scan
    static_assert(kBins == kBinThreads, "one bin per thread");
    const uint32_t mine = h[tid], ln = tid & 63u;
    uint32_t incl = mine;
#pragma unroll
    for (uint32_t s = 1; s < 64u; s <<= 1) {
        const uint32_t u = static_cast<uint32_t>(__shfl_up(static_cast<int>(incl), s));
        incl += ln >= s ? u : 0u;
    }
    if (ln == 63u) wsum[tid >> 6] = incl;
    __syncthreads();
    uint32_t pre = 0, kept_n = 0;                            // (COMPACT: kept_n = the tile's kept records)
#pragma unroll
    for (uint32_t w = 0; w < kBinThreads / 64u; ++w) {
        pre += w < (tid >> 6) ? wsum[w] : 0u;
        kept_n += wsum[w];
    }
    h[tid] = pre + incl - mine;                              // first slot of bin tid in the tile
    __syncthreads();
    const uint64_t full = COMPACT ? ntiles : n / kBinTile;    // T
    const bool interleave = COMPACT || blk < full;
    if constexpr (COMPACT) {
        if (tid == 0) count[blk] = kept_n;
        for (uint32_t srt = kept_n + tid; srt < kBinTile; srt += kBinThreads)        // the padding
            rec[((srt / kpk) * full + blk) * kpk + srt % kpk] = make_uint4(0u, 0u, 0u, static_cast<uint32_t>(n));
    }
#pragma unroll
    for (uint32_t r = 0; r < kBinItems; ++r) {
        const uint64_t i = base + r * kBinThreads + tid;
        const uint32_t srt = IDENT ? r * kBinThreads + tid : h[bin_of(L[r], o[r])] + slot[r];   // rank inside the tile
        const uint64_t dst = (interleave && !IDENT) ? ((srt / kpk) * full + blk) * kpk + srt % kpk : base + srt;
        if (kept(r)) {
            if constexpr (VERIFY) {
                rec[2 * dst] = make_uint4(L[r], static_cast<uint32_t>(o[r]), static_cast<uint32_t>(o[r] >> 32), slot_off[i]);
                rec[2 * dst + 1] = make_uint4(connect[i], static_cast<uint32_t>(i), 0u, 0u);
            } else {
                rec[dst] = make_uint4(L[r], static_cast<uint32_t>(o[r]), static_cast<uint32_t>(o[r] >> 32),
                                      static_cast<uint32_t>(i));
            }
        }
    }
}

template <bool VERIFY, bool COMPACT = false, bool IDENT = false>
__global__ void __launch_bounds__(kBinThreads) bin_tile_kernel(const uint32_t* len, const uint64_t* off, uint64_t n,
                                                               uint32_t kpk, const uint32_t* slot_off,
                                                               const uint32_t* connect, uint4* rec, uint32_t small,
                                                               uint32_t* count) {
    bin_tile_body<VERIFY, COMPACT, IDENT>(blockIdx.x, gridDim.x, len, off, n, kpk, slot_off, connect, rec, small, count);
}

#ifdef ENET_HIP_DIAG
// The binned gather's first launch: blocks [0, tiles) are the compact length-binning
// tiles of the segments, blocks [tiles, tiles + pj) the split join's pre-join
// (gather_join.hpp, one thread per DGRAM: short segments folded, out[d] = finalize(A),
// info[q] for the long ones).  78 VGPRs (6 waves per SIMD): cfg5's 588 + 784 blocks are
// resident at once.  The two need nothing from each other, so one launch
// overlaps the pre-join's dependent loads (segFirst, then lengths and offsets, then
// bytes) with the binning instead of running them after the records pass.
__global__ void __launch_bounds__(kBinThreads) __attribute__((amdgpu_waves_per_eu(6))) gather_bin_prejoin_kernel(GatherArgs ga, uint2* info, KernelTables tb,
                                                                         uint32_t small, uint32_t pj, uint32_t kpk,
                                                                         uint4* rec, uint32_t* count) {
    const uint32_t tiles = gridDim.x - pj;
    if (blockIdx.x < tiles) {
        bin_tile_body<false, true>(blockIdx.x, tiles, ga.seg_len, ga.seg_off, ga.segs, kpk, nullptr, nullptr, rec,
                                   small, count);
        return;
    }
    __shared__ uint32_t t4[4][256];
    fill_t4<kBinThreads>(t4, tb.image);
    for (uint64_t d = static_cast<uint64_t>(blockIdx.x - tiles) * kBinThreads + threadIdx.x; d < ga.n;
         d += static_cast<uint64_t>(pj) * kBinThreads)
        gather_prejoin_dgram(ga, info, tb, small, d, t4);
}
#endif  // ENET_HIP_DIAG

size_t length_bin_workspace(uint64_t n, bool verify) { return (verify ? 32u : 16u) * n; }

int length_bin(const uint32_t* len, const uint64_t* off, const uint32_t* slot_off, const uint32_t* connect, uint64_t n,
               uint32_t kpk, void* workspace, hipStream_t st, bool identity) {
    if (n == 0) return 0;
    if (n > 0xFFFFFFFFull || !workspace || kpk == 0 || kBinTile % kpk) return -static_cast<int>(hipErrorInvalidValue);
    const unsigned tiles = static_cast<unsigned>((n + kBinTile - 1) / kBinTile);
#ifdef ENET_HIP_DIAG
    if (identity && !(slot_off && connect))
        hipLaunchKernelGGL((bin_tile_kernel<false, false, true>), dim3(tiles), dim3(kBinThreads), 0, st, len, off, n, kpk,
                           nullptr, nullptr, static_cast<uint4*>(workspace), 0u, nullptr);
    else
#else
    (void)identity;
#endif
    if (slot_off && connect)
        hipLaunchKernelGGL(bin_tile_kernel<true>, dim3(tiles), dim3(kBinThreads), 0, st, len, off, n, kpk, slot_off,
                           connect, static_cast<uint4*>(workspace), 0u, nullptr);
    else
        hipLaunchKernelGGL(bin_tile_kernel<false>, dim3(tiles), dim3(kBinThreads), 0, st, len, off, n, kpk, nullptr,
                           nullptr, static_cast<uint4*>(workspace), 0u, nullptr);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : -static_cast<int>(e);
}

int length_bin_compact(const uint32_t* len, const uint64_t* off, uint64_t n, uint32_t kpk, uint32_t small,
                       void* records, uint32_t* counts, hipStream_t st) {
    if (n == 0) return 0;
    if (n > 0xFFFFFFFFull || !records || !counts || kpk == 0 || kBinTile % kpk)
        return -static_cast<int>(hipErrorInvalidValue);
    const unsigned tiles = static_cast<unsigned>((n + kBinTile - 1) / kBinTile);
    hipLaunchKernelGGL((bin_tile_kernel<false, true>), dim3(tiles), dim3(kBinThreads), 0, st, len, off, n, kpk, nullptr,
                       nullptr, static_cast<uint4*>(records), small, counts);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : -static_cast<int>(e);
}

#ifdef ENET_HIP_DIAG
int gather_bin_prejoin(const GatherArgs& ga, uint2* info, const KernelTables& tb, uint32_t small, uint32_t kpk,
                       void* records, uint32_t* counts, unsigned prejoin_blocks, hipStream_t st) {
    if (ga.segs > 0xFFFFFFFFull || (ga.segs && (!records || !counts)) || kpk == 0 || kBinTile % kpk ||
        prejoin_blocks == 0)
        return -static_cast<int>(hipErrorInvalidValue);
    const unsigned tiles = static_cast<unsigned>((ga.segs + kBinTile - 1) / kBinTile);
    hipLaunchKernelGGL(gather_bin_prejoin_kernel, dim3(prejoin_blocks + tiles), dim3(kBinThreads), 0, st, ga, info, tb,
                       small, prejoin_blocks, kpk, static_cast<uint4*>(records), counts);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : -static_cast<int>(e);
}
#endif  // ENET_HIP_DIAG

}  // namespace enethip
