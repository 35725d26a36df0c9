// crc32_vring.hip -- the VGPR-ring CRC32 kernel for gfx950 (MI355X): the default
// batched checksum path of libenethip.  Path replaced: ENet.enet_crc32
// (/root/reference/enet-csharp/ENet/c/packet.cs:142-160) over a whole batch of
// DGRAMs, one CRC per packet, in wire order (packet.cs:159).
//
// Arithmetic (tests/kernel_model.py): P = 2^LG lanes per packet
// fold its 32-byte window blocks strided -- lane k folds blocks k, k+P, k+2P, ...
// -- with the advancing slicing-by-32 tables T'_t = T_{t+32(P-1)} of the P image
// in LDS, so every fold also skips the P-1 blocks the other lanes own.
//   * Window: starts at the 64-byte boundary at or before the packet's first
//     byte (lz < 64 leading bytes) and spans nb = ceil((lz + L)/32) blocks, so
//     tz = 32 nb - lz - L < 32 trailing bytes.  Block 0's lane starts at INIT[lz]
//     (the register that lz zero bytes carry to 0xFFFFFFFF, packet.cs:144).
//   * Lane k ends o = (k - nb) mod P blocks past the window end: one multiply by
//     x^(-256 o) (four byte-indexed lookups in the image's correction columns),
//     a DPP XOR of the P lanes, then x^(-8 tz) (CINV[tz]) on the packet's lane 0.
//   * Data goes straight into VGPRs: stage s of a packet = its window bytes
//     [256 s, 256 s + 256) at P = 8, lane k loading its own block k + P s as two
//     16-byte loads, a two-slot register ring (one stage in flight while one is
//     folded).  A 16-byte piece wholly outside [lz, lz + L) is read from a zero
//     line instead; a partly covered piece (a packet start or end off a 16-byte
//     boundary) is masked on the fold side in a wave-uniform edge branch.
//   * LDS holds only the 64 KiB table image (rebuilt per workgroup from a 2.5 KiB
//     GF(2) basis while the first stage is in flight), so two 16-wave
//     workgroups share a CU (32 waves; VGPRs capped at 64 per lane).
// Measured design choices (tools/pipebench.hip, profiles/r02_*): 64-byte window
// starts beat the end-aligned 16-byte windows of the lean kernel (every DMA run
// then covers whole 64-byte sectors), and the register ring at 32 waves per CU
// beats the LDS-DMA ring at 16.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "crc32_vring.hpp"

namespace enethip {

constexpr int kVrW = 16;                                        // waves per workgroup
constexpr uint32_t kVrStaging = kLdsTableBytes;                 // basis rows land after the image
constexpr int kVrLds = kLdsTableBytes + kVrBasisRows * 256;

// Global loads as inline asm, waited for by explicit counted vmcnt: the
// compiler's own wait insertion loses count across the loop's group-switch
// branches and falls back to vmcnt(0) right after the next stage is issued,
// which empties the ring.  Every wait ties the registers it guards ("+v"), so
// no use of them can be scheduled above it.
__device__ __forceinline__ u32x4 vr_ld16(uint64_t addr) {
    u32x4 v;
    asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(v) : "v"(addr));
    return v;
}
// The metadata loads overwrite the previous load's register whether or not that
// value was used ("+v": the old value is an input, so its register is never
// handed to anything else while a load into it may be in flight).
__device__ __forceinline__ void vr_ld4(uint32_t& v, uint64_t addr) {
    asm volatile("global_load_dword %0, %1, off" : "+v"(v) : "v"(addr));
}
__device__ __forceinline__ void vr_ld8(uint64_t& v, uint64_t addr) {
    asm volatile("global_load_dwordx2 %0, %1, off" : "+v"(v) : "v"(addr));
}
__device__ __forceinline__ void vr_ld16_tied(u32x4& v, uint64_t addr) {
    asm volatile("global_load_dwordx4 %0, %1, off" : "+v"(v) : "v"(addr));
}
template <int N>
__device__ __forceinline__ void vr_wait(u32x4& a, u32x4& b) {
    asm volatile("s_waitcnt vmcnt(%2)" : "+v"(a), "+v"(b) : "n"(N));
}
// (BIN: the record register; else the length and offset registers)
template <int N, int BIN>
__device__ __forceinline__ void vr_wait_meta(uint32_t& L, uint64_t& off, u32x4& rec) {
    if constexpr (BIN) asm volatile("s_waitcnt vmcnt(%1)" : "+v"(rec) : "n"(N));
    else asm volatile("s_waitcnt vmcnt(%2)" : "+v"(L), "+v"(off) : "n"(N));
}
// vmcnt(0) tying every register a load may still land in
template <int BIN, int NB>
__device__ __forceinline__ void vr_drain(u32x4 (&a)[NB], u32x4 (&b)[NB], uint32_t& L, uint64_t& off, u32x4& rec) {
    vr_wait_meta<0, BIN>(L, off, rec);
#pragma unroll
    for (int i = 0; i < NB; ++i) asm volatile("" : "+v"(a[i]), "+v"(b[i]));
}

// Zero the bytes of a block that lie outside the packet, [lo, hi) kept (block
// byte offsets, may lie outside [0, 32)).  A, B in lane order (swapped when hs).
__device__ __forceinline__ void vr_edge_mask(u32x4& A, u32x4& B, uint32_t hs, int32_t lo, int32_t hi) {
    const bool sw = hs != 0;
    const u32x4 h0 = sw ? B : A, h1 = sw ? A : B;
    uint32_t v[8] = {h0.x, h0.y, h0.z, h0.w, h1.x, h1.y, h1.z, h1.w};
    const int l = max(-4, min(lo, 36));
    const int h = max(-4, min(hi, 36));
#pragma unroll
    for (int q = 0; q < 8; ++q) v[q] &= keep_mask(l, h, q);
    const u32x4 n0 = {v[0], v[1], v[2], v[3]}, n1 = {v[4], v[5], v[6], v[7]};
    A = sw ? n1 : n0;
    B = sw ? n0 : n1;
}

// Lane constants of the fold (make_sched's, compressed).  The column byte of
// table t is col_byte(t) = t << 3 | (t >> 4) << 2, GF(2)-linear in t, so the
// column of step i = 4g + h for lane l, col_byte(31 ^ i ^ l5), is the
// compile-time bytes of col_byte(31 ^ i) XOR one per-lane byte col_byte(l5):
// one register instead of eight, one XOR per 4 lookups.
struct VrSched {
    uint32_t cl;        // col_byte(l & 31) in all four bytes
    uint32_t sel[4];    // v_perm selectors (make_sched)
    uint32_t m1, m2, hs;
};

__device__ __forceinline__ VrSched make_vr_sched(uint32_t lane) {
    const LaneSched a = make_sched(lane);
    VrSched s;
    s.cl = col_byte(lane & 31u) * 0x01010101u;
#pragma unroll
    for (int h = 0; h < 4; ++h) s.sel[h] = a.sel[h];
    s.m1 = a.m1;
    s.m2 = a.m2;
    s.hs = a.hs;
    return s;
}

// mulmod (crc32_device.hpp) as a rolled loop: once per packet, so the few
// cycles of loop overhead buy registers (the unrolled form set the kernel's peak)
__device__ __forceinline__ uint32_t vr_mulmod(uint32_t a, uint32_t b) {
    uint32_t p = 0;
#pragma unroll 4
    for (int j = 0; j < 32; ++j) {
        const uint32_t m = static_cast<uint32_t>(static_cast<int32_t>(a) >> 31);
        p = __builtin_amdgcn_bitop3_b32(p, b, m, 0x78);                 // p ^ (b & m)
        const uint32_t r = static_cast<uint32_t>(static_cast<int32_t>(b << 31) >> 31);
        b = __builtin_amdgcn_bitop3_b32(b >> 1, kPoly, r, 0x78);         // (b>>1) ^ (P & r)
        a <<= 1;
    }
    return p;
}

template <int G>
__device__ __forceinline__ constexpr uint32_t vr_col_const() {
    uint32_t r = 0;
    for (int h = 0; h < 4; ++h) r |= col_byte(31u ^ static_cast<uint32_t>(4 * G + h)) << (8 * h);
    return r;
}

// fold_block_lane (crc32_device.hpp) with at most 8 table lookups in flight:
// groups of 4 lookups, group g+1 issued before group g is XOR-reduced, so the
// kernel fits 64 VGPRs (32 waves per CU hide the LDS latency instead of ILP).
__device__ __forceinline__ uint32_t vr_fold(uint32_t reg, u32x4 A, u32x4 B, const VrSched& s, uint32_t lane) {
    const uint32_t a0 = __builtin_amdgcn_bitop3_b32(A.x, reg, s.hs, 0xB4);   // A ^ (reg & ~hs)
    const uint32_t b0 = __builtin_amdgcn_bitop3_b32(B.x, reg, s.hs, 0x78);   // B ^ (reg & hs)
    const uint32_t w[8] = {a0, A.y, A.z, A.w, b0, B.y, B.z, B.w};
    // the dword-swap masks (make_sched's m1, m2) rebuilt per block from the lane
    // id: two VALU ops instead of two VGPRs held across the loop (asm volatile, so
    // the compiler cannot hoist them back out)
    uint32_t m1, m2;
    asm volatile("v_bfe_i32 %0, %1, 2, 1" : "=v"(m1) : "v"(lane));
    asm volatile("v_bfe_i32 %0, %1, 3, 1" : "=v"(m2) : "v"(lane));
    uint32_t x[8], d[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) x[q] = __builtin_amdgcn_bitop3_b32(w[q], w[q ^ 1], m1, 0xD8);
#pragma unroll
    for (int q = 0; q < 8; ++q) d[q] = __builtin_amdgcn_bitop3_b32(x[q], x[q ^ 2], m2, 0xD8);
    uint32_t v[2][4];
    uint32_t acc = 0;
    auto issue = [&](auto gc) __attribute__((always_inline)) {
        constexpr int g = decltype(gc)::value;
        const uint32_t col = vr_col_const<g>() ^ s.cl;
#pragma unroll
        for (int i = 0; i < 4; ++i) v[g & 1][i] = lds_load(__builtin_amdgcn_perm(d[g], col, s.sel[i]));
    };
    auto reduce = [&](int g) __attribute__((always_inline)) {
        const uint32_t(&u)[4] = v[g & 1];
        acc = xor3(acc, u[0], u[1]) ^ (u[2] ^ u[3]);
    };
    issue(std::integral_constant<int, 0>{});
    static_for<1, 8>([&](auto gc) __attribute__((always_inline)) {
        __builtin_amdgcn_sched_barrier(0);
        issue(gc);
        reduce(decltype(gc)::value - 1);
    });
    __builtin_amdgcn_sched_barrier(0);
    reduce(7);
    return acc;
}

// NB = ring slots (NB - 1 stages in flight while one is folded).
// WPE = waves per SIMD the register allocation must allow: 8 = two 16-wave
// workgroups per CU (64 VGPRs), 4 = one (no cap below 128).
// TR = 1: the diagnostics instance that writes the per-wave trace (pa.trace).
// BIN = 1: metadata from the length-ordered records of the *_binned entry points
// (PacketArgs::meta4, 16 B {len, off_lo, off_hi, index} per packet, one load
// instead of two); the CRC goes to out[index].
template <int LG, int NB, int WPE, int TR = 0, int BIN = 0>
__global__ void __launch_bounds__(64 * kVrW) __attribute__((amdgpu_waves_per_eu(WPE, 8)))
crc32_vring_kernel(PacketArgs pa, KernelTables tb, const uint32_t* basis) {
    static_assert(NB >= 2 && NB <= 4, "ring slots");
    constexpr uint32_t P = 1u << LG, kPk = 64u >> LG;
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t ngroups = (pa.n + kPk - 1u) >> (6 - LG);
    const uint64_t wv = static_cast<uint64_t>(blockIdx.x) * kVrW + wave;
    const uint64_t wt = static_cast<uint64_t>(gridDim.x) * kVrW;
    const uint32_t J = wv < ngroups ? static_cast<uint32_t>((ngroups - 1u - wv) / wt) + 1u : 0u;
    const uint32_t k = lane & (P - 1u), p = lane >> LG;
    const uint64_t zero = reinterpret_cast<uint64_t>(tb.zero);
    const uint64_t base = reinterpret_cast<uint64_t>(pa.bytes);
    auto packet_of = [&](uint32_t j) __attribute__((always_inline)) -> uint64_t {
        return (wv + static_cast<uint64_t>(j) * wt) * kPk + p;
    };

    // diagnostics (enet_hip_diag_trace): per-wave timestamps, tools/timeline.py's
    // 8 x u64 layout [start, metadata, table, barrier B, first stage, end, HW_ID, groups]
    uint64_t tmark[5] = {0, 0, 0, 0, 0};
    auto mark = [&](int i) __attribute__((always_inline)) {
        if (TR) tmark[i] = __builtin_amdgcn_s_memrealtime();
    };
    auto trace_end = [&]() __attribute__((always_inline)) {
        if (TR && lane == 0u) {
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
    mark(0);
    // tuning (pa.prio): the SIMD arbiter favours older waves, so wave slots 12-15 of a
    // workgroup finish ~40 % after slots 0-3 (profiles/r02_timeline_*): issue priority
    // by slot quartile, youngest highest
    if (pa.prio == 1u) {
        const uint32_t q = wave >> 2;                        // wave-uniform
        if (q == 1u) __builtin_amdgcn_s_setprio(1);
        else if (q == 2u) __builtin_amdgcn_s_setprio(2);
        else if (q == 3u) __builtin_amdgcn_s_setprio(3);
    }

    // ---- prologue: basis row `wave` (waves < 10) and metadata of group 0
    if (wave < static_cast<uint32_t>(kVrBasisRows))
        dma4(basis + static_cast<size_t>(LG == 2 ? 1 : 2) * kVrBasisDwords + 64u * wave + lane,
             kVrStaging + 256u * wave);
    uint32_t mL = 0;                                         // metadata of the producer's next group
    uint64_t moff = 0;
    u32x4 mrec = {0u, 0u, 0u, 0u};                           // (BIN: the record)
    constexpr int kMetaOps = BIN ? 1 : 2;                    // metadata loads per produce
    auto load_meta = [&](uint32_t j) __attribute__((always_inline)) {
        const uint64_t q = min(packet_of(j), pa.n - 1u);
        if constexpr (BIN) {
            vr_ld16_tied(mrec, reinterpret_cast<uint64_t>(pa.meta4 + 4u * q));
        } else {
            vr_ld4(mL, reinterpret_cast<uint64_t>(pa.len + q));
            vr_ld8(moff, reinterpret_cast<uint64_t>(pa.off + q));
        }
    };
    load_meta(0);                                            // (clamped index: valid for J == 0 too)
    vr_wait_meta<0, BIN>(mL, moff, mrec);                    // basis row and metadata have landed
    mark(1);

    // ---- producer: window of the group it loads, one stage ahead of the consumer
    uint64_t pws = 0;                                        // window start (64-byte aligned)
    uint32_t plz = 0, pe = 0;                                // packet bytes [plz, pe) of the window
    uint32_t pj = 0, pst = 0, pstages = 0;
    bool pdone = J == 0;
    // hand-over of the windows to the consumer, which runs NB - 1 stages behind:
    // with NB == 2 it enters a group right after the producer did and reads plz /
    // pe; deeper rings keep a FIFO of the windows the producer entered ahead
    uint32_t f0lz = 0, f0e = 0, f1lz = 0, f1e = 0, f2lz = 0, f2e = 0, fn = 0;
    uint32_t pidx = 0;                                       // (BIN: caller index of the lane's packet)
    auto producer_enter = [&](uint32_t j) __attribute__((always_inline)) {
        const uint32_t L = packet_of(j) < pa.n ? (BIN ? mrec.x : mL) : 0u;
        const uint64_t a = base + (BIN ? (static_cast<uint64_t>(mrec.y) | (static_cast<uint64_t>(mrec.z) << 32)) : moff);
        if constexpr (BIN) pidx = mrec.w;
        plz = static_cast<uint32_t>(a) & 63u;
        pws = a - plz;
        pe = plz + L;
        const uint32_t nb = L ? (pe + 31u) >> 5 : 0u;
        pstages = max(1u, wave_max_u((nb + P - 1u) >> LG));
        pst = 0;
        if constexpr (NB > 2) {
            if (fn == 0u) { f0lz = plz; f0e = pe; }
            else if (fn == 1u) { f1lz = plz; f1e = pe; }
            else { f2lz = plz; f2e = pe; }
            ++fn;
        }
    };
    const VrSched s = make_vr_sched(lane);
    // Every produce issues the same four loads -- the metadata of the group after
    // the producer's (an L2 hit but at group switches) and the stage's two
    // pieces -- so every wait below has a fixed count.
    u32x4 ra[NB], rb[NB];
    auto produce = [&](auto slot_c) __attribute__((always_inline)) {
        constexpr uint32_t slot = decltype(slot_c)::value;
        if (!pdone && pst == pstages) {
            if (++pj < J) {
                // last produce's metadata loads are older than its two stage loads
                // (and a store): at most those may still be in flight
                vr_wait_meta<2, BIN>(mL, moff, mrec);
                producer_enter(pj);
            } else {
                pdone = true;
                plz = pe = 0;                                // every piece reads the zero line
            }
        }
        load_meta(min(pj + 1u, J - 1u));
        const uint32_t q0 = 32u * (k + P * pst);
        const uint32_t hs16 = s.hs & 16u;                    // this lane takes the block's halves swapped
        const uint32_t a0 = q0 + hs16, a1 = q0 + 16u - hs16;
        const uint64_t s0 = (a0 < pe && a0 + 16u > plz) ? pws + a0 : zero;
        const uint64_t s1 = (a1 < pe && a1 + 16u > plz) ? pws + a1 : zero;
        ra[slot] = vr_ld16(s0);
        rb[slot] = vr_ld16(s1);
        ++pst;
    };
    if (J) {
        producer_enter(0);
        unroll_slots<NB - 1>([&](auto sc) __attribute__((always_inline)) { produce(sc); });
    }

    // ---- the table image, rebuilt in LDS while stage 0 is in flight.  Wave w
    // writes rows w + 16 i: row j = XOR of basis rows b with bit b of j set (Gray
    // order: one XOR per row), except the INIT and CINV dwords (not linear in j),
    // whose rows < 64 come from basis rows 8 and 9.  Raw s_barrier: no vmcnt drain.
    __builtin_amdgcn_s_barrier();                            // (A) every basis row has landed
    {
        uint32_t bb[8];
#pragma unroll
        for (int b = 0; b < 8; ++b) bb[b] = lds_load(kVrStaging + 256u * b + 4u * lane);
        const bool nonlin = lane == kInitDword || lane == kCinvDword;
        const uint32_t row8 = kVrStaging + 256u * (lane == kInitDword ? 8u : 9u);
        uint32_t v = 0;
#pragma unroll
        for (int b = 0; b < 4; ++b) v ^= ((wave >> b) & 1u) ? bb[b] : 0u;
#pragma unroll
        for (uint32_t q = 0; q < 16u; ++q) {
            const uint32_t i = q ^ (q >> 1);
            if (q) v ^= bb[4 + __builtin_ctz(q)];
            uint32_t x = v;
            if (i < 4u) {                                    // rows < 64: INIT / CINV
                const uint32_t e = lds_load(row8 + 4u * (wave + 16u * i));
                x = nonlin ? e : x;
            }
            lds_store(256u * (wave + 16u * i) + 4u * lane, x);
        }
    }
    mark(2);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();                            // (B) the image is complete
    mark(3);
    if (!J) {
        trace_end();
        return;
    }

    // ---- consumer
    uint32_t reg = 0, ccnt = 0, clz = 0, ce = 0, cj = 0, cs = 0, cstages = 0, nedge = ~0u;
    uint32_t cidx = 0;                                       // (BIN: out index of the lane's packet)
    // first stage >= from holding a partly covered head or tail piece (~0u = none)
    auto next_edge = [&](uint32_t from) __attribute__((always_inline)) -> uint32_t {
        const bool live = ce != clz;
        const uint32_t wh = clz >> 5, wl = (ce - 1u) >> 5;
        uint32_t h = (live && (clz & 15u) && (wh & (P - 1u)) == k) ? wh >> LG : ~0u;
        uint32_t t = (live && (ce & 15u) && (wl & (P - 1u)) == k) ? wl >> LG : ~0u;
        h = h >= from ? h : ~0u;
        t = t >= from ? t : ~0u;
        return wave_min_u(min(h, t));
    };
    auto consumer_enter = [&]() __attribute__((always_inline)) {
        if constexpr (NB == 2) {
            clz = plz;
            ce = pe;
            if constexpr (BIN) cidx = pidx;
        } else {
            static_assert(!BIN, "binned records: 2 ring slots only");
            clz = f0lz;
            ce = f0e;
            f0lz = f1lz; f0e = f1e;
            f1lz = f2lz; f1e = f2e;
            --fn;
        }
        const uint32_t nb = ce != clz ? (ce + 31u) >> 5 : 0u;
        ccnt = nb > k ? ((nb - 1u - k) >> LG) + 1u : 0u;
        cstages = max(1u, wave_max_u((nb + P - 1u) >> LG));
        const uint32_t init = lds_load(init_addr(clz));
        reg = k == 0u ? (nb ? init : 0xFFFFFFFFu) : 0u;      // packet.cs:144 (empty packet: ~crc = 0)
        nedge = next_edge(0);
        cs = 0;
    };
    consumer_enter();
    bool done = false;
    auto iteration = [&](auto sc) __attribute__((always_inline)) {
        constexpr uint32_t S = decltype(sc)::value;
        if (pa.prio == 2u) {
            // equal progress: the SIMD arbiter serves high priority first, then older
            // waves; a wave with more of its work left than its neighbours goes first,
            // so no wave is left streaming alone at the end
            const uint32_t left = (J - cj) * 8u - min(8u, (cs * 8u) / cstages);   // eighths of groups left
            const uint32_t q = (left * 4u) / (J * 8u + 1u);                        // 0..3
            if (q >= 3u) __builtin_amdgcn_s_setprio(3);
            else if (q == 2u) __builtin_amdgcn_s_setprio(2);
            else if (q == 1u) __builtin_amdgcn_s_setprio(1);
            else __builtin_amdgcn_s_setprio(0);
        }
        produce(std::integral_constant<uint32_t, (S + NB - 1) % NB>{});
        vr_wait<(kMetaOps + 2) * (NB - 1)>(ra[S], rb[S]);    // stage S has landed (younger: the later produces)
        u32x4 A = ra[S], B = rb[S];
        if (cs == nedge) {                                   // head / tail pieces: keep [clz, ce) only
            const uint32_t q0 = 32u * (k + P * cs);               // windows < 2 GiB: differences fit int32
            vr_edge_mask(A, B, s.hs, static_cast<int32_t>(clz - q0), static_cast<int32_t>(ce - q0));
            nedge = next_edge(cs + 1u);
        }
        const uint32_t nr = vr_fold(reg, A, B, s, lane);
        reg = cs < ccnt ? nr : reg;
        if (cj == 0u && cs == 0u) mark(4);
        if (++cs == cstages) {
            // lane k is o = (k - nb) mod P blocks past the window end: x^(-256 o)
            const uint32_t nb = ce != clz ? (ce + 31u) >> 5 : 0u;
            const uint32_t o = (k - nb) & (P - 1u);
            // (lane-uniform byte order: per-lane rotations hoisted out of the loop cost
            // ten VGPRs; four lookups per packet can afford the bank conflicts)
            const uint32_t kk = o ? o : 1u;
            uint32_t x[4];
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                const uint32_t c = kCorrCol + 4u * (kk - 1u) + static_cast<uint32_t>(b);
                const uint32_t col = 4u * (c < 16u ? 2u * c + 1u : 2u * c);     // free_col(c)
                const uint32_t sel = 0x0C0C0000u | ((4u + b) << 8);          // byte1 = byte b of reg, byte0 = column
                x[b] = lds_load(__builtin_amdgcn_perm(reg, col, sel));
            }
            const uint32_t corr = xor3(x[0], x[1], x[2]) ^ x[3];
            reg = o ? corr : reg;
            reg = xor_lanes<0>(LG, reg);
            const uint32_t tz = nb ? 32u * nb - ce : 0u;
            if (k == 0u && tz) reg = vr_mulmod(reg, lds_load(cinv_addr(tz)));
            const uint64_t pk = packet_of(cj);
            if (k == 0u && pk < pa.n) pa.out[BIN ? cidx : pk] = finalize(reg);   // packet.cs:159
            if (++cj == J) {
                // the producer's last loads (zero lines past the end) are dead: drain
                // them, so no register they land in can be reused while in flight
                vr_drain<BIN>(ra, rb, mL, moff, mrec);
                done = true;
                return;
            }
            consumer_enter();
        }
    };
    // each slot's iteration leaves the loop at once when the wave is done, so the
    // loop head is reached only from a completed ring turn (no path with the drained
    // loads of the last turn in flight: tools/isa_inflight_check.py)
    for (;;) {
        iteration(std::integral_constant<uint32_t, 0>{});
        if (done) break;
        iteration(std::integral_constant<uint32_t, 1>{});
        if (done) break;
        if constexpr (NB > 2) {
            iteration(std::integral_constant<uint32_t, 2>{});
            if (done) break;
        }
        if constexpr (NB > 3) {
            iteration(std::integral_constant<uint32_t, 3>{});
            if (done) break;
        }
    }
    trace_end();
}

// ---------------------------------------------------------------- host side

template <int LG, int NB, int WPE, int TR = 0, int BIN = 0>
const void* vring_fn() {
    return reinterpret_cast<const void*>(crc32_vring_kernel<LG, NB, WPE, TR, BIN>);
}

// The product instance: 2 ring slots, one workgroup per CU per launch, 64 VGPRs
// (WPE 8) so that the next launch's workgroup -- overlapping batches on other
// streams -- can share the CU while this one drains (bench: 4831 GiB/s at 59-62
// VGPRs against 4438 at 66, profiles/r02_*).  With a trace buffer: the same kernel
// writing per-wave timestamps.  Measured and not kept: 3 and 4 ring slots, and two
// workgroups of one launch per CU.
const void* vring_pick(int lg, bool trace, bool bin) {
    if (trace) return lg == 2 ? vring_fn<2, 2, 4, 1>() : vring_fn<3, 2, 4, 1>();
    (void)bin;   // the BIN instance stays uninstantiated (see vring_launch)
    return lg == 2 ? vring_fn<2, 2, 8>() : vring_fn<3, 2, 8>();
}

int vring_setup() {
    for (int lg = 2; lg <= 3; ++lg)
        for (int t = 0; t < 2; ++t) {
            const hipError_t e = hipFuncSetAttribute(vring_pick(lg, t == 1, false),
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, kVrLds);
            if (e != hipSuccess) return -static_cast<int>(e);
        }
    return 0;
}

int vring_launch(int lg, int num_cus, hipStream_t st, const PacketArgs& pa, const KernelTables& tb,
                 const uint32_t* basis2) {
    // binned records (pa.meta4) run on the lean kernel: the BIN instance of this one
    // did not pass tools/isa_inflight_check.py (hipcc copies the record register
    // between its load and its wait), so it is not built
    if ((lg != 2 && lg != 3) || pa.meta4) return -static_cast<int>(hipErrorInvalidValue);
    if (pa.n == 0) return 0;
    const uint64_t kpk = 64u >> lg;
    const uint64_t groups = (pa.n + kpk - 1u) / kpk;
    const unsigned grid = static_cast<unsigned>(std::max<uint64_t>(
        1, std::min<uint64_t>((groups + kVrW - 1) / kVrW, static_cast<uint64_t>(num_cus))));
    void* args[] = {const_cast<PacketArgs*>(&pa), const_cast<KernelTables*>(&tb), const_cast<const uint32_t**>(&basis2)};
    const hipError_t e = hipLaunchKernel(vring_pick(lg, pa.trace != nullptr, false), dim3(grid), dim3(64 * kVrW), args,
                                         kVrLds, st);
    return e == hipSuccess ? 0 : -static_cast<int>(e);
}

}  // namespace enethip
