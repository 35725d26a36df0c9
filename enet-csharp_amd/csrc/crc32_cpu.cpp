// crc32_cpu.cpp -- the per-DGRAM callback path of libenethip (CPU only).
//
// ENet calls host->checksum(buffers, bufferCount) synchronously once per DGRAM
// sent (c/protocol.cs:1696) and once per DGRAM received (c/protocol.cs:1066);
// the field is `delegate* managed<ENetBuffer*, nuint, uint>` (include/enet.cs:666)
// and its default implementation is ENet.enet_crc32 (c/packet.cs:142-160).  A
// single 1.4 KB DGRAM is far below what one kernel launch costs, so this entry
// point never touches the GPU and can never fail (SURVEY.md §8b "Errors").  It is
// slicing-by-8 over the same register algebra, bit-identical to the reference's
// byte loop (tests/test_library_cpu.py checks it against every golden vector and
// random gather lists; tests/test_sanitizers.py runs it under ASan + UBSan).
// Buffers of 64 bytes or more go through carry-less-multiply folding when the CPU
// has PCLMULQDQ (checked once at run time): four 128-bit accumulators folded 64
// bytes at a time by x^(8*64+32) / x^(8*64-32) mod P, folded to one, reduced to
// 32 bits by a Barrett step -- the published reflected-CRC32 folding method; the
// multipliers are derived here from the polynomial (xpow_mod), not copied.
#include <cstddef>
#include <cstdint>
#include <cstring>

#if defined(__x86_64__)
#include <immintrin.h>
#define ENET_HIP_CLMUL 1
#endif

#include "crc32_math.hpp"
#include "enet_hip.h"

namespace {

struct Slice8 {
    uint32_t t[8][256];
    Slice8() {
        for (uint32_t n = 0; n < 256; ++n) t[0][n] = enethip::crc_table_entry(n);
        for (int k = 1; k < 8; ++k)
            for (uint32_t n = 0; n < 256; ++n) t[k][n] = (t[k - 1][n] >> 8) ^ t[0][t[k - 1][n] & 0xFFu];
    }
};

const Slice8& slice8() {
    static const Slice8 s;
    return s;
}

inline uint32_t crc_update(uint32_t reg, const uint8_t* p, size_t n, const Slice8& s) {
    while (n && (reinterpret_cast<uintptr_t>(p) & 7u)) {
        reg = (reg >> 8) ^ s.t[0][(reg ^ *p++) & 0xFFu];
        --n;
    }
    while (n >= 8) {
        uint64_t w;
        std::memcpy(&w, p, 8);
        uint32_t lo = static_cast<uint32_t>(w) ^ reg;
        uint32_t hi = static_cast<uint32_t>(w >> 32);
        reg = s.t[7][lo & 0xFF] ^ s.t[6][(lo >> 8) & 0xFF] ^ s.t[5][(lo >> 16) & 0xFF] ^ s.t[4][lo >> 24] ^
              s.t[3][hi & 0xFF] ^ s.t[2][(hi >> 8) & 0xFF] ^ s.t[1][(hi >> 16) & 0xFF] ^ s.t[0][hi >> 24];
        p += 8;
        n -= 8;
    }
    while (n--) reg = (reg >> 8) ^ s.t[0][(reg ^ *p++) & 0xFFu];
    return reg;
}

#ifdef ENET_HIP_CLMUL
// Bit-reflected GF(2) arithmetic for P = 0x104C11DB7 (reflected 0xEDB88320): the
// folding multipliers are x^k mod P as 33-bit reflected values (x^(k-1) reflected
// then shifted left by one, the usual convention for the 64x64 carry-less multiply)
uint64_t xpow_mod(uint32_t k) {                       // x^k mod P, bit-reflected, 32 bits
    uint32_t r = 0x80000000u;                         // x^0
    for (uint32_t i = 0; i < k; ++i) r = (r >> 1) ^ ((r & 1u) ? 0xEDB88320u : 0u);
    return r;
}
uint64_t fold_k(uint32_t k) { return static_cast<uint64_t>(xpow_mod(k)) << 1; }
uint64_t barrett_mu() {                               // floor(x^64 / P), reflected, 33 bits
    // long division of x^64 by P in the reflected domain: bit i of the quotient
    uint64_t q = 0;
    uint64_t rem = 0;                                 // remainder window (normal order, 33 bits)
    for (int i = 64; i >= 0; --i) {
        rem = (rem << 1) | (i == 64 ? 1u : 0u);
        if (rem & (1ull << 32)) {
            rem ^= 0x104C11DB7ull;
            q |= 1ull << i;
        }
    }
    uint64_t r = 0;                                   // reflect the 33-bit quotient
    for (int i = 0; i < 33; ++i)
        if (q & (1ull << i)) r |= 1ull << (32 - i);
    return r;
}

struct ClmulK {
    __m128i k1k2, k3k4, k5, poly_mu;
    ClmulK() {
        k1k2 = _mm_set_epi64x(static_cast<long long>(fold_k(4 * 128 - 32)), static_cast<long long>(fold_k(4 * 128 + 32)));
        k3k4 = _mm_set_epi64x(static_cast<long long>(fold_k(128 - 32)), static_cast<long long>(fold_k(128 + 32)));
        k5 = _mm_set_epi64x(0, static_cast<long long>(fold_k(64)));
        poly_mu = _mm_set_epi64x(static_cast<long long>(barrett_mu()), 0x1DB710641ll);
    }
};

const ClmulK& clmul_k() {
    static const ClmulK k;
    return k;
}

bool have_clmul() {
    static const bool h = __builtin_cpu_supports("pclmul") && __builtin_cpu_supports("sse4.1");
    return h;
}

#define ENET_CLMUL_TARGET __attribute__((target("pclmul,sse4.1")))
ENET_CLMUL_TARGET inline __m128i ld(const uint8_t* a) { return _mm_loadu_si128(reinterpret_cast<const __m128i*>(a)); }
// x folded over 128 bits (x.lo * k.lo ^ x.hi * k.hi) into the next block
ENET_CLMUL_TARGET inline __m128i fold(__m128i x, __m128i kk, __m128i next) {
    return _mm_xor_si128(_mm_xor_si128(_mm_clmulepi64_si128(x, kk, 0x00), _mm_clmulepi64_si128(x, kk, 0x11)), next);
}

// n >= 64, a multiple of 16: the register after n bytes
ENET_CLMUL_TARGET uint32_t crc_clmul(uint32_t reg, const uint8_t* p, size_t n, const ClmulK& k) {
    __m128i x1 = _mm_xor_si128(ld(p), _mm_cvtsi32_si128(static_cast<int>(reg)));
    __m128i x2 = ld(p + 16), x3 = ld(p + 32), x4 = ld(p + 48);
    p += 64;
    n -= 64;
    while (n >= 64) {                                  // four lanes, 64 bytes a step
        x1 = fold(x1, k.k1k2, ld(p));
        x2 = fold(x2, k.k1k2, ld(p + 16));
        x3 = fold(x3, k.k1k2, ld(p + 32));
        x4 = fold(x4, k.k1k2, ld(p + 48));
        p += 64;
        n -= 64;
    }
    x1 = fold(x1, k.k3k4, x2);                         // four lanes into one
    x1 = fold(x1, k.k3k4, x3);
    x1 = fold(x1, k.k3k4, x4);
    while (n >= 16) {
        x1 = fold(x1, k.k3k4, ld(p));
        p += 16;
        n -= 16;
    }
    // 128 -> 64 bits (appending 32 zero bits), then 64 -> 32 by Barrett
    const __m128i mask32 = _mm_set_epi32(0, 0, 0, -1);
    __m128i t = _mm_clmulepi64_si128(x1, k.k3k4, 0x10);   // x1.lo * k4
    x1 = _mm_xor_si128(_mm_srli_si128(x1, 8), t);
    t = _mm_srli_si128(x1, 4);
    x1 = _mm_xor_si128(_mm_clmulepi64_si128(_mm_and_si128(x1, mask32), k.k5, 0x00), t);
    t = x1;
    x1 = _mm_clmulepi64_si128(_mm_and_si128(x1, mask32), k.poly_mu, 0x10);   // * mu
    x1 = _mm_clmulepi64_si128(_mm_and_si128(x1, mask32), k.poly_mu, 0x00);   // * P
    x1 = _mm_xor_si128(x1, t);
    return static_cast<uint32_t>(_mm_extract_epi32(x1, 1));
}
#endif

inline uint32_t crc_any(uint32_t reg, const uint8_t* p, size_t n, const Slice8& s) {
#ifdef ENET_HIP_CLMUL
    if (n >= 64 && have_clmul()) {
        const size_t body = n & ~static_cast<size_t>(15);
        reg = crc_clmul(reg, p, body, clmul_k());
        p += body;
        n -= body;
    }
#endif
    return n ? crc_update(reg, p, n, s) : reg;
}

}  // namespace

extern "C" uint32_t enet_hip_crc32(const ENetBuffer* buffers, size_t bufferCount) {
    const Slice8& s = slice8();
    uint32_t reg = 0xFFFFFFFFu;                       // packet.cs:144
    for (size_t i = 0; i < bufferCount; ++i)          // packet.cs:146-157
        if (buffers[i].dataLength)
            reg = crc_any(reg, static_cast<const uint8_t*>(buffers[i].data), buffers[i].dataLength, s);
    return enethip::finalize(reg);                    // packet.cs:159
}

extern "C" uint32_t enet_hip_crc32_update(uint32_t reg, const void* data, size_t length) {
    return length ? crc_any(reg, static_cast<const uint8_t*>(data), length, slice8()) : reg;
}
