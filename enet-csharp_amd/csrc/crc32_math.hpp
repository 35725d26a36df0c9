// crc32_math.hpp -- CRC-32 (reflected, poly 0xEDB88320) algebra shared by the
// CPU callback path, the host-side table builder and the gfx950 kernels.
//
// Algorithm of record: /root/reference/enet-csharp/ENet/c/packet.cs:142-160
//   crc = 0xFFFFFFFF; crc = (crc >> 8) ^ T[(crc & 0xFF) ^ b] per byte;
//   return ENET_HOST_TO_NET_32(~crc)   (include/win32.cs:18)
// with T the table literal at packet.cs:106-140 (the standard 0xEDB88320 table).
//
// Everything below is expressed in "register space": reg is the 32-bit Sarwate
// register of packet.cs:153.  Register value r stands for the polynomial
// R(x) = sum_i bit_i(r) * x^(31-i)  (bit 31 = x^0).  Feeding a zero byte maps
// R -> R * x^8 mod P, so  reg(s, A||B) = adv_|B|(reg(s, A)) ^ reg(0, B)  with
// adv_n(r) = r (*) (x^(8n) mod P), (*) the reflected GF(2) product below.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define ENH_HD __host__ __device__ inline
#else
#define ENH_HD inline
#endif

namespace enethip {

constexpr uint32_t kPoly = 0xEDB88320u;
constexpr uint32_t kOneReflected = 0x80000000u;  // the polynomial "1"

// T0[n]: register contribution of byte n (packet.cs:106-140).
ENH_HD constexpr uint32_t crc_table_entry(uint32_t n) {
    uint32_t c = n;
    for (int k = 0; k < 8; ++k) c = (c & 1u) ? (c >> 1) ^ kPoly : (c >> 1);
    return c;
}

// One Sarwate step (packet.cs:153).
ENH_HD constexpr uint32_t sarwate_step(uint32_t reg, uint8_t b) {
    return (reg >> 8) ^ crc_table_entry((reg ^ b) & 0xFFu);
}

// Reflected product a(x)*b(x) mod P (branch-free bit loop; zlib's multmodp).
ENH_HD constexpr uint32_t gf2_mulmod(uint32_t a, uint32_t b) {
    uint32_t p = 0;
    for (int j = 0; j < 32; ++j) {
        uint32_t m = 0u - ((a >> (31 - j)) & 1u);
        p ^= b & m;
        b = (b >> 1) ^ (kPoly & (0u - (b & 1u)));
    }
    return p;
}

// x^(8n) mod P by square-and-multiply.
ENH_HD constexpr uint32_t x8n_modp(uint64_t n) {
    uint32_t result = kOneReflected;
    uint32_t sq = 0x00800000u;  // x^8  (bit 31-8)
    while (n) {
        if (n & 1u) result = gf2_mulmod(result, sq);
        sq = gf2_mulmod(sq, sq);
        n >>= 1;
    }
    return result;
}

ENH_HD constexpr uint32_t adv_bytes(uint32_t reg, uint64_t n) { return gf2_mulmod(reg, x8n_modp(n)); }

// Inverse of one zero-byte Sarwate step.  T0[n] >> 24 is a bijection of n, so
// from reg' = (reg >> 8) ^ T0[reg & 0xFF] the low byte of reg is recovered from
// the top byte of reg'.
ENH_HD constexpr uint32_t unstep_zero(uint32_t reg_next) {
    uint32_t top = reg_next >> 24, n = 0;
    for (uint32_t k = 0; k < 256; ++k)
        if ((crc_table_entry(k) >> 24) == top) n = k;
    return ((reg_next ^ crc_table_entry(n)) << 8) | n;
}

ENH_HD constexpr uint32_t bswap32(uint32_t v) {
    return (v >> 24) | ((v >> 8) & 0x0000FF00u) | ((v << 8) & 0x00FF0000u) | (v << 24);
}

// Wire value returned by the checksum callback (packet.cs:159, little-endian host).
ENH_HD constexpr uint32_t finalize(uint32_t reg) { return bswap32(~reg); }

}  // namespace enethip
