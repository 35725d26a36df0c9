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
#include <cstddef>
#include <cstdint>
#include <cstring>

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

}  // namespace

extern "C" uint32_t enet_hip_crc32(const ENetBuffer* buffers, size_t bufferCount) {
    const Slice8& s = slice8();
    uint32_t reg = 0xFFFFFFFFu;                       // packet.cs:144
    for (size_t i = 0; i < bufferCount; ++i)          // packet.cs:146-157
        if (buffers[i].dataLength)
            reg = crc_update(reg, static_cast<const uint8_t*>(buffers[i].data), buffers[i].dataLength, s);
    return enethip::finalize(reg);                    // packet.cs:159
}

extern "C" uint32_t enet_hip_crc32_update(uint32_t reg, const void* data, size_t length) {
    return length ? crc_update(reg, static_cast<const uint8_t*>(data), length, slice8()) : reg;
}
