/* oracle_san.c -- the oracle (test infrastructure) under AddressSanitizer + UBSan:
 * batch (1 and 8 threads), gather, verify (incl. a 200 000-byte DGRAM, heap copy),
 * range coder round trips, over exact-size heap blocks.  Built by
 * `make -C oracle san`, run by tests/test_sanitizers.py. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

typedef struct { size_t dataLength; const void* data; } OracleENetBuffer;
uint32_t oracle_enet_crc32(const OracleENetBuffer* buffers, size_t bufferCount);
void oracle_crc32_batch(const uint8_t*, const uint64_t*, const uint32_t*, size_t, uint32_t*);
int oracle_crc32_batch_mt(const uint8_t*, const uint64_t*, const uint32_t*, size_t, uint32_t*, int);
void oracle_crc32_gather(const uint8_t*, const uint64_t*, const uint32_t*, const uint32_t*, size_t, uint32_t*);
void oracle_verify_batch(const uint8_t*, const uint64_t*, const uint32_t*, const uint32_t*, const uint32_t*, size_t,
                         uint8_t*, uint32_t*);
size_t oracle_range_compress(const uint8_t*, size_t, uint8_t*, size_t);
size_t oracle_range_decompress(const uint8_t*, size_t, uint8_t*, size_t);

static uint64_t s = 0x4F5241;
static uint64_t rnd(void) {
    s += 0x9E3779B97F4A7C15ull;
    uint64_t z = s;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

int main(void) {
    int fails = 0;
    const size_t n = 3000, cap = n * 1500;
    uint8_t* bytes = malloc(cap);
    for (size_t i = 0; i < cap; ++i) bytes[i] = (uint8_t)rnd();
    uint64_t* off = malloc(n * 8);
    uint32_t* len = malloc(n * 4);
    uint32_t* a = malloc(n * 4);
    uint32_t* b = malloc(n * 4);
    for (size_t i = 0; i < n; ++i) {
        len[i] = (uint32_t)(rnd() % 1500);
        off[i] = rnd() % (cap - len[i] + 1);
    }
    oracle_crc32_batch(bytes, off, len, n, a);
    oracle_crc32_batch_mt(bytes, off, len, n, b, 8);
    fails += memcmp(a, b, n * 4) != 0;
    uint32_t* first = malloc((n / 3 + 1) * 4);
    for (size_t d = 0; d <= n / 3; ++d) first[d] = (uint32_t)(3 * d);
    oracle_crc32_gather(bytes, off, len, first, n / 3, b);
    for (size_t d = 0; d < n / 3; ++d) {
        OracleENetBuffer bb[3];
        for (int k = 0; k < 3; ++k) {
            bb[k].dataLength = len[3 * d + k];
            bb[k].data = bytes + off[3 * d + k];
        }
        fails += b[d] != oracle_enet_crc32(bb, 3);
    }
    uint32_t* so = malloc(n * 4);
    uint32_t* cid = malloc(n * 4);
    uint8_t* ok = malloc(n);
    for (size_t i = 0; i < n; ++i) {
        so[i] = (uint32_t)(rnd() % 8);
        cid[i] = (uint32_t)rnd();
    }
    oracle_verify_batch(bytes, off, len, so, cid, n, ok, b);
    const uint32_t L = 200000;
    uint8_t* big = malloc(L);
    for (uint32_t i = 0; i < L; ++i) big[i] = (uint8_t)rnd();
    uint64_t bo = 0;
    uint32_t bs = 4, bc = 7;
    oracle_verify_batch(big, &bo, &L, &bs, &bc, 1, ok, b);
    for (int t = 0; t < 200; ++t) {                         /* range coder round trips */
        const size_t m = rnd() % 3000;
        uint8_t* in = malloc(m + 1);
        for (size_t i = 0; i < m; ++i) in[i] = (uint8_t)(rnd() % (t % 7 + 1));
        uint8_t* c = malloc(m + 64);
        uint8_t* d = malloc(m + 1);
        const size_t cl = oracle_range_compress(in, m, c, m + 64);
        if (cl) fails += oracle_range_decompress(c, cl, d, m) != m || memcmp(in, d, m) != 0;
        free(in);
        free(c);
        free(d);
    }
    printf("{\"oracle_san\": \"%s\", \"fails\": %d}\n", fails ? "FAIL" : "ok", fails);
    free(bytes); free(off); free(len); free(a); free(b); free(first); free(so); free(cid); free(ok); free(big);
    return fails ? 1 : 0;
}
