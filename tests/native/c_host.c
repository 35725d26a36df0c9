/* c_host.c -- a plain C host of libenethip.so: what a native ENet host (or the C#
 * P/Invoke shim) sees of the boundary.  Only include/enet_hip.h and
 * the C library: no HIP headers, no Python.  Built and run by tests/test_c_host.py.
 *
 * Checks, against a bit-at-a-time CRC-32 written out below (the reflected
 * polynomial 0xEDB88320 that c/packet.cs:106-140's table encodes; the callback value
 * is ENET_HOST_TO_NET_32(~crc), c/packet.cs:159):
 *   - the CPU callback enet_hip_crc32 (c/packet.cs:142-160) over gather lists;
 *   - with a device: enet_hip_crc32_batch_device, _batch_list_device (two batches in
 *     one launch), enet_hip_verify_batch_device (the receive check of
 *     c/protocol.cs:1052-1068, one DGRAM in seven corrupted) and the host-memory
 *     enet_hip_crc32_batch_host, on packets of every length 0..1500 at random
 *     offsets; device memory through the library's own helpers;
 *   - the error contract: a bad argument returns -1 (hipErrorInvalidValue) before any
 *     launch, an empty batch returns 0, and without a device enet_hip_context_create
 *     fails (-100), so no batch entry can run: there is no CPU fallback.
 * Exit status 0 = all passed; prints "c_host: ok (device|no device)". */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "enet_hip.h"

#define CHECK(cond, ...)                                                      \
    do {                                                                      \
        if (!(cond)) {                                                        \
            fprintf(stderr, "c_host: FAILED %s:%d: ", __FILE__, __LINE__);    \
            fprintf(stderr, __VA_ARGS__);                                     \
            fputc('\n', stderr);                                              \
            exit(1);                                                          \
        }                                                                     \
    } while (0)

static uint32_t bitwise_reg(uint32_t reg, const uint8_t* p, size_t n) {
    for (size_t i = 0; i < n; ++i) {
        reg ^= p[i];
        for (int b = 0; b < 8; ++b) reg = (reg >> 1) ^ (0xEDB88320u & (0u - (reg & 1u)));
    }
    return reg;
}
static uint32_t wire(uint32_t reg) { /* ENET_HOST_TO_NET_32(~reg) as stored bytes */
    const uint32_t c = ~reg;
    return (c >> 24) | ((c >> 8) & 0xFF00u) | ((c << 8) & 0xFF0000u) | (c << 24);
}
static uint64_t rng_state = 0x9E3779B97F4A7C15ull;
static uint32_t rnd(void) { /* xorshift64* */
    rng_state ^= rng_state >> 12;
    rng_state ^= rng_state << 25;
    rng_state ^= rng_state >> 27;
    return (uint32_t)((rng_state * 0x2545F4914F6CDD1Dull) >> 32);
}

static void* dev_copy(enet_hip_context* ctx, const void* src, size_t bytes) {
    void* d = NULL;
    int rc = enet_hip_device_alloc(ctx, bytes ? bytes : 16, &d);
    CHECK(rc == 0 && d, "device_alloc %zu: %d %s", bytes, rc, enet_hip_error_string(rc));
    if (src && bytes) {                                 /* (src NULL: allocate only) */
        rc = enet_hip_memcpy_h2d(ctx, d, src, bytes);
        CHECK(rc == 0, "memcpy_h2d %zu: %d %s", bytes, rc, enet_hip_error_string(rc));
    }
    return d;
}

int main(void) {
    /* ---- the callback: gather lists of one and three buffers, every length 0..600 */
    uint8_t buf[4096];
    for (size_t i = 0; i < sizeof buf; ++i) buf[i] = (uint8_t)rnd();
    for (size_t len = 0; len <= 600; ++len) {
        const size_t cut1 = len / 3, cut2 = len / 2;
        ENetBuffer parts[3] = {{cut1, buf + 7}, {cut2 - cut1, buf + 7 + cut1}, {len - cut2, buf + 7 + cut2}};
        const uint32_t want = wire(bitwise_reg(0xFFFFFFFFu, buf + 7, len));
        CHECK(enet_hip_crc32(parts, 3) == want, "callback, len %zu", len);
        CHECK(enet_hip_crc32(parts, 1) == wire(bitwise_reg(0xFFFFFFFFu, buf + 7, cut1)), "one buffer, len %zu", cut1);
        CHECK(wire(enet_hip_crc32_update(0xFFFFFFFFu, buf + 7, len)) == want, "update, len %zu", len);
    }
    CHECK(enet_hip_crc32(NULL, 0) == wire(0xFFFFFFFFu), "empty list");

    int ndev = 0;
    enet_hip_device_count(&ndev);
    enet_hip_context* ctx = NULL;
    const int cc = enet_hip_context_create(0, &ctx);
    if (ndev <= 0) {
        /* no device: no context, so no batch entry can run (no CPU fallback); a null
         * context is an argument error */
        uint64_t off = 0;
        uint32_t len = 0, out = 0;
        CHECK(cc < 0 && ctx == NULL, "context_create without a device returned %d", cc);
        CHECK(enet_hip_crc32_batch_host(NULL, buf, sizeof buf, &off, &len, 1, &out) == -1, "null context");
        printf("c_host: ok (no device; context_create %d: %s)\n", cc, enet_hip_error_string(cc));
        return 0;
    }
    CHECK(cc == 0 && ctx != NULL, "context_create %d", cc);

    /* ---- packets of every length 0..1500 at random offsets of one arena */
    enum { N = 1501 };
    const size_t arena_bytes = 1u << 21;
    uint8_t* arena = (uint8_t*)malloc(arena_bytes);
    CHECK(arena != NULL, "malloc");
    for (size_t i = 0; i < arena_bytes; ++i) arena[i] = (uint8_t)rnd();
    /* host arrays on the heap, as a host's packet tables would be */
    uint64_t* off = (uint64_t*)calloc(N, sizeof *off);
    uint32_t* len = (uint32_t*)calloc(N, sizeof *len);
    uint32_t* want = (uint32_t*)calloc(N, sizeof *want);
    uint32_t* out = (uint32_t*)calloc(2 * N, sizeof *out);
    CHECK(off && len && want && out, "calloc");
    for (int i = 0; i < N; ++i) {
        len[i] = (uint32_t)i;
        off[i] = rnd() % (arena_bytes - 1600);
        want[i] = wire(bitwise_reg(0xFFFFFFFFu, arena + off[i], len[i]));
    }
    uint8_t* d_arena = (uint8_t*)dev_copy(ctx, arena, arena_bytes);
    uint64_t* d_off = (uint64_t*)dev_copy(ctx, off, N * sizeof *off);
    uint32_t* d_len = (uint32_t*)dev_copy(ctx, len, N * sizeof *len);
    uint32_t* d_out = (uint32_t*)dev_copy(ctx, NULL, 2 * N * sizeof *out);

    /* enet_hip_crc32_batch_device on the context's stream */
    CHECK(enet_hip_crc32_batch_device(ctx, d_arena, d_off, d_len, N, d_out, NULL) == 0, "batch_device");
    CHECK(enet_hip_synchronize(ctx) == 0, "synchronize");
    CHECK(enet_hip_memcpy_d2h(ctx, out, d_out, N * sizeof *out) == 0, "memcpy_d2h");
    for (int i = 0; i < N; ++i) CHECK(out[i] == want[i], "batch_device packet %d: %08x against %08x", i, out[i], want[i]);

    /* two batches in one launch: the second is the first half again, written after it */
    ENetHipBatch list[2] = {{d_arena, d_off, d_len, N, d_out}, {d_arena, d_off, d_len, N / 2, d_out + N}};
    CHECK(enet_hip_crc32_batch_list_device(ctx, list, 2, NULL) == 0, "batch_list_device");
    CHECK(enet_hip_synchronize(ctx) == 0, "synchronize");
    CHECK(enet_hip_memcpy_d2h(ctx, out, d_out, 2 * N * sizeof *out) == 0, "memcpy_d2h");
    for (int i = 0; i < N; ++i) CHECK(out[i] == want[i], "list batch 0 packet %d", i);
    for (int i = 0; i < N / 2; ++i) CHECK(out[N + i] == want[i], "list batch 1 packet %d", i);

    /* receive verify (c/protocol.cs:1052-1068): DGRAMs of >= 8 bytes carrying their CRC,
     * computed with connectID in the slot, in the slot; one in seven corrupted */
    enum { M = 1200 };
    uint8_t* dg = (uint8_t*)malloc((size_t)M * 1600);
    uint64_t* voff = (uint64_t*)calloc(M, sizeof *voff);
    uint32_t* vlen = (uint32_t*)calloc(M, sizeof *vlen);
    uint32_t* slot = (uint32_t*)calloc(M, sizeof *slot);
    uint32_t* conn = (uint32_t*)calloc(M, sizeof *conn);
    uint8_t* expect_ok = (uint8_t*)calloc(M, 1);
    uint8_t* ok = (uint8_t*)calloc(M, 1);
    CHECK(dg && voff && vlen && slot && conn && expect_ok && ok, "calloc");
    for (int i = 0; i < M; ++i) {
        vlen[i] = 8u + (uint32_t)(rnd() % 1400u);
        voff[i] = (uint64_t)i * 1600u + (rnd() % 64u);
        slot[i] = (rnd() & 1u) ? 2u : 4u;
        conn[i] = rnd();
        uint8_t* p = dg + voff[i];
        for (uint32_t b = 0; b < vlen[i]; ++b) p[b] = (uint8_t)rnd();
        memcpy(p + slot[i], &conn[i], 4);
        const uint32_t crc = wire(bitwise_reg(0xFFFFFFFFu, p, vlen[i]));
        memcpy(p + slot[i], &crc, 4);
        expect_ok[i] = 1;
        if (i % 7 == 3) {
            p[vlen[i] - 1] ^= 0x5A;
            expect_ok[i] = 0;
        }
    }
    uint8_t* d_dg = (uint8_t*)dev_copy(ctx, dg, (size_t)M * 1600);
    uint64_t* d_voff = (uint64_t*)dev_copy(ctx, voff, M * sizeof *voff);
    uint32_t* d_vlen = (uint32_t*)dev_copy(ctx, vlen, M * sizeof *vlen);
    uint32_t* d_slot = (uint32_t*)dev_copy(ctx, slot, M * sizeof *slot);
    uint32_t* d_conn = (uint32_t*)dev_copy(ctx, conn, M * sizeof *conn);
    uint8_t* d_ok = (uint8_t*)dev_copy(ctx, NULL, M);
    CHECK(enet_hip_verify_batch_device(ctx, d_dg, d_voff, d_vlen, d_slot, d_conn, M, d_ok, NULL, NULL) == 0,
          "verify_batch_device");
    CHECK(enet_hip_synchronize(ctx) == 0, "synchronize");
    CHECK(enet_hip_memcpy_d2h(ctx, ok, d_ok, M) == 0, "memcpy_d2h");
    for (int i = 0; i < M; ++i) CHECK(ok[i] == expect_ok[i], "verify DGRAM %d: ok %d against %d", i, ok[i], expect_ok[i]);

    /* host-memory batch (pinned arena from the library's allocator) */
    uint8_t* pinned = NULL;
    CHECK(enet_hip_host_alloc(arena_bytes, (void**)&pinned) == 0 && pinned, "host_alloc");
    memcpy(pinned, arena, arena_bytes);
    memset(out, 0, N * sizeof *out);
    CHECK(enet_hip_crc32_batch_host(ctx, pinned, arena_bytes, off, len, N, out) == 0, "batch_host");
    for (int i = 0; i < N; ++i) CHECK(out[i] == want[i], "batch_host packet %d", i);

    /* the error contract: rejected before any launch; an empty batch is a no-op */
    CHECK(enet_hip_crc32_batch_device(ctx, NULL, d_off, d_len, N, d_out, NULL) == -1, "null bytes");
    CHECK(enet_hip_crc32_batch_device(ctx, d_arena, d_off, d_len, 0, d_out, NULL) == 0, "empty batch");
    CHECK(enet_hip_crc32_batch_list_device(ctx, list, 0, NULL) == 0, "empty list");

    enet_hip_host_free(pinned);
    void* frees[] = {d_arena, d_off, d_len, d_out, d_dg, d_voff, d_vlen, d_slot, d_conn, d_ok};
    for (size_t k = 0; k < sizeof frees / sizeof frees[0]; ++k) CHECK(enet_hip_device_free(ctx, frees[k]) == 0, "free");
    CHECK(enet_hip_context_destroy(ctx) == 0, "context_destroy");
    free(arena);
    free(dg);
    free(off);
    free(len);
    free(want);
    free(out);
    free(voff);
    free(vlen);
    free(slot);
    free(conn);
    free(expect_ok);
    free(ok);
    printf("c_host: ok (device)\n");
    return 0;
}
