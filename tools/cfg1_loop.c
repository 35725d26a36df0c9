/* cfg1_loop.c -- BASELINE config 1: the per-DGRAM checksum
 * callback as ENet's protocol engine drives it in the loopback echo test
 * (reference Test/TestWave.cs), with the checksum enabled on both hosts.
 *
 * No ENet here (out of scope): the loop restates only what the protocol engine
 * does around host->checksum for one reliable echo round trip, per DGRAM:
 *   send    (c/protocol.cs:1690-1698): slot <- connectID, crc <- checksum(buffers,
 *           bufferCount) over [header+slot][command][payload], slot <- crc;
 *   receive (c/protocol.cs:1052-1068): desired <- slot, slot <- connectID,
 *           crc <- checksum(&whole DGRAM, 1), drop unless crc == desired.
 * DGRAM shapes (include/protocol.cs:55-73, 136-140): ENetProtocolHeader 4 B
 * (peerID with the SENT_TIME flag, sentTime) + the 4-B slot; SendReliable 6 B +
 * payload; Acknowledge 8 B.  One round trip = client send (3 buffers, 270 B),
 * server ack (2 buffers, 16 B), server echo (270 B), client ack (16 B), each
 * stamped once and verified once: 8 checksum calls.
 *
 * Timed for two callbacks over the same DGRAMs: libenethip's enet_hip_crc32
 * (the drop-in CPU callback) and the oracle's byte-serial restatement of
 * ENet.enet_crc32 (c/packet.cs:142-160), which stands in for the C# reference
 * (no .NET toolchain here or on the GPU box: DESIGN.md §3).  Every CRC of the
 * two is compared and every verify must pass.
 *
 *   cfg1_loop <libenethip.so> <liboracle.so> [packets=1024] [payload=256] [min_seconds=1.0]
 * prints one JSON line. */
#define _GNU_SOURCE
#include <dlfcn.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

typedef struct {
    size_t dataLength;
    void* data;
} Buf; /* ENetBuffer: length first (include/win32.cs:25-29) */
typedef uint32_t (*Checksum)(const Buf*, size_t);

enum { HDR = 4, SLOT = 4, CMD_REL = 6, CMD_ACK = 8 };

typedef struct {
    uint8_t hdr[HDR + SLOT];
    uint8_t cmd[CMD_ACK];
    size_t cmd_len;
    const uint8_t* payload;
    size_t payload_len;
    uint8_t wire[HDR + SLOT + CMD_ACK + 4096];
    size_t wire_len;
} Dgram;

static uint64_t sm_state = 0x454E6574ull;
static uint64_t splitmix64(void) {
    uint64_t z = (sm_state += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

static double now_s(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec + 1e-9 * t.tv_nsec;
}

/* protocol.cs:1690-1698: connectID into the slot, CRC over the gather list, CRC into the slot */
static uint32_t stamp(Checksum cb, Dgram* d, uint32_t connect) {
    memcpy(d->hdr + HDR, &connect, 4);
    Buf b[3] = {{HDR + SLOT, d->hdr}, {d->cmd_len, d->cmd}, {d->payload_len, (void*)d->payload}};
    const uint32_t crc = cb(b, d->payload_len ? 3 : 2);
    memcpy(d->hdr + HDR, &crc, 4);
    /* the socket layer sends the buffers back to back (c/win32.cs:168-194) */
    memcpy(d->wire, d->hdr, HDR + SLOT);
    memcpy(d->wire + HDR + SLOT, d->cmd, d->cmd_len);
    if (d->payload_len) /* (an ack carries no payload: payload may be NULL) */
        memcpy(d->wire + HDR + SLOT + d->cmd_len, d->payload, d->payload_len);
    d->wire_len = HDR + SLOT + d->cmd_len + d->payload_len;
    return crc;
}

/* protocol.cs:1052-1068: desired <- slot, slot <- connectID, CRC over the DGRAM, compare */
static int verify(Checksum cb, Dgram* d, uint32_t connect, uint32_t* computed) {
    uint32_t desired;
    memcpy(&desired, d->wire + HDR, 4);
    memcpy(d->wire + HDR, &connect, 4);
    Buf b = {d->wire_len, d->wire};
    *computed = cb(&b, 1);
    memcpy(d->wire + HDR, &desired, 4);
    return *computed == desired;
}

static void make_reliable(Dgram* d, uint16_t peer, uint16_t seq, const uint8_t* payload, size_t n) {
    const uint16_t pid = (uint16_t)(peer | 0x8000u); /* ENET_PROTOCOL_HEADER_FLAG_SENT_TIME = 1 << 15 */
    const uint16_t sent = (uint16_t)(seq * 7u);
    d->hdr[0] = (uint8_t)(pid >> 8), d->hdr[1] = (uint8_t)pid; /* network order */
    d->hdr[2] = (uint8_t)(sent >> 8), d->hdr[3] = (uint8_t)sent;
    d->cmd[0] = 6 | 0x80; /* ENET_PROTOCOL_COMMAND_SEND_RELIABLE | ACKNOWLEDGE flag */
    d->cmd[1] = 0;
    d->cmd[2] = (uint8_t)(seq >> 8), d->cmd[3] = (uint8_t)seq;
    d->cmd[4] = (uint8_t)(n >> 8), d->cmd[5] = (uint8_t)n;
    d->cmd_len = CMD_REL;
    d->payload = payload;
    d->payload_len = n;
}

static void make_ack(Dgram* d, uint16_t peer, uint16_t seq) {
    const uint16_t pid = (uint16_t)(peer | 0x8000u); /* SENT_TIME */
    const uint16_t sent = (uint16_t)(seq * 7u + 1u);
    d->hdr[0] = (uint8_t)(pid >> 8), d->hdr[1] = (uint8_t)pid;
    d->hdr[2] = (uint8_t)(sent >> 8), d->hdr[3] = (uint8_t)sent;
    d->cmd[0] = 1; /* ENET_PROTOCOL_COMMAND_ACKNOWLEDGE */
    d->cmd[1] = 0xFF;
    d->cmd[2] = (uint8_t)(seq >> 8), d->cmd[3] = (uint8_t)seq;
    d->cmd[4] = (uint8_t)(seq >> 8), d->cmd[5] = (uint8_t)seq;
    d->cmd[6] = (uint8_t)((seq * 7u) >> 8), d->cmd[7] = (uint8_t)(seq * 7u);
    d->cmd_len = CMD_ACK;
    d->payload = NULL;
    d->payload_len = 0;
}

typedef struct {
    double seconds;
    long reps, calls, verify_fail;
    uint64_t bytes;
    uint32_t digest;
} Run;

/* one pass: every round trip's 4 DGRAMs stamped and verified; crcs[] collects the stamps */
static void pass(Checksum cb, Dgram* dg, long packets, uint32_t* crcs, Run* r) {
    const uint32_t connect = 0x1234ABCDu;
    for (long i = 0; i < packets; ++i) {
        for (int q = 0; q < 4; ++q) {
            Dgram* d = &dg[4 * i + q];
            const uint32_t c = stamp(cb, d, connect);
            uint32_t got;
            if (!verify(cb, d, connect, &got)) r->verify_fail++;
            crcs[4 * i + q] = c;
            r->digest = r->digest * 31u + c;
            r->calls += 2;
            r->bytes += 2 * d->wire_len;
        }
    }
}

static Run timed(Checksum cb, Dgram* dg, long packets, uint32_t* crcs, double min_s) {
    Run r;
    memset(&r, 0, sizeof r);
    pass(cb, dg, packets, crcs, &r); /* warm */
    memset(&r, 0, sizeof r);
    const double t0 = now_s();
    do {
        pass(cb, dg, packets, crcs, &r);
        r.reps++;
    } while (now_s() - t0 < min_s);
    r.seconds = now_s() - t0;
    return r;
}

int main(int argc, char** argv) {
    if (argc < 3) {
        fprintf(stderr, "usage: %s libenethip.so liboracle.so [packets] [payload] [min_seconds]\n", argv[0]);
        return 2;
    }
    const long packets = argc > 3 ? atol(argv[3]) : 1024;
    const size_t plen = argc > 4 ? (size_t)atol(argv[4]) : 256;
    const double min_s = argc > 5 ? atof(argv[5]) : 1.0;
    if (packets <= 0 || plen > 4096 - 14) return 2;
    void* hl = dlopen(argv[1], RTLD_NOW | RTLD_LOCAL);
    void* ol = dlopen(argv[2], RTLD_NOW | RTLD_LOCAL);
    if (!hl || !ol) {
        fprintf(stderr, "dlopen: %s\n", dlerror());
        return 2;
    }
    Checksum lib = (Checksum)dlsym(hl, "enet_hip_crc32");
    Checksum ora = (Checksum)dlsym(ol, "oracle_enet_crc32");
    if (!lib || !ora) {
        fprintf(stderr, "dlsym failed\n");
        return 2;
    }
    uint8_t* payload = malloc((size_t)packets * plen + 1);
    for (size_t i = 0; i < (size_t)packets * plen; i += 8) {
        const uint64_t v = splitmix64();
        memcpy(payload + i, &v, ((size_t)packets * plen - i) < 8 ? ((size_t)packets * plen - i) : 8);
    }
    Dgram* dg = calloc((size_t)packets * 4, sizeof(Dgram));
    for (long i = 0; i < packets; ++i) {
        const uint16_t seq = (uint16_t)(i + 1);
        make_reliable(&dg[4 * i + 0], 0, seq, payload + (size_t)i * plen, plen); /* client send */
        make_ack(&dg[4 * i + 1], 0, seq);                                       /* server ack */
        make_reliable(&dg[4 * i + 2], 0, seq, payload + (size_t)i * plen, plen); /* server echo */
        make_ack(&dg[4 * i + 3], 0, seq);                                       /* client ack */
    }
    uint32_t* c_lib = malloc(sizeof(uint32_t) * 4 * (size_t)packets);
    uint32_t* c_ora = malloc(sizeof(uint32_t) * 4 * (size_t)packets);
    const Run rl = timed(lib, dg, packets, c_lib, min_s);
    const Run ro = timed(ora, dg, packets, c_ora, min_s);
    long mismatch = 0;
    for (long i = 0; i < 4 * packets; ++i) mismatch += c_lib[i] != c_ora[i];
    const double dg_per_pass = 4.0 * packets;
    printf("{\"config\": \"cfg1: loopback echo round trips, checksum on both hosts\", \"packets\": %ld, "
           "\"payload\": %zu, \"dgrams_per_round_trip\": 4, \"checksum_calls_per_round_trip\": 8, "
           "\"callback\": {\"name\": \"enet_hip_crc32 (libenethip, CPU)\", \"round_trips_per_s\": %.1f, "
           "\"calls_per_s\": %.1f, \"ns_per_call\": %.1f, \"GiBps\": %.3f, \"verify_fail\": %ld}, "
           "\"reference_port\": {\"name\": \"oracle_enet_crc32 (byte-serial restatement of packet.cs:142-160)\", "
           "\"round_trips_per_s\": %.1f, \"calls_per_s\": %.1f, \"ns_per_call\": %.1f, \"GiBps\": %.3f, "
           "\"verify_fail\": %ld}, \"bytes_per_round_trip\": %.1f, \"mismatch\": %ld, \"speedup\": %.2f}\n",
           packets, plen, rl.reps * packets / rl.seconds, rl.calls / rl.seconds, 1e9 * rl.seconds / rl.calls,
           rl.bytes / rl.seconds / 1073741824.0, rl.verify_fail, ro.reps * packets / ro.seconds,
           ro.calls / ro.seconds, 1e9 * ro.seconds / ro.calls, ro.bytes / ro.seconds / 1073741824.0, ro.verify_fail,
           (double)rl.bytes / rl.reps / packets, mismatch, (ro.seconds / ro.calls) / (rl.seconds / rl.calls));
    (void)dg_per_pass;
    free(c_lib);
    free(c_ora);
    free(dg);
    free(payload);
    return (mismatch || rl.verify_fail || ro.verify_fail) ? 1 : 0;
}
