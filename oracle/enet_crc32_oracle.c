/*
 * enet_crc32_oracle.c -- CPU ORACLE for the ENet per-datagram CRC32 path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the shipped library links or calls this
 * file; only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load it, and only as the checker (or as the timed CPU baseline, kind "port").
 *
 * It is a plain-C restatement of the reference algorithm in
 *   /root/reference/enet-csharp/ENet/c/packet.cs
 *     :106-140  crcTable  (256 x uint32, reflected poly 0xEDB88320)
 *     :142-160  enet_crc32(ENetBuffer* buffers, nuint bufferCount)
 *   /root/reference/enet-csharp/ENet/include/win32.cs
 *     :18       ENET_HOST_TO_NET_32  (ReverseEndianness on little-endian)
 *     :25-29    struct ENetBuffer { nuint dataLength; void* data; }  (length FIRST)
 * and of the two checksum call sites in c/protocol.cs (:1052-1068 receive
 * verify, :1690-1698 send stamp), used by the batched verify oracle below.
 *
 * Parity pinning: the reference's own tests pin no CRC value;
 * the C# reference cannot be built here (no dotnet/mono).  This restatement is
 * pinned instead by (1) the reference's crcTable, extracted verbatim from
 * packet.cs:106-140 into tests/golden/crc_table_ref.json by
 * tests/golden/make_golden.py and compared entry-for-entry with the table
 * generated here, (2) the CRC-32/ISO-HDLC check value (crc32("123456789") =
 * 0xCBF43926, i.e. enet_crc32 = 0x2639F4CB on little-endian), and (3) zlib.crc32
 * on every golden vector.
 */
#include <stddef.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* include/win32.cs:25-29 -- Win32 WSABUF order: length first, then pointer. */
typedef struct {
    size_t dataLength;
    const void* data;
} OracleENetBuffer;

static uint32_t g_table[256];
static int g_table_ready = 0;

/* The reference ships the table as a literal (packet.cs:106-140); we regenerate
 * it from the polynomial and check it against the literal in the tests. */
static void oracle_init_table(void) {
    if (g_table_ready) return;
    for (uint32_t n = 0; n < 256; ++n) {
        uint32_t c = n;
        for (int k = 0; k < 8; ++k) c = (c & 1u) ? (c >> 1) ^ 0xEDB88320u : (c >> 1);
        g_table[n] = c;
    }
    g_table_ready = 1;
}

/* ENET_HOST_TO_NET_32 on a little-endian host (include/win32.cs:18). */
static uint32_t oracle_host_to_net_32(uint32_t v) {
    return (v >> 24) | ((v >> 8) & 0x0000FF00u) | ((v << 8) & 0x00FF0000u) | (v << 24);
}

void oracle_crc_table(uint32_t* out256) {
    oracle_init_table();
    memcpy(out256, g_table, sizeof(g_table));
}

/* packet.cs:142-160, byte for byte: init 0xFFFFFFFF (:144), for each buffer in
 * order (:146-157), for each byte crc = (crc >> 8) ^ T[(crc & 0xFF) ^ b] (:153),
 * return ENET_HOST_TO_NET_32(~crc) (:159). */
uint32_t oracle_enet_crc32(const OracleENetBuffer* buffers, size_t bufferCount) {
    oracle_init_table();
    uint32_t crc = 0xFFFFFFFFu;
    while (bufferCount-- > 0) {
        const uint8_t* data = (const uint8_t*)buffers->data;
        const uint8_t* dataEnd = data + buffers->dataLength;
        while (data < dataEnd) crc = (crc >> 8) ^ g_table[(crc & 0xFFu) ^ *data++];
        ++buffers;
    }
    return oracle_host_to_net_32(~crc);
}

/* Batched form used by the parity tests: packet i is bytes[off[i] .. off[i]+len[i]). */
void oracle_crc32_batch(const uint8_t* bytes, const uint64_t* off, const uint32_t* len,
                        size_t n, uint32_t* out) {
    for (size_t i = 0; i < n; ++i) {
        OracleENetBuffer b = {len[i], bytes + off[i]};
        out[i] = oracle_enet_crc32(&b, 1);
    }
}

/* Same, multithreaded over the host cores by static contiguous partitioning
 * (SURVEY.md §8d "all cores"); each thread runs the byte-serial reference loop. */
#include <pthread.h>
typedef struct {
    const uint8_t* bytes; const uint64_t* off; const uint32_t* len; uint32_t* out;
    size_t lo, hi;
} oracle_job;
static void* oracle_worker(void* p) {
    oracle_job* j = (oracle_job*)p;
    oracle_crc32_batch(j->bytes, j->off + j->lo, j->len + j->lo, j->hi - j->lo, j->out + j->lo);
    return NULL;
}
int oracle_crc32_batch_mt(const uint8_t* bytes, const uint64_t* off, const uint32_t* len,
                          size_t n, uint32_t* out, int threads) {
    oracle_init_table();
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    pthread_t tid[256];
    oracle_job jobs[256];
    for (int t = 0; t < threads; ++t) {
        jobs[t].bytes = bytes; jobs[t].off = off; jobs[t].len = len; jobs[t].out = out;
        jobs[t].lo = n * (size_t)t / (size_t)threads;
        jobs[t].hi = n * (size_t)(t + 1) / (size_t)threads;
        if (pthread_create(&tid[t], NULL, oracle_worker, &jobs[t]) != 0) return -1;
    }
    for (int t = 0; t < threads; ++t) pthread_join(tid[t], NULL);
    return 0;
}

/* Gather-list batch (send path, protocol.cs:1690-1698 passes host->buffers with
 * bufferCount <= 65): DGRAM i is segments seg_first[i] .. seg_first[i+1]-1, each
 * segment a (offset,length) into `bytes`. */
void oracle_crc32_gather(const uint8_t* bytes, const uint64_t* seg_off, const uint32_t* seg_len,
                         const uint32_t* seg_first, size_t n_dgrams, uint32_t* out) {
    enum { CHUNK = 65 }; /* ENET_BUFFER_MAXIMUM, include/enet.cs:417 */
    OracleENetBuffer bufs[CHUNK];
    for (size_t i = 0; i < n_dgrams; ++i) {
        uint32_t a = seg_first[i], b = seg_first[i + 1];
        size_t k = 0;
        for (uint32_t s = a; s < b && k < CHUNK; ++s, ++k) {
            bufs[k].dataLength = seg_len[s];
            bufs[k].data = bytes + seg_off[s];
        }
        out[i] = oracle_enet_crc32(bufs, k); /* callers keep b - a <= 65 */
    }
}

/* Batched receive verify (protocol.cs:1052-1068): desired = slot; slot = connectID
 * (or 0 when there is no peer); crc over the whole DGRAM; drop on mismatch.  The
 * slot sits at slot_off[i] bytes into DGRAM i.  `bytes` is NOT modified: the
 * substitution is applied on a private copy (heap, as long as the longest DGRAM:
 * no length limit beyond the reference's).  A slot that does not lie wholly inside
 * the DGRAM (slot_off + 4 > L) is dropped (ok = 0, computed = 0): the reference
 * reads those bytes from past receivedDataLength in its 4096-byte receive buffer
 * (protocol.cs:1001-1014 check only L >= 2), which a batch API has no content for. */
void oracle_verify_batch(const uint8_t* bytes, const uint64_t* off, const uint32_t* len,
                         const uint32_t* slot_off, const uint32_t* connect_id, size_t n,
                         uint8_t* ok, uint32_t* computed) {
    uint32_t maxL = 8;
    for (size_t i = 0; i < n; ++i)
        if (len[i] > maxL) maxL = len[i];
    uint8_t* tmp = (uint8_t*)malloc(maxL);
    if (!tmp) abort();
    for (size_t i = 0; i < n; ++i) {
        uint32_t L = len[i];
        if ((uint64_t)slot_off[i] + 4u > L) { ok[i] = 0; if (computed) computed[i] = 0; continue; }
        memcpy(tmp, bytes + off[i], L);
        uint32_t desired;
        memcpy(&desired, tmp + slot_off[i], 4);
        uint32_t sub = connect_id[i];
        memcpy(tmp + slot_off[i], &sub, 4);
        OracleENetBuffer b = {L, tmp};
        uint32_t c = oracle_enet_crc32(&b, 1);
        if (computed) computed[i] = c;
        ok[i] = (c == desired) ? 1 : 0;
    }
    free(tmp);
}

/* Batched fragment reassembly, sequential, as c/protocol.cs:529-637
 * (enet_protocol_handle_send_fragment) treats each command once the caller has
 * matched its reassembly slot: the -1 checks of 546-552 / 571-577 / 598-601, the
 * bitmap duplicate test (619), --fragmentsRemaining (621), the bit set (623) and
 * the memcpy with the length clamp (625-630).  Command fields are network order
 * (include/protocol.cs:156-165).  status: -1 rejected, 0 skipped/duplicate, 1 copied. */
static uint32_t be16_(const uint8_t* p) { return ((uint32_t)p[0] << 8) | p[1]; }
static uint32_t be32_(const uint8_t* p) {
    return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}
void oracle_fragment_reassemble(const uint8_t* bytes, const uint64_t* cmd_off, const uint32_t* cmd_avail,
                                const int32_t* slots, size_t n, uint32_t max_packet, uint8_t* msg_bytes,
                                const uint64_t* msg_off, const uint32_t* msg_len, const uint32_t* msg_count,
                                uint32_t* fragments, uint32_t words, uint32_t* remaining, size_t slot_count,
                                int8_t* status) {
    for (size_t i = 0; i < n; ++i) {
        int32_t s = slots[i];
        if (s < 0) { status[i] = 0; continue; }
        if ((size_t)s >= slot_count) { status[i] = -1; continue; }
        const uint8_t* c = bytes + cmd_off[i];
        uint32_t fragmentLength = be16_(c + 6);
        uint32_t fragmentCount = be32_(c + 8), fragmentNumber = be32_(c + 12);
        uint32_t totalLength = be32_(c + 16), fragmentOffset = be32_(c + 20);
        if (fragmentLength == 0 || fragmentLength > max_packet || fragmentLength > cmd_avail[i]) { status[i] = -1; continue; }
        if (fragmentCount > 1024u * 1024u || fragmentNumber >= fragmentCount || totalLength > max_packet ||
            totalLength < fragmentCount || fragmentOffset >= totalLength || fragmentLength > totalLength - fragmentOffset) {
            status[i] = -1;
            continue;
        }
        if (totalLength != msg_len[s] || fragmentCount != msg_count[s]) { status[i] = -1; continue; }
        if (fragmentCount > 32u * words) { status[i] = -1; continue; }
        uint32_t* fr = fragments + (size_t)s * words;
        if ((fr[fragmentNumber / 32] & (1u << (fragmentNumber % 32))) == 0) {
            --remaining[s];
            fr[fragmentNumber / 32] |= 1u << (fragmentNumber % 32);
            if (fragmentOffset + fragmentLength > msg_len[s]) fragmentLength = msg_len[s] - fragmentOffset;
            memcpy(msg_bytes + msg_off[s] + fragmentOffset, c + 24, fragmentLength);
            status[i] = 1;
        } else {
            status[i] = 0;
        }
    }
}
