/*
 * dropin_caller.c — a plain C caller of the drop-in (tests/test_boundary_cpu.py).
 *
 * Built against host/net_util_mi355x.c in one of its modes and linked with libnetcsum_mi355x.so
 * (tests/c/Makefile): standalone (include/netcsum_netbuf.h layout) or in-stack (-DNETCSUM_IN_STACK
 * with the stand-in stack headers of tests/instack/, whose NET_BUF layout differs), with or without
 * the NET_ERR_CFG_ARG_CHK_DBG_EN checks (NETCSUM_TEST_DBG), under -fsanitize=address,undefined on
 * the CPU. It builds real NET_BUF chains (1 to 1000 buffers, odd lengths, empty middles, every
 * protocol type's index selection), and checks
 *   - NetUtil_MI355X_ChainToSpans against the caller's own concatenation of the chain,
 *   - the four functions against an RFC 1071 sum of that concatenation written here,
 *   - the error paths (invalid protocol; with DBG: NULL, size 0, zero-length chain, ix NONE),
 *   - two threads calling the drop-in at once (each its own chains), their first CRC calls racing
 *     for the host table's one-time build (the tsan variant checks for data races).
 * Without a GPU every device call must FAIL with NET_UTIL_ERR_MI355X_DEV (no CPU fallback); with
 * one (NETCSUM_EXPECT_GPU=1) every call must succeed and match. Exit status 0 = all checks passed.
 */
#ifdef NETCSUM_IN_STACK
#include <cpu_core.h>
#include <net_util.h>
#include <net_buf.h>
#define NETCSUM_HAVE_MICRIUM_TYPES 1
#include "netcsum_mi355x.h"
#else
#include "netcsum_mi355x.h"
#include "netcsum_netbuf.h"
#endif

#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static int g_fail, g_checks, g_dev_ok, g_dev_missing, g_expect_gpu;

#define CHECK(cond, ...)                                              \
    do {                                                              \
        __atomic_fetch_add(&g_checks, 1, __ATOMIC_RELAXED);           \
        if (!(cond)) {                                                \
            __atomic_fetch_add(&g_fail, 1, __ATOMIC_RELAXED);         \
            fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__);      \
            fprintf(stderr, __VA_ARGS__);                             \
            fputc('\n', stderr);                                      \
        }                                                             \
    } while (0)

static __thread uint64_t rng_state = 0x9E3779B97F4A7C15ull;
static uint32_t rnd(void)
{
    rng_state ^= rng_state << 13;
    rng_state ^= rng_state >> 7;
    rng_state ^= rng_state << 17;
    return (uint32_t)(rng_state >> 11);
}

/* RFC 1071 over one contiguous byte string: big-endian words, odd tail padded, u32 sum. */
static uint32_t rfc1071_sum32(const uint8_t *p, size_t n)
{
    uint32_t s = 0;
    size_t i;
    for (i = 0; i + 1 < n; i += 2) s += (uint32_t)p[i] << 8 | p[i + 1];
    if (n & 1u) s += (uint32_t)p[n - 1] << 8;
    return s;
}
static uint16_t fold(uint32_t s)
{
    while (s >> 16) s = (s & 0xFFFFu) + (s >> 16);
    return (uint16_t)s;
}
static uint16_t bswap(uint16_t v) { return (uint16_t)(v << 8 | v >> 8); }

/* A chain of n buffers; each buffer's checksummed piece is placed via its protocol's fields. */
typedef struct {
    NET_BUF  *bufs;
    uint8_t **mem;
    uint8_t  *stream;          /* the caller's own concatenation (pseudo-header first) */
    size_t    stream_len;
    uint32_t  n;
} chain_t;

static void chain_build(chain_t *c, uint32_t n, const uint8_t *ph, uint16_t plen)
{
    static const int protos[] = { NET_PROTOCOL_TYPE_UDP_V4, NET_PROTOCOL_TYPE_TCP_V4, NET_PROTOCOL_TYPE_ICMP_V4,
                                  NET_PROTOCOL_TYPE_ICMP_V6, NET_PROTOCOL_TYPE_UDP_V6, NET_PROTOCOL_TYPE_TCP_V6,
                                  NET_PROTOCOL_TYPE_IP_V6_EXT_NONE };
    uint32_t i;
    size_t cap = plen;
    c->n = n;
    c->bufs = calloc(n ? n : 1, sizeof(NET_BUF));
    c->mem = calloc(n ? n : 1, sizeof(uint8_t *));
    for (i = 0; i < n; ++i) cap += 700;
    c->stream = malloc(cap + 1);
    memcpy(c->stream, ph, plen);
    c->stream_len = plen;
    for (i = 0; i < n; ++i) {
        NET_BUF_HDR *h = &c->bufs[i].Hdr;
        uint16_t len = (i % 11u == 5u) ? 0u : (uint16_t)(rnd() % 600u + 1u);
        uint16_t lead = (uint16_t)(rnd() % 40u), hdr = (uint16_t)(len ? rnd() % (len < 60u ? len : 60u) : 0u);
        uint8_t *m = malloc((size_t)lead + len + 8u);
        uint32_t k;
        for (k = 0; k < (uint32_t)lead + len + 8u; ++k) m[k] = (uint8_t)rnd();
        c->mem[i] = m;
        c->bufs[i].DataPtr = m + (rnd() & 3u);          /* odd data addresses */
        h->ProtocolHdrType = (NET_PROTOCOL_TYPE)protos[rnd() % 7u];
        switch ((int)h->ProtocolHdrType) {
        case NET_PROTOCOL_TYPE_ICMP_V4:
        case NET_PROTOCOL_TYPE_ICMP_V6:
            h->ICMP_MsgIx = lead; h->ICMP_HdrLen = hdr; h->DataLen = (uint16_t)(len - hdr);
            break;
        case NET_PROTOCOL_TYPE_IP_V6_EXT_NONE:
            h->TotLen = (uint16_t)(lead + len); h->DataLen = len;
            break;
        default:
            h->TransportHdrIx = lead; h->TransportHdrLen = hdr; h->DataLen = (uint16_t)(len - hdr);
        }
        h->NextBufPtr = (i + 1u < n) ? &c->bufs[i + 1u] : NULL;
        memcpy(c->stream + c->stream_len, c->bufs[i].DataPtr + lead, len);
        c->stream_len += len;
    }
    if (n == 0 && (plen & 1u)) c->stream_len -= 1u;     /* net_util.c:1601-1611: dropped octet */
}

static void chain_free(chain_t *c)
{
    uint32_t i;
    for (i = 0; i < c->n; ++i) free(c->mem[i]);
    free(c->mem);
    free(c->bufs);
    free(c->stream);
}

/* One device call's outcome: counts it, and checks the no-fallback rule without a GPU. */
static int dev_result(NET_ERR err, const char *what)
{
    if ((unsigned)err == NET_UTIL_ERR_NONE) {
        __atomic_fetch_add(&g_dev_ok, 1, __ATOMIC_RELAXED);
        return 1;
    }
    __atomic_fetch_add(&g_dev_missing, 1, __ATOMIC_RELAXED);
    CHECK((unsigned)err == NET_UTIL_ERR_MI355X_DEV && !g_expect_gpu, "%s: err %u", what, (unsigned)err);
    return 0;
}

static void check_chain(uint32_t nbuf, uint16_t plen)
{
    uint8_t ph[40];
    chain_t c;
    NETCSUM_SPAN *spans;
    uint32_t need = 0, got = 0, i;
    size_t pos = 0;
    NET_ERR err;
    uint16_t v, want;
    CPU_BOOLEAN ok;
    for (i = 0; i < sizeof ph; ++i) ph[i] = (uint8_t)rnd();
    chain_build(&c, nbuf, ph, plen);

    err = NetUtil_MI355X_ChainToSpans(nbuf ? c.bufs : NULL, plen ? ph : NULL, plen, NULL, 0, &need, 0);
    CHECK((unsigned)err == NET_UTIL_ERR_NONE, "count walk err %u (n=%u)", (unsigned)err, nbuf);
    spans = malloc(sizeof(NETCSUM_SPAN) * (need ? need : 1));
    err = NetUtil_MI355X_ChainToSpans(nbuf ? c.bufs : NULL, plen ? ph : NULL, plen, spans, need, &got, 0);
    CHECK((unsigned)err == NET_UTIL_ERR_NONE && got == need, "walk err %u got %u need %u", (unsigned)err, got, need);
    for (i = 0; i < got && pos <= c.stream_len; ++i) {
        CHECK(pos + spans[i].len <= c.stream_len && memcmp(spans[i].p, c.stream + pos, spans[i].len) == 0,
              "span %u of %u-buffer chain differs", i, nbuf);
        pos += spans[i].len;
    }
    CHECK(pos == c.stream_len, "spans cover %zu of %zu bytes (n=%u)", pos, c.stream_len, nbuf);
    free(spans);

#ifdef NETCSUM_TEST_DBG
    if (nbuf == 0) {                                       /* DBG: NULL chain (net_util.c:1566-1570) */
        v = NetUtil_16BitOnesCplChkSumDataCalc(NULL, plen ? ph : NULL, plen, &err);
        CHECK(v == 0 && (unsigned)err == NET_ERR_FAULT_NULL_PTR, "DBG DataCalc(NULL) -> %u", (unsigned)err);
        chain_free(&c);
        return;
    }
#endif
    want = bswap((uint16_t)~fold(rfc1071_sum32(c.stream, c.stream_len)));
    v = NetUtil_16BitOnesCplChkSumDataCalc(nbuf ? c.bufs : NULL, plen ? ph : NULL, plen, &err);
    if (dev_result(err, "DataCalc")) CHECK(v == want, "DataCalc n=%u plen=%u: %04x != %04x", nbuf, plen, v, want);
    ok = NetUtil_16BitOnesCplChkSumDataVerify(nbuf ? c.bufs : NULL, plen ? ph : NULL, plen, &err);
    if (dev_result(err, "DataVerify")) {
        CHECK(ok == (bswap(fold(rfc1071_sum32(c.stream, c.stream_len))) == 0xFFFFu ? DEF_OK : DEF_FAIL),
              "DataVerify n=%u", nbuf);
    }
    chain_free(&c);
}

static void check_headers(void)
{
    static const uint8_t kat[20] = { 0x45, 0x00, 0x00, 0x73, 0x00, 0x00, 0x40, 0x00, 0x40, 0x11,
                                     0x00, 0x00, 0xc0, 0xa8, 0x00, 0x01, 0xc0, 0xa8, 0x00, 0xc7 };
    uint8_t hdr[21];
    NET_ERR err;
    uint16_t v;
    memcpy(hdr + 1, kat, 20);                              /* odd address */
    v = NetUtil_16BitOnesCplChkSumHdrCalc(hdr + 1, 20, &err);
    if (dev_result(err, "HdrCalc")) {
        CPU_BOOLEAN ok;
        CHECK(v == 0x61B8u, "IPv4 KAT %04x", v);
        memcpy(hdr + 11, &v, 2);                           /* NET_UTIL_VAL_COPY_16 of the host-order value */
        ok = NetUtil_16BitOnesCplChkSumHdrVerify(hdr + 1, 20, &err);
        if (dev_result(err, "HdrVerify")) CHECK(ok == DEF_OK, "HdrVerify of the KAT");
    }
}

static void check_errors(void)
{
    NET_BUF b[2];
    uint8_t data[64] = { 1, 2, 3 };
    NET_ERR err;
    memset(b, 0, sizeof b);
    b[0].DataPtr = data;
    b[0].Hdr.ProtocolHdrType = NET_PROTOCOL_TYPE_IGMP;      /* net_util.c:1637-1639 */
    b[0].Hdr.DataLen = 8;
    CHECK(NetUtil_16BitOnesCplChkSumDataCalc(b, NULL, 0, &err) == 0 &&
          (unsigned)err == NET_UTIL_ERR_INVALID_PROTOCOL, "invalid protocol -> %u", (unsigned)err);
    CHECK(NetUtil_16BitOnesCplChkSumDataVerify(b, NULL, 0, &err) == DEF_FAIL &&
          (unsigned)err == NET_UTIL_ERR_INVALID_PROTOCOL, "invalid protocol (verify) -> %u", (unsigned)err);
#ifdef NETCSUM_TEST_DBG
    /* NET_ERR_CFG_ARG_CHK_DBG_EN paths, all before any device work. */
    CHECK(NetUtil_16BitOnesCplChkSumHdrCalc(NULL, 20, &err) == 0 && (unsigned)err == NET_ERR_FAULT_NULL_PTR,
          "HdrCalc(NULL) -> %u (net_util.c:168-172)", (unsigned)err);
    CHECK(NetUtil_16BitOnesCplChkSumHdrVerify(data, 0, &err) == DEF_FAIL && (unsigned)err == NET_UTIL_ERR_NULL_SIZE,
          "HdrVerify(size 0) -> %u (net_util.c:261-265)", (unsigned)err);
    CHECK(NetUtil_16BitOnesCplChkSumHdrCalc(data, 0, &err) == 0 && (unsigned)err == NET_UTIL_ERR_NULL_SIZE,
          "HdrCalc(size 0) -> %u (net_util.c:174-178)", (unsigned)err);
    CHECK(NetUtil_16BitOnesCplChkSumDataCalc(NULL, data, 12, &err) == 0 && (unsigned)err == NET_ERR_FAULT_NULL_PTR,
          "DataCalc(NULL) -> %u (net_util.c:1566-1570)", (unsigned)err);
    b[0].Hdr.ProtocolHdrType = NET_PROTOCOL_TYPE_UDP_V4;
    b[0].Hdr.DataLen = 0;
    b[0].Hdr.TransportHdrLen = 0;
    CHECK(NetUtil_16BitOnesCplChkSumDataCalc(b, NULL, 0, &err) == 0 && (unsigned)err == NET_UTIL_ERR_NULL_SIZE,
          "single zero-length buffer -> %u (net_util.c:1660-1672)", (unsigned)err);
    b[0].Hdr.DataLen = 8;
    b[0].Hdr.TransportHdrIx = NET_BUF_IX_NONE;
    CHECK(NetUtil_16BitOnesCplChkSumDataVerify(b, NULL, 0, &err) == DEF_FAIL &&
          (unsigned)err == NET_BUF_ERR_INVALID_IX, "ix NONE -> %u (net_util.c:1642-1647)", (unsigned)err);
#else
    {   /* DBG checks off: size 0 is a legal header (0xFFFF) and reaches the device path. */
        uint16_t v = NetUtil_16BitOnesCplChkSumHdrCalc(data, 0, &err);
        if (dev_result(err, "HdrCalc(size 0)")) CHECK(v == 0xFFFFu, "HdrCalc(size 0) = %04x", v);
    }
#endif
}

/* CRC-32 drop-ins (net_util.c:485-636): the EXT argument checks answered on the host, the
 * complement relation, the CRC-32 check value and MAC hashes on the host (calls of up to 4096
 * octets), a 5000-octet buffer through the device, and the bit reflection. */
static uint32_t crc_bitwise(const uint8_t *p, uint32_t n)
{
    uint32_t c = 0xFFFFFFFFu, i, j;
    for (i = 0; i < n; ++i) {
        c ^= p[i];
        for (j = 0; j < 8; ++j) c = (c & 1u) ? (c >> 1) ^ 0xEDB88320u : c >> 1;
    }
    return c;
}

static void check_crc(void)
{
    static uint8_t kat[] = "123456789";
    uint8_t mac[6] = { 0x01, 0x00, 0x5E, 0x12, 0x34, 0x56 };
    NET_ERR err;
    CPU_INT32U v;
    uint32_t i, r;
    CHECK(NetUtil_32BitCRC_Calc(NULL, 6, &err) == 0u && (unsigned)err == NET_ERR_FAULT_NULL_PTR,
          "CRC(NULL) -> %u (net_util.c:499-503)", (unsigned)err);
    CHECK(NetUtil_32BitCRC_CalcCpl(mac, 0, &err) == 0u && (unsigned)err == NET_UTIL_ERR_NULL_SIZE,
          "CRC(len 0) -> %u (net_util.c:504-508)", (unsigned)err);
    v = NetUtil_32BitCRC_CalcCpl(kat, 9, &err);
    CHECK((unsigned)err == NET_UTIL_ERR_NONE && v == 0xCBF43926u, "CRC-32 check value %08x", (unsigned)v);
    v = NetUtil_32BitCRC_Calc(mac, 6, &err);
    CHECK((unsigned)err == NET_UTIL_ERR_NONE && v == crc_bitwise(mac, 6), "CRC of a MAC %08x (host)", (unsigned)v);
    {
        static uint8_t big[5000];
        for (i = 0; i < sizeof big; ++i) big[i] = (uint8_t)(i * 131u + 7u);
        v = NetUtil_32BitCRC_Calc(big, 4096, &err);
        CHECK((unsigned)err == NET_UTIL_ERR_NONE && v == crc_bitwise(big, 4096), "CRC of 4096 B %08x", (unsigned)v);
        v = NetUtil_32BitCRC_Calc(big, sizeof big, &err);
        if (dev_result(err, "CRC32 Calc 5000 B")) CHECK(v == crc_bitwise(big, sizeof big), "CRC of 5000 B %08x", (unsigned)v);
    }
    for (i = 0; i < 32; ++i) {
        r = NetUtil_32BitReflect(1u << i);
        CHECK(r == (1u << (31u - i)), "Reflect(bit %u) = %08x", i, r);
    }
    CHECK(NetUtil_32BitReflect(0x12345678u) == 0x1E6A2C48u, "Reflect(0x12345678)");
}

static pthread_barrier_t g_start;

/* Both threads start together, so their first CRC calls race for the host table's one-time build
 * (pthread_once in net_util_mi355x.c); the -fsanitize=thread variant (tsan) checks that race and the
 * chain walks for data races. */
static void *thread_main(void *arg)
{
    uint32_t t = (uint32_t)(uintptr_t)arg, k, i;
    uint8_t buf[300];
    NET_ERR err;
    pthread_barrier_wait(&g_start);
    for (k = 0; k < 64; ++k) {
        for (i = 0; i < sizeof buf; ++i) buf[i] = (uint8_t)(i * 7u + k + t);
        CHECK(NetUtil_32BitCRC_Calc(buf, 6u + k * 4u, &err) == crc_bitwise(buf, 6u + k * 4u) &&
              (unsigned)err == NET_UTIL_ERR_NONE, "thread %u CRC %u", t, k);
    }
    for (k = 0; k < 40; ++k) check_chain(1u + (k % 9u) * 7u, (uint16_t)((k & 1u) ? 12u : 11u));
    NetUtil_MI355X_ThreadRelease();
    return NULL;
}

int main(void)
{
    static const uint32_t lens[] = { 0, 1, 2, 3, 63, 64, 65, 120, 200, 1000 };
    static const uint16_t plens[] = { 0, 1, 11, 12, 40 };
    const char *e = getenv("NETCSUM_EXPECT_GPU");
    uint32_t i, j;
    pthread_t th[2];
    g_expect_gpu = e && e[0] == '1';
    /* two host threads on the same device, each with its own chains and context, started first so
     * that they make the process's first CRC calls */
    pthread_barrier_init(&g_start, NULL, 2);
    for (i = 0; i < 2; ++i) pthread_create(&th[i], NULL, thread_main, (void *)(uintptr_t)i);
    for (i = 0; i < 2; ++i) pthread_join(th[i], NULL);
    pthread_barrier_destroy(&g_start);
    for (i = 0; i < sizeof lens / sizeof lens[0]; ++i) {
        for (j = 0; j < sizeof plens / sizeof plens[0]; ++j) check_chain(lens[i], plens[j]);
    }
    check_headers();
    check_errors();
    check_crc();
    NetUtil_MI355X_ThreadRelease();
    printf("%s checks=%d failed=%d device_ok=%d device_missing=%d\n", g_fail ? "FAIL" : "ok",
           g_checks, g_fail, g_dev_ok, g_dev_missing);
    return g_fail ? 1 : 0;
}
