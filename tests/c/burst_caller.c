/*
 * burst_caller.c — a plain C NIC-driver-side caller of the checksum-offload burst adapters
 * (include/netcsum_mi355x.h (2b''), (2e)), as INTEGRATION.md §2 wires them: the stack is built with
 * every NET_*_CFG_CHK_SUM_OFFLOAD_{RX,TX}_EN enabled (in-stack mode: the stand-in net_cfg.h with
 * NETCSUM_TEST_OFFLOAD, and this file refuses to build unless the stack maps them to
 * NET_*_CHK_SUM_OFFLOAD_* as Source/net_cfg_net.h:174-190, 305-366 does), and the driver runs one
 * adapter call per burst of frames in its host Rx ring / Tx queue.
 *
 *   Rx: a ring of 1520-B buffers (Cfg/Template/net_dev_cfg.c:146-149: 1518-B buffers, 4-B aligned),
 *       each an Ethernet frame whose IPv4 or IPv6 datagram starts at +14; some datagrams carry a bad
 *       IPv4 header checksum, a bad TCP / UDP / ICMP checksum, no UDP checksum. RxBurstHost gives one
 *       action per frame: drop the failures with the reference's counter, deliver the rest
 *       (RxBurstTally sums the counters the stack's Net_ErrCtrs would have seen).
 *   Tx: the frames as the offloading stack builds them (0 in the IPv4 / TCP fields, 0xFFFF in UDP,
 *       0 for "no UDP checksum"); TxBurstHost fills the checksums in place; every frame then
 *       verifies with the caller's own RFC 1071 sum.
 * Without a GPU both calls must FAIL with NET_UTIL_ERR_MI355X_DEV (no CPU fallback) after their
 * argument checks; with one (NETCSUM_EXPECT_GPU=1) they must succeed and match. Exit 0 = passed.
 */
#ifdef NETCSUM_IN_STACK
#include <cpu_core.h>
#include <net_cfg_net.h>
#if !defined(NET_IPV4_CHK_SUM_OFFLOAD_RX) || !defined(NET_TCP_CHK_SUM_OFFLOAD_RX) || \
    !defined(NET_UDP_CHK_SUM_OFFLOAD_RX) || !defined(NET_ICMP_CHK_SUM_OFFLOAD_RX) || \
    !defined(NET_IPV4_CHK_SUM_OFFLOAD_TX) || !defined(NET_TCP_CHK_SUM_OFFLOAD_TX) || \
    !defined(NET_UDP_CHK_SUM_OFFLOAD_TX)
#error "the burst adapters replace the stack's checksum calls: build it with NET_*_CFG_CHK_SUM_OFFLOAD_{RX,TX}_EN enabled"
#endif
#include <net_util.h>
#define NETCSUM_HAVE_MICRIUM_TYPES 1
#endif
#include "netcsum_mi355x.h"

#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define NET_UTIL_ERR_MI355X_DEV_CODE  218u
#define RING_N      4096u
#define BUF_SIZE    1520u              /* 1518 rounded up to the 4-B buffer alignment */
#define IP_AT       14u                /* after the Ethernet header */

static int g_fail, g_checks, g_expect_gpu;

#define CHECK(cond, ...)                                              \
    do {                                                              \
        ++g_checks;                                                   \
        if (!(cond)) {                                                \
            ++g_fail;                                                 \
            fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__);      \
            fprintf(stderr, __VA_ARGS__);                             \
            fputc('\n', stderr);                                      \
        }                                                             \
    } while (0)

static uint64_t rng_state = 0x5EED0003ull;
static uint32_t rnd(void)
{
    rng_state ^= rng_state << 13;
    rng_state ^= rng_state >> 7;
    rng_state ^= rng_state << 17;
    return (uint32_t)(rng_state >> 11);
}

static uint32_t sum_be(const uint8_t *p, size_t n, uint32_t s)
{
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
static void put16(uint8_t *p, uint16_t v) { p[0] = (uint8_t)(v >> 8); p[1] = (uint8_t)v; }
static uint16_t get16(const uint8_t *p) { return (uint16_t)(p[0] << 8 | p[1]); }

/* The transport checksum's one's-complement sum incl. the pseudo-header (IPv4 12 B / IPv6 40 B). */
static uint32_t l4_sum(const uint8_t *ip, int v6, uint8_t proto, const uint8_t *l4, uint16_t l4len)
{
    uint32_t s = sum_be(l4, l4len, 0);
    if (proto == 1) return s;                                   /* ICMPv4: no pseudo-header */
    if (v6) {
        s = sum_be(ip + 8, 32, s);
        return s + l4len + proto;
    }
    s = sum_be(ip + 12, 8, s);
    return s + proto + l4len;
}

typedef struct {
    uint8_t  v6, proto, kind;      /* kind: 0 valid, 1 bad IP checksum, 2 bad L4, 3 UDP no checksum */
    uint16_t l4len;
} frame_t;

/* Writes the frame as the offloading stack hands it over (fields 0 / 0xFFFF / 0) into buf + IP_AT. */
static void build(uint8_t *buf, frame_t *f)
{
    uint8_t *ip = buf + IP_AT, *l4;
    uint16_t pay = (uint16_t)(20u + rnd() % 1300u), i;
    memset(buf, 0, BUF_SIZE);
    buf[12] = f->v6 ? 0x86 : 0x08;
    buf[13] = f->v6 ? 0xDD : 0x00;
    f->l4len = (uint16_t)((f->proto == 6 ? 20u : f->proto == 17 ? 8u : 8u) + pay);
    if (f->v6) {
        ip[0] = 0x60;
        put16(ip + 4, f->l4len);
        ip[6] = f->proto;
        ip[7] = 64;
        for (i = 8; i < 40; ++i) ip[i] = (uint8_t)rnd();
        l4 = ip + 40;
    } else {
        ip[0] = 0x45;
        put16(ip + 2, (uint16_t)(20u + f->l4len));
        ip[6] = 0x40;
        ip[8] = 64;
        ip[9] = f->proto;
        for (i = 12; i < 20; ++i) ip[i] = (uint8_t)rnd();
        l4 = ip + 20;
    }
    for (i = 0; i < f->l4len; ++i) l4[i] = (uint8_t)rnd();
    if (f->proto == 6) {
        l4[12] = 0x50;
        put16(l4 + 16, 0);                                      /* net_tcp.c:29813-29815 */
    } else if (f->proto == 17) {
        put16(l4 + 4, f->l4len);
        put16(l4 + 6, f->kind == 3 ? 0u : 0xFFFFu);             /* net_udp.c:2929-2935 */
    } else {
        l4[0] = 8;                                              /* ICMPv4 echo request */
        l4[1] = 0;
        put16(l4 + 2, 0);
    }
}

/* The checksums a stack without the offload would have written (for the Rx ring). */
static void finalize_host(uint8_t *buf, const frame_t *f)
{
    uint8_t *ip = buf + IP_AT, *l4 = ip + (f->v6 ? 40 : 20);
    uint16_t c;
    if (!f->v6) {
        put16(ip + 10, 0);
        put16(ip + 10, (uint16_t)~fold(sum_be(ip, 20, 0)));
    }
    if (f->proto == 17 && f->kind == 3) return;
    if (f->proto == 6) {
        put16(l4 + 16, 0);
        put16(l4 + 16, (uint16_t)~fold(l4_sum(ip, f->v6, 6, l4, f->l4len)));
    } else if (f->proto == 17) {
        put16(l4 + 6, 0);
        c = (uint16_t)~fold(l4_sum(ip, f->v6, 17, l4, f->l4len));
        put16(l4 + 6, c ? c : 0xFFFFu);
    } else {
        put16(l4 + 2, 0);
        put16(l4 + 2, (uint16_t)~fold(l4_sum(ip, 0, 1, l4, f->l4len)));
    }
}

static int verifies(const uint8_t *buf, const frame_t *f)
{
    const uint8_t *ip = buf + IP_AT, *l4 = ip + (f->v6 ? 40 : 20);
    if (!f->v6 && fold(sum_be(ip, 20, 0)) != 0xFFFFu) return 0;
    if (f->proto == 17 && get16(l4 + 6) == 0) return f->kind == 3;
    return fold(l4_sum(ip, f->v6, f->proto, l4, f->l4len)) == 0xFFFFu;
}

int main(void)
{
    static frame_t fr[RING_N];
    static uint8_t want_act[RING_N], act[RING_N];
    uint8_t *ring = (uint8_t *)malloc((size_t)RING_N * BUF_SIZE);
    uint32_t ctr[NETCSUM_RX_NBR_ACTIONS], want_ctr[NETCSUM_RX_NBR_ACTIONS], i;
    const char *e = getenv("NETCSUM_EXPECT_GPU");
    NET_ERR err;
    g_expect_gpu = e && e[0] == '1';
    memset(want_ctr, 0, sizeof want_ctr);
    for (i = 0; i < RING_N; ++i) {
        uint32_t r = rnd() % 16u;
        fr[i].v6 = (uint8_t)(rnd() & 1u);
        fr[i].proto = (uint8_t)(r < 6 ? 6 : r < 12 ? 17 : (fr[i].v6 ? 17 : 1));
        fr[i].kind = (uint8_t)(rnd() % 8u);
        if (fr[i].kind > 3 || (fr[i].kind == 1 && fr[i].v6) || (fr[i].kind == 3 && fr[i].proto != 17)) fr[i].kind = 0;
        build(ring + (size_t)i * BUF_SIZE, &fr[i]);
        finalize_host(ring + (size_t)i * BUF_SIZE, &fr[i]);
        if (fr[i].kind == 1) ring[(size_t)i * BUF_SIZE + IP_AT + 8] ^= 0x01u;               /* TTL */
        if (fr[i].kind == 2) ring[(size_t)i * BUF_SIZE + IP_AT + (fr[i].v6 ? 40 : 20) + fr[i].l4len - 1] ^= 0x10u;
        want_act[i] = fr[i].kind == 1 ? NETCSUM_RX_DROP_IPV4_CHK_SUM
                    : fr[i].kind == 2 ? (fr[i].proto == 6 ? NETCSUM_RX_DROP_TCP_CHK_SUM
                                        : fr[i].proto == 17 ? NETCSUM_RX_DROP_UDP_CHK_SUM
                                        : NETCSUM_RX_DROP_ICMPV4_CHK_SUM)
                    : NETCSUM_RX_DELIVER;
        ++want_ctr[want_act[i]];
    }
    /* --- Rx: one call per burst of the host ring (device pipelined in 4 chunks) */
    CHECK(NetUtil_MI355X_RxBurstHost(ring + IP_AT, NULL, NULL, BUF_SIZE, BUF_SIZE - IP_AT, RING_N, 0u, NULL,
                                     NULL, 4u) == NET_ERR_FAULT_NULL_PTR, "RxBurstHost without actions");
    memset(act, 0xEE, sizeof act);
    err = NetUtil_MI355X_RxBurstHost(ring + IP_AT, NULL, NULL, BUF_SIZE, BUF_SIZE - IP_AT, RING_N, 0u, act, NULL, 4u);
    if (!g_expect_gpu) {
        CHECK((unsigned)err == NET_UTIL_ERR_MI355X_DEV_CODE, "no GPU: RxBurstHost -> %u, not DEV", (unsigned)err);
    } else {
        CHECK((unsigned)err == NET_UTIL_ERR_NONE, "RxBurstHost -> %u", (unsigned)err);
        for (i = 0; i < RING_N; ++i) CHECK(act[i] == want_act[i], "frame %u action %u want %u", i, act[i], want_act[i]);
        memset(ctr, 0, sizeof ctr);
        CHECK(NetUtil_MI355X_RxBurstTally(act, RING_N, ctr) == NET_UTIL_ERR_NONE, "tally");
        for (i = 0; i < NETCSUM_RX_NBR_ACTIONS; ++i) CHECK(ctr[i] == want_ctr[i], "counter %u: %u want %u", i, ctr[i], want_ctr[i]);
    }
    /* --- Tx: the frames as the offloading stack leaves them, finished in place by one call */
    for (i = 0; i < RING_N; ++i) {
        if (fr[i].kind != 3) fr[i].kind = 0;
        build(ring + (size_t)i * BUF_SIZE, &fr[i]);
    }
    err = NetUtil_MI355X_TxBurstHost(ring + IP_AT, NULL, NULL, BUF_SIZE, BUF_SIZE - IP_AT, RING_N, NULL, 4u);
    if (!g_expect_gpu) {
        CHECK((unsigned)err == NET_UTIL_ERR_MI355X_DEV_CODE, "no GPU: TxBurstHost -> %u, not DEV", (unsigned)err);
    } else {
        CHECK((unsigned)err == NET_UTIL_ERR_NONE, "TxBurstHost -> %u", (unsigned)err);
        for (i = 0; i < RING_N; ++i) CHECK(verifies(ring + (size_t)i * BUF_SIZE, &fr[i]), "frame %u does not verify", i);
    }
    NetUtil_MI355X_ThreadRelease();
    free(ring);
    printf("%s checks=%d failed=%d gpu=%d\n", g_fail ? "FAIL" : "ok", g_checks, g_fail, g_expect_gpu);
    return g_fail ? 1 : 0;
}
