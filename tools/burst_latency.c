/*
 * burst_latency.c — what a NIC driver thread written in C waits for one checksum-offload burst
 * (include/netcsum_mi355x.h (2b''), (2e)), without the Python binding that
 * tools/burst_size_probe.py goes through.
 *
 * Frames: 1500-B IPv4/TCP datagrams in the reference's template Rx buffers (1520-B slots, the IP
 * header at +14, Cfg/Template/net_dev_cfg.c:146-149), random payloads, checksums made valid by one
 * TxBurst. Per burst size n, the median wall time of 300 calls (after 20 warm-up calls) of
 *   rx_dev / tx_dev    RxBurst / TxBurst on a device-resident ring + hipStreamSynchronize
 *   rx_host / tx_host  RxBurstHost / TxBurstHost on a pinned host ring in one chunk, which return
 *                      with the results in host memory (_auto: n_chunks 0, the library's choice —
 *                      up to 4096 frames the resident burst server reads the pinned ring in place
 *                      and the host polls the results; _auto_copy: the same with
 *                      NETCSUM_TUNE_BURST_ZERO_COPY 0, the copy pipeline; _launch: 2, a kernel launch
 *                      per burst; from 1024 frames also in 2-16 chunks: _cK)
 * and a check that every Rx action is DELIVER. One JSON line per n on stdout.
 *
 * Built here (the binary travels with the tree; tools/build/ is git-ignored), run on the GPU box:
 *   gcc -O2 -std=c11 -D__HIP_PLATFORM_AMD__ -I include -I /opt/rocm/include tools/burst_latency.c \
 *       -o tools/build/burst_latency -L uc-tcp-ip_amd -lnetcsum_mi355x \
 *       -Wl,-rpath,'$ORIGIN/../../uc-tcp-ip_amd' -L /opt/rocm/lib -lamdhip64 -Wl,-rpath,/opt/rocm/lib
 *   timeout -k 10 120 tools/build/burst_latency > gpurun_out/TAG_burst_latency.jsonl
 */
#define _POSIX_C_SOURCE 200809L
#include <hip/hip_runtime_api.h>

#include "netcsum_mi355x.h"

#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#define SLOT   1520u
#define IP_AT  14u
#define DGRAM  1500u
#define NMAX   262144u
#define REPS   300
#define WARM   20

#define HIP_OK(x)                                                                         \
    do {                                                                                  \
        hipError_t e_ = (x);                                                              \
        if (e_ != hipSuccess) {                                                           \
            fprintf(stderr, "%s:%d: %s -> %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(2);                                                                      \
        }                                                                                 \
    } while (0)
#define NET_OK(x)                                                                         \
    do {                                                                                  \
        NET_ERR r_ = (x);                                                                 \
        if (r_ != NET_UTIL_ERR_NONE) {                                                    \
            fprintf(stderr, "%s:%d: %s -> NET_ERR %u\n", __FILE__, __LINE__, #x, (unsigned)r_); \
            exit(3);                                                                      \
        }                                                                                 \
    } while (0)

static double now_us(void)
{
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (double)t.tv_sec * 1e6 + (double)t.tv_nsec * 1e-3;
}

static int cmp_d(const void *a, const void *b)
{
    double x = *(const double *)a, y = *(const double *)b;
    return (x > y) - (x < y);
}

static double median(double *v, int n)
{
    qsort(v, (size_t)n, sizeof *v, cmp_d);
    return v[n / 2];
}

static uint64_t rng = 0x5EED0011ull;
static uint8_t rnd8(void)
{
    rng ^= rng << 13;
    rng ^= rng >> 7;
    rng ^= rng << 17;
    return (uint8_t)(rng >> 29);
}

/* An IPv4/TCP datagram as the offloading stack leaves it (checksum fields 0). */
static void build(uint8_t *slot)
{
    uint8_t *ip = slot + IP_AT, *tcp = ip + 20;
    uint32_t i;
    for (i = 0; i < SLOT; ++i) slot[i] = rnd8();
    slot[12] = 0x08;
    slot[13] = 0x00;
    ip[0] = 0x45;
    ip[1] = 0;
    ip[2] = (uint8_t)(DGRAM >> 8);
    ip[3] = (uint8_t)DGRAM;
    ip[6] = 0x40;
    ip[7] = 0;
    ip[8] = 64;
    ip[9] = 6;
    ip[10] = ip[11] = 0;
    tcp[12] = 0x50;
    tcp[16] = tcp[17] = 0;
}

typedef enum { RX_DEV, TX_DEV, RX_HOST, TX_HOST } kind_t;

static uint8_t *g_dring, *g_hring, *g_dact, *g_hact;
static hipStream_t g_st;

static uint32_t g_chunks;

static void call(kind_t k, uint32_t n)
{
    const uint32_t chunks = g_chunks;
    switch (k) {
    case RX_DEV:
        NET_OK(NetUtil_MI355X_RxBurst(g_dring + IP_AT, NULL, NULL, SLOT, DGRAM, n, 0u, g_dact, NULL, g_st));
        HIP_OK(hipStreamSynchronize(g_st));
        break;
    case TX_DEV:
        NET_OK(NetUtil_MI355X_TxBurst(g_dring + IP_AT, NULL, NULL, SLOT, DGRAM, n, NULL, g_st));
        HIP_OK(hipStreamSynchronize(g_st));
        break;
    case RX_HOST:
        NET_OK(NetUtil_MI355X_RxBurstHost(g_hring + IP_AT, NULL, NULL, SLOT, DGRAM, n, 0u, g_hact, NULL, chunks));
        break;
    case TX_HOST:
        NET_OK(NetUtil_MI355X_TxBurstHost(g_hring + IP_AT, NULL, NULL, SLOT, DGRAM, n, NULL, chunks));
        break;
    }
}

static double time_us(kind_t k, uint32_t n)
{
    static double t[REPS];
    int r;
    for (r = 0; r < WARM; ++r) call(k, n);
    for (r = 0; r < REPS; ++r) {
        const double t0 = now_us();
        call(k, n);
        t[r] = now_us() - t0;
    }
    return median(t, REPS);
}

/* "zc": only the zero-copy bursts of 1 / 64 frames, 2000 calls each, plus the host-side pieces of
 * their cost (pointer-attribute queries, an empty-stream synchronise) — the program rocprofv3 traces
 * for the per-call breakdown. */
static int zc_only(void)
{
    static const uint32_t sizes[] = {1u, 64u};
    hipPointerAttribute_t at;
    double t0, t[2000];
    uint32_t s;
    int r, b;
    for (r = 0; r < 2000; ++r) {
        t0 = now_us();
        HIP_OK(hipPointerGetAttributes(&at, g_hring));
        t[r] = now_us() - t0;
    }
    printf("{\"pointer_attributes_us\": %.3f", median(t, 2000));
    for (r = 0; r < 2000; ++r) {
        t0 = now_us();
        HIP_OK(hipStreamSynchronize(g_st));
        t[r] = now_us() - t0;
    }
    printf(", \"empty_stream_sync_us\": %.3f", median(t, 2000));
    /* b = 0: a completion kernel and word (TUNE_BURST_ZERO_COPY 1); 1: results polled (2); 2: polled,
     * live-piece stream with piece 0 during the parse (TUNE_PKT_BOUND 2) instead of the whole-span
     * form; 3: the resident burst server (TUNE_BURST_ZERO_COPY 3) */
    for (b = 0; b <= 3; b += 1) {
        NET_OK(NetUtil_MI355X_Tune(NETCSUM_TUNE_PKT_BOUND, b == 2 ? 2 : -1));
        NET_OK(NetUtil_MI355X_Tune(NETCSUM_TUNE_BURST_ZERO_COPY, b == 3 ? 3 : b >= 1 ? 2 : 1));
        for (s = 0; s < 2; ++s) {
            int ok = 1;
            uint32_t i;
            for (r = 0; r < 2000; ++r) {
                memset(g_hact, 0xEE, sizes[s]);
                t0 = now_us();
                NET_OK(NetUtil_MI355X_RxBurstHost(g_hring + IP_AT, NULL, NULL, SLOT, DGRAM, sizes[s], 0u, g_hact, NULL, 0u));
                t[r] = now_us() - t0;
                for (i = 0; i < sizes[s]; ++i) ok &= g_hact[i] == NETCSUM_RX_DELIVER;
            }
            printf(", \"rx_host_zc_v%d_%u_us\": %.2f", b, sizes[s], median(t, 2000));
            if (!ok) {
                printf(", \"rx_host_zc_v%d_%u_delivered\": false}\n", b, sizes[s]);
                return 1;
            }
            for (r = 0; r < 2000; ++r) {
                t0 = now_us();
                NET_OK(NetUtil_MI355X_TxBurstHost(g_hring + IP_AT, NULL, NULL, SLOT, DGRAM, sizes[s], NULL, 0u));
                t[r] = now_us() - t0;
            }
            printf(", \"tx_host_zc_v%d_%u_us\": %.2f", b, sizes[s], median(t, 2000));
        }
    }
    NET_OK(NetUtil_MI355X_Tune(NETCSUM_TUNE_PKT_BOUND, -1));
    NET_OK(NetUtil_MI355X_Tune(NETCSUM_TUNE_BURST_ZERO_COPY, 3));
    printf("}\n");
    return 0;
}

int main(int argc, char **argv)
{
    static const uint32_t sizes[] = {1u, 10u, 16u, 32u, 64u, 128u, 256u, 1024u, 4096u, 16384u, 65536u, 262144u};
    const size_t bytes = (size_t)NMAX * SLOT;
    uint32_t i, s;
    HIP_OK(hipSetDevice(0));
    HIP_OK(hipStreamCreateWithFlags(&g_st, hipStreamNonBlocking));
    HIP_OK(hipMalloc((void **)&g_dring, bytes));
    HIP_OK(hipMalloc((void **)&g_dact, NMAX));
    HIP_OK(hipHostMalloc((void **)&g_hring, bytes, 0));
    HIP_OK(hipHostMalloc((void **)&g_hact, NMAX, 0));
    for (i = 0; i < NMAX; ++i) build(g_hring + (size_t)i * SLOT);
    NET_OK(NetUtil_MI355X_TxBurstHost(g_hring + IP_AT, NULL, NULL, SLOT, DGRAM, NMAX, NULL, 8u));   /* valid sums */
    HIP_OK(hipMemcpy(g_dring, g_hring, bytes, hipMemcpyHostToDevice));
    if (argc > 1 && strcmp(argv[1], "zc") == 0) return zc_only();
    for (s = 0; s < sizeof sizes / sizeof sizes[0]; ++s) {
        const uint32_t n = sizes[s];
        double rx_dev, tx_dev, rx_host, tx_host;
        int ok = 1;
        HIP_OK(hipMemset(g_dact, 0xEE, NMAX));
        memset(g_hact, 0xEE, NMAX);
        g_chunks = 1u;
        rx_dev = time_us(RX_DEV, n);
        tx_dev = time_us(TX_DEV, n);
        rx_host = time_us(RX_HOST, n);
        tx_host = time_us(TX_HOST, n);
        {
            static uint8_t act[NMAX];
            HIP_OK(hipMemcpy(act, g_dact, n, hipMemcpyDeviceToHost));
            for (i = 0; i < n; ++i) ok &= act[i] == NETCSUM_RX_DELIVER && g_hact[i] == NETCSUM_RX_DELIVER;
        }
        printf("{\"frames\": %u, \"rx_dev_sync_us\": %.2f, \"tx_dev_sync_us\": %.2f, \"rx_host_us\": %.2f, "
               "\"tx_host_us\": %.2f, \"all_delivered\": %s", n, rx_dev, tx_dev, rx_host, tx_host, ok ? "true" : "false");
        g_chunks = 0u;                                          /* the library's choice */
        memset(g_hact, 0xEE, NMAX);
        printf(", \"rx_host_us_auto\": %.2f, \"tx_host_us_auto\": %.2f", time_us(RX_HOST, n), time_us(TX_HOST, n));
        for (i = 0; i < n; ++i) ok &= g_hact[i] == NETCSUM_RX_DELIVER;
        /* n_chunks 0 without the zero-copy burst path (the copy pipeline in one chunk) */
        NET_OK(NetUtil_MI355X_Tune(NETCSUM_TUNE_BURST_ZERO_COPY, 0));
        printf(", \"rx_host_us_auto_copy\": %.2f", time_us(RX_HOST, n));
        NET_OK(NetUtil_MI355X_Tune(NETCSUM_TUNE_BURST_ZERO_COPY, 3));
        /* ... and with a kernel launch per burst, results polled (TUNE_BURST_ZERO_COPY 2) */
        NET_OK(NetUtil_MI355X_Tune(NETCSUM_TUNE_BURST_ZERO_COPY, 2));
        if (n <= 4096u) {
            memset(g_hact, 0xEE, NMAX);
            printf(", \"rx_host_us_launch\": %.2f, \"tx_host_us_launch\": %.2f", time_us(RX_HOST, n), time_us(TX_HOST, n));
            for (i = 0; i < n; ++i) ok &= g_hact[i] == NETCSUM_RX_DELIVER;
        }
        NET_OK(NetUtil_MI355X_Tune(NETCSUM_TUNE_BURST_ZERO_COPY, 3));
        for (g_chunks = 2u; g_chunks <= 16u && n >= 1024u; g_chunks *= 2u) {
            printf(", \"rx_host_us_c%u\": %.2f", g_chunks, time_us(RX_HOST, n));
            printf(", \"tx_host_us_c%u\": %.2f", g_chunks, time_us(TX_HOST, n));
        }
        printf(", \"all_delivered_auto\": %s}\n", ok ? "true" : "false");
        fflush(stdout);
        if (!ok) return 1;
    }
    NetUtil_MI355X_ThreadRelease();
    HIP_OK(hipFree(g_dring));
    HIP_OK(hipFree(g_dact));
    HIP_OK(hipHostFree(g_hring));
    HIP_OK(hipHostFree(g_hact));
    HIP_OK(hipStreamDestroy(g_st));
    return 0;
}
