/*
 * net_util_mi355x.c — drop-in host C for µC/TCP-IP's four public checksum functions
 * (Source/net_util.h:422-438), with the byte summation done on an MI355X through the C ABI in
 * include/netcsum_mi355x.h. Plain C11; no HIP headers.
 *
 * What stays on the host is what the reference does around the sum and cannot move to the GPU:
 * the NET_BUF chain walk over host memory (net_util.c:1611-1687, per-buffer (ix, len) selection
 * by ProtocolHdrType), the argument checks of NET_ERR_CFG_ARG_CHK_DBG_EN, and the 2-op epilogue
 * on the returned 32-bit accumulator (fold :1690-1692, complement / compare :187-188, :275-276,
 * :358, :443-444). The bytes themselves are summed by the gfx950 stream kernel
 * (NetUtil_MI355X_StreamSum32). There is no CPU summation path: a device failure is reported as
 * NET_UTIL_ERR_MI355X_DEV.
 *
 * Build modes:
 *   standalone (this repo)  — NET_BUF comes from include/netcsum_netbuf.h (template-config
 *                             mirror); exported from libnetcsum_mi355x.so.
 *   inside a µC/TCP-IP tree — compile with -DNETCSUM_IN_STACK and the stack's include paths so
 *                             the real net_util.h / net_buf.h (and its configured layout) are
 *                             used; see INTEGRATION.md.
 */
#ifdef NETCSUM_IN_STACK
#include <cpu_core.h>
#include <net_util.h>
#include <net_buf.h>
#define NETCSUM_HAVE_MICRIUM_TYPES 1
#include "../../include/netcsum_mi355x.h"
#define NC_NET_TO_HOST_16(v) ((CPU_INT16U)NET_UTIL_NET_TO_HOST_16((CPU_INT16U)(v)))
#ifndef NETCSUM_ARG_CHK_DBG_EN
#define NETCSUM_ARG_CHK_DBG_EN (NET_ERR_CFG_ARG_CHK_DBG_EN == DEF_ENABLED)
#endif
#ifndef NETCSUM_ARG_CHK_EXT_EN
#define NETCSUM_ARG_CHK_EXT_EN (NET_ERR_CFG_ARG_CHK_EXT_EN == DEF_ENABLED)
#endif
#else
#include "../../include/netcsum_mi355x.h"
#include "../../include/netcsum_netbuf.h"
/* Little-endian host: MEM_VAL_BIG_TO_HOST_16 is a byte swap (uC-LIB lib_mem.h semantics). */
#define NC_NET_TO_HOST_16(v) ((CPU_INT16U)__builtin_bswap16((uint16_t)(v)))
#ifndef NETCSUM_ARG_CHK_DBG_EN
#define NETCSUM_ARG_CHK_DBG_EN 0          /* template default: DEF_DISABLED (net_cfg.h:184) */
#endif
#ifndef NETCSUM_ARG_CHK_EXT_EN
#define NETCSUM_ARG_CHK_EXT_EN 1          /* template default: DEF_ENABLED (net_cfg.h:178) */
#endif
#endif

#include <pthread.h>
#include <stddef.h>
#include <stdio.h>
#include <stdlib.h>

#define NC_NEG_ZERO     0xFFFFu            /* NET_UTIL_16_BIT_ONES_CPL_NEG_ZERO (net_util.c:56) */
#define NC_STACK_SPANS  64u                /* spans on the stack; longer chains use the heap */

static CPU_INT16U nc_fold(uint32_t sum)
{
    while (sum >> 16) {
        sum = (sum & 0xFFFFu) + (sum >> 16);
    }
    return (CPU_INT16U)sum;
}

/* ------------------------------------------------------------------------------------------
 * NET_BUF chain -> byte spans. Host-logic restatement of net_util.c:1589-1687.
 * ---------------------------------------------------------------------------------------- */
NET_ERR NetUtil_MI355X_ChainToSpans(const void *pdata_buf, const void *ppseudo_hdr,
                                    CPU_INT16U pseudo_hdr_size, NETCSUM_SPAN *spans,
                                    uint32_t max_spans, uint32_t *p_n_spans, int dbg_chk)
{
    const NET_BUF *pbuf = (const NET_BUF *)pdata_buf;
    uint32_t n = 0u;                                          /* spans the chain needs */
    int first = 1;

    if (p_n_spans == NULL) {
        return NET_ERR_FAULT_NULL_PTR;
    }
    if (spans == NULL) {                                      /* count-only walk */
        max_spans = 0u;
    }
    *p_n_spans = 0u;
    if (dbg_chk && pdata_buf == NULL) {                       /* :1566-1570 */
        return NET_ERR_FAULT_NULL_PTR;
    }

    if (ppseudo_hdr != NULL && pseudo_hdr_size != 0u) {      /* :1591-1609 */
        CPU_INT16U len = pseudo_hdr_size;
        if (pbuf == NULL && (len & 1u) != 0u) {
            /* The odd last pseudo-header octet is carried toward a first buffer that never
             * comes (the while loop at :1611 does not run), so it is never summed. */
            len = (CPU_INT16U)(len - 1u);
        }
        if (len != 0u) {
            if (n < max_spans) {
                spans[n].p = ppseudo_hdr;
                spans[n].len = len;
                spans[n].rsvd = 0u;
            }
            ++n;
        }
    }

    while (pbuf != NULL) {                                    /* :1611-1687, any chain length */
        const NET_BUF_HDR *h = &pbuf->Hdr;
        CPU_INT16U ix, len;

        switch ((int)h->ProtocolHdrType) {                    /* :1613-1640 */
        case NET_PROTOCOL_TYPE_ICMP_V4:
        case NET_PROTOCOL_TYPE_ICMP_V6:
            ix  = h->ICMP_MsgIx;
            len = (CPU_INT16U)(h->ICMP_HdrLen + (CPU_INT16U)h->DataLen);
            break;
        case NET_PROTOCOL_TYPE_UDP_V4:
        case NET_PROTOCOL_TYPE_UDP_V6:
#if !defined(NETCSUM_IN_STACK) || defined(NET_TCP_MODULE_EN)     /* as net_util.c:1625-1628 */
        case NET_PROTOCOL_TYPE_TCP_V4:
        case NET_PROTOCOL_TYPE_TCP_V6:
#endif
            ix  = h->TransportHdrIx;
            len = (CPU_INT16U)(h->TransportHdrLen + (CPU_INT16U)h->DataLen);
            break;
        case NET_PROTOCOL_TYPE_IP_V6_EXT_NONE:
            ix  = (CPU_INT16U)(h->TotLen - h->DataLen);
            len = (CPU_INT16U)h->DataLen;
            break;
        default:
            return NET_UTIL_ERR_INVALID_PROTOCOL;            /* :1637-1639 */
        }
        if (dbg_chk && ix == NET_BUF_IX_NONE) {               /* :1642-1647 */
            return NET_BUF_ERR_INVALID_IX;
        }
        if (dbg_chk && first) {                               /* :1660-1672 */
            first = 0;
            if (h->NextBufPtr == NULL && len == 0u) {
                return NET_UTIL_ERR_NULL_SIZE;
            }
        }
        if (len != 0u) {                                      /* zero-length buffers only pass */
            if (n < max_spans) {                              /* the carried octet through     */
                spans[n].p = pbuf->DataPtr + ix;
                spans[n].len = len;
                spans[n].rsvd = 0u;
            }
            ++n;
        }
        pbuf = (const NET_BUF *)h->NextBufPtr;
    }
    *p_n_spans = n;
    if (spans != NULL && n > max_spans) {
        return NET_UTIL_ERR_BUF_TOO_SMALL;                    /* *p_n_spans = the count needed */
    }
    return NET_UTIL_ERR_NONE;
}

/* The reference's u32 accumulator for one packet, summed on the GPU. */
/* The chain may be any length (net_util.c:1611-1687 has no bound; e.g. a 64 KiB datagram
 * reassembled from 576-B-MTU fragments is ~120 buffers, net_ipv4.c:6523): short chains use a
 * stack array, longer ones a heap array sized by the walk's own count. */
static NET_ERR nc_data_sum32(void *pdata_buf, void *ppseudo_hdr, CPU_INT16U pseudo_hdr_size,
                             uint32_t *p_sum32)
{
    NETCSUM_SPAN stack_spans[NC_STACK_SPANS];
    NETCSUM_SPAN *spans = stack_spans;
    uint32_t n = 0u;
    NET_ERR err = NetUtil_MI355X_ChainToSpans(pdata_buf, ppseudo_hdr, pseudo_hdr_size, spans,
                                              NC_STACK_SPANS, &n, NETCSUM_ARG_CHK_DBG_EN);
    if (err == NET_UTIL_ERR_BUF_TOO_SMALL) {
        spans = (NETCSUM_SPAN *)malloc((size_t)n * sizeof(NETCSUM_SPAN));
        if (spans == NULL) {
            fprintf(stderr, "[netcsum-mi355x] out of host memory for a %u-buffer chain\n", (unsigned)n);
            return (NET_ERR)NET_UTIL_ERR_MI355X_DEV;
        }
        err = NetUtil_MI355X_ChainToSpans(pdata_buf, ppseudo_hdr, pseudo_hdr_size, spans, n, &n,
                                          NETCSUM_ARG_CHK_DBG_EN);
    }
    if (err == NET_UTIL_ERR_NONE) {
        err = NetUtil_MI355X_StreamSum32(spans, n, p_sum32);
    }
    if (spans != stack_spans) {
        free(spans);
    }
    return err;
}

static NET_ERR nc_hdr_sum32(void *phdr, CPU_INT16U hdr_size, uint32_t *p_sum32)
{
    NETCSUM_SPAN span;
#if NETCSUM_ARG_CHK_DBG_EN
    if (phdr == NULL) {                                       /* :168-172, :255-259 */
        return NET_ERR_FAULT_NULL_PTR;
    }
    if (hdr_size < 1u) {                                      /* :174-178, :261-265 */
        return NET_UTIL_ERR_NULL_SIZE;
    }
#endif
    span.p = phdr;
    span.len = hdr_size;
    span.rsvd = 0u;
    return NetUtil_MI355X_StreamSum32(&span, hdr_size ? 1u : 0u, p_sum32);
}

/* Replaces Source/net_util.c:159-195. */
NET_CHK_SUM NetUtil_16BitOnesCplChkSumHdrCalc(void *phdr, CPU_INT16U hdr_size, NET_ERR *p_err)
{
    uint32_t sum32 = 0u;
    NET_ERR err = nc_hdr_sum32(phdr, hdr_size, &sum32);
    if (err != NET_UTIL_ERR_NONE) {
        *p_err = err;
        return 0u;
    }
    *p_err = NET_UTIL_ERR_NONE;
    return NC_NET_TO_HOST_16((CPU_INT16U)~nc_fold(sum32));
}

/* Replaces Source/net_util.c:245-284. */
CPU_BOOLEAN NetUtil_16BitOnesCplChkSumHdrVerify(void *phdr, CPU_INT16U hdr_size, NET_ERR *p_err)
{
    uint32_t sum32 = 0u;
    NET_ERR err = nc_hdr_sum32(phdr, hdr_size, &sum32);
    if (err != NET_UTIL_ERR_NONE) {
        *p_err = err;
        return DEF_FAIL;
    }
    *p_err = NET_UTIL_ERR_NONE;
    return (NC_NET_TO_HOST_16(nc_fold(sum32)) == NC_NEG_ZERO) ? DEF_OK : DEF_FAIL;
}

/* Replaces Source/net_util.c:344-363. */
NET_CHK_SUM NetUtil_16BitOnesCplChkSumDataCalc(void *pdata_buf, void *ppseudo_hdr,
                                               CPU_INT16U pseudo_hdr_size, NET_ERR *p_err)
{
    uint32_t sum32 = 0u;
    NET_ERR err = nc_data_sum32(pdata_buf, ppseudo_hdr, pseudo_hdr_size, &sum32);
    if (err != NET_UTIL_ERR_NONE) {
        *p_err = err;
        return 0u;
    }
    *p_err = NET_UTIL_ERR_NONE;
    return (NET_CHK_SUM)~NC_NET_TO_HOST_16(nc_fold(sum32));
}

/* Replaces Source/net_util.c:428-449. */
CPU_BOOLEAN NetUtil_16BitOnesCplChkSumDataVerify(void *pdata_buf, void *ppseudo_hdr,
                                                 CPU_INT16U pseudo_hdr_size, NET_ERR *p_err)
{
    uint32_t sum32 = 0u;
    NET_ERR err = nc_data_sum32(pdata_buf, ppseudo_hdr, pseudo_hdr_size, &sum32);
    if (err != NET_UTIL_ERR_NONE) {
        *p_err = err;
        return DEF_FAIL;
    }
    *p_err = NET_UTIL_ERR_NONE;
    return (NC_NET_TO_HOST_16(nc_fold(sum32)) == NC_NEG_ZERO) ? DEF_OK : DEF_FAIL;
}

/* The reference's optional native-inner-loop seam (Source/net_util.h:486-490, declared when
 * NET_CFG_OPTIMIZE_ASM_EN is enabled; ports Ports/<cpu>/<compiler>/net_util_a.*): the unfolded sum
 * of the network-order 16-bit words of a 4-byte-aligned region of `size` bytes (a multiple of 4),
 * which NetUtil_16BitSumDataCalc adds to its accumulator (net_util.c:1407-1415). Summed on the GPU
 * (exact, mod 2^32 — sizes passed by the reference are < 2^16, so the sum is exact). The reference
 * signature has no error channel: a device failure returns 0 and is reported on stderr (there is no
 * CPU path). */
CPU_INT32U NetUtil_16BitSumDataCalcAlign_32(void *pdata_32, CPU_INT32U size)
{
    NETCSUM_SPAN span;
    uint32_t sum32 = 0u;
    NET_ERR err;
    if (size == 0u) {
        return 0u;
    }
    span.p = pdata_32;
    span.len = size;
    span.rsvd = 0u;
    err = NetUtil_MI355X_StreamSum32(&span, 1u, &sum32);
    if (err != NET_UTIL_ERR_NONE) {
        fprintf(stderr, "[netcsum-mi355x] NetUtil_16BitSumDataCalcAlign_32: NET_ERR %d, returning 0\n", (int)err);
        return 0u;
    }
    return (CPU_INT32U)sum32;
}

/* ------------------------------------------------------------------------------------------
 * CRC-32 (net_util.c:485-636). SURVEY §2 row 10 keeps the CRC a host function: the stack calls it
 * per 6-octet MAC address (the drivers' multicast hash, e.g. Dev/Ether/GMAC/net_dev_gmac.c:2673-2683),
 * where a GPU round trip (~9 us) would cost ~1000 x the reference's loop. So a call of up to
 * NETCSUM_CRC_HOST_MAX octets runs the reference's register update (net_util.c:515-529: per octet,
 * eight shift / conditional-xor steps of the reflected polynomial) one table lookup per octet here;
 * a longer buffer is sent to the GPU kernel (NetUtil_MI355X_CRC32Host). Batches of CRCs use
 * NetUtil_MI355X_CRC32Batch* directly. The argument checks of NET_ERR_CFG_ARG_CHK_EXT_EN and the
 * final complement are the reference's.
 * ---------------------------------------------------------------------------------------- */
#define NETCSUM_CRC_HOST_MAX  4096u

/* T[v] = the eight steps of net_util.c:518-525 applied to the octet value v. */
static uint32_t crc_step_table(uint32_t v)
{
    uint32_t j;
    for (j = 0u; j < 8u; ++j) {
        v = (v & 1u) ? ((v >> 1) ^ 0xEDB88320u) : (v >> 1);   /* NET_UTIL_32_BIT_CRC_POLY_REFLECT */
    }
    return v;
}

/* The 256-entry table is built once per process (pthread_once): the drop-in may be called from
 * several host threads (one per device), and the table must be complete before any lookup. */
static uint32_t crc_tab[256];
static pthread_once_t crc_tab_once = PTHREAD_ONCE_INIT;

static void crc_tab_build(void)
{
    uint32_t i;
    for (i = 0u; i < 256u; ++i) {
        crc_tab[i] = crc_step_table(i);
    }
}

static uint32_t crc_host(const CPU_INT08U *p, uint32_t n)
{
    uint32_t crc = 0xFFFFFFFFu, i;                          /* NET_UTIL_32_BIT_ONES_CPL_NEG_ZERO */
    (void)pthread_once(&crc_tab_once, crc_tab_build);
    for (i = 0u; i < n; ++i) {
        crc = (crc >> 8) ^ crc_tab[(crc ^ p[i]) & 0xFFu];   /* :518, :527 */
    }
    return crc;
}

/* Replaces Source/net_util.c:485-530. */
CPU_INT32U NetUtil_32BitCRC_Calc(CPU_INT08U *p_data, CPU_INT32U data_len, NET_ERR *p_err)
{
    uint32_t crc = 0u;
    NET_ERR err;
#if NETCSUM_ARG_CHK_EXT_EN
    if (p_data == NULL) {                                     /* :499-503 */
        *p_err = NET_ERR_FAULT_NULL_PTR;
        return 0u;
    }
    if (data_len < 1u) {                                      /* :504-508 */
        *p_err = NET_UTIL_ERR_NULL_SIZE;
        return 0u;
    }
#endif
    if (data_len <= NETCSUM_CRC_HOST_MAX) {
        *p_err = NET_UTIL_ERR_NONE;
        return (CPU_INT32U)crc_host(p_data, (uint32_t)data_len);   /* 0 octets: 0xFFFFFFFF (:518-528) */
    }
    err = NetUtil_MI355X_CRC32Host(p_data, data_len, &crc);
    if (err != NET_UTIL_ERR_NONE) {
        *p_err = err;
        return 0u;
    }
    /* without the EXT checks a zero length leaves the register at its initial value (:518-528) */
    *p_err = NET_UTIL_ERR_NONE;
    return (data_len == 0u) ? 0xFFFFFFFFu : (CPU_INT32U)crc;
}

/* Replaces Source/net_util.c:571-588. */
CPU_INT32U NetUtil_32BitCRC_CalcCpl(CPU_INT08U *p_data, CPU_INT32U data_len, NET_ERR *p_err)
{
    CPU_INT32U crc = NetUtil_32BitCRC_Calc(p_data, data_len, p_err);
    if (*p_err != NET_UTIL_ERR_NONE) {
        return 0u;
    }
    return crc ^ 0xFFFFFFFFu;                                 /* :583 */
}

/* Replaces Source/net_util.c:610-636: bit i of val -> bit 31 - i. */
CPU_INT32U NetUtil_32BitReflect(CPU_INT32U val)
{
    uint32_t v = (uint32_t)val;
    v = ((v >> 1) & 0x55555555u) | ((v & 0x55555555u) << 1);
    v = ((v >> 2) & 0x33333333u) | ((v & 0x33333333u) << 2);
    v = ((v >> 4) & 0x0F0F0F0Fu) | ((v & 0x0F0F0F0Fu) << 4);
    v = ((v >> 8) & 0x00FF00FFu) | ((v & 0x00FF00FFu) << 8);
    return (CPU_INT32U)((v >> 16) | (v << 16));
}
