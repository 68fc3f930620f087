/*
 * ORACLE — TEST INFRASTRUCTURE ONLY (see net_util_oracle.h for the parity status and the rules
 * on who may call this). CPU restatement of µC/TCP-IP V3.06.01 Source/net_util.c, checksum part.
 *
 * Structure deliberately follows the reference (one routine per reference routine, the same
 * aligned/unaligned paths, the same 32-bit-word inner loop with two 16-bit swaps per word as
 * net_util.c:1423-1435 with NET_CFG_OPTIMIZE_ASM_EN disabled), so that its speed is a faithful
 * stand-in for the reference C path when bench.py times it as the CPU baseline.
 */
#include "net_util_oracle.h"

#include <stddef.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#include "../include/netcsum_netbuf.h"

/* uC-LIB MEM_VAL_{HOST_TO_BIG,BIG_TO_HOST}_16 on a little-endian CPU (net_util.h:102,105). */
#define ORC_SWAP16(v) ((uint16_t)__builtin_bswap16((uint16_t)(v)))

/* psum_err bits of NetUtil_16BitSumDataCalc (net_util.c:60-62). */
#define ORC_SUM_ERR_NONE       0x00u
#define ORC_SUM_ERR_NULL_SIZE  0x02u   /* DEF_BIT_01 */
#define ORC_SUM_ERR_LAST_OCTET 0x04u   /* DEF_BIT_02 */

#define ORC_NEG_ZERO 0xFFFFu           /* NET_UTIL_16_BIT_ONES_CPL_NEG_ZERO, net_util.c:56 */

static inline uint16_t ld16(const uint8_t *p) { uint16_t v; memcpy(&v, p, 2); return v; }
static inline uint32_t ld32(const uint8_t *p) { uint32_t v; memcpy(&v, p, 4); return v; }

/* ---------------------------------------------------------------------------------------------
 * Restates NetUtil_16BitSumHdrCalc, net_util.c:1160-1208.
 * Unfolded network-order sum of one contiguous header. 16-bit-aligned headers are read as host
 * 16-bit words and swapped to network order; unaligned headers are combined octet pairs; an odd
 * last octet is summed as the high half of a word (right-padded).
 * ------------------------------------------------------------------------------------------- */
static uint32_t orc_sum_hdr(const uint8_t *p, uint16_t size)
{
    uint32_t acc = 0u;
    uint32_t left = size;

    if (size < 1u) {                                   /* :1171-1173 */
        return 0u;
    }
    if (((uintptr_t)p & 1u) == 0u) {                   /* :1179-1188 word path */
        for (; left >= 2u; left -= 2u, p += 2) {
            acc += (uint32_t)ORC_SWAP16(ld16(p));
        }
    } else {                                           /* :1190-1198 octet-pair path */
        for (; left >= 2u; left -= 2u, p += 2) {
            acc += ((uint32_t)p[0] << 8) + (uint32_t)p[1];
        }
    }
    if (left > 0u) {                                   /* :1201-1203 */
        acc += (uint32_t)p[0] << 8;
    }
    return acc;
}

/* ---------------------------------------------------------------------------------------------
 * Restates NetUtil_16BitSumDataCalc, net_util.c:1321-1475 (NET_CFG_OPTIMIZE_ASM_EN disabled).
 * One buffer's unfolded network-order sum, with the odd octet carried between buffers:
 *   - prev_valid: *octet_prev is the dangling octet of the previous piece, prepended here;
 *   - last_buf:   a dangling octet at the end is padded (summed <<8) instead of carried out
 *                 through *octet_last with ORC_SUM_ERR_LAST_OCTET.
 * ------------------------------------------------------------------------------------------- */
static uint32_t orc_sum_buf(const uint8_t *p, uint16_t size,
                            const uint8_t *octet_prev, uint8_t *octet_last,
                            int prev_valid, int last_buf, uint8_t *flags)
{
    uint32_t acc = 0u;
    uint32_t word = 0u;
    uint32_t left;
    int      even_path;

    if (size < 1u) {                                   /* :1350-1371 null-size buffer */
        *flags = ORC_SUM_ERR_NULL_SIZE;
        if (prev_valid) {
            if (last_buf) {
                acc = (uint32_t)*octet_prev << 8;      /* pad the carried octet */
            } else {
                *octet_last = *octet_prev;             /* pass it through to the next buffer */
                *flags |= ORC_SUM_ERR_LAST_OCTET;
            }
        }
        return acc;
    }

    left   = size;
    *flags = ORC_SUM_ERR_NONE;
    /* :1379-1381 — the word path applies when, after any prepended octet, reads are 2-aligned. */
    even_path = ((((uintptr_t)p & 1u) == 0u) && !prev_valid) ||
                ((((uintptr_t)p & 1u) != 0u) &&  prev_valid);

    if (prev_valid) {                                  /* :1385-1393 prepend carried octet */
        acc  += ((uint32_t)*octet_prev << 8) + (uint32_t)p[0];
        p    += 1;
        left -= 1u;
    }

    if (even_path) {
        if ((((uintptr_t)p & 3u) != 0u) && (left >= 2u)) {   /* :1398-1405 lead word to 4-align */
            acc  += (uint32_t)ORC_SWAP16(ld16(p));
            p    += 2;
            left -= 2u;
        }
        for (; left >= 4u; left -= 4u, p += 4) {      /* :1423-1435 32-bit word loop */
            uint32_t w = ld32(p);
            acc += (uint32_t)ORC_SWAP16((uint16_t)(w >> 16));
            acc += (uint32_t)ORC_SWAP16((uint16_t)(w & 0xFFFFu));
        }
        for (; left >= 2u; left -= 2u, p += 2) {      /* :1439-1444 16-bit tail */
            acc += (uint32_t)ORC_SWAP16(ld16(p));
        }
        if (left > 0u) {
            word = (uint32_t)p[0];
        }
    } else {                                           /* :1450-1460 octet-pair path */
        for (; left >= 2u; left -= 2u, p += 2) {
            acc += ((uint32_t)p[0] << 8) + (uint32_t)p[1];
        }
        if (left > 0u) {
            word = (uint32_t)p[0];
        }
    }

    if (left > 0u) {                                   /* :1463-1471 dangling octet */
        if (last_buf) {
            acc += word << 8;
        } else {
            *octet_last = (uint8_t)word;
            *flags |= ORC_SUM_ERR_LAST_OCTET;
        }
    }
    return acc;
}

/* ---------------------------------------------------------------------------------------------
 * Restates the chain walk of NetUtil_16BitOnesCplSumDataCalc, net_util.c:1545-1687, returning
 * the u32 accumulator BEFORE the fold. Return value is the NET_ERR code.
 * ------------------------------------------------------------------------------------------- */
static uint32_t orc_sum_chain(const void *pdata_buf, const void *ppseudo_hdr,
                              uint16_t pseudo_hdr_size, int dbg_chk, uint32_t *p_sum)
{
    const NET_BUF *pbuf = (const NET_BUF *)pdata_buf;
    uint32_t sum = 0u;
    uint8_t  octet_prev = 0u, octet_last = 0u, flags = 0u;
    int      prev_valid = 0;
    int      first = 1;

    *p_sum = 0u;
    if (dbg_chk && pdata_buf == NULL) {                /* :1566-1570 */
        return NET_ERR_FAULT_NULL_PTR;
    }

    if (ppseudo_hdr != NULL) {                         /* :1591-1609, never the last piece */
        sum += orc_sum_buf((const uint8_t *)ppseudo_hdr, pseudo_hdr_size,
                           &octet_prev, &octet_last, prev_valid, 0, &flags);
        if (flags & ORC_SUM_ERR_LAST_OCTET) {
            octet_prev = octet_last;
            prev_valid = 1;
        } else {
            octet_prev = 0u;
            prev_valid = 0;
        }
    }

    while (pbuf != NULL) {                             /* :1611-1687 */
        const NET_BUF_HDR *h = &pbuf->Hdr;
        uint16_t ix, len;
        int last;

        switch ((int)h->ProtocolHdrType) {             /* :1613-1640 */
        case NET_PROTOCOL_TYPE_ICMP_V4:
        case NET_PROTOCOL_TYPE_ICMP_V6:
            ix  = h->ICMP_MsgIx;
            len = (uint16_t)(h->ICMP_HdrLen + h->DataLen);        /* 16-bit wrap, :1617 */
            break;
        case NET_PROTOCOL_TYPE_UDP_V4:
        case NET_PROTOCOL_TYPE_UDP_V6:
        case NET_PROTOCOL_TYPE_TCP_V4:                 /* NET_TCP_MODULE_EN (template cfg) */
        case NET_PROTOCOL_TYPE_TCP_V6:
            ix  = h->TransportHdrIx;
            len = (uint16_t)(h->TransportHdrLen + h->DataLen);    /* 16-bit wrap, :1628 */
            break;
        case NET_PROTOCOL_TYPE_IP_V6_EXT_NONE:
            ix  = (uint16_t)(h->TotLen - h->DataLen);
            len = h->DataLen;
            break;
        default:
            return NET_UTIL_ERR_INVALID_PROTOCOL;      /* :1637-1639 */
        }
        if (dbg_chk && ix == NET_BUF_IX_NONE) {        /* :1642-1647 */
            return NET_BUF_ERR_INVALID_IX;
        }

        last = (h->NextBufPtr == NULL);
        {
            uint32_t part = orc_sum_buf(pbuf->DataPtr + ix, len, &octet_prev, &octet_last,
                                        prev_valid, last, &flags);
            if (dbg_chk && first) {                    /* :1660-1672 */
                first = 0;
                if (last && (flags & ORC_SUM_ERR_NULL_SIZE)) {
                    return NET_UTIL_ERR_NULL_SIZE;
                }
            }
            if (!last) {                               /* :1674-1683 */
                if (flags & ORC_SUM_ERR_LAST_OCTET) {
                    octet_prev = octet_last;
                    prev_valid = 1;
                } else {
                    octet_prev = 0u;
                    prev_valid = 0;
                }
            }
            sum += part;                               /* u32 accumulate, wraps mod 2^32 */
        }
        pbuf = h->NextBufPtr;
    }
    *p_sum = sum;
    return NET_UTIL_ERR_NONE;
}

static uint16_t orc_fold(uint32_t sum)                 /* :184-186, :1690-1692 */
{
    while (sum >> 16) {
        sum = (sum & 0xFFFFu) + (sum >> 16);
    }
    return (uint16_t)sum;
}

/* Restates NetUtil_16BitOnesCplChkSumHdrCalc, net_util.c:159-195. */
uint16_t Oracle_HdrCalc(const void *phdr, uint16_t hdr_size, uint32_t *p_err, int dbg_chk)
{
    uint16_t folded;
    if (dbg_chk) {                                     /* :168-179 */
        if (phdr == NULL)   { *p_err = NET_ERR_FAULT_NULL_PTR; return 0u; }
        if (hdr_size < 1u)  { *p_err = NET_UTIL_ERR_NULL_SIZE; return 0u; }
    }
    folded = orc_fold(orc_sum_hdr((const uint8_t *)phdr, hdr_size));
    *p_err = NET_UTIL_ERR_NONE;
    return ORC_SWAP16((uint16_t)~folded);              /* :187-188 */
}

/* Restates NetUtil_16BitOnesCplChkSumHdrVerify, net_util.c:245-284. */
uint8_t Oracle_HdrVerify(const void *phdr, uint16_t hdr_size, uint32_t *p_err, int dbg_chk)
{
    uint16_t folded;
    if (dbg_chk) {                                     /* :255-266 */
        if (phdr == NULL)   { *p_err = NET_ERR_FAULT_NULL_PTR; return 0u; }
        if (hdr_size < 1u)  { *p_err = NET_UTIL_ERR_NULL_SIZE; return 0u; }
    }
    folded = orc_fold(orc_sum_hdr((const uint8_t *)phdr, hdr_size));
    *p_err = NET_UTIL_ERR_NONE;
    return (ORC_SWAP16(folded) == ORC_NEG_ZERO) ? 1u : 0u;   /* :275-278 */
}

/* Restates NetUtil_16BitOnesCplSumDataCalc's tail (:1690-1695): folded sum in host order. */
static uint16_t orc_ones_cpl_sum(const void *pdata_buf, const void *ppseudo_hdr,
                                 uint16_t pseudo_hdr_size, uint32_t *p_err, int dbg_chk)
{
    uint32_t sum;
    uint32_t err = orc_sum_chain(pdata_buf, ppseudo_hdr, pseudo_hdr_size, dbg_chk, &sum);
    *p_err = err;
    if (err != NET_UTIL_ERR_NONE) {
        return 0u;
    }
    return ORC_SWAP16(orc_fold(sum));
}

/* Restates NetUtil_16BitOnesCplChkSumDataCalc, net_util.c:344-363. */
uint16_t Oracle_DataCalc(const void *pdata_buf, const void *ppseudo_hdr, uint16_t pseudo_hdr_size,
                         uint32_t *p_err, int dbg_chk)
{
    uint16_t s = orc_ones_cpl_sum(pdata_buf, ppseudo_hdr, pseudo_hdr_size, p_err, dbg_chk);
    if (*p_err != NET_UTIL_ERR_NONE) {
        return 0u;
    }
    return (uint16_t)~s;
}

/* Restates NetUtil_16BitOnesCplChkSumDataVerify, net_util.c:428-449. */
uint8_t Oracle_DataVerify(const void *pdata_buf, const void *ppseudo_hdr, uint16_t pseudo_hdr_size,
                          uint32_t *p_err, int dbg_chk)
{
    uint16_t s = orc_ones_cpl_sum(pdata_buf, ppseudo_hdr, pseudo_hdr_size, p_err, dbg_chk);
    if (*p_err != NET_UTIL_ERR_NONE) {
        return 0u;
    }
    return (s == ORC_NEG_ZERO) ? 1u : 0u;
}

uint32_t Oracle_DataSum32(const void *pdata_buf, const void *ppseudo_hdr, uint16_t pseudo_hdr_size,
                          uint32_t *p_sum32)
{
    return orc_sum_chain(pdata_buf, ppseudo_hdr, pseudo_hdr_size, 0, p_sum32);
}

/* ------------------------------ batch drivers (test/bench only) --------------------------- */

static void orc_one_segment(const uint8_t *seg, uint16_t len, const uint8_t *pseudo,
                            uint16_t pseudo_len, void *out, uint32_t i, int op)
{
    uint32_t err;
    if (op >= 2) {                                     /* HdrCalc / HdrVerify */
        if (op == 2) {
            ((uint16_t *)out)[i] = Oracle_HdrCalc(seg, len, &err, 0);
        } else {
            ((uint8_t *)out)[i] = Oracle_HdrVerify(seg, len, &err, 0);
        }
        return;
    }
    {
        NET_BUF buf;                                   /* one-buffer chain, as a TCP_V4 Rx; */
        buf.Hdr.NextBufPtr      = NULL;                /* only the fields the walk reads    */
        buf.Hdr.ProtocolHdrType = NET_PROTOCOL_TYPE_TCP_V4;
        buf.Hdr.TransportHdrIx  = 0u;
        buf.Hdr.TransportHdrLen = 0u;
        buf.Hdr.DataLen         = len;
        buf.DataPtr             = (CPU_INT08U *)seg;
        if (op == 0) {
            ((uint16_t *)out)[i] = Oracle_DataCalc(&buf, pseudo, pseudo_len, &err, 0);
        } else {
            ((uint8_t *)out)[i] = Oracle_DataVerify(&buf, pseudo, pseudo_len, &err, 0);
        }
    }
}

void Oracle_BatchStrided(const uint8_t *seg, uint64_t seg_stride, uint16_t seg_len,
                         const uint8_t *pseudo, uint32_t pseudo_stride, uint16_t pseudo_len,
                         uint32_t n_seg, void *out, int op, int n_threads)
{
    int64_t i;
#ifdef _OPENMP
    int nt = (n_threads > 0) ? n_threads : omp_get_max_threads();
#pragma omp parallel for schedule(static) num_threads(nt)
#else
    (void)n_threads;
#endif
    for (i = 0; i < (int64_t)n_seg; ++i) {
        orc_one_segment(seg + (uint64_t)i * seg_stride, seg_len,
                        pseudo ? pseudo + (uint64_t)i * pseudo_stride : NULL, pseudo_len,
                        out, (uint32_t)i, op);
    }
}

void Oracle_BatchVarLen(const uint8_t *base, const uint64_t *seg_off, const uint16_t *seg_len,
                        const uint8_t *pseudo, uint32_t pseudo_stride, uint16_t pseudo_len,
                        uint32_t n_seg, void *out, int op, int n_threads)
{
    int64_t i;
#ifdef _OPENMP
    int nt = (n_threads > 0) ? n_threads : omp_get_max_threads();
#pragma omp parallel for schedule(static) num_threads(nt)
#else
    (void)n_threads;
#endif
    for (i = 0; i < (int64_t)n_seg; ++i) {
        orc_one_segment(base + seg_off[i], seg_len[i],
                        pseudo ? pseudo + (uint64_t)i * pseudo_stride : NULL, pseudo_len,
                        out, (uint32_t)i, op);
    }
}

/* Chain i = pieces [chain_first[i], chain_first[i+1]) linked as a NET_BUF chain (TCP_V4 buffers,
 * DataPtr = base + piece_off[j], DataLen = piece_len[j]) and walked by Oracle_DataCalc/Verify with
 * its pseudo-header — the reference's multi-buffer call (net_util.c:1611-1687). No pieces => the
 * pdata_buf == NULL call. ops 0/1 only. */
void Oracle_BatchChains(const uint8_t *base, const uint64_t *piece_off, const uint16_t *piece_len,
                        const uint32_t *chain_first, const uint8_t *pseudo, uint32_t pseudo_stride,
                        uint16_t pseudo_len, uint32_t n_chains, void *out, int op, int n_threads)
{
    int64_t i;
#ifdef _OPENMP
    int nt = (n_threads > 0) ? n_threads : omp_get_max_threads();
#pragma omp parallel for schedule(dynamic, 64) num_threads(nt)
#else
    (void)n_threads;
#endif
    for (i = 0; i < (int64_t)n_chains; ++i) {
        uint32_t p0 = chain_first[i], p1 = chain_first[i + 1], j, err;
        uint32_t n = p1 - p0;
        NET_BUF *bufs = (n != 0u) ? (NET_BUF *)malloc((size_t)n * sizeof(NET_BUF)) : NULL;
        const uint8_t *ph = pseudo ? pseudo + (uint64_t)i * pseudo_stride : NULL;
        for (j = 0; j < n; ++j) {
            NET_BUF *b = &bufs[j];
            b->Hdr.NextBufPtr      = (j + 1u < n) ? &bufs[j + 1u] : NULL;
            b->Hdr.ProtocolHdrType = NET_PROTOCOL_TYPE_TCP_V4;
            b->Hdr.TransportHdrIx  = 0u;
            b->Hdr.TransportHdrLen = 0u;
            b->Hdr.DataLen         = piece_len[p0 + j];
            b->DataPtr             = (CPU_INT08U *)(base + piece_off[p0 + j]);
        }
        if (op == 0) {
            ((uint16_t *)out)[i] = Oracle_DataCalc(bufs, ph, pseudo_len, &err, 0);
        } else {
            ((uint8_t *)out)[i] = Oracle_DataVerify(bufs, ph, pseudo_len, &err, 0);
        }
        free(bufs);
    }
}

/* Per-datagram Rx / Tx checksum sequence of the stack on a strided batch (the CPU line of the fused
 * packet rows): IPv4 — Rx HdrVerify(IP header) (net_ipv4.c:5247) then, for TCP / UDP, DataVerify of
 * the transport over a one-buffer NET_BUF with the 12-B pseudo-header {src, dst, 0, proto, length}
 * (net_tcp.c:7851-7857, net_udp.c:1918-1934; UDP checksum 0 not checked, :1920); Tx the fields
 * zeroed, HdrCalc written (net_ipv4.c:9573-9586), DataCalc written, UDP 0 -> 0xFFFF
 * (net_tcp.c:29824-29862, net_udp.c:2891-2937). IPv6 without extension headers — the transport over
 * the 40-B pseudo-header {src, dst, length, 0, next header} (net_tcp.c:7871-7876, net_udp.c:1947-1953).
 * The version nibble picks the path per datagram. flags[i]: bit 0 IP header OK (IPv6: 1), bit 1
 * transport OK, bit 2 transport checked. No length / shape checks: the batch is well formed (the
 * configs' synthetic datagrams); test and bench use only. */
static uint16_t orc_be16(const uint8_t *p) { return (uint16_t)((p[0] << 8) | p[1]); }

static void orc_one_datagram(uint8_t *p, uint16_t avail, int tx, uint8_t *flag)
{
    uint8_t  pseudo[40];
    uint16_t plen, hlen, tot, l4len, c;
    uint8_t  proto;
    uint32_t err;
    NET_BUF  buf;
    uint8_t  f = 0u;
    int      v6 = (p[0] >> 4) == 6;
    if (v6) {
        hlen  = 40u;
        l4len = orc_be16(p + 4);
        tot   = (uint16_t)(40u + l4len);
        proto = p[6];
        memcpy(pseudo, p + 8, 32);
        pseudo[32] = 0u; pseudo[33] = 0u; pseudo[34] = (uint8_t)(l4len >> 8); pseudo[35] = (uint8_t)l4len;
        pseudo[36] = 0u; pseudo[37] = 0u; pseudo[38] = 0u; pseudo[39] = proto;
        plen  = 40u;
        f     = 1u;
    } else {
        hlen  = (uint16_t)((p[0] & 0x0Fu) * 4u);
        tot   = orc_be16(p + 2);
        proto = p[9];
        l4len = (uint16_t)(tot - hlen);
        if (tx) {
            p[10] = 0u; p[11] = 0u;
            c = Oracle_HdrCalc(p, hlen, &err, 0);
            memcpy(p + 10, &c, 2);
            f = 1u;
        } else {
            f = Oracle_HdrVerify(p, hlen, &err, 0) ? 1u : 0u;
        }
        memcpy(pseudo, p + 12, 8);
        pseudo[8] = 0u; pseudo[9] = proto; pseudo[10] = (uint8_t)(l4len >> 8); pseudo[11] = (uint8_t)l4len;
        plen  = 12u;
    }
    if (tot <= avail && (proto == 6u || proto == 17u)) {
        uint16_t fo = (uint16_t)(hlen + (proto == 6u ? 16u : 6u));
        buf.Hdr.NextBufPtr      = NULL;
        buf.Hdr.ProtocolHdrType = (proto == 6u) ? (v6 ? NET_PROTOCOL_TYPE_TCP_V6 : NET_PROTOCOL_TYPE_TCP_V4)
                                                : (v6 ? NET_PROTOCOL_TYPE_UDP_V6 : NET_PROTOCOL_TYPE_UDP_V4);
        buf.Hdr.TransportHdrIx  = hlen;
        buf.Hdr.TransportHdrLen = 0u;
        buf.Hdr.DataLen         = l4len;
        buf.DataPtr             = p;
        if (tx) {
            p[fo] = 0u; p[fo + 1u] = 0u;
            c = Oracle_DataCalc(&buf, pseudo, plen, &err, 0);
            if (proto == 17u && c == 0u) c = 0xFFFFu;
            memcpy(p + fo, &c, 2);
            f |= 6u;
        } else if (proto == 6u || orc_be16(p + fo) != 0u) {
            f |= (uint8_t)(4u | (Oracle_DataVerify(&buf, pseudo, plen, &err, 0) ? 2u : 0u));
        }
    }
    *flag = f;
}

void Oracle_PktBatch(uint8_t *base, uint64_t stride, uint16_t avail, uint32_t n, int tx, uint8_t *flags,
                     int n_threads)
{
    int64_t i;
#ifdef _OPENMP
    int nt = (n_threads > 0) ? n_threads : omp_get_max_threads();
#pragma omp parallel for schedule(static) num_threads(nt)
#else
    (void)n_threads;
#endif
    for (i = 0; i < (int64_t)n; ++i) {
        orc_one_datagram(base + (uint64_t)i * stride, avail, tx, &flags[i]);
    }
}

uint32_t Oracle_C1Loop(const void *pdata_buf, const void *ppseudo_hdr, uint16_t pseudo_hdr_size,
                       const void *ip_hdr, uint64_t iters)
{
    uint32_t acc = 0u, err = 0u;
    uint64_t k;
    for (k = 0; k < iters; ++k) {
        acc ^= Oracle_DataCalc(pdata_buf, ppseudo_hdr, pseudo_hdr_size, &err, 0);
        acc ^= (uint32_t)Oracle_HdrCalc(ip_hdr, 20u, &err, 0) << 16;
        acc += Oracle_HdrVerify(ip_hdr, 20u, &err, 0);
        acc += Oracle_DataVerify(pdata_buf, ppseudo_hdr, pseudo_hdr_size, &err, 0);
        __asm__ __volatile__("" : "+r"(acc) : : "memory");   /* one full sequence per iteration */
    }
    return acc ^ err;
}

int Oracle_MaxThreads(void)
{
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}

/* ------------------------------ synthetic bytes (== NetUtil_MI355X_Fill) ------------------ */

static inline uint64_t orc_splitmix64(uint64_t x)
{
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

void Oracle_Fill(uint8_t *buf, uint64_t first_byte, uint64_t n_bytes, uint64_t seed, int pattern)
{
    static const uint8_t carry_pat[4] = { 0xFFu, 0xFFu, 0x00u, 0x01u };
    uint64_t k;
    for (k = 0; k < n_bytes; ++k) {
        uint64_t a = first_byte + k;
        switch (pattern) {
        case 1:  buf[k] = 0x00u; break;
        case 2:  buf[k] = 0xFFu; break;
        case 3:  buf[k] = carry_pat[a & 3u]; break;
        default: buf[k] = (uint8_t)(orc_splitmix64(seed + (a >> 3)) >> (8u * (unsigned)(a & 7u)));
        }
    }
}

/* The same bytes, first-touched by the OpenMP workers that will read them: units of `unit` bytes
 * are distributed schedule(static) over n_threads threads, the partition Oracle_Batch* uses for
 * n_bytes / unit segments of `unit` bytes each (CPU-baseline setup). */
void Oracle_FillParallel(uint8_t *buf, uint64_t first_byte, uint64_t n_bytes, uint64_t seed, int pattern,
                         int n_threads, uint64_t unit)
{
    int nt = (n_threads > 0) ? n_threads : omp_get_max_threads();
    uint64_t n_units = unit ? (n_bytes + unit - 1u) / unit : 1u;
    int64_t u;
    if (unit == 0u) unit = n_bytes;
#pragma omp parallel for schedule(static) num_threads(nt)
    for (u = 0; u < (int64_t)n_units; ++u) {
        uint64_t lo = (uint64_t)u * unit;
        uint64_t len = (lo + unit <= n_bytes) ? unit : n_bytes - lo;
        Oracle_Fill(buf + lo, first_byte + lo, len, seed, pattern);
    }
}

/* ------------------------------ CRC-32 (net_util.c:485-636) ------------------------------- */

/* Restates NetUtil_32BitCRC_Calc (net_util.c:485-530): register starts at
 * NET_UTIL_32_BIT_ONES_CPL_NEG_ZERO (0xFFFFFFFF, :58), each octet is XORed into the low byte and
 * shifted out bit by bit against the reflected IEEE 802.3 polynomial 0xEDB88320 (:77), no final
 * complement. Argument checks of NET_ERR_CFG_ARG_CHK_EXT_EN (template default enabled,
 * net_cfg.h:178): NULL -> NET_ERR_FAULT_NULL_PTR (23), zero length -> NET_UTIL_ERR_NULL_SIZE (210),
 * both returning 0. */
uint32_t Oracle_CRC32Calc(const uint8_t *p_data, uint32_t data_len, uint32_t *p_err)
{
    uint32_t crc = 0xFFFFFFFFu, i, j;
    if (p_data == NULL) {
        *p_err = 23u;
        return 0u;
    }
    if (data_len < 1u) {
        *p_err = 210u;
        return 0u;
    }
    for (i = 0u; i < data_len; ++i) {
        uint32_t v = (crc ^ p_data[i]) & 0xFFu;
        for (j = 0u; j < 8u; ++j) {
            v = (v & 1u) ? ((v >> 1) ^ 0xEDB88320u) : (v >> 1);
        }
        crc = (crc >> 8) ^ v;
    }
    *p_err = 200u;
    return crc;
}

/* NetUtil_32BitCRC_CalcCpl (net_util.c:571-588): the same, complemented; 0 on error. */
uint32_t Oracle_CRC32CalcCpl(const uint8_t *p_data, uint32_t data_len, uint32_t *p_err)
{
    uint32_t crc = Oracle_CRC32Calc(p_data, data_len, p_err);
    if (*p_err != 200u) {
        return 0u;
    }
    return crc ^ 0xFFFFFFFFu;
}

/* NetUtil_32BitReflect (net_util.c:610-636): bit i -> bit 31 - i. */
uint32_t Oracle_Reflect32(uint32_t val)
{
    uint32_t r = 0u, i;
    for (i = 0u; i < 32u; ++i) {
        if (val & (1u << i)) {
            r |= 1u << (31u - i);
        }
    }
    return r;
}

/* Batch driver: out[i] = Calc (cpl 0) or CalcCpl (cpl 1) of segment i (base + off[i] or
 * base + i*stride, len[i] or len bytes); 0 for an empty segment (the reference's NULL_SIZE). */
void Oracle_CRC32Batch(const uint8_t *base, const uint64_t *off, const uint32_t *lens, uint64_t stride,
                       uint32_t len, uint32_t n, uint32_t *out, int cpl)
{
    uint32_t i, err;
    for (i = 0u; i < n; ++i) {
        const uint8_t *p = base + (off ? off[i] : (uint64_t)i * stride);
        const uint32_t l = lens ? lens[i] : len;
        out[i] = cpl ? Oracle_CRC32CalcCpl(p, l, &err) : Oracle_CRC32Calc(p, l, &err);
    }
}
