/*
 * netcsum_netbuf.h — standalone mirror of the NET_BUF fields the checksum path reads.
 *
 * Reference: struct net_buf_hdr   Source/net_buf.h:394-562
 *            struct net_buf       Source/net_buf.h:595-598
 * Fields read by NetUtil_16BitOnesCplSumDataCalc (Source/net_util.c:1611-1687):
 *   NextBufPtr, ProtocolHdrType, ICMP_MsgIx, ICMP_HdrLen, TransportHdrIx, TransportHdrLen,
 *   DataLen, TotLen, DataPtr.
 *
 * The reference layout changes with configuration macros (#ifdef blocks at net_buf.h:436-440,
 * 442-445,457-460,475-478,484-521,526-554). This mirror reproduces the layout of the TEMPLATE
 * configuration (Cfg/Template/net_cfg.h: IPv4 + TCP + ARP + IGMP, no IPv6/DAD/NDP/MLDP) on an
 * LP64 little-endian gcc/clang target. Offsets derived field by field from net_buf.h:394-562
 * (enums 4 B, pointers 8 B):
 *
 *     Flags            6   NextBufPtr      72   ProtocolHdrType 104   ICMP_MsgIx   146
 *     ICMP_HdrLen    150   TransportHdrIx 156   TransportHdrLen 158   DataLen      166
 *     TotLen         168   sizeof(NET_BUF_HDR) 304                    DataPtr      304
 *
 * Inside a real µC/TCP-IP build, DO NOT use this header: compile host/net_util_mi355x.c against the
 * stack's own net_buf.h — the field NAMES below are identical, so the same C
 * source works with either definition.
 */
#ifndef NETCSUM_NETBUF_H
#define NETCSUM_NETBUF_H

#include <stddef.h>
#include <stdint.h>
#include "netcsum_types.h"

#ifndef NET_BUF_MODULE_PRESENT

typedef struct net_buf NET_BUF;

typedef struct net_buf_hdr {
    uint8_t            _rsvd_000[6];          /* Type, Size                                   */
    CPU_INT16U         Flags;                 /* @6                                           */
    uint8_t            _rsvd_008[64];         /* ID, RefCtr, IF_Nbr*, Prev/Next list ptrs      */
    NET_BUF           *NextBufPtr;            /* @72                                          */
    uint8_t            _rsvd_080[24];         /* TmrPtr, UnlinkFnctPtr, UnlinkObjPtr           */
    NET_PROTOCOL_TYPE  ProtocolHdrType;       /* @104                                         */
    uint8_t            _rsvd_108[38];         /* ProtocolHdrType{IF,...}, IF/ARP/IP ix & lens  */
    CPU_INT16U         ICMP_MsgIx;            /* @146                                         */
    CPU_INT16U         ICMP_MsgLen;           /* @148                                         */
    CPU_INT16U         ICMP_HdrLen;           /* @150                                         */
    CPU_INT16U         IGMP_MsgIx;            /* @152                                         */
    CPU_INT16U         IGMP_MsgLen;           /* @154                                         */
    CPU_INT16U         TransportHdrIx;        /* @156                                         */
    CPU_INT16U         TransportHdrLen;       /* @158                                         */
    CPU_INT16U         TransportTotLen;       /* @160                                         */
    CPU_INT16U         TransportDataLen;      /* @162                                         */
    CPU_INT16U         DataIx;                /* @164                                         */
    CPU_INT16U         DataLen;               /* @166  (NET_BUF_SIZE = CPU_INT16U, :272)      */
    CPU_INT16U         TotLen;                /* @168                                         */
    uint8_t            _rsvd_170[134];        /* ARP ptrs, IP frag/addr fields, TCP fields ... */
} NET_BUF_HDR;

struct net_buf {
    NET_BUF_HDR  Hdr;
    CPU_INT08U  *DataPtr;                     /* @304                                         */
};

#if defined(__cplusplus)
#define NETCSUM_STATIC_ASSERT static_assert
#else
#define NETCSUM_STATIC_ASSERT _Static_assert
#endif
NETCSUM_STATIC_ASSERT(offsetof(NET_BUF_HDR, Flags)           ==   6, "NET_BUF_HDR.Flags");
NETCSUM_STATIC_ASSERT(offsetof(NET_BUF_HDR, NextBufPtr)      ==  72, "NET_BUF_HDR.NextBufPtr");
NETCSUM_STATIC_ASSERT(offsetof(NET_BUF_HDR, ProtocolHdrType) == 104, "NET_BUF_HDR.ProtocolHdrType");
NETCSUM_STATIC_ASSERT(offsetof(NET_BUF_HDR, ICMP_MsgIx)      == 146, "NET_BUF_HDR.ICMP_MsgIx");
NETCSUM_STATIC_ASSERT(offsetof(NET_BUF_HDR, ICMP_HdrLen)     == 150, "NET_BUF_HDR.ICMP_HdrLen");
NETCSUM_STATIC_ASSERT(offsetof(NET_BUF_HDR, TransportHdrIx)  == 156, "NET_BUF_HDR.TransportHdrIx");
NETCSUM_STATIC_ASSERT(offsetof(NET_BUF_HDR, TransportHdrLen) == 158, "NET_BUF_HDR.TransportHdrLen");
NETCSUM_STATIC_ASSERT(offsetof(NET_BUF_HDR, DataLen)         == 166, "NET_BUF_HDR.DataLen");
NETCSUM_STATIC_ASSERT(offsetof(NET_BUF_HDR, TotLen)          == 168, "NET_BUF_HDR.TotLen");
NETCSUM_STATIC_ASSERT(sizeof(NET_BUF_HDR)                    == 304, "sizeof NET_BUF_HDR");
NETCSUM_STATIC_ASSERT(offsetof(NET_BUF, DataPtr)             == 304, "NET_BUF.DataPtr");
NETCSUM_STATIC_ASSERT(sizeof(NET_BUF)                        == 312, "sizeof NET_BUF");

#endif /* !NET_BUF_MODULE_PRESENT */

#endif /* NETCSUM_NETBUF_H */
