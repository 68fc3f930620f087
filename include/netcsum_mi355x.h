/*
 * netcsum_mi355x.h — C ABI of the MI355X (gfx950) Internet-checksum path.
 *
 * Drop-in for µC/TCP-IP V3.06.01 Source/net_util.c's 16-bit one's-complement checksum
 * (RFC 1071). Everything here is plain C: pointers, sizes, NET_ERR codes. No torch or HIP
 * types cross this boundary; HIP streams are passed as `void *` (a hipStream_t, NULL = the
 * legacy default stream of the current device).
 *
 * Library: uc-tcp-ip_amd/libnetcsum_mi355x.so (built by `make -C uc-tcp-ip_amd`).
 *
 * Three groups of entry points:
 *
 *  (1) The reference's four public checksum functions, SAME signatures and semantics
 *      (Source/net_util.h:422-438). Callers in net_ipv4.c, net_icmpv4.c, net_igmp.c,
 *      net_tcp.c, net_udp.c, net_icmpv6.c link against these unchanged (SURVEY §8(b) lists all
 *      23 call sites). The host side walks the NET_BUF chain and the bytes are summed on the GPU.
 *
 *  (2) The additive batch ABI (the throughput path): N independent segments resident in HBM,
 *      one output element per segment, results bit-identical to calling (1) once per segment
 *      with a one-buffer NET_BUF chain.
 *
 *  (3) Support: the exact stream sum used by (1), the NET_BUF chain walk (host logic, exported
 *      so it can be tested without a GPU), synthetic-input generation and a read-stream
 *      roofline probe for the bench.
 */
#ifndef NETCSUM_MI355X_H
#define NETCSUM_MI355X_H

#include <stddef.h>
#include <stdint.h>
#include "netcsum_types.h"

#ifdef __cplusplus
extern "C" {
#endif

/* ============================================================================================
 * (1) Reference signatures (Source/net_util.h:422-438, implemented in net_util.c:159-449).
 *
 *  NetUtil_16BitOnesCplChkSumHdrCalc      replaces Source/net_util.c:159  (decl net_util.h:422)
 *  NetUtil_16BitOnesCplChkSumHdrVerify    replaces Source/net_util.c:245  (decl net_util.h:426)
 *  NetUtil_16BitOnesCplChkSumDataCalc     replaces Source/net_util.c:344  (decl net_util.h:430)
 *  NetUtil_16BitOnesCplChkSumDataVerify   replaces Source/net_util.c:428  (decl net_util.h:435)
 *
 * Return-value convention is the reference's: Calc returns the checksum in HOST order such that
 * a memcpy into the header yields network byte order (net_util.c:187-188, :358); Verify returns
 * DEF_OK/DEF_FAIL. *p_err = NET_UTIL_ERR_NONE on success; NET_UTIL_ERR_INVALID_PROTOCOL for an
 * unknown ProtocolHdrType (net_util.c:1637-1639). With NETCSUM_ARG_CHK_DBG_EN=1 at build time the
 * NET_ERR_CFG_ARG_CHK_DBG_EN checks of net_util.c:168-179,255-266,1566-1577,1642-1672 apply.
 * A device failure returns 0 / DEF_FAIL with *p_err = NET_UTIL_ERR_MI355X_DEV (never a CPU path).
 * ============================================================================================ */
NET_CHK_SUM  NetUtil_16BitOnesCplChkSumHdrCalc   (void        *phdr,
                                                  CPU_INT16U   hdr_size,
                                                  NET_ERR     *p_err);

CPU_BOOLEAN  NetUtil_16BitOnesCplChkSumHdrVerify (void        *phdr,
                                                  CPU_INT16U   hdr_size,
                                                  NET_ERR     *p_err);

NET_CHK_SUM  NetUtil_16BitOnesCplChkSumDataCalc  (void        *pdata_buf,
                                                  void        *ppseudo_hdr,
                                                  CPU_INT16U   pseudo_hdr_size,
                                                  NET_ERR     *p_err);

CPU_BOOLEAN  NetUtil_16BitOnesCplChkSumDataVerify(void        *pdata_buf,
                                                  void        *ppseudo_hdr,
                                                  CPU_INT16U   pseudo_hdr_size,
                                                  NET_ERR     *p_err);

/* The reference's optional native-loop seam (net_util.h:486-490; NET_CFG_OPTIMIZE_ASM_EN): unfolded
 * sum of the network-order 16-bit words of [pdata_32, pdata_32 + size), size a multiple of 4, as
 * NetUtil_16BitSumDataCalc adds it (net_util.c:1407-1415). A stack that keeps its own net_util.c with
 * the ASM option enabled links this instead of a Ports/<cpu>/net_util_a.* file. Per-buffer and
 * synchronous (one GPU round trip per call); a device failure returns 0 with a message on stderr
 * (the signature has no error channel). */
CPU_INT32U   NetUtil_16BitSumDataCalcAlign_32    (void        *pdata_32,
                                                  CPU_INT32U   size);

/* CRC-32 of net_util.c:485-636 (IEEE 802.3 polynomial, reflected, register initialised to
 * 0xFFFFFFFF): Calc returns the register, CalcCpl its complement (the Ethernet FCS value), Reflect
 * reverses the 32 bits (net_util.c:610-636; the drivers' multicast hash, e.g.
 * Dev/Ether/GMAC/net_dev_gmac.c:2673-2683). With NETCSUM_ARG_CHK_EXT_EN (default 1, the template's
 * NET_ERR_CFG_ARG_CHK_EXT_EN = DEF_ENABLED, net_cfg.h:178): p_data NULL -> 0 and
 * NET_ERR_FAULT_NULL_PTR, data_len 0 -> 0 and NET_UTIL_ERR_NULL_SIZE. A call of up to 4096 octets
 * (the stack's only use: 6-octet multicast MAC hashes) runs the reference's register update in host
 * C — a GPU round trip would cost ~1000 x the CPU loop; a longer buffer goes to the GPU kernel
 * (NetUtil_MI355X_CRC32Host). Reflect is a bit permutation of one register, done in host C. A stack
 * may equally keep its own net_util.c CRC functions: throughput CRCs are the batch
 * entry points below.
 *  NetUtil_32BitCRC_Calc     replaces Source/net_util.c:485  (decl net_util.h:442)
 *  NetUtil_32BitCRC_CalcCpl  replaces Source/net_util.c:571  (decl net_util.h:446)
 *  NetUtil_32BitReflect      replaces Source/net_util.c:610  (decl net_util.h:450) */
CPU_INT32U   NetUtil_32BitCRC_Calc               (CPU_INT08U  *p_data,
                                                  CPU_INT32U   data_len,
                                                  NET_ERR     *p_err);

CPU_INT32U   NetUtil_32BitCRC_CalcCpl            (CPU_INT08U  *p_data,
                                                  CPU_INT32U   data_len,
                                                  NET_ERR     *p_err);

CPU_INT32U   NetUtil_32BitReflect                (CPU_INT32U   val);

/* ============================================================================================
 * (2) Batch ABI — device-resident segments.
 *
 * Segment i is the byte span [seg_i, seg_i + len_i) in device memory, any alignment (odd starts
 * are fine); its optional pseudo-header is [d_pseudo + i*pseudo_stride, +pseudo_len).
 * out[i] equals what the reference returns for ONE NET_BUF whose data area holds the segment
 * (ProtocolHdrType TCP/UDP, TransportHdrIx -> segment start) and ppseudo_hdr -> the pseudo-header:
 *
 *   NETCSUM_OP_DATA_CALC    uint16_t out[i] = NetUtil_16BitOnesCplChkSumDataCalc(...)
 *   NETCSUM_OP_DATA_VERIFY  uint8_t  out[i] = NetUtil_16BitOnesCplChkSumDataVerify(...)
 *   NETCSUM_OP_HDR_CALC     uint16_t out[i] = NetUtil_16BitOnesCplChkSumHdrCalc(seg_i, len_i)
 *   NETCSUM_OP_HDR_VERIFY   uint8_t  out[i] = NetUtil_16BitOnesCplChkSumHdrVerify(seg_i, len_i)
 *
 * (HDR ops take no pseudo-header: pass d_pseudo = NULL.) Lengths are CPU_INT16U as in the
 * reference (net_util.c:1617,1628: per-buffer data_len is 16-bit). The call is asynchronous
 * on `hip_stream`; returns NET_UTIL_ERR_NONE when the launch was queued. n_seg <= 2^31 - 1.
 * ============================================================================================ */
typedef enum netcsum_op {
    NETCSUM_OP_DATA_CALC   = 0,
    NETCSUM_OP_DATA_VERIFY = 1,
    NETCSUM_OP_HDR_CALC    = 2,
    NETCSUM_OP_HDR_VERIFY  = 3
} NETCSUM_OP;

/* Uniform segments: seg_i = d_seg + i*seg_stride, len_i = seg_len (config C2/C3/C5). */
NET_ERR  NetUtil_MI355X_ChkSumBatchStrided (const void  *d_seg,
                                            uint64_t     seg_stride,
                                            CPU_INT16U   seg_len,
                                            const void  *d_pseudo,
                                            uint32_t     pseudo_stride,
                                            CPU_INT16U   pseudo_len,
                                            uint32_t     n_seg,
                                            void        *d_out,
                                            NETCSUM_OP   op,
                                            void        *hip_stream);

/* Variable-length segments: seg_i = d_base + d_seg_off[i], len_i = d_seg_len[i] (config C4). */
NET_ERR  NetUtil_MI355X_ChkSumBatchVarLen  (const void      *d_base,
                                            const uint64_t  *d_seg_off,
                                            const uint16_t  *d_seg_len,
                                            const void      *d_pseudo,
                                            uint32_t         pseudo_stride,
                                            CPU_INT16U       pseudo_len,
                                            uint32_t         n_seg,
                                            void            *d_out,
                                            NETCSUM_OP       op,
                                            void            *hip_stream);

/* Host-memory variant of the strided batch (the path starts and ends in host memory: NIC Rx
 * buffers / socket Tx buffers). h_seg/h_pseudo/h_out should be pinned (hipHostMalloc) for
 * overlap; the call pipelines H2D -> kernel -> D2H over `n_chunks` chunks on internal streams of
 * the current device and returns when h_out is complete. */
NET_ERR  NetUtil_MI355X_ChkSumBatchStridedHost(const void  *h_seg,
                                               uint64_t     seg_stride,
                                               CPU_INT16U   seg_len,
                                               const void  *h_pseudo,
                                               uint32_t     pseudo_stride,
                                               CPU_INT16U   pseudo_len,
                                               uint32_t     n_seg,
                                               void        *h_out,
                                               NETCSUM_OP   op,
                                               uint32_t     n_chunks);

/* ============================================================================================
 * (2b) IPv4 packet batches. Packet i = one IPv4 datagram starting at
 * its IP header: d_base + d_off[i] with d_len[i] bytes present (d_off/d_len non-NULL), or
 * d_base + i*stride with pkt_len bytes present (d_off = d_len = NULL). Any alignment. Strided
 * batches need 7 * stride + 65536 < 2^32 (packets at most ~613 MB apart), else
 * NET_UTIL_ERR_MI355X_INVALID_ARG; offset/length batches have no such bound.
 *
 * RxValidateIPv4 — one HBM pass per packet, d_flags[i] = NETCSUM_PKT_* bits:
 *   IP_OK       NetUtil_16BitOnesCplChkSumHdrVerify(ip_hdr, IHL*4) == DEF_OK      (net_ipv4.c:5247)
 *   L4_CHECKED  a transport checksum was verified: TCP (6), UDP (17) with a non-zero checksum
 *               field, ICMP (1), IGMP (2); pseudo-header {src, dst, 0, proto, len} built from
 *               the IP header (net_tcp.c:7851-7857, net_udp.c:1918-1934)
 *   L4_OK       that verification passed (also set for UDP_NO_CSUM: accepted, net_udp.c:1971)
 *   UDP_NO_CSUM UDP checksum field 0 (no checksum transmitted)
 *   MALFORMED   IP version/IHL/total length inconsistent with the bytes present: no verdict
 *   FRAGMENT    MF or fragment offset set: IP verdict only
 *   L4_MALFORMED transport length invalid (TCP < 20 B, UDP length != IP datagram length)
 * TxFinalizeIPv4 — computes and writes back, IN PLACE, the IPv4 header checksum and the
 *   TCP/UDP/ICMP/IGMP checksum (fields treated as zero; UDP 0x0000 sent as 0xFFFF, RFC 768;
 *   udp_tx_csum = 0 writes 0 = no UDP checksum, NET_UDP_CFG_TX_CHK_SUM_EN); d_flags optional
 *   (IP_OK = IP checksum written, L4_CHECKED = transport checksum written).
 * ============================================================================================ */
#define NETCSUM_PKT_IP_OK         0x01u
#define NETCSUM_PKT_L4_OK         0x02u
#define NETCSUM_PKT_L4_CHECKED    0x04u
#define NETCSUM_PKT_UDP_NO_CSUM   0x08u
#define NETCSUM_PKT_MALFORMED     0x10u
#define NETCSUM_PKT_FRAGMENT      0x20u
#define NETCSUM_PKT_L4_MALFORMED  0x40u
#define NETCSUM_PKT_EXT_HDR       0x80u   /* IPv6 only: next header is an extension header */

NET_ERR  NetUtil_MI355X_RxValidateIPv4     (const void      *d_base,
                                            const uint64_t  *d_off,
                                            const uint16_t  *d_len,
                                            uint64_t         stride,
                                            CPU_INT16U       pkt_len,
                                            uint32_t         n_pkt,
                                            uint8_t         *d_flags,
                                            void            *hip_stream);

NET_ERR  NetUtil_MI355X_TxFinalizeIPv4     (void            *d_base,
                                            const uint64_t  *d_off,
                                            const uint16_t  *d_len,
                                            uint64_t         stride,
                                            CPU_INT16U       pkt_len,
                                            uint32_t         n_pkt,
                                            uint8_t         *d_flags,
                                            int              udp_tx_csum,
                                            void            *hip_stream);

/* ============================================================================================
 * (2b') IPv6 packet batches (the 40-B pseudo-header of net_ipv6.h:844-852). Same
 * layout and arguments as (2b); packet i starts at its 40-B IPv6 header. Flags:
 *   IP_OK       header well-formed (version 6, 40 + payload length <= bytes present); IPv6 has no
 *               header checksum (MALFORMED otherwise)
 *   L4_CHECKED / L4_OK / UDP_NO_CSUM / L4_MALFORMED   as (2b), for a transport header directly after
 *               the IPv6 header, pseudo-header {src, dst, payload length, 0, next header}:
 *               TCP (net_tcp.c:7871-7879), UDP (net_udp.c:1947-1957), ICMPv6 (58): types 128-131 and
 *               134-137 with the pseudo-header (net_icmpv6.c:2923-2942); types 1, 3, 4 HdrVerify over
 *               the message alone, as the reference does (net_icmpv6.c:2910-2920); other types get no
 *               verdict (the reference rejects them before any checksum, net_icmpv6.c:2945)
 *   Extension headers: Hop-by-Hop (0, first only), Routing (43) and Destination Options (60) are
 *               skipped, a chain of any length as NetIPv6_RxPktProcessExtHdr walks it
 *               (net_ipv6.c:8396-8510; upper-layer length = payload length - their bytes,
 *               net_ipv6.c:5682), each judged as the reference's handler judges it: the options of
 *               Hop-by-Hop / Destination Options headers are walked and one whose type & 0x1F is not
 *               Pad1 / PadN / Router Alert with non-"skip" action bits drops the datagram
 *               (NetIPv6_RxOptHdr, net_ipv6.c:8604-8672); a routing type > 2 with Segments Left != 0
 *               drops it (NetIPv6_RxRoutingHdr, :8735-8753). The batch kernel walks accepted Routing
 *               headers its first loads hold; a second pass (netcsum_v6walk.hip, launched work only
 *               when the batch deferred a datagram) the option headers and longer chains; a Fragment
 *               header (44) gives FRAGMENT; a header running past the payload gives MALFORMED (the
 *               reference does not check this, and reads on past the payload)
 *   EXT_HDR     a datagram the reference drops in its extension-header processing: a dropping option
 *               or routing header (above), any other extension header (50, 51, 59, 135, 139, 140, 253,
 *               254) or a late Hop-by-Hop header: no transport verdict. ESP and Mobility:
 *               NET_IPv6_ERR_INVALID_EH, net_ipv6.c:8837-8846, :8956-8965; AH: the next header is read
 *               from the IPv6 header's first octet, 0x6X, and rejected as NET_IPv6_ERR_INVALID_PROTOCOL,
 *               :8885-8894, :8357-8360; No Next Header: no upper layer, :8460-8462
 * TxFinalizeIPv6 writes the TCP / UDP / ICMPv6 checksum in place (net_tcp.c:29839-29862,
 *   net_udp.c:2909-2937, net_icmpv6.c:1439 and :949-965); UDP 0x0000 -> 0xFFFF, udp_tx_csum = 0
 *   writes 0; no header checksum to write.
 * ============================================================================================ */
NET_ERR  NetUtil_MI355X_RxValidateIPv6     (const void      *d_base,
                                            const uint64_t  *d_off,
                                            const uint16_t  *d_len,
                                            uint64_t         stride,
                                            CPU_INT16U       pkt_len,
                                            uint32_t         n_pkt,
                                            uint8_t         *d_flags,
                                            void            *hip_stream);

NET_ERR  NetUtil_MI355X_TxFinalizeIPv6     (void            *d_base,
                                            const uint64_t  *d_off,
                                            const uint16_t  *d_len,
                                            uint64_t         stride,
                                            CPU_INT16U       pkt_len,
                                            uint32_t         n_pkt,
                                            uint8_t         *d_flags,
                                            int              udp_tx_csum,
                                            void            *hip_stream);

/* Mixed IPv4 / IPv6 batches (a NIC ring carrying both): packet i goes through (2b) when the version
 * nibble of its first byte is 4 (or anything but 6) and through (2b') when it is 6; same arguments,
 * same flags, one launch. */
NET_ERR  NetUtil_MI355X_RxValidateIP       (const void      *d_base,
                                            const uint64_t  *d_off,
                                            const uint16_t  *d_len,
                                            uint64_t         stride,
                                            CPU_INT16U       pkt_len,
                                            uint32_t         n_pkt,
                                            uint8_t         *d_flags,
                                            void            *hip_stream);

NET_ERR  NetUtil_MI355X_TxFinalizeIP       (void            *d_base,
                                            const uint64_t  *d_off,
                                            const uint16_t  *d_len,
                                            uint64_t         stride,
                                            CPU_INT16U       pkt_len,
                                            uint32_t         n_pkt,
                                            uint8_t         *d_flags,
                                            int              udp_tx_csum,
                                            void            *hip_stream);

/* ============================================================================================
 * (2b'') Burst adapters for the reference's own checksum-offload seam.
 *
 * The reference builds with NET_{IPV4,ICMP,UDP,TCP}_CFG_CHK_SUM_OFFLOAD_{RX,TX}_EN
 * (Cfg/Template/net_cfg.h:669-682, mapped to NET_*_CHK_SUM_OFFLOAD_{RX,TX} at
 * Source/net_cfg_net.h:174-190, 305-366) when "the controller" computes the checksums: the stack
 * then skips those calls. These two entry points ARE that controller, one launch per NIC burst:
 *
 * RxBurst — run before the burst is handed to the stack (NetIF_Rx). d_action[i] is one of
 *   NETCSUM_RX_* below. With the Rx offload flags enabled the stack assumes every checksum valid
 *   (net_ipv4.c:5243-5244, net_tcp.c:7847-7848 / :7868-7869, net_udp.c:1925-1927 / :1944-1946,
 *   net_icmpv4.c:1673-1674 / :1683-1684, net_icmpv6.c:2931-2932), so a frame whose checksum fails
 *   must be dropped HERE; a frame the reference would reject for any other reason (header shape,
 *   lengths, types, addresses, ports) is delivered and the stack's own checks, which the offload
 *   flags do not remove, reject it. Decisions therefore equal the reference's with the flags off:
 *   a frame is delivered iff its checksums pass (or it carries none), and every frame the
 *   reference drops at a checksum check is dropped. The DROP code names the counter the reference
 *   increments at that check; for a frame that ALSO fails an earlier non-checksum check (an
 *   ICMPv4 type/code/length, net_icmpv4.c:1500-1659) the reference counts that check instead.
 *   IPv4 fragments: the transport checksum covers the reassembled datagram (net_ipv4.c:6523), which
 *   a per-frame burst does not hold; they are verified at the IP header only (DELIVER_L4_UNVERIFIED,
 *   what any offloading NIC does; ChkSumBatchChains verifies reassembled datagrams).
 *   IGMP (net_igmp.c:1332) and ICMPv6 types 1/3/4 (net_icmpv6.c:2913) have no offload flag; the
 *   adapter drops their checksum failures too (same decision, same counter), so the stack's own
 *   per-packet call only ever sees valid ones.
 *   rx_cfg: NETCSUM_RXCFG_UDP_DISCARD_NO_CHK_SUM = the stack's NET_UDP_CFG_RX_CHK_SUM_DISCARD_EN
 *   (net_udp.c:1972-1977: UDP datagrams without a checksum are dropped); 0 = the template default.
 *   d_flags (optional, NULL allowed) receives the NETCSUM_PKT_* verdicts of RxValidateIP.
 *
 * TxBurst — run on frames the stack built with the Tx offload flags, before they go to the NIC:
 *   the stack left 0 in the IPv4 header checksum (net_ipv4.c:9575-9586, :10160-10171), 0 in TCP
 *   (net_tcp.c:29813-29815, :29845-29847) and ICMPv4 (net_icmpv4.c:1046, :2225, :2245, :3093,
 *   :3124), and in UDP the placeholder 0xFFFF: its own 0 -> 0xFFFF mapping (net_udp.c:2929-2931)
 *   runs on the offload's 0 (:2877-2878, :2901-2902). A UDP field of 0 means "no checksum"
 *   (NET_UDP_CFG_TX_CHK_SUM_EN / NET_UDP_FLAG_TX_CHK_SUM_DIS, net_udp.c:2863-2867, :2934-2935) and
 *   is left 0. Every other checksum field is computed as if zero and written in place (as
 *   TxFinalizeIP, UDP 0 -> 0xFFFF). Fields the stack computed itself — ICMPv6 and ICMPv4 echo
 *   requests, whose guards test the never-defined NET_ICMP_CFG_CHK_SUM_OFFLOAD_TX
 *   (net_icmpv6.c:1439, :1521, :2224, :2273, :2322, :2354; net_icmpv4.c:2201), and IGMP, which has
 *   no flag (net_igmp.c:1692) — are rewritten with the value they already hold. Frames starting at
 *   the IP header, mixed IPv4 / IPv6 as RxValidateIP / TxFinalizeIP.
 * ============================================================================================ */
#define NETCSUM_RX_DELIVER                 0u  /* hand to the stack                                  */
#define NETCSUM_RX_DROP_IPV4_CHK_SUM       1u  /* IPv4.RxInvChkSumCtr      net_ipv4.c:5251-5254        */
#define NETCSUM_RX_DROP_TCP_CHK_SUM        2u  /* TCP.RxHdrChkSumCtr       net_tcp.c:7886-7889         */
#define NETCSUM_RX_DROP_UDP_CHK_SUM        3u  /* UDP.RxHdrChkSumCtr       net_udp.c:1963-1967         */
#define NETCSUM_RX_DROP_UDP_NO_CHK_SUM     4u  /* UDP.RxHdrChkSumCtr       net_udp.c:1973-1977         */
#define NETCSUM_RX_DROP_ICMPV4_CHK_SUM     5u  /* ICMPv4.RxInvChkSumCtr    net_icmpv4.c:1697-1700      */
#define NETCSUM_RX_DROP_IGMP_CHK_SUM       6u  /* IGMP.RxHdrChkSumCtr      net_igmp.c:1335-1339        */
#define NETCSUM_RX_DROP_ICMPV6_CHK_SUM     7u  /* ICMPv6.RxHdrChkSumCtr    net_icmpv6.c:2952-2955      */
#define NETCSUM_RX_DELIVER_L4_UNVERIFIED   8u  /* IPv4 / IPv6 fragment: IP layer verified only       */
#define NETCSUM_RX_NBR_ACTIONS             9u

#define NETCSUM_RXCFG_UDP_DISCARD_NO_CHK_SUM  0x1u

NET_ERR  NetUtil_MI355X_RxBurst            (const void      *d_base,
                                            const uint64_t  *d_off,
                                            const uint16_t  *d_len,
                                            uint64_t         stride,
                                            CPU_INT16U       pkt_len,
                                            uint32_t         n_pkt,
                                            uint32_t         rx_cfg,
                                            uint8_t         *d_action,
                                            uint8_t         *d_flags,
                                            void            *hip_stream);

NET_ERR  NetUtil_MI355X_TxBurst            (void            *d_base,
                                            const uint64_t  *d_off,
                                            const uint16_t  *d_len,
                                            uint64_t         stride,
                                            CPU_INT16U       pkt_len,
                                            uint32_t         n_pkt,
                                            uint8_t         *d_flags,
                                            void            *hip_stream);

/* The action of one datagram from its RxValidateIP verdict `flags` (NETCSUM_PKT_*), the transport
 * protocol its checksum verdict covers (6, 17, 1, 2, 58) and its IP version: the function the Rx
 * burst kernels apply per frame, as host logic (no device work). */
uint8_t  NetUtil_MI355X_RxAction           (uint8_t          flags,
                                            uint8_t          proto,
                                            int              ipv6,
                                            uint32_t         rx_cfg);

/* Host tally of a burst's actions (after copying d_action to the host): ctr[a] += number of frames
 * with action a, a < NETCSUM_RX_NBR_ACTIONS — the increments the stack's Net_ErrCtrs would have seen
 * (NET_CTR_ERR_INC at the lines above). Host logic, no device work. */
NET_ERR  NetUtil_MI355X_RxBurstTally       (const uint8_t   *h_action,
                                            uint32_t         n_pkt,
                                            uint32_t        *ctr);

/* ============================================================================================
 * (2e) Host-memory forms (the path starts in NIC Rx buffers, IF/net_if.c:6593,
 * and socket Tx buffers, Source/net_sock.c:5531). Same arguments and results as the device forms
 * above with every pointer in HOST memory. The call splits the batch into n_chunks chunks and
 * pipelines, on three streams of the calling thread's context, H2D of each chunk's byte span
 * [min offset, max end) (plus its descriptors) -> the device form -> D2H of the results (Tx: one
 * 8-B record of the fields written per datagram, which the call writes into the host buffer, so
 * the call owns those bytes while it runs; a Tx batch's datagrams must not overlap one another,
 * as the stack's buffers do not). n_chunks 0 = the library's choice: one chunk, except TxFinalizeIPHost /
 * TxBurstHost from 32 Ki datagrams (n / 16 Ki chunks, at most 16). Every chunk adds 15-20 us to a
 * call and PCIe stays the bound, so bursts of a few thousand frames are fastest in one
 * (tools/burst_latency.c). Host buffers should be pinned (hipHostMalloc / hipHostRegister) for the
 * copies to run at PCIe rate. Returns when every result is in
 * host memory. IP = mixed IPv4 / IPv6 (per datagram by the version nibble).
 * Packet bursts (RxValidateIPHost, TxFinalizeIPHost, RxBurstHost, TxBurstHost) of <= 4096 frames with
 * n_chunks 0 whose frames lie in ONE pinned allocation (<= 64 MiB span) are not copied: the calling
 * thread's resident burst server kernel reads them in place over PCIe and writes the results into
 * coherent pinned memory the call polls (NETCSUM_TUNE_BURST_ZERO_COPY; 1 frame ~7 us, 64 frames
 * ~11 us). The server stays resident until idle for NETCSUM_TUNE_BURST_SERVER_IDLE_US (500 us), so a
 * device-wide synchronisation right after a burst may wait up to that long, and never longer than
 * NETCSUM_TUNE_BURST_SERVER_LIFE_US (1000 us) per launch while bursts keep coming: work on other
 * streams that share the server's hardware queue waits at most that long plus one burst.
 * ============================================================================================ */
NET_ERR  NetUtil_MI355X_ChkSumBatchVarLenHost(const void      *h_base,
                                              const uint64_t  *h_seg_off,
                                              const uint16_t  *h_seg_len,
                                              const void      *h_pseudo,
                                              uint32_t         pseudo_stride,
                                              CPU_INT16U       pseudo_len,
                                              uint32_t         n_seg,
                                              void            *h_out,
                                              NETCSUM_OP       op,
                                              uint32_t         n_chunks);

NET_ERR  NetUtil_MI355X_RxValidateIPHost   (const void      *h_base,
                                            const uint64_t  *h_off,
                                            const uint16_t  *h_len,
                                            uint64_t         stride,
                                            CPU_INT16U       pkt_len,
                                            uint32_t         n_pkt,
                                            uint8_t         *h_flags,
                                            uint32_t         n_chunks);

NET_ERR  NetUtil_MI355X_TxFinalizeIPHost   (void            *h_base,
                                            const uint64_t  *h_off,
                                            const uint16_t  *h_len,
                                            uint64_t         stride,
                                            CPU_INT16U       pkt_len,
                                            uint32_t         n_pkt,
                                            uint8_t         *h_flags,
                                            int              udp_tx_csum,
                                            uint32_t         n_chunks);

NET_ERR  NetUtil_MI355X_RxBurstHost        (const void      *h_base,
                                            const uint64_t  *h_off,
                                            const uint16_t  *h_len,
                                            uint64_t         stride,
                                            CPU_INT16U       pkt_len,
                                            uint32_t         n_pkt,
                                            uint32_t         rx_cfg,
                                            uint8_t         *h_action,
                                            uint8_t         *h_flags,
                                            uint32_t         n_chunks);

NET_ERR  NetUtil_MI355X_TxBurstHost        (void            *h_base,
                                            const uint64_t  *h_off,
                                            const uint16_t  *h_len,
                                            uint64_t         stride,
                                            CPU_INT16U       pkt_len,
                                            uint32_t         n_pkt,
                                            uint8_t         *h_flags,
                                            uint32_t         n_chunks);

/* ============================================================================================
 * (2c) Batched NET_BUF chains. Chain i = its pseudo-header
 * (d_pseudo + i*pseudo_stride, pseudo_len bytes; none if pseudo_len = 0) followed by pieces
 * [d_chain_first[i], d_chain_first[i+1]) in order, piece j = d_base + d_piece_off[j] with
 * d_piece_len[j] bytes (any alignment; d_chain_first holds n_chains + 1 entries). Each chain is
 * checksummed as the single byte stream NetUtil_16BitOnesCplChkSumDataCalc / DataVerify
 * (net_util.c:590, :716) walks for a NET_BUF chain whose buffers' (DataPtr + ix, len) are the
 * pieces (NetUtil_MI355X_ChainToSpans resolves them): an odd-length piece carries its dangling
 * octet into the next (net_util.c:1385-1393), the u32 accumulator wraps like the reference's
 * (net_util.c:1685), so chains of any total length are bit-exact. A chain with NO pieces is the
 * reference's pdata_buf == NULL case (an odd pseudo-header loses its last octet,
 * net_util.c:1601-1611); describe a chain of empty buffers with one zero-length piece.
 * op: NETCSUM_OP_DATA_CALC (u16 out) or NETCSUM_OP_DATA_VERIFY (u8 DEF_OK/DEF_FAIL out).
 * Forms: by default two launches on the stream — the pieces read as a segment stream (live 64-B
 * sectors, runs of 12 pieces), each piece's exact half-word sum into this thread's device scratch
 * for the stream (4 B per piece, room for max(2^20, 128 * n_chains) pieces; a batch with more pieces
 * is done in the wave-per-chain form instead, same results), then one combine per chain, modulo
 * 65535 up to 131 072 stream bytes and in the exact u32-wrapping form beyond;
 * NETCSUM_TUNE_KERNEL 1 selects the wave-per-chain form, 4 the round-5 two-pass form (tiled 16-lane
 * groups, 8-B even / odd records), NETCSUM_TUNE_GROUP_LANES 16 / 32 / 64 a lane group per chain.
 * Graph capture: as for the Tx scratch (one uncaptured call first).
 * ============================================================================================ */
NET_ERR  NetUtil_MI355X_ChkSumBatchChains  (const void      *d_base,
                                            const uint64_t  *d_piece_off,
                                            const uint16_t  *d_piece_len,
                                            const uint32_t  *d_chain_first,
                                            const void      *d_pseudo,
                                            uint32_t         pseudo_stride,
                                            CPU_INT16U       pseudo_len,
                                            uint32_t         n_chains,
                                            void            *d_out,
                                            NETCSUM_OP       op,
                                            void            *hip_stream);

/* ============================================================================================
 * (3) Support entry points.
 * ============================================================================================ */

/* One contiguous piece of the checksummed byte stream (host memory). */
typedef struct netcsum_span {
    const void  *p;
    uint32_t     len;
    uint32_t     rsvd;
} NETCSUM_SPAN;

/* Reference-exact 32-bit accumulator of the concatenated spans, computed on the GPU:
 *   *p_sum32 = ( Σ big-endian 16-bit words of span_0 ‖ span_1 ‖ … , odd tail padded with 0x00 )
 *              mod 2^32
 * which is exactly the u32 `sum` of net_util.c:1554/:1163 before its end-around-carry fold
 * (per-buffer partials never exceed 2^31, net_util.c:1321-1475, so only the cross-buffer u32
 * accumulation wraps, at :1685). Spans are staged through pinned memory of the calling
 * thread's context. */
NET_ERR  NetUtil_MI355X_StreamSum32        (const NETCSUM_SPAN *spans,
                                            uint32_t            n_spans,
                                            uint32_t           *p_sum32);

/* Multi-GPU partition of a variable-length batch by bytes: rank r of `world`
 * checksums segments [first[r], first[r+1]) — contiguous ranges whose len + pseudo_len byte totals
 * are equal to within one segment (prefix sum; first[0] = 0, first[world] = n_seg; `first` holds
 * world + 1 entries). Host logic, no device work; per-segment results are independent, so the
 * union of the ranks' outputs is the single-GPU result. */
NET_ERR  NetUtil_MI355X_ShardVarLen        (const uint16_t *seg_len,
                                            uint32_t        n_seg,
                                            CPU_INT16U      pseudo_len,
                                            uint32_t        world,
                                            uint32_t       *first);

/* CRC-32 batches (device memory): d_out[i] = NetUtil_32BitCRC_Calc (cpl = 0) or _CalcCpl (cpl != 0)
 * of segment i — base + i * stride, `len` bytes (strided) or base + d_off[i], d_len[i] bytes
 * (varlen) — any alignment and length; an empty segment gives 0 (the reference's NULL_SIZE case).
 * Strided segments up to 96 B take one lane each (crc_tiny_kernel up to 16 B, else crc_lane_kernel,
 * byte tables in LDS); longer ones and every varlen batch the interleaved form crc_ilv_kernel: 8 lanes
 * per segment for strided segments >= 1 KiB, else 4, over interleaved 16-B chunks with 11-bit slicing
 * tables in LDS (netcsum_crc.hip). NETCSUM_TUNE_CRC_KERNEL 1 selects the 16-lane block-combine form. */
NET_ERR  NetUtil_MI355X_CRC32BatchStrided  (const void *d_base,
                                            uint64_t    stride,
                                            uint32_t    len,
                                            uint32_t    n,
                                            uint32_t   *d_out,
                                            int         cpl,
                                            void       *hip_stream);

NET_ERR  NetUtil_MI355X_CRC32BatchVarLen   (const void     *d_base,
                                            const uint64_t *d_off,
                                            const uint32_t *d_len,
                                            uint32_t        n,
                                            uint32_t       *d_out,
                                            int             cpl,
                                            void           *hip_stream);

/* One CRC-32 register value (NetUtil_32BitCRC_Calc's result) of a host buffer, computed on the GPU
 * from this thread's pinned staging (the per-call path of the drop-in CRC functions). */
NET_ERR  NetUtil_MI355X_CRC32Host          (const void *h_data,
                                            uint32_t    len,
                                            uint32_t   *p_crc);

/* Frees the calling thread's per-device contexts (stream, pinned staging, device buffers) used by
 * the four drop-in functions, NetUtil_MI355X_StreamSum32 and ..._ChkSumBatchStridedHost. They are
 * also freed automatically when the thread exits; the next call re-creates them. */
NET_ERR  NetUtil_MI355X_ThreadRelease      (void);

/* NET_BUF chain walk of NetUtil_16BitOnesCplSumDataCalc (net_util.c:1589-1687) as pure host
 * logic: emits the spans whose concatenation is the checksummed stream (pseudo-header first).
 * Chains of any length are walked. spans == NULL counts only (*p_n_spans = spans needed).
 * Returns NET_UTIL_ERR_NONE, NET_UTIL_ERR_INVALID_PROTOCOL, NET_UTIL_ERR_BUF_TOO_SMALL (more
 * than max_spans pieces: the first max_spans are written and *p_n_spans is the count needed,
 * so the caller can size an array and walk again) or — with dbg_chk != 0 — the
 * NET_ERR_CFG_ARG_CHK_DBG_EN errors. On any other error *p_n_spans is 0. */
NET_ERR  NetUtil_MI355X_ChainToSpans       (const void   *pdata_buf,
                                            const void   *ppseudo_hdr,
                                            CPU_INT16U    pseudo_hdr_size,
                                            NETCSUM_SPAN *spans,
                                            uint32_t      max_spans,
                                            uint32_t     *p_n_spans,
                                            int           dbg_chk);

/* Deterministic synthetic bytes, generated on the device. Byte k of the buffer is byte g of one
 * global stream, g = first_byte + k: pattern 0 = byte (g & 7) of splitmix64(seed + (g >> 3));
 * 1 = all 0x00; 2 = all 0xFF; 3 = 0xFF,0xFF,0x00,0x01 repeating by g (maximal carries). Shards of
 * one global batch are generated independently per GPU by passing their global byte offset.
 * d_buf must be 8-byte aligned. Asynchronous on hip_stream. */
NET_ERR  NetUtil_MI355X_Fill               (void      *d_buf,
                                            uint64_t   n_bytes,
                                            uint64_t   first_byte,
                                            uint64_t   seed,
                                            int        pattern,
                                            void      *hip_stream);

/* Roofline probe: a pure HBM read stream over [d_buf, d_buf + n_bytes) (16-B aligned, n_bytes a
 * multiple of 16) summing dwords into *d_sink (device uint64). Same launch geometry policy as the
 * checksum kernels; used by bench.py as the measured achievable read bandwidth. */
NET_ERR  NetUtil_MI355X_ReadStream         (const void *d_buf,
                                            uint64_t    n_bytes,
                                            uint64_t   *d_sink,
                                            void       *hip_stream);

/* Launch tuning knobs (0 = automatic). A setting applies to the CALLING host thread's launches only;
 * every thread starts from the defaults. */
typedef enum netcsum_tune_key {
    NETCSUM_TUNE_GRID_BLOCKS   = 1,   /* workgroups per launch (0: exactly fill the chip)        */
    NETCSUM_TUNE_GROUP_LANES   = 2,   /* lanes per segment: 0 auto, else 1,4,8,16,32,64          */
    NETCSUM_TUNE_NT_LOADS      = 3,   /* -1 auto (default), 0 plain, 1 non-temporal segment loads */
    NETCSUM_TUNE_BLOCK_THREADS = 4,   /* threads per workgroup: 64, 128 or 256 (0 = 256)         */
    NETCSUM_TUNE_KERNEL        = 5,   /* 0 auto (default: 8 where it applies, else 7, else 5 where it
                                         applies, 6 for packed strided segments of >= 1 KiB and for
                                         offset/length batches, else 2), 1 simple,
                                         2 pipelined register loads, 3 pipelined LDS-DMA, 4 wave-tile
                                         LDS image (strided; else falls back to 2), 5 small aligned
                                         segments (strided, no pseudo-header, 1-64 B, base and stride
                                         multiples of 4; else falls back to 2), 6 segmented stream
                                         (strided, stride in [len, len+64], len >= 256, or any
                                         offset/length batch; pseudo-header <= 64 B; one wave per run
                                         of segments, streamed when packed; else falls back to 2;
                                         CHUNKS = pieces in flight per wave: 4, 6 or 8), 7 header
                                         tiles through LDS (kernel 5's domain with stride <= 64 B;
                                         CHUNKS = tiles in flight per wave: 2, 3 or 4), 8 packed
                                         16 / 20-B headers streamed by one wave per run (stride ==
                                         len, base a multiple of 4, no pseudo-header; else 7;
                                         CHUNKS 4 / 8 = pieces in flight; TILE = headers per run,
                                         auto: the most that fit 4 KiB from any 128-B lead, 192 for
                                         20-B headers). Chain batches: 1 = the wave-per-chain form
                                         (default / 5: two passes, the first in the segment
                                         live-sector stream with one record per piece, see (2c)), 3 =
                                         two passes with round 5's live-sector pass 1 (two sums per
                                         piece), 4 = two passes with tiled 16-lane groups in pass 1;
                                         3 / 5: TILE = pieces per run, CHUNKS 4 / 8 = pieces in
                                         flight                                                       */
    NETCSUM_TUNE_CHUNKS        = 6,   /* 16-B chunks per lane per pass: 0 auto, 1,2,3,4,6,8;
                                         run-stream kernels: 1-KiB pieces in flight (4 / 8)        */
    NETCSUM_TUNE_PROBE         = 7,   /* read-stream probe: 0 register loads, 1 LDS-DMA (default),
                                         2 run-stream form of the checksum kernels (24-KiB runs per
                                         wave, 4 nt pieces in flight, row touch, 5 waves per SIMD),
                                         3 the same with a ~128-clock pause after each piece        */
    NETCSUM_TUNE_GRID_MULT     = 8,   /* auto grid = resident blocks x CUs x this (0 = 1)          */
    NETCSUM_TUNE_TILE          = 9,   /* J > 0: each block owns a contiguous tile of J segments per
                                         group (grid = tiles); 0: grid-stride; -1: auto (J = 4).
                                         Kernel 6: J > 0 = segments per wave run (<= 128; auto 16);
                                         varlen batches whose plan is the live-sector stream (segments
                                         one per pool buffer): its runs (<= 64; auto from the plan).
                                         Kernel 7: headers per lane, 1, 2 or 4 (auto 2).
                                         IPv4 packet batches: packets per wave run of the run-stream
                                         form (<= 64; auto 8); TUNE_KERNEL 2 forces the lane-group
                                         packet kernel                                              */
    NETCSUM_TUNE_TX_PASSES     = 10,  /* run-stream Tx finalize: 0 auto (2 from 64 Ki datagrams up,
                                         else 1), 1 checksum fields written by the checksum pass
                                         (IPv6 chains past the window walked in the same launch),
                                         2 checksum pass writes 8-B records, a scatter pass writes
                                         the fields (and walks IPv6 chains past the window)      */
    NETCSUM_TUNE_STREAM_WAVES  = 11,  /* run-stream kernels (segments, packets): resident waves per
                                         SIMD, 3..8, enforced by reserving LDS per workgroup; 0 = as
                                         many as registers allow; -1 = each kernel's default (dense
                                         segment batches 5, others 0)                               */
    NETCSUM_TUNE_STREAM_TOUCH  = 12,  /* run-stream kernels: row-touch prologue (the first dword of
                                         every 1-KiB piece of a wave's run loaded up front): 1 on,
                                         0 off, -1 each kernel's default (segment batches on, packet
                                         batches off)                                               */
    NETCSUM_TUNE_STREAM_XCD    = 13,  /* segment / varlen / header / packet stream kernels: 1 = XCD-
                                         aware block order (each XCD's blocks take one contiguous 1/8
                                         of the runs), 0 = the dispatch order, 2..4096 = (segment
                                         and varlen batches, chain pass 1) each XCD takes chunks of
                                         that many blocks in turn, the other kernels reading any
                                         value >= 1 as 1; -1 = each kernel's default (strided segment
                                         batches chunks of 256 when an XCD's slice would span >= 1 GiB,
                                         else one slice per XCD, as for varlen batches and chain pass
                                         1; header and packet batches off)                           */
    NETCSUM_TUNE_TX_FLUSH      = 14,  /* run-stream Tx finalize, write-back of the dirty checksum-field
                                         lines: -1 / 0 none (they are evicted during later launches),
                                         1 scatter stores written through at system scope, 2 an L2
                                         release at the end of every scatter wave, 3 / 4 a write-back
                                         launch of 8 / 256 workgroups after the Tx launch(es)         */
    NETCSUM_TUNE_CRC_KERNEL    = 15,  /* CRC-32 batches: 0 auto (strided segments <= 96 B one lane
                                         each, longer ones and every varlen batch the interleaved
                                         form), 1 block combine (GF(2) multiplications by bit loops,
                                         the round-2 form), 2 interleaved for every length, 3 one lane
                                         per segment for every length                                 */
    NETCSUM_TUNE_CRC_NT        = 16,  /* CRC-32 interleaved form: 1 non-temporal chunk loads, 0 plain */
    NETCSUM_TUNE_CRC_LANES     = 17,  /* CRC-32 interleaved form: lanes per segment, 1, 2, 4, 8, 16;
                                         0 auto (8 for strided segments >= 1 KiB, else 4)             */
    NETCSUM_TUNE_CRC_WIDE      = 18,  /* CRC-32 interleaved form: 1 (default) 11-bit slicing tables
                                         (3 LDS lookups per dword), 0 byte tables (4), 2 lane-private
                                         6-bit replicas (6, conflict-free)                            */
    NETCSUM_TUNE_HDR_BURST     = 19,  /* header stream kernel (C3): 1 = a run's results gathered in LDS
                                         and written as whole 16-B pieces, 0 = one store per piece,
                                         -1 = the default                                             */
    NETCSUM_TUNE_VARLEN_RUN_BYTES = 20,/* varlen stream kernel (C4): B > 0 = runs of about B bytes, the
                                         run length chosen on the device from sampled lengths; 0 =
                                         runs of 8 segments; -1 = the default (16 KiB)                 */
    NETCSUM_TUNE_PKT_BOUND     = 21,  /* packet batches (run-stream form): which bytes are read. 0 = every
                                         byte of each wave's span (dense strided layouts: gaps <= 64 B),
                                         1 = only the 64-B sectors holding summed bytes (live pieces), the
                                         parse first; 2 = live pieces with the run's first piece loaded
                                         during the parse; 3 = live pieces with the run's first 4 (8)
                                         pieces loaded during the parse (dense strided layouts);
                                         4 = ring plans (strided batches that are not packed): each launch
                                         samples 1024 of its datagrams on the device (one extra block)
                                         and leaves the form and run length for the next batch on the
                                         same ring (base, stride, pkt_len, count, IP version): form 0
                                         when the datagrams fill their slots, else live pieces in runs
                                         of 8 / 16 / 32 by the bytes they stream; a ring's first batch
                                         runs as 2; -1 = the default: 0 for packed batches (stride ==
                                         pkt_len), 4 for other strided batches of >= 16 Ki datagrams, 2
                                         for smaller ones and offset/length batches                  */
    NETCSUM_TUNE_BURST_ZERO_COPY = 22,/* host-memory packet batches with n_chunks 0 of <= 4096 frames whose
                                         ring is pinned host memory: the kernel reads the ring in place;
                                         3 (default) = a resident server kernel (one per calling thread,
                                         on a stream of its own) takes each burst from a 64-B post in
                                         coherent host memory, no launch per burst; 2 = a launch per
                                         burst, the results go straight to coherent pinned memory and the
                                         host polls them; 1 = a completion kernel copies the results out
                                         and stores a completion word the host polls; 0 = the copy
                                         pipeline (H2D, kernel, D2H, stream synchronisation)            */
    NETCSUM_TUNE_BURST_SERVER_IDLE_US = 23,/* mode 3: microseconds without a burst after which the server
                                         stops (the next burst relaunches it); a device-wide
                                         synchronisation waits up to this long. 1..1000000, default 500 */
    NETCSUM_TUNE_BURST_SERVER_LIFE_US = 24,/* mode 3: microseconds one server launch stays resident even
                                         while bursts keep coming (kernels of other streams sharing its
                                         hardware queue wait behind it at most this long plus one
                                         burst); the next burst relaunches it. 1..1000000, default 1000 */
    NETCSUM_TUNE_FAULT_INJECT  = 25,  /* TEST ONLY. 1: the calling thread's next offset/length packet
                                         batch that has a deferred pass enqueues its stream kernel,
                                         skips the deferred pass and fails (NET_UTIL_ERR_MI355X_DEV):
                                         the state a failed launch leaves; one-shot. 0: cleared      */
    NETCSUM_TUNE_PLAN_AHEAD    = 26,  /* planned batches (NIC rings, offset/length rings, segments one
                                         per pool buffer) whose plan has no sample yet — the first batch
                                         on a layout (NetUtil_MI355X_PlanBind) — : 1 = sample the layout
                                         first (a one-block launch on the same stream; the call waits
                                         for its plan word, i.e. for the stream's earlier work too) and
                                         run this batch in its plan; 0 = run the first batch unplanned
                                         (its own sampler block leaves the plan for the next batch);
                                         -1 (default) = 1 from 4 Mi frames (rings) / 512 Ki segments
                                         (pools), else 0. Never under stream capture.                 */
    NETCSUM_TUNE_LIVE_COMPACT  = 27,  /* live-sector streams (segments one per pool buffer): 1 / -1
                                         (default) the run's live 64-B sectors read compacted, 16 per
                                         wave-instruction; 0 the live 1-KiB pieces of the run's span,
                                         each lane loading its 16 B where its sector is live          */
    NETCSUM_TUNE_STORE_GATHER  = 28,  /* dense strided segment batches (C2 / C5): 1 / -1 (default) the
                                         results of a workgroup's 4 runs gathered in LDS and written as
                                         whole lines by its last wave; 0 each wave writes its own run's
                                         results (partial lines)                                      */
    NETCSUM_TUNE_CHAIN_GRID    = 29,  /* NET_BUF chain batches, tiled pass 1 (TUNE_KERNEL 4): 0 / -1
                                         (default) one tile of 64 consecutive pieces per block; k =
                                         1..16 a grid of k x the resident blocks, each owning an equal
                                         contiguous share                                             */
    NETCSUM_TUNE_CHAIN_COMBINE = 30   /* NET_BUF chain batches, the one-record form's combine pass:
                                         16 or 64 lanes per chain; -1 (default) = chosen by the
                                         library                                                      */
} NETCSUM_TUNE_KEY;

NET_ERR  NetUtil_MI355X_Tune               (int key, int value);

/* Plan identity. The planned batch kinds — strided and offset/length NIC rings
 * (RxValidate / TxFinalize / bursts) and offset/length segment batches one per pool buffer — choose
 * their form from a plan the previous batch on the same layout sampled on the device, keyed on the
 * batch's addresses (base, descriptor arrays / stride, count, IP version). A caller that places a
 * DIFFERENT layout at the same addresses binds each layout to an id of its own: the calling thread's
 * later batches key their plans on (addresses, plan_id) until it binds another id, so each layout keeps
 * its plan and never runs one batch in the other's form. 0 (the default) = addresses only. Host-only;
 * never fails. */
NET_ERR  NetUtil_MI355X_PlanBind           (uint32_t plan_id);

/* The calling thread's last batch launch: kernel form and geometry (for profiling / logs). */
const char *NetUtil_MI355X_LastLaunch      (void);

/* Version / build identification string ("netcsum-mi355x <ver> gfx950"). */
const char *NetUtil_MI355X_Version         (void);

#ifdef __cplusplus
}
#endif

#endif /* NETCSUM_MI355X_H */
