"""ORACLE — test infrastructure only (never used by the product). The reference's per-frame outcome
around its checksum checks, with and without its checksum-offload configuration, so that the burst
adapters (NetUtil_MI355X_RxBurst / TxBurst, include/netcsum_mi355x.h (2b'')) can be checked to make
the reference's decisions.

Rx, `rx_reference(pkt, udp_discard, offload)`: the checks a received frame meets, in the reference's
order, each one a drop (with the Net_ErrCtrs counter it increments) or a pass:

  IPv4  header shape: version / IHL / total length vs. bytes present   net_ipv4.c:5123-5235
        header checksum  HdrVerify(ip_hdr, IHL*4)                       net_ipv4.c:5243-5254  [offload: IPV4]
        fragment: the transport checks run on the reassembled datagram  net_ipv4.c:6523      -> deliver
  TCP   length >= 20                                                   net_tcp.c:7808-7818
        checksum DataVerify + pseudo {src, dst, 0, 6, len}             net_tcp.c:7845-7890   [offload: TCP]
  UDP   length == IP datagram length                                   net_udp.c:1893-1911
        field 0: "no checksum" -> accepted, or dropped with
        NET_UDP_CFG_RX_CHK_SUM_DISCARD_EN                              net_udp.c:1916-1920, 1971-1977
        checksum DataVerify + pseudo {src, dst, 0, 17, len}            net_udp.c:1916-1968   [offload: UDP]
  ICMPv4 type accepted (3, 4, 11, 12, 0, 8, 13, 14, 18)                net_icmpv4.c:1500-1640
        checksum                                                       net_icmpv4.c:1665-1700 [offload: ICMP]
  IGMP  checksum HdrVerify (no offload flag exists)                    net_igmp.c:1332-1339
  IPv6  header shape, extension-header chain (oracle_packets._parse6), fragment -> deliver
        TCP / UDP as above with the 40-B pseudo-header                 net_tcp.c:7866-7879, net_udp.c:1941-1957
        ICMPv6 types 1, 3, 4: HdrVerify, no offload flag               net_icmpv6.c:2910-2920
               types 128-131, 134-137: DataVerify + pseudo             net_icmpv6.c:2923-2942 [offload: ICMP]
               other types: dropped (RxHdrTypeCtr)                      net_icmpv6.c:2945-2948
  anything else: delivered (the protocol demultiplexer decides).

`offload=True` is the stack built with every NET_*_CFG_CHK_SUM_OFFLOAD_RX_EN enabled: the checks
marked [offload] assume a valid checksum (net_ipv4.c:5243-5244, net_tcp.c:7847-7848, :7868-7869,
net_udp.c:1925-1927, :1944-1946, net_icmpv4.c:1673-1674, :1683-1684, net_icmpv6.c:2931-2932).
Non-checksum drops are reported as (\"drop\", \"<LAYER>.hdr\"): their exact counters are the
stack's business and equal on both sides of the seam. ICMPv4 codes and per-type lengths are not
modelled (the tests use valid ones).

`rx_with_adapter(pkt, action, udp_discard)`: a frame first meets the adapter's action, then — if
delivered — the stack built with the offload flags.

Tx, `tx_stack_offload(pkt, udp_tx_csum)`: the frame as the stack builds it with every
*_CHK_SUM_OFFLOAD_TX flag enabled (from the reference-built frame oracle_packets.tx_finalize_ip):
IPv4 / TCP / ICMPv4 fields 0 (net_ipv4.c:9575-9586, net_tcp.c:29813-29815, :29845-29847,
net_icmpv4.c:1046, :2225, :2245, :3093, :3124), the UDP field 0xFFFF when checksums are on (the
offload's 0 mapped by net_udp.c:2929-2931) and 0 when off (:2934-2935); ICMPv4 echo requests and
ICMPv6 keep their computed value (their guards test the never-defined macro
NET_ICMP_CFG_CHK_SUM_OFFLOAD_TX: net_icmpv4.c:2201, net_icmpv6.c:1439), IGMP too (no flag,
net_igmp.c:1692). `tx_burst_model(frame)`: the adapter's rule on such a frame.
"""
from __future__ import annotations

import struct

import oracle
import oracle_packets as op
import netcsum

ICMPV4_RX_TYPES = {0, 3, 4, 8, 11, 12, 13, 14, 18}           # net_icmpv4.c:1500-1640 (supported types)
ICMPV4_CSUM_TYPES = ICMPV4_RX_TYPES                           # every accepted type is checksummed (:1665-1690)

DROP_COUNTER = {netcsum.RX_DROP_IPV4_CHK_SUM: "IPv4.RxInvChkSumCtr",
                netcsum.RX_DROP_TCP_CHK_SUM: "TCP.RxHdrChkSumCtr",
                netcsum.RX_DROP_UDP_CHK_SUM: "UDP.RxHdrChkSumCtr",
                netcsum.RX_DROP_UDP_NO_CHK_SUM: "UDP.RxHdrChkSumCtr",
                netcsum.RX_DROP_ICMPV4_CHK_SUM: "ICMPv4.RxInvChkSumCtr",
                netcsum.RX_DROP_IGMP_CHK_SUM: "IGMP.RxHdrChkSumCtr",
                netcsum.RX_DROP_ICMPV6_CHK_SUM: "ICMPv6.RxHdrChkSumCtr"}
CHECKSUM_COUNTERS = set(DROP_COUNTER.values())


def _v4_l4_ok(pkt, hlen, tot, proto, src, dst):
    """The transport checksum verdict of an IPv4 datagram, through the oracle's four functions."""
    l4len = tot - hlen
    if proto in (6, 17):
        ptype = netcsum.NET_PROTOCOL_TYPE_TCP_V4 if proto == 6 else netcsum.NET_PROTOCOL_TYPE_UDP_V4
        ch = op._l4_chain(pkt, ptype, hlen, l4len)
        ph = netcsum.HostBytes(struct.pack("!4s4sBBH", src, dst, 0, proto, l4len))
        return oracle.data_verify(ch.ptr, ph.ptr, 12)[0] == 1
    if proto == 1:
        ch = op._l4_chain(pkt, netcsum.NET_PROTOCOL_TYPE_ICMP_V4, hlen, l4len, icmp=True)
        return oracle.data_verify(ch.ptr, None, 0)[0] == 1
    hb = netcsum.HostBytes(pkt[hlen:tot])
    return oracle.hdr_verify(hb.ptr, l4len)[0] == 1


def _rx_v4(pkt, udp_discard, offload):
    p = op._parse(pkt)
    if p is None:
        return "drop", "IPv4.hdr"
    hlen, tot, frag, proto, src, dst = p
    if not offload:
        hb = netcsum.HostBytes(pkt)
        if oracle.hdr_verify(hb.ptr, hlen)[0] != 1:
            return "drop", "IPv4.RxInvChkSumCtr"
    if frag:
        return "deliver", None
    l4len = tot - hlen
    if proto == 6:
        if l4len < 20:
            return "drop", "TCP.hdr"
        if not offload and not _v4_l4_ok(pkt, hlen, tot, proto, src, dst):
            return "drop", "TCP.RxHdrChkSumCtr"
        return "deliver", None
    if proto == 17:
        if l4len < 8 or struct.unpack("!H", pkt[hlen + 4:hlen + 6])[0] != l4len:
            return "drop", "UDP.hdr"
        if pkt[hlen + 6:hlen + 8] == b"\x00\x00":
            return ("drop", "UDP.RxHdrChkSumCtr") if udp_discard else ("deliver", None)
        if not offload and not _v4_l4_ok(pkt, hlen, tot, proto, src, dst):
            return "drop", "UDP.RxHdrChkSumCtr"
        return "deliver", None
    if proto == 1:
        if l4len < 4 or pkt[hlen] not in ICMPV4_RX_TYPES:
            return "drop", "ICMPv4.hdr"
        if not offload and not _v4_l4_ok(pkt, hlen, tot, proto, src, dst):
            return "drop", "ICMPv4.RxInvChkSumCtr"
        return "deliver", None
    if proto == 2:
        if l4len < 4:
            return "drop", "IGMP.hdr"
        if not _v4_l4_ok(pkt, hlen, tot, proto, src, dst):      # no offload flag for IGMP
            return "drop", "IGMP.RxHdrChkSumCtr"
        return "deliver", None
    return "deliver", None


def _rx_v6(pkt, udp_discard, offload):
    p = op._parse6(pkt)
    if p is None:
        return "drop", "IPv6.hdr"
    fx, off, plen, nh, addrs = p
    if fx & op.FRAGMENT:
        return "deliver", None
    if fx:                                                     # EXT_HDR: the reference rejects it
        return "drop", "IPv6.ext"
    body = pkt[:40] + pkt[off:40 + struct.unpack("!H", pkt[4:6])[0]]

    def verify(ptype, nhv, icmp=False):
        ch = op._l4_chain6(body, ptype, plen, icmp)
        ph = netcsum.HostBytes(op.pseudo6(addrs, plen, nhv))
        return oracle.data_verify(ch.ptr, ph.ptr, 40)[0] == 1

    if nh == 6:
        if plen < 20:
            return "drop", "TCP.hdr"
        if not offload and not verify(netcsum.NET_PROTOCOL_TYPE_TCP_V6, 6):
            return "drop", "TCP.RxHdrChkSumCtr"
        return "deliver", None
    if nh == 17:
        if plen < 8 or struct.unpack("!H", body[44:46])[0] != plen:
            return "drop", "UDP.hdr"
        if body[46:48] == b"\x00\x00":
            return ("drop", "UDP.RxHdrChkSumCtr") if udp_discard else ("deliver", None)
        if not offload and not verify(netcsum.NET_PROTOCOL_TYPE_UDP_V6, 17):
            return "drop", "UDP.RxHdrChkSumCtr"
        return "deliver", None
    if nh == 58:
        if plen < 4:
            return "drop", "ICMPv6.hdr"
        t = body[40]
        if t in op.ICMPV6_NOPSEUDO_TYPES:                      # no offload flag (net_icmpv6.c:2913)
            hb = netcsum.HostBytes(body[40:40 + plen])
            if oracle.hdr_verify(hb.ptr, plen)[0] != 1:
                return "drop", "ICMPv6.RxHdrChkSumCtr"
            return "deliver", None
        if t in op.ICMPV6_PSEUDO_TYPES:
            if not offload and not verify(netcsum.NET_PROTOCOL_TYPE_ICMP_V6, 58, icmp=True):
                return "drop", "ICMPv6.RxHdrChkSumCtr"
            return "deliver", None
        return "drop", "ICMPv6.hdr"
    return "deliver", None


def rx_reference(pkt: bytes, udp_discard: bool = False, offload: bool = False):
    """-> ("deliver", None) or ("drop", counter)."""
    pkt = bytes(pkt)
    if len(pkt) and pkt[0] >> 4 == 6:
        return _rx_v6(pkt, udp_discard, offload)
    return _rx_v4(pkt, udp_discard, offload)


def rx_with_adapter(pkt: bytes, action: int, udp_discard: bool = False):
    """The adapter's action, then the stack built with the Rx offload flags."""
    if action in DROP_COUNTER:
        return "drop", DROP_COUNTER[action]
    assert action in (netcsum.RX_DELIVER, netcsum.RX_DELIVER_L4_UNVERIFIED), action
    return rx_reference(pkt, udp_discard, offload=True)


def transport_proto(pkt: bytes) -> int:
    """The protocol whose checksum RxValidateIP's verdict covers (0: none)."""
    pkt = bytes(pkt)
    if len(pkt) and pkt[0] >> 4 == 6:
        p = op._parse6(pkt)
        return 0 if p is None else p[3]
    return pkt[9] if len(pkt) >= 20 else 0


def tx_stack_offload(pkt: bytes, udp_tx_csum: bool = True) -> bytes:
    """The frame the stack hands to the NIC when built with every Tx offload flag (see the header)."""
    ref, _ = op.tx_finalize_ip(pkt, udp_tx_csum)
    b = bytearray(ref)
    if len(b) and b[0] >> 4 == 6:
        p = op._parse6(bytes(b))
        if p is None or p[0]:
            return bytes(b)
        off, nh = p[1], p[3]
        if nh == 17 and p[2] >= 8 and udp_tx_csum and struct.unpack("!H", bytes(b[off + 4:off + 6]))[0] == p[2]:
            b[off + 6:off + 8] = b"\xff\xff"
        elif nh == 6 and p[2] >= 20:
            b[off + 16:off + 18] = b"\x00\x00"
        return bytes(b)                                        # ICMPv6: computed by the stack
    p = op._parse(bytes(b))
    if p is None:
        return bytes(b)
    hlen, tot, frag, proto, _, _ = p
    b[10:12] = b"\x00\x00"
    l4len = tot - hlen
    if not frag:
        if proto == 6 and l4len >= 20:
            b[hlen + 16:hlen + 18] = b"\x00\x00"
        elif proto == 17 and l4len >= 8 and struct.unpack("!H", bytes(b[hlen + 4:hlen + 6]))[0] == l4len:
            b[hlen + 6:hlen + 8] = b"\xff\xff" if udp_tx_csum else b"\x00\x00"
        elif proto == 1 and l4len >= 4 and b[hlen] != 8:      # echo requests: computed (net_icmpv4.c:2201)
            b[hlen + 2:hlen + 4] = b"\x00\x00"
    return bytes(b)


def tx_burst_model(frame: bytes) -> bytes:
    """The Tx adapter's rule: every checksum field computed as if zero, except a UDP field of 0,
    which means "no checksum" and stays 0."""
    frame = bytes(frame)
    v6 = len(frame) and frame[0] >> 4 == 6
    if v6:
        p = op._parse6(frame)
        udp_none = p is not None and not p[0] and p[3] == 17 and frame[p[1] + 6:p[1] + 8] == b"\x00\x00"
    else:
        p = op._parse(frame)
        udp_none = (p is not None and not p[2] and p[3] == 17 and
                    frame[p[0] + 6:p[0] + 8] == b"\x00\x00")
    return op.tx_finalize_ip(frame, udp_tx_csum=not udp_none)[0]
