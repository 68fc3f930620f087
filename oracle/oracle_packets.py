"""ORACLE — test infrastructure only. Per-packet IPv4 Rx validation / Tx finalization composed from
the C oracle's restatements of the four reference functions, called the way the reference's call
sites call them (never used by the product):

  Rx  IP header   HdrVerify(ip_hdr, IHL*4)                          net_ipv4.c:5247
      TCP         DataVerify(NET_BUF{TCP_V4, TransportHdrIx = IHL*4}, pseudo{src,dst,0,6,len}, 12)
                                                                    net_tcp.c:7851-7857
      UDP         field 0 -> no checksum (accepted); else DataVerify(NET_BUF{UDP_V4}, pseudo{..,17,len})
                                                                    net_udp.c:1893-1934
      ICMP        DataVerify(NET_BUF{ICMP_V4, ICMP_MsgIx = IHL*4}, NULL, 0)    net_icmpv4.c:1676
      IGMP        HdrVerify(igmp_hdr, msg len)                      net_igmp.c:1332
  Tx  the same sums through the Calc functions with the checksum fields zeroed first, written back
      as the host-order value (net_ipv4.c:9573-9586, net_tcp.c:29824-29862, net_udp.c:2891-2937).

Flag bits mirror include/netcsum_mi355x.h NETCSUM_PKT_*.
"""
from __future__ import annotations

import ctypes
import struct

import netcsum
import oracle

IP_OK, L4_OK, L4_CHECKED, UDP_NO_CSUM, MALFORMED, FRAGMENT, L4_MALFORMED = 1, 2, 4, 8, 16, 32, 64


def _parse(pkt: bytes):
    if len(pkt) < 20:
        return None
    ver, ihl = pkt[0] >> 4, pkt[0] & 0xF
    hlen = ihl * 4
    tot = struct.unpack("!H", pkt[2:4])[0]
    if ver != 4 or hlen < 20 or tot < hlen or tot > len(pkt):
        return None
    frag = struct.unpack("!H", pkt[6:8])[0] & 0x3FFF
    return hlen, tot, frag, pkt[9], pkt[12:16], pkt[16:20]


def _l4_chain(pkt: bytes, proto_type: int, hlen: int, l4len: int, icmp=False):
    if icmp:
        return netcsum.Chain([{"data": pkt, "proto": proto_type, "icmp_ix": hlen, "icmp_hdr_len": 0,
                               "data_len": l4len}])
    return netcsum.Chain([{"data": pkt, "proto": proto_type, "transport_ix": hlen, "transport_hdr_len": 0,
                           "data_len": l4len}])


def rx_validate(pkt: bytes) -> int:
    pkt = bytes(pkt)
    p = _parse(pkt)
    if p is None:
        return MALFORMED
    hlen, tot, frag, proto, src, dst = p
    hb = netcsum.HostBytes(pkt)
    ok, _ = oracle.hdr_verify(hb.ptr, hlen)
    f = IP_OK if ok else 0
    if frag:
        return f | FRAGMENT
    l4len = tot - hlen
    if proto == 6:
        if l4len < 20:
            return f | L4_MALFORMED
        ch = _l4_chain(pkt, netcsum.NET_PROTOCOL_TYPE_TCP_V4, hlen, l4len)
        ph = netcsum.HostBytes(struct.pack("!4s4sBBH", src, dst, 0, 6, l4len))
        v, err = oracle.data_verify(ch.ptr, ph.ptr, 12)
        return f | L4_CHECKED | (L4_OK if v else 0)
    if proto == 17:
        if l4len < 8:
            return f | L4_MALFORMED
        udp_len = struct.unpack("!H", pkt[hlen + 4:hlen + 6])[0]
        if udp_len != l4len:
            return f | L4_MALFORMED
        if pkt[hlen + 6:hlen + 8] == b"\x00\x00":
            return f | UDP_NO_CSUM | L4_OK
        ch = _l4_chain(pkt, netcsum.NET_PROTOCOL_TYPE_UDP_V4, hlen, udp_len)
        ph = netcsum.HostBytes(struct.pack("!4s4sBBH", src, dst, 0, 17, udp_len))
        v, err = oracle.data_verify(ch.ptr, ph.ptr, 12)
        return f | L4_CHECKED | (L4_OK if v else 0)
    if proto == 1:
        if l4len < 4:
            return f | L4_MALFORMED
        ch = _l4_chain(pkt, netcsum.NET_PROTOCOL_TYPE_ICMP_V4, hlen, l4len, icmp=True)
        v, err = oracle.data_verify(ch.ptr, None, 0)
        return f | L4_CHECKED | (L4_OK if v else 0)
    if proto == 2:
        if l4len < 4:
            return f | L4_MALFORMED
        v, err = oracle.hdr_verify(ctypes.addressof(hb.arr) + hlen, l4len)
        return f | L4_CHECKED | (L4_OK if v else 0)
    return f


def tx_finalize(pkt: bytes, udp_tx_csum: bool = True):
    """-> (finalized packet bytes, flags)."""
    pkt = bytearray(pkt)
    p = _parse(bytes(pkt))
    if p is None:
        return bytes(pkt), MALFORMED
    hlen, tot, frag, proto, src, dst = p
    f = 0
    l4len = tot - hlen
    if not frag:
        if proto == 6 and l4len >= 20:
            pkt[hlen + 16:hlen + 18] = b"\x00\x00"
            ch = _l4_chain(bytes(pkt), netcsum.NET_PROTOCOL_TYPE_TCP_V4, hlen, l4len)
            ph = netcsum.HostBytes(struct.pack("!4s4sBBH", src, dst, 0, 6, l4len))
            c, _ = oracle.data_calc(ch.ptr, ph.ptr, 12)
            pkt[hlen + 16:hlen + 18] = c.to_bytes(2, "little")
            f |= L4_CHECKED | L4_OK
        elif proto == 17 and l4len >= 8 and struct.unpack("!H", bytes(pkt[hlen + 4:hlen + 6]))[0] == l4len:
            pkt[hlen + 6:hlen + 8] = b"\x00\x00"
            if udp_tx_csum:
                ch = _l4_chain(bytes(pkt), netcsum.NET_PROTOCOL_TYPE_UDP_V4, hlen, l4len)
                ph = netcsum.HostBytes(struct.pack("!4s4sBBH", src, dst, 0, 17, l4len))
                c, _ = oracle.data_calc(ch.ptr, ph.ptr, 12)
                if c == 0:
                    c = 0xFFFF
                pkt[hlen + 6:hlen + 8] = c.to_bytes(2, "little")
                f |= L4_CHECKED | L4_OK
            else:
                f |= UDP_NO_CSUM
        elif proto in (1, 2) and l4len >= 4:
            pkt[hlen + 2:hlen + 4] = b"\x00\x00"
            if proto == 1:
                ch = _l4_chain(bytes(pkt), netcsum.NET_PROTOCOL_TYPE_ICMP_V4, hlen, l4len, icmp=True)
                c, _ = oracle.data_calc(ch.ptr, None, 0)
            else:
                hb = netcsum.HostBytes(bytes(pkt[hlen:hlen + l4len]))
                c, _ = oracle.hdr_calc(hb.ptr, l4len)
            pkt[hlen + 2:hlen + 4] = c.to_bytes(2, "little")
            f |= L4_CHECKED | L4_OK
        elif proto in (6, 17, 1, 2):
            f |= L4_MALFORMED
    else:
        f |= FRAGMENT
    pkt[10:12] = b"\x00\x00"
    hb = netcsum.HostBytes(bytes(pkt[:hlen]))
    c, _ = oracle.hdr_calc(hb.ptr, hlen)
    pkt[10:12] = c.to_bytes(2, "little")
    return bytes(pkt), f | IP_OK


# ---------------------------------------------------------------------------------------------
# IPv6 (40-B fixed header). Pseudo-header {src(16), dst(16), upper-layer length (32), zero (16),
# next header (16, network order)} = NET_IPv6_PSEUDO_HDR (net_ipv6.h:844-852), as the call sites fill it:
#   TCP     Rx DataVerify(NET_BUF{TCP_V6}, pseudo{.., 6}, 40)         net_tcp.c:7871-7879
#           Tx DataCalc                                               net_tcp.c:29839-29862
#   UDP     Rx field 0 -> accepted, no checksum; else DataVerify      net_udp.c:1940-1957, 1971
#           Tx DataCalc, 0 -> 0xFFFF; disabled -> 0                   net_udp.c:2909-2937
#   ICMPv6  Rx types 1, 3, 4: HdrVerify(msg, len) -- no pseudo-header net_icmpv6.c:2910-2920
#              types 128-131, 134-137: DataVerify(NET_BUF{ICMP_V6}, pseudo{.., 58}, 40)  :2923-2942
#              other types: rejected before the checksum (no verdict) :2945-2948
#           Tx DataCalc(NET_BUF{ICMP_V6}, pseudo, 40) for every type   net_icmpv6.c:1439 (the error
#              messages' ~HdrCalc(pseudo) field trick, :949-965, is tested equal in tests/)
# Extension headers (net_ipv6.c:8290-8360, 8396-8510): Hop-by-Hop (0, first only), Routing (43),
# Destination Options (60), length (HdrExtLen + 1) * 8 (net_ipv6.c:8601), are skipped -- a chain of
# any length, as NetIPv6_RxPktProcessExtHdr walks it -- and the upper-layer length becomes payload -
# extension bytes (net_ipv6.c:5682). Each is checked as the reference's handler checks it:
#   Hop-by-Hop / Destination Options (NetIPv6_RxOptHdr, net_ipv6.c:8604-8672): the options are walked
#     while the offset into them is < length - 2; an option whose type & 0x1F is not Pad1 (0), PadN (1)
#     or Router Alert (5) and whose action bits (type & 0xC0) are not "skip" drops the datagram
#     (NET_IPv6_ERR_INVALID_EH_OPT); Pad1 advances 1 octet, every other option Len + 2;
#   Routing (NetIPv6_RxRoutingHdr, net_ipv6.c:8735-8753): a routing type other than 0, 1, 2 with
#     Segments Left != 0 drops the datagram (NET_IPv6_ERR_INVALID_EH_OPT_SEQ).
# A dropped datagram, any other extension header, or a Hop-by-Hop header after the first -> EXT_HDR:
# the reference never reaches a transport checksum for them. Fragment (44) -> FRAGMENT. An extension
# header running past the payload -> MALFORMED: the reference has no such check (its
# NET_IPv6_ERR_INVALID_EH_LEN, net_ipv6.c:8381, is never raised; it reads on past the payload and its
# DataLen -= eh_len wraps, net_ipv6.c:8602), so the datagram gets no transport verdict here instead of
# reading past the bytes present.
# ---------------------------------------------------------------------------------------------
EXT_HDR = 128
IPV6_EXT = {0, 43, 44, 50, 51, 59, 60, 135, 139, 140, 253, 254}
ICMPV6_PSEUDO_TYPES = {128, 129, 130, 131, 134, 135, 136, 137}
ICMPV6_NOPSEUDO_TYPES = {1, 3, 4}


def opt_hdr_accepts(pkt: bytes, off: int, eh_len: int) -> bool:
    """NetIPv6_RxOptHdr's option walk (net_ipv6.c:8604-8672) over the header at pkt[off:off+eh_len]."""
    nto = 0
    while nto < eh_len - 2:
        t = pkt[off + 2 + nto]
        opt, act = t & 0x1F, t & 0xC0
        if opt not in (0, 1, 5) and act != 0:
            return False                       # DISCARD, DISCARD_IPPM or DISCARD_IPPM_MC
        # an option starting at the header's last octet reads its Len one past the header; any value
        # ends the walk there, so it is not needed
        nto += 1 if opt == 0 else (pkt[off + 3 + nto] if nto + 3 < eh_len else 0) + 2
    return True


def routing_hdr_accepts(pkt: bytes, off: int) -> bool:
    """NetIPv6_RxRoutingHdr (net_ipv6.c:8735-8753): types 0-2 pass; others need Segments Left 0."""
    return pkt[off + 2] <= 2 or pkt[off + 3] == 0


def _parse6(pkt: bytes):
    """-> None (malformed) or (flags_so_far, transport offset, upper-layer length, next header, addrs)."""
    if len(pkt) < 40 or pkt[0] >> 4 != 6:
        return None
    plen = struct.unpack("!H", pkt[4:6])[0]
    tot = 40 + plen
    if tot > len(pkt):
        return None
    nh, off = pkt[6], 40
    while nh in (0, 43, 60):                   # net_ipv6.c:8411-8418: until a non-extension header
        if nh == 0 and off != 40:              # Hop-by-Hop only first (net_ipv6.c:8307-8309)
            return EXT_HDR, off, 0, nh, pkt[8:40]
        if off + 8 > tot:                      # the header itself would run past the payload
            return None
        eh_len = (pkt[off + 1] + 1) * 8
        if off + eh_len > tot:
            return None
        if not (routing_hdr_accepts(pkt, off) if nh == 43 else opt_hdr_accepts(pkt, off, eh_len)):
            return EXT_HDR, off, 0, nh, pkt[8:40]
        nh, off = pkt[off], off + eh_len
    if nh == 44:
        return FRAGMENT, off, 0, nh, pkt[8:40]
    if nh in IPV6_EXT:
        return EXT_HDR, off, 0, nh, pkt[8:40]
    return 0, off, tot - off, nh, pkt[8:40]


def pseudo6(addrs: bytes, length: int, nh: int) -> bytes:
    return addrs + struct.pack("!IHH", length, 0, nh)


def _l4_chain6(pkt: bytes, proto_type: int, l4len: int, icmp=False, ix=40):
    if icmp:
        return netcsum.Chain([{"data": pkt, "proto": proto_type, "icmp_ix": ix, "icmp_hdr_len": 0,
                               "data_len": l4len}])
    return netcsum.Chain([{"data": pkt, "proto": proto_type, "transport_ix": ix, "transport_hdr_len": 0,
                           "data_len": l4len}])


def rx_validate_v6(pkt: bytes) -> int:
    pkt = bytes(pkt)
    p = _parse6(pkt)
    if p is None:
        return MALFORMED
    fx, off, plen, nh, addrs = p
    f = IP_OK | fx
    if fx:
        return f
    if off != 40:                              # transport after extension headers
        pkt = pkt[:40] + pkt[off:]
    if nh == 6:
        if plen < 20:
            return f | L4_MALFORMED
        ch = _l4_chain6(pkt, netcsum.NET_PROTOCOL_TYPE_TCP_V6, plen)
        ph = netcsum.HostBytes(pseudo6(addrs, plen, 6))
        v, _ = oracle.data_verify(ch.ptr, ph.ptr, 40)
        return f | L4_CHECKED | (L4_OK if v else 0)
    if nh == 17:
        if plen < 8:
            return f | L4_MALFORMED
        if struct.unpack("!H", pkt[44:46])[0] != plen:
            return f | L4_MALFORMED
        if pkt[46:48] == b"\x00\x00":
            return f | UDP_NO_CSUM | L4_OK
        ch = _l4_chain6(pkt, netcsum.NET_PROTOCOL_TYPE_UDP_V6, plen)
        ph = netcsum.HostBytes(pseudo6(addrs, plen, 17))
        v, _ = oracle.data_verify(ch.ptr, ph.ptr, 40)
        return f | L4_CHECKED | (L4_OK if v else 0)
    if nh == 58:
        if plen < 4:
            return f | L4_MALFORMED
        t = pkt[40]
        if t in ICMPV6_NOPSEUDO_TYPES:
            hb = netcsum.HostBytes(pkt[40:40 + plen])
            v, _ = oracle.hdr_verify(hb.ptr, plen)
        elif t in ICMPV6_PSEUDO_TYPES:
            ch = _l4_chain6(pkt, netcsum.NET_PROTOCOL_TYPE_ICMP_V6, plen, icmp=True)
            ph = netcsum.HostBytes(pseudo6(addrs, plen, 58))
            v, _ = oracle.data_verify(ch.ptr, ph.ptr, 40)
        else:
            return f
        return f | L4_CHECKED | (L4_OK if v else 0)
    return f


def tx_finalize_v6(pkt: bytes, udp_tx_csum: bool = True):
    """-> (finalized packet bytes, flags)."""
    pkt = bytes(pkt)
    p = _parse6(pkt)
    if p is None:
        return pkt, MALFORMED
    fx, off, plen, nh, addrs = p
    f = IP_OK | fx
    if fx:
        return pkt, f
    if off != 40:                              # finalize the transport part as if it followed the header
        hdr = pkt[:4] + struct.pack("!HB", plen, nh) + pkt[7:40]
        body, fl = tx_finalize_v6(hdr + pkt[off:], udp_tx_csum)
        return pkt[:off] + body[40:], fl
    pkt = bytearray(pkt)

    def calc(proto_type, nhv, icmp=False):
        ch = _l4_chain6(bytes(pkt), proto_type, plen, icmp)
        ph = netcsum.HostBytes(pseudo6(addrs, plen, nhv))
        c, _ = oracle.data_calc(ch.ptr, ph.ptr, 40)
        return c

    if nh == 6 and plen >= 20:
        pkt[56:58] = b"\x00\x00"
        pkt[56:58] = calc(netcsum.NET_PROTOCOL_TYPE_TCP_V6, 6).to_bytes(2, "little")
        f |= L4_CHECKED | L4_OK
    elif nh == 17 and plen >= 8 and struct.unpack("!H", bytes(pkt[44:46]))[0] == plen:
        pkt[46:48] = b"\x00\x00"
        if udp_tx_csum:
            c = calc(netcsum.NET_PROTOCOL_TYPE_UDP_V6, 17)
            pkt[46:48] = (c or 0xFFFF).to_bytes(2, "little")
            f |= L4_CHECKED | L4_OK
        else:
            f |= UDP_NO_CSUM
    elif nh == 58 and plen >= 4:
        pkt[42:44] = b"\x00\x00"
        pkt[42:44] = calc(netcsum.NET_PROTOCOL_TYPE_ICMP_V6, 58, icmp=True).to_bytes(2, "little")
        f |= L4_CHECKED | L4_OK
    elif nh in (6, 17, 58):
        f |= L4_MALFORMED
    return bytes(pkt), f


def rx_validate_ip(pkt: bytes) -> int:
    """Mixed batches: version nibble 6 -> IPv6, anything else -> IPv4 (include/netcsum_mi355x.h)."""
    return rx_validate_v6(pkt) if len(pkt) and pkt[0] >> 4 == 6 else rx_validate(pkt)


def tx_finalize_ip(pkt: bytes, udp_tx_csum: bool = True):
    if len(pkt) and pkt[0] >> 4 == 6:
        return tx_finalize_v6(pkt, udp_tx_csum)
    return tx_finalize(pkt, udp_tx_csum)
