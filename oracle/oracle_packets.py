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
