"""CPU checks of the IPv6 packet oracle (oracle/oracle_packets.py *_v6, tests/packets.py
make_packet_v6): the restatement agrees with an independent RFC 1071 / RFC 8200 §8.1 checksum written
here from the RFC text, Tx-finalized packets validate on Rx, the reference's ICMPv6 quirks hold, and
every malformation class maps to its flag."""
import random
import struct

import netcsum
import oracle
import oracle_packets as op
from packets import KINDS6, make_packet_v6


def rfc1071(data: bytes) -> int:
    """Plain RFC 1071: one's-complement of the one's-complement sum of big-endian 16-bit words."""
    if len(data) & 1:
        data += b"\x00"
    s = sum(struct.unpack(f"!{len(data) // 2}H", data))
    while s >> 16:
        s = (s & 0xFFFF) + (s >> 16)
    return (~s) & 0xFFFF


def rfc_l4_checksum(pkt: bytes, field: int) -> int:
    """RFC 8200 §8.1 upper-layer checksum of an IPv6 packet (network-order value), field zeroed."""
    plen = struct.unpack("!H", pkt[4:6])[0]
    l4 = bytearray(pkt[40:40 + plen])
    l4[field:field + 2] = b"\x00\x00"
    return rfc1071(pkt[8:40] + struct.pack("!IHH", plen, 0, pkt[6]) + bytes(l4))


def test_tx_matches_independent_rfc_checksum():
    rng = random.Random(61)
    for _ in range(300):
        kind = rng.choice(["tcp", "udp", "icmp_echo", "icmp_err", "icmp_nd", "icmp_other"])
        pkt = make_packet_v6(rng, kind, payload=rng.randint(0, 700))
        field = {6: 16, 17: 6, 58: 2}[pkt[6]]
        got = struct.unpack("!H", pkt[40 + field:42 + field])[0]
        want = rfc_l4_checksum(pkt, field)
        if pkt[6] == 17 and want == 0:
            want = 0xFFFF
        assert got == want, kind


def test_tx_then_rx_per_kind():
    rng = random.Random(62)
    for _ in range(400):
        kind = rng.choice(["tcp", "udp", "icmp_echo", "icmp_nd", "icmp_other", "ext", "other", "udp0"])
        f = op.rx_validate_v6(make_packet_v6(rng, kind))
        assert f & op.IP_OK
        if kind in ("tcp", "udp", "icmp_echo", "icmp_nd"):
            assert f == op.IP_OK | op.L4_CHECKED | op.L4_OK, (kind, f)
        elif kind == "udp0":
            assert f == op.IP_OK | op.UDP_NO_CSUM | op.L4_OK
        elif kind == "ext":
            assert f == op.IP_OK | op.EXT_HDR
        else:
            assert f == op.IP_OK, (kind, f)


def test_icmpv6_error_types_are_verified_without_pseudo_header():
    """net_icmpv6.c:2910-2920: types 1/3/4 are checked by HdrVerify over the message alone, so the
    verdict equals 'RFC 1071 over the message == 0' (a pseudo-header-correct message usually fails)."""
    rng = random.Random(63)
    fails = 0
    for _ in range(200):
        pkt = make_packet_v6(rng, "icmp_err", payload=rng.randint(0, 300))
        plen = struct.unpack("!H", pkt[4:6])[0]
        f = op.rx_validate_v6(pkt)
        ok = rfc1071(pkt[40:40 + plen]) == 0
        assert f == op.IP_OK | op.L4_CHECKED | (op.L4_OK if ok else 0)
        fails += not ok
    assert fails > 190


def test_icmpv6_error_tx_trick_equals_datacalc_with_pseudo():
    """net_icmpv6.c:949-965 computes error-message checksums as HdrCalc(msg) with the field set to
    ~HdrCalc(pseudo); the oracle's Tx uses DataCalc(msg, pseudo). Same value."""
    rng = random.Random(64)
    for _ in range(200):
        pkt = make_packet_v6(rng, "icmp_err", payload=rng.randint(0, 300))
        plen = struct.unpack("!H", pkt[4:6])[0]
        ph = netcsum.HostBytes(op.pseudo6(pkt[8:40], plen, 58))
        c1, _ = oracle.hdr_calc(ph.ptr, 40)
        msg = bytearray(pkt[40:40 + plen])
        msg[2:4] = ((~c1) & 0xFFFF).to_bytes(2, "little")         # host-order store, as the C does
        mb = netcsum.HostBytes(bytes(msg))
        c2, _ = oracle.hdr_calc(mb.ptr, plen)
        assert c2.to_bytes(2, "little") == pkt[42:44]


def test_malformed_and_corrupt_flags():
    rng = random.Random(65)
    for _ in range(40):
        assert op.rx_validate_v6(make_packet_v6(rng, "bad_ver")) == op.MALFORMED
        assert op.rx_validate_v6(make_packet_v6(rng, "bad_plen")) == op.MALFORMED
        assert op.rx_validate_v6(make_packet_v6(rng, "udp_badlen")) == op.IP_OK | op.L4_MALFORMED
        assert op.rx_validate_v6(make_packet_v6(rng, "tcp_short")) == op.IP_OK | op.L4_MALFORMED
        p = make_packet_v6(rng, "corrupt_l4", payload=rng.randint(30, 500))
        assert op.rx_validate_v6(p) == op.IP_OK | op.L4_CHECKED
    assert op.rx_validate_v6(b"\x60" + bytes(38)) == op.MALFORMED


def test_every_v6_kind_generates():
    rng = random.Random(66)
    for k in KINDS6:
        assert isinstance(op.rx_validate_v6(make_packet_v6(rng, k)), int)


def test_extension_headers_walked_and_flagged():
    """Hop-by-Hop / Routing / Destination Options are skipped (upper-layer length = payload - their
    bytes), the transport checksum then equals the RFC checksum of the transport part with that
    length; Fragment -> FRAGMENT; opaque ones and late Hop-by-Hop -> EXT_HDR; chains of any length walked."""
    rng = random.Random(67)
    for _ in range(200):
        pkt = make_packet_v6(rng, "ext_ok", payload=rng.randint(0, 300))
        f = op.rx_validate_v6(pkt)
        assert f & op.IP_OK and not f & (op.EXT_HDR | op.FRAGMENT | op.MALFORMED)
        fx, off, ulen, nh, _ = op._parse6(pkt)
        assert fx == 0 and off > 40 and nh in (6, 17, 58)
        flat = pkt[:4] + struct.pack("!HB", ulen, nh) + pkt[7:40] + pkt[off:]
        if nh in (6, 17):
            field = {6: 16, 17: 6}[nh]
            want = rfc_l4_checksum(flat, field)
            got = struct.unpack("!H", flat[40 + field:42 + field])[0]
            assert got == (want or 0xFFFF if nh == 17 else want)
            assert f == op.IP_OK | op.L4_CHECKED | op.L4_OK
    for _ in range(50):
        assert op.rx_validate_v6(make_packet_v6(rng, "ext_frag")) == op.IP_OK | op.FRAGMENT
        assert op.rx_validate_v6(make_packet_v6(rng, "ext_hbh_late")) == op.IP_OK | op.EXT_HDR
        assert op.rx_validate_v6(make_packet_v6(rng, "ext_bad")) == op.MALFORMED
        f = op.rx_validate_v6(make_packet_v6(rng, "ext_long"))          # walked to the end, any length
        assert f & op.L4_CHECKED and not f & op.EXT_HDR
        assert op.rx_validate_v6(make_packet_v6(rng, "ext")) == op.IP_OK | op.EXT_HDR


def test_mixed_dispatch_follows_the_version_nibble():
    """rx_validate_ip / tx_finalize_ip (the mixed-ring oracle): version 6 -> IPv6 rules, anything
    else -> IPv4 rules (an IPv4 packet relabelled 6 is judged as IPv6, and vice versa)."""
    from packets import make_packet
    rng = random.Random(68)
    for _ in range(100):
        p4 = make_packet(rng, "tcp")
        p6 = make_packet_v6(rng, "tcp")
        assert op.rx_validate_ip(p4) == op.rx_validate(p4)
        assert op.rx_validate_ip(p6) == op.rx_validate_v6(p6)
        swapped = bytes([0x60 | (p4[0] & 0xF)]) + p4[1:]
        assert op.rx_validate_ip(swapped) == op.rx_validate_v6(swapped)
        assert op.tx_finalize_ip(p6) == op.tx_finalize_v6(p6)
    assert op.rx_validate_ip(b"") == op.MALFORMED


def test_chains_of_any_length_and_their_outcomes():
    """The oracle walks Hop-by-Hop / Routing / Destination Options chains of any length and header
    count (net_ipv6.c:8411-8418): 1..20 headers of 1..140 units reach the transport header; a chain
    cut at the payload end or running past it is MALFORMED; Fragment / an opaque header / a late
    Hop-by-Hop after a long chain keep their outcomes."""
    from packets import _ext_chain
    rng = random.Random(69)
    for _ in range(200):
        inner = make_packet_v6(rng, rng.choice(["tcp", "udp", "icmp_echo"]), payload=rng.randint(0, 200))
        kinds = [(rng.choice([43, 60]), rng.randint(1, 140 if k == 0 else 3)) for k in range(rng.randint(1, 20))]
        if rng.random() < 0.3:
            kinds = [(0, rng.randint(1, 4))] + kinds                 # Hop-by-Hop first: allowed
        nh, ext = _ext_chain(rng, kinds, inner[6])
        body = ext + inner[40:]
        pkt, ft = op.tx_finalize_v6(inner[:4] + struct.pack("!HB", len(body), nh) + inner[7:40] + body)
        assert ft == op.IP_OK | op.L4_CHECKED | op.L4_OK
        assert op.rx_validate_v6(pkt) == op.IP_OK | op.L4_CHECKED | op.L4_OK
        fx, off, ulen, nh2, _ = op._parse6(pkt)
        assert fx == 0 and off == 40 + len(ext) and ulen == len(inner) - 40 and nh2 == inner[6]
    for tail, want in ((44, op.IP_OK | op.FRAGMENT), (50, op.IP_OK | op.EXT_HDR), (0, op.IP_OK | op.EXT_HDR)):
        kinds = [(60, 100), (43, 2)] + ([(44, 1)] if tail == 44 else [(0, 1)] if tail == 0 else [])
        nh, ext = _ext_chain(rng, kinds, 6 if tail != 50 else 50)
        body = ext + bytes(40)
        pkt = struct.pack("!IHBB32s", 6 << 28, len(body), nh, 64, bytes(32)) + body
        assert op.rx_validate_v6(pkt) == want, tail
    nh, ext = _ext_chain(rng, [(60, 100)], 43)                        # next header 43, no bytes left
    pkt = struct.pack("!IHBB32s", 6 << 28, len(ext), nh, 64, bytes(32)) + ext
    assert op.rx_validate_v6(pkt) == op.MALFORMED
    nh, ext = _ext_chain(rng, [(60, 100), (43, 1)], 6)
    b = bytearray(struct.pack("!IHBB32s", 6 << 28, len(ext) + 20, nh, 64, bytes(32)) + ext + bytes(20))
    b[40 + 800 + 1] = 200                                             # the Routing header runs past the payload
    assert op.rx_validate_v6(bytes(b)) == op.MALFORMED


def test_option_and_routing_header_rules():
    """Hand-made headers against NetIPv6_RxOptHdr (net_ipv6.c:8604-8672) and NetIPv6_RxRoutingHdr
    (:8735-8753): an option is judged by type & 0x1F (Pad1 0, PadN 1, Router Alert 5 pass under any
    action bits) and otherwise by its action bits (0x00 skip passes; 0x40 / 0x80 / 0xC0 drop); the walk
    only sees options it reaches; a routing type > 2 drops iff Segments Left != 0. A dropped datagram
    gets EXT_HDR (no transport verdict), its neighbours' verdicts are unchanged."""
    inner = make_packet_v6(random.Random(70), "tcp", payload=40)

    def dgram(nh, ext):
        body = ext + inner[40:]
        return op.tx_finalize_v6(inner[:4] + struct.pack("!HB", len(body), nh) + inner[7:40] + body)[0]

    ok = op.IP_OK | op.L4_CHECKED | op.L4_OK
    rej = op.IP_OK | op.EXT_HDR
    opts = [  # (6 option octets of an 8-B header, accepted?)
        (bytes([0, 0, 0, 0, 0, 0]), True),                       # Pad1 x 6
        (bytes([1, 4, 0, 0, 0, 0]), True),                       # PadN
        (bytes([5, 2, 0, 0, 1, 4, 0, 0][:6]), True),             # Router Alert, PadN cut by the end
        (bytes([0x3E, 4, 9, 9, 9, 9]), True),                    # unknown, skip (+ change bit)
        (bytes([0x1E, 0, 0x01, 2, 0, 0]), True),
        (bytes([0x7E, 4, 9, 9, 9, 9]), False),                   # unknown, discard
        (bytes([0xBE, 4, 9, 9, 9, 9]), False),                   # discard + ICMP
        (bytes([0xFE, 4, 9, 9, 9, 9]), False),                   # discard + ICMP unless multicast
        (bytes([0, 0, 0, 0, 0, 0xDE]), False),                   # reached at the last octet
        (bytes([0x40, 0x80, 0xC0, 0x20, 0, 0]), True),           # opt 0 under any action: Pad1
        (bytes([0xC5, 2, 1, 1, 0xC1, 0]), True),                 # Router Alert / PadN with action bits
        (bytes([1, 4, 0xDE, 0, 0, 0]), True),                    # the discard option is PadN's data
        (bytes([0x01, 200, 0xDE, 0, 0, 0]), True),               # a Len past the header ends the walk
    ]
    for first in (0, 60):
        for o, accepted in opts:
            nh, ext = first, bytes([6, 0]) + o
            assert op.rx_validate_v6(dgram(nh, ext)) == (ok if accepted else rej), (first, o.hex())
            # second in a chain behind an accepted Destination Options header
            nh2, ext2 = 60, bytes([first if first == 60 else 60, 0]) + bytes(6) + ext
            assert op.rx_validate_v6(dgram(nh2, ext2)) == (ok if accepted else rej), (first, o.hex())
    for rt, sl, accepted in ((0, 7, True), (1, 1, True), (2, 255, True), (3, 0, True), (3, 1, False),
                             (4, 2, False), (255, 255, False), (200, 0, True)):
        ext = bytes([6, 0, rt, sl]) + bytes(4)
        assert op.rx_validate_v6(dgram(43, ext)) == (ok if accepted else rej), (rt, sl)
