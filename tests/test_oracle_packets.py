"""CPU checks of the packet oracle (tests/packets.py + oracle/oracle_packets.py): Tx-finalized
packets validate on Rx, every malformation class maps to its flag, corruption is detected."""
import random
import struct

import oracle_packets as op
from packets import KINDS, make_packet


def test_tx_then_rx_accepts_every_wellformed_kind():
    rng = random.Random(1)
    for _ in range(300):
        kind = rng.choice(["tcp", "udp", "icmp", "igmp", "other"])
        f = op.rx_validate(make_packet(rng, kind))
        assert f & op.IP_OK
        if kind in ("tcp", "udp", "icmp", "igmp"):
            assert f & op.L4_CHECKED and f & op.L4_OK, (kind, f)
        else:
            assert not f & op.L4_CHECKED


def test_flags_per_kind():
    rng = random.Random(2)
    expect = {"udp0": op.IP_OK | op.UDP_NO_CSUM | op.L4_OK, "bad_ver": op.MALFORMED, "bad_ihl": op.MALFORMED,
              "bad_tot": op.MALFORMED}
    for kind, want in expect.items():
        for _ in range(20):
            assert op.rx_validate(make_packet(rng, kind)) == want, kind
    for _ in range(40):
        assert op.rx_validate(make_packet(rng, "frag")) == op.IP_OK | op.FRAGMENT
        assert op.rx_validate(make_packet(rng, "udp_badlen")) == op.IP_OK | op.L4_MALFORMED
        assert op.rx_validate(make_packet(rng, "tcp_short")) == op.IP_OK | op.L4_MALFORMED
        assert not op.rx_validate(make_packet(rng, "corrupt_ip")) & op.IP_OK
        p = make_packet(rng, "corrupt_l4", payload=rng.randint(1, 500))
        assert op.rx_validate(p) == op.IP_OK | op.L4_CHECKED


def test_udp_zero_checksum_maps_to_ffff_on_tx():
    """Find a UDP payload whose checksum computes to 0 and check it is sent as 0xFFFF (RFC 768)."""
    rng = random.Random(3)
    base = make_packet(rng, "udp", payload=10)
    hlen = (base[0] & 0xF) * 4
    b = bytearray(base)
    b[hlen + 6:hlen + 8] = b"\x00\x00"
    pk, _ = op.tx_finalize(bytes(b))
    c = int.from_bytes(pk[hlen + 6:hlen + 8], "little")
    # adjust the last two payload bytes so that the one's-complement sum becomes 0xFFFF
    word = struct.unpack("!H", bytes(b[-2:]))[0]
    host_c = ((c & 0xFF) << 8) | (c >> 8)            # checksum value in network order
    new = (word + host_c) % 0xFFFF
    b[-2:] = struct.pack("!H", new)
    pk2, _ = op.tx_finalize(bytes(b))
    assert pk2[hlen + 6:hlen + 8] == b"\xff\xff"
    assert op.rx_validate(pk2) & op.L4_OK


def test_every_kind_generates():
    rng = random.Random(4)
    for k in KINDS:
        assert isinstance(op.rx_validate(make_packet(rng, k)), int)
