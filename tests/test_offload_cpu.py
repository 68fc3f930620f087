"""The checksum-offload seam on CPU (include/netcsum_mi355x.h (2b''); no GPU needed).

Rx: for every frame kind the packet generators make (IPv4 and IPv6: valid, corrupted IP header,
corrupted transport, UDP without a checksum, malformed headers and lengths, fragments, ICMP types,
IGMP, extension headers), the reference's outcome with its offload flags OFF
(oracle/oracle_offload.py rx_reference: net_ipv4.c:5243-5255, net_tcp.c:7845-7890,
net_udp.c:1916-1977, net_icmpv4.c:1665-1700, net_igmp.c:1332-1339, net_icmpv6.c:2910-2955) equals
the outcome of the adapter's action followed by the stack built with every
NET_*_CFG_CHK_SUM_OFFLOAD_RX_EN ON — both with and without NET_UDP_CFG_RX_CHK_SUM_DISCARD_EN. The
action is the library's own host function (NetUtil_MI355X_RxAction, the one the Rx kernels apply)
of the oracle's RxValidateIP verdict. Decisions must be equal for every frame; the counter too
whenever the reference drops the frame at a checksum check.

Tx: the adapter's per-datagram rule, applied to the frame the stack builds with every Tx offload
flag ON (IPv4 / TCP / ICMPv4 fields 0, UDP field 0xFFFF or 0 for "no checksum"), gives the frame the
reference builds with the flags OFF, for UDP checksums on and off (net_udp.c:2863-2935).
"""
import random
import struct

import netcsum
import oracle_offload as oo
import oracle_packets as op
from packets import KINDS, KINDS6, make_packet, make_packet_v6


def _frames(seed, n):
    rng = random.Random(seed)
    out = []
    for _ in range(n):
        if rng.random() < 0.5:
            out.append(make_packet(rng, rng.choice(KINDS), payload=rng.randint(0, 300)))
        else:
            out.append(make_packet_v6(rng, rng.choice(KINDS6), payload=rng.randint(0, 300)))
    # ICMPv4 types the reference rejects before the checksum, with good and bad checksums
    for t in (5, 9, 10, 15, 17, 42):
        p = bytearray(make_packet(rng, "icmp", payload=20))
        hlen = (p[0] & 0xF) * 4
        p[hlen] = t
        out.append(bytes(p))                                    # checksum now wrong
        out.append(op.tx_finalize(bytes(p))[0])                 # recomputed
    # every accepted ICMPv4 type, valid and corrupted
    for t in sorted(oo.ICMPV4_RX_TYPES):
        p = bytearray(make_packet(rng, "icmp", payload=24))
        hlen = (p[0] & 0xF) * 4
        p[hlen] = t
        good = op.tx_finalize(bytes(p))[0]
        out.append(good)
        bad = bytearray(good)
        bad[-1] ^= 0x10
        out.append(bytes(bad))
    # IGMP with a corrupted checksum
    g = bytearray(make_packet(rng, "igmp"))
    g[-1] ^= 1
    out.append(bytes(g))
    # UDP with a corrupted payload (IPv4 and IPv6)
    for mk in (make_packet, make_packet_v6):
        for _ in range(10):
            u = bytearray(mk(rng, "udp", payload=rng.randint(1, 200)))
            u[-1] ^= 1 << rng.randint(0, 7)
            out.append(bytes(u))
    return out


def _action(pkt, cfg):
    flags = op.rx_validate_ip(pkt)
    v6 = len(pkt) and pkt[0] >> 4 == 6
    return netcsum.rx_action(flags, oo.transport_proto(pkt), v6, cfg)


def test_rx_adapter_decisions_equal_the_reference():
    frames = _frames(1, 1500)
    seen = {}
    for discard in (False, True):
        cfg = netcsum.RXCFG_UDP_DISCARD_NO_CHK_SUM if discard else 0
        for k, pkt in enumerate(frames):
            want = oo.rx_reference(pkt, udp_discard=discard)
            a = _action(pkt, cfg)
            got = oo.rx_with_adapter(pkt, a, udp_discard=discard)
            assert got[0] == want[0], (k, discard, want, got, a, pkt[:48].hex())
            if want[0] == "drop" and want[1] in oo.CHECKSUM_COUNTERS:
                assert got[1] == want[1], (k, discard, want, got, a)
            seen[a] = seen.get(a, 0) + 1
    # every action the adapter can take occurred
    assert set(seen) == set(range(netcsum.RX_NBR_ACTIONS)), seen


def test_rx_checksum_failures_are_dropped_by_the_adapter_itself():
    """With the offload flags on, the stack accepts any checksum: every frame the reference drops at
    an offloaded checksum check must be dropped by the adapter's action, with that counter."""
    frames = _frames(2, 800)
    for pkt in frames:
        want = oo.rx_reference(pkt)
        a = _action(pkt, 0)
        if want[0] == "drop" and want[1] in oo.CHECKSUM_COUNTERS:
            assert oo.DROP_COUNTER.get(a) == want[1], (want, a, pkt[:48].hex())
        if a in oo.DROP_COUNTER:
            assert want[0] == "drop", (want, a)


def test_rx_udp_no_checksum_policy():
    rng = random.Random(3)
    for mk, kind in ((make_packet, "udp0"), (make_packet_v6, "udp0")):
        for _ in range(20):
            pkt = mk(rng, kind, payload=rng.randint(0, 200))
            assert _action(pkt, 0) == netcsum.RX_DELIVER
            assert _action(pkt, netcsum.RXCFG_UDP_DISCARD_NO_CHK_SUM) == netcsum.RX_DROP_UDP_NO_CHK_SUM
            assert oo.rx_reference(pkt, udp_discard=True) == ("drop", "UDP.RxHdrChkSumCtr")


def test_rx_action_table():
    """The action function itself, verdict by verdict (host logic of NetUtil_MI355X_RxAction)."""
    A = netcsum.rx_action
    IP, L4OK, CHK, NOCS, MAL, FRAG, L4MAL, EXT = 1, 2, 4, 8, 16, 32, 64, 128
    assert A(MAL, 6, False) == netcsum.RX_DELIVER                      # the stack rejects it itself
    assert A(MAL | IP, 6, True) == netcsum.RX_DELIVER
    assert A(CHK | L4OK, 6, False) == netcsum.RX_DROP_IPV4_CHK_SUM       # IP checksum first
    assert A(FRAG, 6, False) == netcsum.RX_DROP_IPV4_CHK_SUM
    assert A(IP | FRAG, 6, False) == netcsum.RX_DELIVER_L4_UNVERIFIED
    assert A(IP | FRAG, 6, True) == netcsum.RX_DELIVER_L4_UNVERIFIED
    assert A(FRAG, 6, True) == netcsum.RX_DELIVER_L4_UNVERIFIED          # IPv6: no header checksum
    assert A(IP | L4MAL, 17, False) == netcsum.RX_DELIVER
    assert A(IP | EXT, 0, True) == netcsum.RX_DELIVER
    for proto, v6, want in ((6, False, netcsum.RX_DROP_TCP_CHK_SUM), (6, True, netcsum.RX_DROP_TCP_CHK_SUM),
                            (17, False, netcsum.RX_DROP_UDP_CHK_SUM), (17, True, netcsum.RX_DROP_UDP_CHK_SUM),
                            (1, False, netcsum.RX_DROP_ICMPV4_CHK_SUM), (2, False, netcsum.RX_DROP_IGMP_CHK_SUM),
                            (58, True, netcsum.RX_DROP_ICMPV6_CHK_SUM)):
        assert A(IP | CHK, proto, v6) == want
        assert A(IP | CHK | L4OK, proto, v6) == netcsum.RX_DELIVER
    assert A(IP | NOCS | L4OK, 17, False) == netcsum.RX_DELIVER
    assert A(IP | NOCS | L4OK, 17, False, netcsum.RXCFG_UDP_DISCARD_NO_CHK_SUM) == netcsum.RX_DROP_UDP_NO_CHK_SUM
    assert A(IP, 47, False) == netcsum.RX_DELIVER


def test_rx_burst_tally():
    acts = [0, 1, 1, 2, 3, 3, 3, 4, 5, 6, 7, 8, 8]
    assert netcsum.rx_burst_tally(acts) == [1, 2, 1, 3, 1, 1, 1, 1, 2]
    assert netcsum.rx_burst_tally([]) == [0] * netcsum.RX_NBR_ACTIONS
    lib = netcsum.lib()
    import numpy as np
    bad = np.array([0, 9], np.uint8)
    ctr = np.zeros(netcsum.RX_NBR_ACTIONS, np.uint32)
    assert lib.NetUtil_MI355X_RxBurstTally(bad.ctypes.data, 2, ctr.ctypes.data) == netcsum.NET_UTIL_ERR_MI355X_INVALID_ARG
    assert not ctr.any()                                         # nothing counted on a bad action
    assert lib.NetUtil_MI355X_RxBurstTally(None, 0, None) == netcsum.NET_ERR_FAULT_NULL_PTR


def test_tx_adapter_rebuilds_the_reference_frames():
    rng = random.Random(4)
    n_udp_none = 0
    for k in range(600):
        v6 = k % 2 == 1
        kinds = ["tcp", "udp", "udp", "icmp", "igmp", "other", "frag"] if not v6 else \
            ["tcp", "udp", "udp", "icmp_echo", "icmp_err", "icmp_nd", "other", "ext_ok", "ext_frag"]
        kind = rng.choice(kinds)
        pkt = (make_packet_v6 if v6 else make_packet)(rng, kind, payload=rng.randint(0, 400))
        for csum in (True, False):
            want = op.tx_finalize_ip(pkt, udp_tx_csum=csum)[0]
            frame = oo.tx_stack_offload(pkt, udp_tx_csum=csum)
            assert oo.tx_burst_model(frame) == want, (kind, csum)
            if kind == "udp" and not csum:
                n_udp_none += 1
    assert n_udp_none > 20


def test_tx_offload_frames_carry_the_placeholders():
    """What the model of the offloading stack leaves in the fields (the seam's contract)."""
    rng = random.Random(5)
    p = make_packet(rng, "udp", payload=40)
    hlen = (p[0] & 0xF) * 4
    f = oo.tx_stack_offload(p)
    assert f[10:12] == b"\x00\x00" and f[hlen + 6:hlen + 8] == b"\xff\xff"
    assert oo.tx_stack_offload(p, udp_tx_csum=False)[hlen + 6:hlen + 8] == b"\x00\x00"
    t = make_packet(rng, "tcp", payload=40)
    hlen = (t[0] & 0xF) * 4
    assert oo.tx_stack_offload(t)[hlen + 16:hlen + 18] == b"\x00\x00"
    e = bytearray(make_packet(rng, "icmp", payload=8))          # echo request: computed anyway
    hlen = (e[0] & 0xF) * 4
    assert e[hlen] == 8 and oo.tx_stack_offload(bytes(e))[hlen + 2:hlen + 4] == bytes(e[hlen + 2:hlen + 4])
