"""Random IPv4 packet generator for the packet-batch tests (TCP, UDP, UDP without checksum, ICMP,
IGMP, other protocols, fragments, IP options, malformed headers/lengths, corrupted checksums)."""
from __future__ import annotations

import random
import struct

import numpy as np

import oracle_packets as op

KINDS = ["tcp", "tcp", "udp", "udp", "udp0", "icmp", "igmp", "other", "frag", "bad_ver", "bad_ihl",
         "bad_tot", "udp_badlen", "tcp_short", "corrupt_ip", "corrupt_l4"]


def make_packet(rng: random.Random, kind: str, payload: int | None = None) -> bytes:
    ihl = rng.choice([5, 5, 5, 6, 8, 15])
    opts = bytes(rng.getrandbits(8) for _ in range(ihl * 4 - 20))
    payload = rng.randint(0, 1600) if payload is None else payload
    data = bytes(rng.getrandbits(8) for _ in range(payload))
    if kind in ("tcp", "tcp_short", "corrupt_l4", "frag", "corrupt_ip"):
        proto = 6
        thl = rng.choice([20, 20, 32, 60])
        l4 = struct.pack("!HHIIBBHHH", rng.getrandbits(16), rng.getrandbits(16), rng.getrandbits(32),
                         rng.getrandbits(32), (thl // 4) << 4, 0x18, 0xFFFF, 0, 0) + bytes(thl - 20) + data
        if kind == "tcp_short":
            l4 = l4[:rng.randint(0, 19)]
    elif kind in ("udp", "udp0", "udp_badlen"):
        proto = 17
        ulen = 8 + len(data)
        if kind == "udp_badlen":
            ulen = (ulen + rng.choice([-3, -1, 1, 5])) & 0xFFFF
        l4 = struct.pack("!HHHH", rng.getrandbits(16), rng.getrandbits(16), ulen, 0) + data
    elif kind == "icmp":
        proto = 1
        l4 = struct.pack("!BBHHH", 8, 0, 0, rng.getrandbits(16), rng.getrandbits(16)) + data
    elif kind == "igmp":
        proto = 2
        l4 = struct.pack("!BBH4s", 0x16, 0, 0, bytes(rng.getrandbits(8) for _ in range(4)))
    else:
        proto = rng.choice([41, 47, 50, 89, 132])
        l4 = data
    tot = ihl * 4 + len(l4)
    frag = 0x4000
    if kind == "frag":
        frag = rng.choice([0x2000, 0x2000 | rng.randint(1, 0x1FFF), rng.randint(1, 0x1FFF)])
    ver_ihl = (4 << 4) | ihl
    if kind == "bad_ver":
        ver_ihl = (rng.choice([0, 6, 15]) << 4) | ihl
    if kind == "bad_ihl":
        ver_ihl = (4 << 4) | rng.randint(0, 4)
    hdr = struct.pack("!BBHHHBBH4s4s", ver_ihl, 0, tot & 0xFFFF, rng.getrandbits(16), frag, 64, proto, 0,
                      bytes(rng.getrandbits(8) for _ in range(4)), bytes(rng.getrandbits(8) for _ in range(4)))
    pkt = hdr + opts + l4
    if kind not in ("bad_ver", "bad_ihl", "bad_tot"):
        pkt, _ = op.tx_finalize(pkt, udp_tx_csum=(kind != "udp0"))
    if kind == "bad_tot":
        b = bytearray(pkt)
        b[2:4] = struct.pack("!H", len(pkt) + rng.randint(1, 40))
        pkt = bytes(b)
    if kind == "corrupt_ip":
        b = bytearray(pkt)
        b[8] ^= 1 << rng.randint(0, 7)
        pkt = bytes(b)
    if kind == "corrupt_l4" and len(pkt) > ihl * 4 + 20:
        b = bytearray(pkt)
        k = rng.randint(ihl * 4, len(b) - 1)
        b[k] ^= 1 << rng.randint(0, 7)
        pkt = bytes(b)
    return pkt


def packed_batch(pkts, rng: random.Random, trailer=True, lead=1):
    """Pack packets back to back (odd starts) with optional trailing bytes (e.g. Ethernet padding).
    -> (buffer uint8, offsets uint64, lengths uint16 = bytes present per packet)."""
    offs, lens, parts = [], [], [bytes(lead)]
    pos = lead
    for p in pkts:
        extra = bytes(rng.getrandbits(8) for _ in range(rng.randint(0, 5))) if trailer else b""
        offs.append(pos)
        lens.append(len(p) + len(extra))
        parts.append(p + extra)
        pos += len(p) + len(extra)
    parts.append(bytes(64))
    buf = np.frombuffer(b"".join(parts), dtype=np.uint8).copy()
    return buf, np.array(offs, np.uint64), np.array(lens, np.uint16)


KINDS6 = ["tcp", "tcp", "udp", "udp", "udp0", "icmp_echo", "icmp_err", "icmp_nd", "icmp_other", "ext",
          "other", "bad_ver", "bad_plen", "udp_badlen", "tcp_short", "corrupt_l4", "ext_ok", "ext_ok",
          "ext_frag", "ext_long", "ext_bad", "ext_hbh_late", "ext_opt_drop", "ext_rt_drop"]
EXT_OPAQUE = [50, 51, 59, 135, 139, 140, 253, 254]       # extension headers the batch does not walk


def _options(rng: random.Random, n: int) -> bytes:
    """n octets of Hop-by-Hop / Destination Options that NetIPv6_RxOptHdr accepts (net_ipv6.c:8604-
    8672): Pad1 and PadN, Router Alert, unknown options with the "skip" action, option types whose
    low 5 bits are 0 / 1 / 5 under any action bits, and a last option whose Len runs past the header
    (the walk just ends there)."""
    out = b""
    while len(out) < n:
        r = n - len(out)
        c = rng.random()
        if r == 1 or c < 0.15:
            out += bytes([rng.choice([0x00, 0x20, 0x40, 0x80, 0xC0])])                 # Pad1 (any action bits)
        elif c < 0.4:
            k = rng.randint(0, min(r - 2, 255))
            out += bytes([rng.choice([0x01, 0x21, 0xC1]), k]) + bytes(k)             # PadN
        elif c < 0.55 and r >= 4:
            out += bytes([rng.choice([0x05, 0x85]), 2]) + rng.randbytes(2)          # Router Alert
        elif c < 0.9 or r > 256:
            k = rng.randint(0, min(r - 2, 255))
            t = rng.choice([x for x in range(2, 32) if x != 5]) | rng.choice([0x00, 0x20])
            out += bytes([t, k]) + rng.randbytes(k)                                 # unknown, skip
        else:
            out += bytes([0x01, rng.randint(r - 1, 255)]) + rng.randbytes(r - 2)    # Len past the end
    return out[:n]


def ext_body(rng: random.Random, t: int, n: int) -> bytes:
    """The n octets after NextHdr / HdrExtLen of an extension header of type t that the reference
    accepts (random octets for other types)."""
    if t == 43:
        rt = rng.choice([0, 1, 2]) if rng.random() < 0.6 else rng.randint(3, 255)
        return bytes([rt, rng.randint(0, 255) if rt <= 2 else 0]) + rng.randbytes(n - 2)
    if t in (0, 60):
        return _options(rng, n)
    return rng.randbytes(n)


def _ext_chain(rng: random.Random, kinds, final_nh: int, reject: int | None = None) -> tuple[int, bytes]:
    """Extension headers of the given types (units of 8 B each) ending in final_nh -> (first nh, bytes).
    Option headers carry options the reference accepts and Routing headers a type / Segments Left it
    accepts (net_ipv6.c:8735-8753), except header number `reject`, which carries what it drops: an
    unknown option with a discard action, or a routing type > 2 with Segments Left != 0."""
    out, nh = b"", final_nh
    for j in reversed(range(len(kinds))):
        t, units = kinds[j]
        n = units * 8 - 2
        body = ext_body(rng, t, n)
        if t == 43 and reject == j:
            body = bytes([rng.randint(3, 255), rng.randint(1, 255)]) + body[2:]
        elif t in (0, 60):
            if reject == j:
                k = rng.randint(0, n - 2)                                          # reachable: valid options before
                pre = _options(rng, k) if k else b""
                while pre and (len(pre) < k or _ends_walk(pre)):
                    pre = _options(rng, k)
                bad = rng.choice([x for x in range(2, 32) if x != 5]) | rng.choice([0x40, 0x80, 0xC0])
                body = pre + bytes([bad]) + rng.randbytes(n - k - 1)
        out = struct.pack("!BB", nh, units - 1) + body + out
        nh = t
    return nh, out


def _ends_walk(opts: bytes) -> bool:
    """Does the option walk over `opts` (as a prefix of a longer area) end before its last octet?"""
    i = 0
    while i < len(opts):
        t = opts[i]
        if t & 0x1F == 0:
            i += 1
        elif i + 1 < len(opts):
            i += opts[i + 1] + 2
        else:
            return True
    return i != len(opts)


def make_packet_v6(rng: random.Random, kind: str, payload: int | None = None) -> bytes:
    """Random IPv6 datagram of one kind, finalized by the packet oracle (except the malformed and
    corrupted kinds). ICMPv6 error messages (types 1, 3, 4) are finalized as the reference's Tx does
    (pseudo-header included), so its Rx verdict for them (no pseudo-header) is usually a failure."""
    payload = rng.randint(0, 1600) if payload is None else payload
    data = rng.randbytes(payload)
    nh = 6
    if kind in ("tcp", "tcp_short", "corrupt_l4"):
        thl = rng.choice([20, 20, 32, 60])
        l4 = struct.pack("!HHIIBBHHH", rng.getrandbits(16), rng.getrandbits(16), rng.getrandbits(32),
                         rng.getrandbits(32), (thl // 4) << 4, 0x18, 0xFFFF, 0, 0) + bytes(thl - 20) + data
        if kind == "tcp_short":
            l4 = l4[:rng.randint(0, 19)]
    elif kind in ("udp", "udp0", "udp_badlen"):
        nh = 17
        ulen = 8 + len(data)
        if kind == "udp_badlen":
            ulen = (ulen + rng.choice([-3, -1, 1, 5])) & 0xFFFF
        l4 = struct.pack("!HHHH", rng.getrandbits(16), rng.getrandbits(16), ulen, 0) + data
    elif kind.startswith("icmp"):
        nh = 58
        t = {"icmp_echo": rng.choice([128, 129]), "icmp_err": rng.choice([1, 3, 4]),
             "icmp_nd": rng.choice([130, 131, 134, 135, 136, 137]),
             "icmp_other": rng.choice([2, 132, 133, 143, 200])}[kind]
        l4 = struct.pack("!BBH", t, rng.getrandbits(8), 0) + data
    elif kind == "ext":
        nh = rng.choice(EXT_OPAQUE)
        l4 = data
    elif kind.startswith("ext_"):
        inner = rng.choice(["tcp", "udp", "icmp_echo", "icmp_err"])
        body = make_packet_v6(rng, inner, payload)[40:]
        inner_nh = {"tcp": 6, "udp": 17}.get(inner, 58)
        if kind == "ext_ok":                                   # <= 48 B: inside every group's window
            chain = [(0, 1)] if rng.random() < 0.5 else []
            chain += [(rng.choice([43, 60]), rng.choice([1, 2])) for _ in range(rng.randint(0 if chain else 1, 2))]
            nh, ext = _ext_chain(rng, chain, inner_nh)
        elif kind == "ext_frag":
            nh, ext = _ext_chain(rng, [(60, 1)] * rng.randint(0, 1) + [(44, 1)], inner_nh)
        elif kind == "ext_long":                               # 1032+ B: beyond every batch kernel's window (walk pass)
            nh, ext = _ext_chain(rng, [(60, rng.randint(129, 200))], inner_nh)
        elif kind == "ext_hbh_late":
            nh, ext = _ext_chain(rng, [(60, 1), (0, 1)], inner_nh)
        elif kind == "ext_opt_drop":                           # an option the reference discards on
            chain = [(rng.choice([0, 60]), rng.choice([1, 1, 2, 3]))] + [(60, 1)] * rng.randint(0, 1)
            nh, ext = _ext_chain(rng, chain, inner_nh, reject=rng.randrange(len(chain)))
        elif kind == "ext_rt_drop":                            # routing type > 2, Segments Left != 0
            chain = [(60, 1)] * rng.randint(0, 1) + [(43, rng.choice([1, 2, 3]))]
            nh, ext = _ext_chain(rng, chain, inner_nh, reject=len(chain) - 1)
        else:                                                  # ext_bad: length past the payload
            nh, ext = _ext_chain(rng, [(43, 1)], inner_nh)
            ext = ext[:1] + bytes([rng.randint(20, 255)]) + ext[2:]
            body = body[:rng.randint(0, 40)]
        l4 = ext + body
    else:
        nh = rng.choice([4, 41, 47, 89, 132])
        l4 = data
    hdr = struct.pack("!IHBB16s16s", (6 << 28) | rng.getrandbits(20), len(l4), nh, 64, rng.randbytes(16),
                      rng.randbytes(16))
    pkt = hdr + l4
    if kind not in ("bad_ver", "bad_plen"):
        pkt, _ = op.tx_finalize_v6(pkt, udp_tx_csum=(kind != "udp0"))
    b = bytearray(pkt)
    if kind == "bad_ver":
        b[0] = (rng.choice([0, 4, 15]) << 4) | (b[0] & 0xF)
    if kind == "bad_plen":
        b[4:6] = struct.pack("!H", len(l4) + rng.randint(1, 40))
    if kind == "corrupt_l4" and len(b) > 60:
        k = rng.randint(8, len(b) - 1)                            # addresses are covered too
        b[k] ^= 1 << rng.randint(0, 7)
    return bytes(b)
