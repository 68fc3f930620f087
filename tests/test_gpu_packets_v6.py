"""GPU parity of the IPv6 packet batches (NetUtil_MI355X_RxValidateIPv6 / TxFinalizeIPv6) against
the IPv6 packet oracle (oracle/oracle_packets.py *_v6, pinned to an independent RFC 8200 checksum in
tests/test_oracle_packets_v6.py): every packet kind, packed odd-aligned and strided layouts, every lane
group width, grid-stride and tiled launches, Tx write-back in place."""
import random
import struct

import numpy as np
import pytest

import netcsum
import oracle_packets as op
from packets import KINDS6, ext_body, make_packet_v6, packed_batch

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(autouse=True)
def _defaults():
    def reset():
        for k in (netcsum.TUNE_GRID_BLOCKS, netcsum.TUNE_GROUP_LANES):
            netcsum.tune(k, 0)
        netcsum.tune(netcsum.TUNE_NT_LOADS, -1)
        netcsum.tune(netcsum.TUNE_TILE, -1)
        netcsum.tune(netcsum.TUNE_KERNEL, 0)
    reset()
    yield
    reset()


def _dev(buf, offs, lens):
    return (torch.from_numpy(buf).to(DEV), torch.from_numpy(offs.view(np.int64)).to(DEV),
            torch.from_numpy(lens.view(np.int16)).to(DEV))


def _auto_group(varlen, pkt_len=0):
    """The ABI's lane-group choice for packet batches (netcsum_abi.hip pkt_batch)."""
    if varlen:
        return 32
    want = max(1, ((pkt_len + 30) // 16 + 5) // 6)
    return max(8, next((g for g in (1, 4, 8, 16, 32, 64) if g >= want), 64))


def _rx_gpu(buf, offs, lens):
    b, o, ln = _dev(buf, offs, lens)
    f = torch.zeros(len(offs), dtype=torch.uint8, device=DEV)
    netcsum.rx_validate_ipv6(b, len(offs), f, off=o, lens=ln)
    torch.cuda.synchronize()
    return f.cpu().numpy()


@pytest.mark.parametrize("group", [0, 8, 16, 32, 64])
@pytest.mark.parametrize("grid,tile", [(0, -1), (3, 0)])
def test_rx_validate_v6_mixed_varlen(group, grid, tile):
    rng = random.Random(600 + group * 7 + grid)
    pkts = [make_packet_v6(rng, rng.choice(KINDS6)) for _ in range(1500)]
    buf, offs, lens = packed_batch(pkts, rng)
    netcsum.tune(netcsum.TUNE_GROUP_LANES, group)
    netcsum.tune(netcsum.TUNE_GRID_BLOCKS, grid)
    netcsum.tune(netcsum.TUNE_TILE, tile)
    got = _rx_gpu(buf, offs, lens)
    g = group or _auto_group(True)
    want = np.array([op.rx_validate_v6(bytes(buf[o:o + n]))
                     for o, n in zip(offs.tolist(), lens.tolist())], np.uint8)
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, [(pkts[i][:48].hex(), int(got[i]), int(want[i])) for i in bad[:5]]
    assert (want & op.EXT_HDR).any() and (want & op.FRAGMENT).any()


def test_rx_validate_v6_strided_c2_shape():
    """1500-B TCP/IPv6 datagrams, strided (the C2 shape with real IPv6/TCP headers), nt on and off."""
    rng = random.Random(611)
    n, L = 4000, 1500
    buf = np.zeros(n * L + 64, np.uint8)
    for i in range(n):
        p = make_packet_v6(rng, rng.choice(["tcp", "tcp", "corrupt_l4", "udp"]), payload=L - 60)[:L]
        buf[i * L:i * L + len(p)] = np.frombuffer(p, np.uint8)
    want = np.array([op.rx_validate_v6(bytes(buf[i * L:(i + 1) * L])) for i in range(n)], np.uint8)
    b = torch.from_numpy(buf).to(DEV)
    for nt in (-1, 0, 1):
        netcsum.tune(netcsum.TUNE_NT_LOADS, nt)
        f = torch.zeros(n, dtype=torch.uint8, device=DEV)
        netcsum.rx_validate_ipv6(b, n, f, stride=L, pkt_len=L)
        torch.cuda.synchronize()
        assert np.array_equal(f.cpu().numpy(), want), nt


@pytest.mark.parametrize("udp_tx_csum", [True, False])
@pytest.mark.parametrize("group", [0, 8, 64])
def test_tx_finalize_v6_varlen_then_rx_accepts(udp_tx_csum, group):
    rng = random.Random(620 + udp_tx_csum + group)
    kinds = ["tcp", "udp", "udp", "icmp_echo", "icmp_err", "icmp_nd", "icmp_other", "ext", "other",
             "udp_badlen", "tcp_short", "bad_ver", "bad_plen", "ext_ok", "ext_ok", "ext_frag", "ext_long",
             "ext_bad", "ext_hbh_late"]
    pkts = []
    for _ in range(2000):
        p = bytearray(make_packet_v6(rng, rng.choice(kinds)))
        if len(p) >= 60 and rng.random() < 0.5:
            for fo in (42, 46, 56):                               # stale transport checksum fields
                p[fo:fo + 2] = rng.randbytes(2)
        pkts.append(bytes(p))
    buf, offs, lens = packed_batch(pkts, rng)
    netcsum.tune(netcsum.TUNE_GROUP_LANES, group)
    b, o, ln = _dev(buf, offs, lens)
    f = torch.zeros(len(pkts), dtype=torch.uint8, device=DEV)
    netcsum.tx_finalize_ipv6(b, len(pkts), f, off=o, lens=ln, udp_tx_csum=udp_tx_csum)
    torch.cuda.synchronize()
    out, flags = b.cpu().numpy(), f.cpu().numpy()
    g = group or _auto_group(True)
    for i, (off, n) in enumerate(zip(offs.tolist(), lens.tolist())):
        pkt = bytes(buf[off:off + n])
        want_pkt, want_f = op.tx_finalize_v6(pkt, udp_tx_csum)
        assert bytes(out[off:off + n]) == want_pkt, (i, pkt[:48].hex())
        assert flags[i] == want_f, (i, int(flags[i]), want_f)
    assert np.array_equal(out[:offs[0]], buf[:offs[0]])
    got = _rx_gpu(out, offs, lens)
    want = np.array([op.rx_validate_v6(bytes(out[o:o + n]))
                     for o, n in zip(offs.tolist(), lens.tolist())], np.uint8)
    assert np.array_equal(got, want)
    tcp_udp = np.array([len(p) >= 48 and p[0] >> 4 == 6 and p[6] in (6, 17) for p in pkts])
    checked = tcp_udp & ((got & op.L4_CHECKED) != 0)
    assert checked.sum() > 50 and ((got[checked] & op.L4_OK) != 0).all()


@pytest.mark.parametrize("stride,pkt_len", [(1500, 1500), (1540, 1514), (200, 184), (96, 72)])
@pytest.mark.parametrize("group", [0, 16, 32])
def test_tx_finalize_v6_strided_vs_oracle(stride, pkt_len, group):
    """Strided IPv6 Tx through the lane-group kernel (TUNE_KERNEL 2; the run-stream form has its own
    tests in test_gpu_pktstream.py): packets finalized exactly as the oracle does with the group's
    window, bytes between packets untouched."""
    netcsum.tune(netcsum.TUNE_KERNEL, 2)
    rng = random.Random(stride * 5 + pkt_len + group)
    n = 600
    kinds = ["tcp", "tcp", "udp", "udp0", "icmp_echo", "icmp_err", "ext", "other", "tcp_short", "bad_ver",
             "ext_ok", "ext_frag", "ext_hbh_late"]
    buf = np.frombuffer(rng.randbytes(n * stride + 64), np.uint8).copy()
    for i in range(n):
        p = make_packet_v6(rng, rng.choice(kinds), payload=rng.randint(0, max(0, pkt_len - 110)))[:pkt_len]
        buf[i * stride:i * stride + len(p)] = np.frombuffer(p, np.uint8)
    netcsum.tune(netcsum.TUNE_GROUP_LANES, group)
    g = group or _auto_group(False, pkt_len)
    b = torch.from_numpy(buf).to(DEV)
    assert b.data_ptr() % 64 == 0
    f = torch.zeros(n, dtype=torch.uint8, device=DEV)
    netcsum.tx_finalize_ipv6(b, n, f, stride=stride, pkt_len=pkt_len)
    torch.cuda.synchronize()
    out = b.cpu().numpy()
    want = buf.copy()
    want_f = np.zeros(n, np.uint8)
    for i in range(n):
        pk, want_f[i] = op.tx_finalize_v6(bytes(buf[i * stride:i * stride + pkt_len]), True)
        want[i * stride:i * stride + pkt_len] = np.frombuffer(pk, np.uint8)
    bad = np.nonzero(out != want)[0]
    assert bad.size == 0, [(int(j), int(j) // stride, int(j) % stride, int(out[j]), int(want[j])) for j in bad[:8]]
    assert np.array_equal(f.cpu().numpy(), want_f)


def test_v6_empty_batch_and_null_flags():
    b = torch.zeros(64, dtype=torch.uint8, device=DEV)
    assert netcsum.rx_validate_ipv6(b, 0, None, stride=64, pkt_len=64) == netcsum.NET_UTIL_ERR_NONE
    assert netcsum.rx_validate_ipv6(b, 1, None, stride=64, pkt_len=64, check=False) != netcsum.NET_UTIL_ERR_NONE


def _long_chain_pkts(rng, max_units, n_hdrs=(1,), reps=3):
    """Valid datagrams whose transport follows Routing / Destination Options chains of n headers of
    1..max_units 8-B units each (the walk pass finishes whatever the batch kernel's window holds not)."""
    pkts = []
    for units in range(1, max_units + 1):
        for h in n_hdrs:
            for _ in range(reps):
                inner = make_packet_v6(rng, rng.choice(["tcp", "udp", "icmp_echo", "icmp_err"]), payload=rng.randint(24, 200))
                nh, ext = inner[6], b""
                for _k in range(h):
                    u = rng.randint(1, units)
                    t = rng.choice([43, 60])
                    ext = struct.pack("!BB", nh, u - 1) + ext_body(rng, t, u * 8 - 2) + ext
                    nh = t
                body = ext + inner[40:]
                hdr = inner[:4] + struct.pack("!HB", len(body), nh) + inner[7:40]
                pkts.append(op.tx_finalize_v6(hdr + body)[0])
    return pkts


@pytest.mark.parametrize("group", [8, 16, 64])
def test_rx_tx_v6_extension_chains_of_any_length(group):
    """Extension-header chains of every length around and far past the group's window (16 G bytes of
    the frame minus the packet's lead) and of 1..12 headers, at every lead 0-15: every one walked to
    its transport header like the reference (net_ipv6.c:8396-8510), Rx verdicts and Tx bytes equal
    the oracle's, no EXT_HDR left."""
    rng = random.Random(700 + group)
    pkts = _long_chain_pkts(rng, 2 * group + 5) + _long_chain_pkts(rng, 3, n_hdrs=(4, 5, 8, 12), reps=4)
    rng.shuffle(pkts)
    buf, offs, lens = packed_batch(pkts, rng)
    netcsum.tune(netcsum.TUNE_GROUP_LANES, group)
    got = _rx_gpu(buf, offs, lens)
    want = np.array([op.rx_validate_v6(bytes(buf[o:o + n]))
                     for o, n in zip(offs.tolist(), lens.tolist())], np.uint8)
    assert np.array_equal(got, want), np.nonzero(got != want)[0][:8]
    assert not (want & op.EXT_HDR).any() and (want & op.L4_CHECKED).all() and ((want & op.L4_OK) != 0).any()
    # Tx of the same datagrams with stale transport fields: the oracle's bytes and flags
    stale = buf.copy()
    for o, n in zip(offs.tolist(), lens.tolist()):
        fx, off, _ul, nh, _ = op._parse6(bytes(buf[o:o + n]))
        fld = o + off + {6: 16, 17: 6, 58: 2}[nh]
        stale[fld:fld + 2] = np.frombuffer(rng.randbytes(2), np.uint8)
    b, o, ln = _dev(stale, offs, lens)
    fl = torch.zeros(len(lens), dtype=torch.uint8, device=DEV)
    netcsum.tx_finalize_ipv6(b, len(lens), fl, off=o, lens=ln)
    torch.cuda.synchronize()
    assert np.array_equal(b.cpu().numpy(), buf)
    assert (fl.cpu().numpy() == (op.IP_OK | op.L4_CHECKED | op.L4_OK)).all()
    # Tx without flags: the walk pass keeps its flags in scratch, the bytes are the same
    b, o, ln = _dev(stale, offs, lens)
    netcsum.tx_finalize_ipv6(b, len(lens), None, off=o, lens=ln)
    torch.cuda.synchronize()
    assert np.array_equal(b.cpu().numpy(), buf)


@pytest.mark.parametrize("group", [0, 16, 64])
@pytest.mark.parametrize("udp_tx_csum", [True, False])
def test_mixed_ip_batch_rx_and_tx(group, udp_tx_csum):
    """NetUtil_MI355X_RxValidateIP / TxFinalizeIP: one launch over a ring carrying IPv4 and IPv6
    datagrams (every kind of both, incl. IPv4 packets with version 6 / IPv6 with version 4), each
    dispatched on its version nibble, equal to the per-version oracles."""
    from packets import KINDS, make_packet
    rng = random.Random(800 + group + udp_tx_csum)
    pkts = [make_packet_v6(rng, rng.choice(KINDS6)) if rng.random() < 0.5 else make_packet(rng, rng.choice(KINDS))
            for _ in range(2000)]
    buf, offs, lens = packed_batch(pkts, rng)
    netcsum.tune(netcsum.TUNE_GROUP_LANES, group)
    g = group or _auto_group(True)
    b, o, ln = _dev(buf, offs, lens)
    f = torch.zeros(len(pkts), dtype=torch.uint8, device=DEV)
    netcsum.rx_validate_ip(b, len(pkts), f, off=o, lens=ln)
    torch.cuda.synchronize()
    want = np.array([op.rx_validate_ip(bytes(buf[p:p + n]))
                     for p, n in zip(offs.tolist(), lens.tolist())], np.uint8)
    got = f.cpu().numpy()
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, [(pkts[i][:24].hex(), int(got[i]), int(want[i])) for i in bad[:5]]
    netcsum.tx_finalize_ip(b, len(pkts), f, off=o, lens=ln, udp_tx_csum=udp_tx_csum)
    torch.cuda.synchronize()
    out, flags = b.cpu().numpy(), f.cpu().numpy()
    for i, (p, n) in enumerate(zip(offs.tolist(), lens.tolist())):
        want_pkt, want_f = op.tx_finalize_ip(bytes(buf[p:p + n]), udp_tx_csum)
        assert bytes(out[p:p + n]) == want_pkt, (i, pkts[i][:24].hex())
        assert flags[i] == want_f, (i, int(flags[i]), want_f)


def test_mixed_ip_strided_c2_shape():
    """1500-B TCP datagrams, alternating IPv4 / IPv6, strided: Tx then Rx accepts every one."""
    rng = random.Random(811)
    from packets import make_packet
    n, L = 2000, 1500
    buf = np.zeros(n * L + 64, np.uint8)
    for i in range(n):
        p = make_packet_v6(rng, "tcp", payload=1390) if i % 2 else make_packet(rng, "tcp", payload=1380)
        p = bytearray(p)
        p[-2:] = b"\x00\x00"                                     # force a Tx rewrite of stale fields
        buf[i * L:i * L + len(p)] = np.frombuffer(bytes(p), np.uint8)
    b = torch.from_numpy(buf).to(DEV)
    f = torch.zeros(n, dtype=torch.uint8, device=DEV)
    netcsum.tx_finalize_ip(b, n, f, stride=L, pkt_len=L)
    netcsum.rx_validate_ip(b, n, f, stride=L, pkt_len=L)
    torch.cuda.synchronize()
    out = b.cpu().numpy()
    want = np.array([op.rx_validate_ip(bytes(out[i * L:(i + 1) * L])) for i in range(n)], np.uint8)
    assert np.array_equal(f.cpu().numpy(), want)
    assert (want == (op.IP_OK | op.L4_CHECKED | op.L4_OK)).sum() > n * 0.9


@pytest.mark.parametrize("group", [0, 64])
def test_v6_extreme_sizes(group):
    """IPv6 datagrams at the size limits: header only (40 B), empty UDP (48 B), minimal TCP (60 B),
    and payloads up to 65495 B (65535 B present, the 16-bit length limit), packed at odd offsets;
    Rx verdicts and Tx write-back equal the oracle."""
    rng = random.Random(900 + group)
    pkts = [make_packet_v6(rng, "other", payload=0), make_packet_v6(rng, "udp", payload=0),
            make_packet_v6(rng, "tcp", payload=0)]
    for size in (65495 - 60, 65495 - 8, 40000, 65495 - 4):
        kind = {65495 - 60: "tcp", 65495 - 8: "udp", 40000: "icmp_echo", 65495 - 4: "icmp_nd"}[size]
        p = make_packet_v6(rng, kind, payload=size)
        assert len(p) <= 65535
        pkts.append(p)
    buf, offs, lens = packed_batch(pkts, rng, trailer=False)
    netcsum.tune(netcsum.TUNE_GROUP_LANES, group)
    g = group or _auto_group(True)
    got = _rx_gpu(buf, offs, lens)
    want = np.array([op.rx_validate_v6(bytes(buf[o:o + n]))
                     for o, n in zip(offs.tolist(), lens.tolist())], np.uint8)
    assert np.array_equal(got, want), (got, want)
    assert ((want[1:] & op.L4_OK) != 0).all()
    stale = buf.copy()
    for o in offs.tolist()[1:]:
        stale[o + 42:o + 44] ^= 0x5A                              # ICMPv6 / UDP length byte / TCP seq
    b, o_, ln = _dev(stale, offs, lens)
    f = torch.zeros(len(pkts), dtype=torch.uint8, device=DEV)
    netcsum.tx_finalize_ipv6(b, len(pkts), f, off=o_, lens=ln)
    torch.cuda.synchronize()
    out = b.cpu().numpy()
    for i, (o, n) in enumerate(zip(offs.tolist(), lens.tolist())):
        want_pkt, want_f = op.tx_finalize_v6(bytes(stale[o:o + n]), True)
        assert bytes(out[o:o + n]) == want_pkt, i
        assert f.cpu().numpy()[i] == want_f, i


_TAILS = ["tcp", "udp", "udp0", "udp_badlen", "tcp_short", "icmp_echo", "icmp_err", "icmp_nd", "icmp_other",
          "corrupt_l4", "frag", "esp", "hbh_late", "overrun", "trunc"]


def _long_prefix_pkt(rng, tail, big):
    """An IPv6 datagram whose chain starts with a Destination Options header of `big` 8-B units (past
    every batch kernel's window) and ends in `tail`: every transport outcome, Fragment, an opaque
    header, a late Hop-by-Hop, a header running past the payload, a chain cut at the payload end."""
    from packets import _ext_chain
    if tail in ("frag", "esp", "hbh_late", "overrun", "trunc"):
        inner = make_packet_v6(rng, "tcp", payload=rng.randint(0, 200))
        chain = {"frag": [(60, big), (44, 1)], "esp": [(60, big)], "hbh_late": [(60, big), (0, 1)],
                 "overrun": [(60, big), (43, 1)], "trunc": [(60, big)]}[tail]
        final = {"esp": 50, "trunc": 43}.get(tail, 6)
        nh, ext = _ext_chain(rng, chain, final)
        body = ext + (b"" if tail == "trunc" else inner[40:])
    else:
        inner = make_packet_v6(rng, "tcp" if tail == "corrupt_l4" else tail, payload=rng.randint(0, 300))
        nh, ext = _ext_chain(rng, [(60, big)] + [(43, 1)] * rng.randint(0, 5), inner[6])
        body = ext + inner[40:]
    p = bytearray(inner[:4] + struct.pack("!HB", len(body), nh) + inner[7:40] + body)
    if tail == "overrun":
        p[40 + 8 * big + 1] = 255
    if tail not in ("overrun", "trunc", "frag", "esp", "hbh_late"):
        p = bytearray(op.tx_finalize_v6(bytes(p), udp_tx_csum=(tail != "udp0"))[0])
    if tail == "corrupt_l4":
        k = rng.randint(40 + 8 * big, len(p) - 1)
        p[k] ^= 1 << rng.randint(0, 7)
    return bytes(p)


@pytest.mark.parametrize("form", ["varlen8", "varlen64", "strided"])
def test_v6_long_chain_outcomes_vs_oracle(form):
    """Every outcome behind a chain the batch kernels cannot hold (the walk pass decides them all):
    Rx verdicts and Tx bytes + flags (stale fields, UDP checksums on) equal the oracle's, in the
    lane-group kernel (G = 8 / 64, packed odd offsets) and the run-stream kernel (strided)."""
    rng = random.Random({"varlen8": 1, "varlen64": 2, "strided": 3}[form] + 4400)
    pkts = [_long_prefix_pkt(rng, t, rng.choice([17, 40, 129, 140])) for t in _TAILS for _ in range(4)]
    rng.shuffle(pkts)
    want_rx = np.array([op.rx_validate_v6(p) for p in pkts], np.uint8)
    want_tx = [op.tx_finalize_v6(p, True) for p in pkts]
    assert (want_rx & op.MALFORMED).any() and (want_rx & op.FRAGMENT).any() and (want_rx & op.EXT_HDR).any()
    assert (want_rx & op.L4_MALFORMED).any() and (want_rx & op.UDP_NO_CSUM).any()
    assert ((want_rx & (op.L4_CHECKED | op.L4_OK)) == op.L4_CHECKED).any() and (want_rx & op.L4_OK).any()
    n = len(pkts)
    if form == "strided":
        L = 2048
        buf = np.frombuffer(rng.randbytes(n * L + 64), np.uint8).copy()
        for i, p in enumerate(pkts):
            buf[i * L:i * L + len(p)] = np.frombuffer(p, np.uint8)
        want_buf = buf.copy()
        for i, (q, _f) in enumerate(want_tx):
            want_buf[i * L:i * L + len(q)] = np.frombuffer(q, np.uint8)
        b = torch.from_numpy(buf).to(DEV)
        f = torch.zeros(n, dtype=torch.uint8, device=DEV)
        netcsum.rx_validate_ipv6(b, n, f, stride=L, pkt_len=L)
        torch.cuda.synchronize()
        assert netcsum.last_launch().startswith("pkt_stream_kernel")
        rx = f.cpu().numpy()
        ft = torch.zeros(n, dtype=torch.uint8, device=DEV)
        netcsum.tx_finalize_ipv6(b, n, ft, stride=L, pkt_len=L)
    else:
        netcsum.tune(netcsum.TUNE_GROUP_LANES, 8 if form == "varlen8" else 64)
        buf, offs, lens = packed_batch(pkts, rng)
        want_buf = buf.copy()
        for o, (q, _f) in zip(offs.tolist(), want_tx):
            want_buf[o:o + len(q)] = np.frombuffer(q, np.uint8)
        b, o, ln = _dev(buf, offs, lens)
        f = torch.zeros(n, dtype=torch.uint8, device=DEV)
        netcsum.rx_validate_ipv6(b, n, f, off=o, lens=ln)
        torch.cuda.synchronize()
        rx = f.cpu().numpy()
        ft = torch.zeros(n, dtype=torch.uint8, device=DEV)
        netcsum.tx_finalize_ipv6(b, n, ft, off=o, lens=ln)
    torch.cuda.synchronize()
    bad = np.nonzero(rx != want_rx)[0]
    assert bad.size == 0, [(int(i), int(rx[i]), int(want_rx[i])) for i in bad[:6]]
    assert np.array_equal(ft.cpu().numpy(), np.array([fl for _q, fl in want_tx], np.uint8))
    assert np.array_equal(b.cpu().numpy(), want_buf)
