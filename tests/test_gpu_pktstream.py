"""GPU parity of the run-stream packet kernel (netcsum_pktstream.hip: strided IPv4, IPv6 and mixed batches, fused Rx
validation and Tx finalize) against the packet oracle (oracle/oracle_packets.py, which composes the
C restatement's HdrVerify / DataVerify / HdrCalc / DataCalc the way net_ipv4.c, net_tcp.c,
net_udp.c, net_icmpv4.c and net_igmp.c call them), and against the lane-group kernel it replaces
for these batches (TUNE_KERNEL 2): every packet kind incl. malformed ones, IP options, stale
checksum fields, odd and even base addresses, dense and gapped strides, run lengths 1..64, plain
and non-temporal loads, UDP Tx checksums on and off. Every byte outside the written fields must be
left as it was (gaps between packets, the bytes past the last one)."""
import random
import struct

import numpy as np
import pytest

import netcsum
import oracle_packets as op
from packets import KINDS, ext_body, make_packet

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(autouse=True)
def _defaults():
    def reset():
        netcsum.tune(netcsum.TUNE_KERNEL, 0)
        netcsum.tune(netcsum.TUNE_TILE, -1)
        netcsum.tune(netcsum.TUNE_NT_LOADS, -1)
        netcsum.tune(netcsum.TUNE_CHUNKS, 0)
        netcsum.tune(netcsum.TUNE_TX_PASSES, 0)
        netcsum.tune(netcsum.TUNE_STREAM_TOUCH, -1)
        netcsum.tune(netcsum.TUNE_STREAM_WAVES, -1)
        netcsum.tune(netcsum.TUNE_PKT_BOUND, -1)
        netcsum.tune(netcsum.TUNE_TX_FLUSH, -1)
    reset()
    yield
    reset()


def _batch(rng, n, stride, pkt_len, lead):
    buf = np.frombuffer(rng.randbytes(lead + n * stride + 96), np.uint8).copy()
    for i in range(n):
        kind = rng.choice(KINDS + ["udp", "tcp", "icmp", "igmp"])
        p = bytearray(make_packet(rng, kind, payload=rng.randint(0, max(0, pkt_len - 80))))
        if rng.random() < 0.1:                                    # longer than the slot: truncated
            p = bytearray(make_packet(rng, kind, payload=pkt_len))
        p = p[:pkt_len]
        if len(p) >= 12 and rng.random() < 0.5:
            p[10:12] = rng.randbytes(2)                           # stale IP checksum field
        o = lead + i * stride
        buf[o:o + len(p)] = np.frombuffer(bytes(p), np.uint8)
    return buf


def _want(buf, n, stride, pkt_len, lead, udp_tx_csum):
    rx = np.zeros(n, np.uint8)
    tx_buf = buf.copy()
    tx_f = np.zeros(n, np.uint8)
    for i in range(n):
        o = lead + i * stride
        pkt = bytes(buf[o:o + pkt_len])
        rx[i] = op.rx_validate(pkt)
        q, tx_f[i] = op.tx_finalize(pkt, udp_tx_csum)
        tx_buf[o:o + pkt_len] = np.frombuffer(q, np.uint8)
    return rx, tx_buf, tx_f


def _run(buf, n, stride, pkt_len, lead, udp_tx_csum):
    b = torch.from_numpy(buf).to(DEV)
    f = torch.zeros(n, dtype=torch.uint8, device=DEV)
    netcsum.rx_validate_ipv4(b[lead:], n, f, stride=stride, pkt_len=pkt_len)
    torch.cuda.synchronize()
    rx_desc = netcsum.last_launch()
    rx = f.cpu().numpy()
    ft = torch.zeros(n, dtype=torch.uint8, device=DEV)
    netcsum.tx_finalize_ipv4(b[lead:], n, ft, stride=stride, pkt_len=pkt_len, udp_tx_csum=udp_tx_csum)
    torch.cuda.synchronize()
    return rx, b.cpu().numpy(), ft.cpu().numpy(), rx_desc, netcsum.last_launch()


@pytest.mark.parametrize("passes", [1, 2])
@pytest.mark.parametrize("flush", [0, 1, 2, 3, 4])
def test_tx_write_back_options_do_not_change_results(passes, flush):
    """NETCSUM_TUNE_TX_FLUSH (measured, profiles/r2z_tx_flush_sweep.jsonl): write-through scatter
    stores, a release per scatter wave, or a write-back launch after Tx: the same bytes."""
    netcsum.tune(netcsum.TUNE_TX_PASSES, passes)
    netcsum.tune(netcsum.TUNE_TX_FLUSH, flush)
    rng = random.Random(97 + flush + 5 * passes)
    stride, pkt_len, lead, n = 1501, 1500, 1, 900
    buf = _batch(rng, n, stride, pkt_len, lead)
    rx_w, tx_w, txf_w = _want(buf, n, stride, pkt_len, lead, True)
    rx, tx, txf, _, d_tx = _run(buf, n, stride, pkt_len, lead, True)
    assert d_tx.startswith("pkt_stream_kernel") and (" +pkt_scatter_kernel" in d_tx) == (passes == 2), d_tx
    assert np.array_equal(rx, rx_w) and np.array_equal(tx, tx_w) and np.array_equal(txf, txf_w)


SHAPES = [(1500, 1500), (1514, 1514), (1540, 1514), (1501, 1500), (64, 64), (100, 64), (577, 577), (9000, 9000),
          (4096, 4040)]


@pytest.mark.parametrize("stride,pkt_len", SHAPES)
@pytest.mark.parametrize("lead", [0, 1, 6])
@pytest.mark.parametrize("passes", [1, 2])
def test_pkt_stream_vs_oracle(stride, pkt_len, lead, passes):
    netcsum.tune(netcsum.TUNE_TX_PASSES, passes)
    rng = random.Random(stride * 131 + pkt_len * 7 + lead)
    n = 700 if stride < 5000 else 200
    udp_tx_csum = lead != 6
    buf = _batch(rng, n, stride, pkt_len, lead)
    rx_w, tx_w, txf_w = _want(buf, n, stride, pkt_len, lead, udp_tx_csum)
    rx, tx, txf, d_rx, d_tx = _run(buf, n, stride, pkt_len, lead, udp_tx_csum)
    assert d_rx.startswith("pkt_stream_kernel") and d_tx.startswith("pkt_stream_kernel"), (d_rx, d_tx)
    bad = np.nonzero(rx != rx_w)[0]
    assert bad.size == 0, [(int(i), int(rx[i]), int(rx_w[i])) for i in bad[:6]]
    bad = np.nonzero(tx != tx_w)[0]
    assert bad.size == 0, [(int(j), (int(j) - lead) // stride, (int(j) - lead) % stride, int(tx[j]), int(tx_w[j]))
                           for j in bad[:8]]
    assert np.array_equal(txf, txf_w)


@pytest.mark.parametrize("spw", [1, 5, 16, 33, 64])
@pytest.mark.parametrize("nt,depth,touch,waves", [(0, 4, -1, -1), (1, 8, -1, -1), (1, 4, 1, 3), (0, 8, 1, 8)])
def test_pkt_stream_run_lengths_and_loads_equal_lane_group_kernel(spw, nt, depth, touch, waves):
    rng = random.Random(spw * 3 + nt + 10 * touch)
    stride, pkt_len, lead, n = 1518, 1514, 3, 1000
    buf = _batch(rng, n, stride, pkt_len, lead)
    netcsum.tune(netcsum.TUNE_KERNEL, 2)                         # the lane-group kernel: reference run
    rx_ref, tx_ref, txf_ref, d_rx, _ = _run(buf, n, stride, pkt_len, lead, True)
    assert d_rx.startswith("pkt_batch_kernel"), d_rx
    netcsum.tune(netcsum.TUNE_KERNEL, 0)
    netcsum.tune(netcsum.TUNE_TILE, spw)
    netcsum.tune(netcsum.TUNE_NT_LOADS, nt)
    netcsum.tune(netcsum.TUNE_CHUNKS, depth)
    netcsum.tune(netcsum.TUNE_STREAM_TOUCH, touch)               # row touch / residency cap: launch options
    netcsum.tune(netcsum.TUNE_STREAM_WAVES, waves)
    rx, tx, txf, d_rx, d_tx = _run(buf, n, stride, pkt_len, lead, True)
    assert f"pkts_per_wave={spw}" in d_rx and f"D={depth}" in d_tx, (d_rx, d_tx)
    assert np.array_equal(rx, rx_ref)
    assert np.array_equal(tx, tx_ref)
    assert np.array_equal(txf, txf_ref)
    rx_w, tx_w, _ = _want(buf, n, stride, pkt_len, lead, True)
    assert np.array_equal(rx, rx_w) and np.array_equal(tx, tx_w)


def test_pkt_stream_c2_shape_round_trip_1M():
    """1 M x 1500-B TCP datagrams (the Tx / Rx config of DESIGN §9): Tx finalize, then Rx accepts
    every packet; one flipped byte per 1000 packets is caught exactly; 4096 sampled packets equal
    the oracle's Tx bytes."""
    n, L = 1 << 20, 1500
    pk = torch.empty(n * L + 256, dtype=torch.uint8, device=DEV)
    netcsum.fill(pk, n * L, 0x5EED0001, 0)
    v = pk[: n * L].view(n, L)
    v[:, 0:12] = torch.tensor([0x45, 0, L >> 8, L & 0xFF, 0, 0, 0x40, 0, 64, 6, 0, 0], dtype=torch.uint8,
                              device=DEV)
    smp = np.sort(np.random.default_rng(5).choice(n, size=4096, replace=False))
    sidx = torch.from_numpy(smp).to(DEV)
    before = v[sidx].cpu().numpy()
    f = torch.zeros(n, dtype=torch.uint8, device=DEV)
    netcsum.tx_finalize_ipv4(pk, n, f, stride=L, pkt_len=L)
    torch.cuda.synchronize()
    assert netcsum.last_launch().startswith("pkt_stream_kernel")
    after = v[sidx].cpu().numpy()
    for j in range(len(smp)):
        assert bytes(after[j]) == op.tx_finalize(bytes(before[j]), True)[0], int(smp[j])
    netcsum.rx_validate_ipv4(pk, n, f, stride=L, pkt_len=L)
    torch.cuda.synchronize()
    ok = op.IP_OK | op.L4_OK | op.L4_CHECKED
    assert bool(((f & ok) == ok).all())
    bad = torch.arange(0, n, 1000, device=DEV)
    v[bad, 777] ^= 0x04
    netcsum.rx_validate_ipv4(pk, n, f, stride=L, pkt_len=L)
    torch.cuda.synchronize()
    failed = torch.nonzero((f & op.L4_OK) == 0).flatten()
    assert torch.equal(failed, bad)


# ---- IPv6 and mixed IPv4 / IPv6 batches in the run-stream form (VER 6 / VER 0) -----------------

def _batch_ip(rng, n, stride, pkt_len, lead, v6_share):
    from packets import KINDS6, make_packet_v6
    buf = np.frombuffer(rng.randbytes(lead + n * stride + 96), np.uint8).copy()
    for i in range(n):
        if rng.random() < v6_share:
            p = bytearray(make_packet_v6(rng, rng.choice(KINDS6), payload=rng.randint(0, max(0, pkt_len - 100))))
        else:
            p = bytearray(make_packet(rng, rng.choice(KINDS + ["udp", "tcp"]), payload=rng.randint(0, max(0, pkt_len - 80))))
        if rng.random() < 0.1:                                    # longer than the slot: truncated
            p = bytearray(make_packet_v6(rng, "tcp", payload=pkt_len))
        p = p[:pkt_len]
        o = lead + i * stride
        buf[o:o + len(p)] = np.frombuffer(bytes(p), np.uint8)
    return buf


def _want_ip(buf, n, stride, pkt_len, lead, udp_tx_csum, ver):
    rx = np.zeros(n, np.uint8)
    tx_buf = buf.copy()
    tx_f = np.zeros(n, np.uint8)
    for i in range(n):
        o = lead + i * stride
        pkt = bytes(buf[o:o + pkt_len])
        if ver == 6:
            rx[i] = op.rx_validate_v6(pkt)
            q, tx_f[i] = op.tx_finalize_v6(pkt, udp_tx_csum)
        else:
            rx[i] = op.rx_validate_ip(pkt)
            q, tx_f[i] = op.tx_finalize_ip(pkt, udp_tx_csum)
        tx_buf[o:o + pkt_len] = np.frombuffer(q, np.uint8)
    return rx, tx_buf, tx_f


def _run_ip(buf, n, stride, pkt_len, lead, udp_tx_csum, ver):
    rxf, txf = ((netcsum.rx_validate_ipv6, netcsum.tx_finalize_ipv6) if ver == 6
                else (netcsum.rx_validate_ip, netcsum.tx_finalize_ip))
    b = torch.from_numpy(buf).to(DEV)
    f = torch.zeros(n, dtype=torch.uint8, device=DEV)
    rxf(b[lead:], n, f, stride=stride, pkt_len=pkt_len)
    torch.cuda.synchronize()
    rx_desc = netcsum.last_launch()
    rx = f.cpu().numpy()
    ft = torch.zeros(n, dtype=torch.uint8, device=DEV)
    txf(b[lead:], n, ft, stride=stride, pkt_len=pkt_len, udp_tx_csum=udp_tx_csum)
    torch.cuda.synchronize()
    return rx, b.cpu().numpy(), ft.cpu().numpy(), rx_desc, netcsum.last_launch()


@pytest.mark.parametrize("ver", [6, 0])
@pytest.mark.parametrize("stride,pkt_len", [(1500, 1500), (1540, 1514), (1501, 1500), (64, 64), (100, 64),
                                            (577, 577), (9000, 9000)])
@pytest.mark.parametrize("lead", [0, 1, 6, 13])
@pytest.mark.parametrize("passes", [1, 2])
def test_pkt_stream_v6_and_mixed_vs_oracle(ver, stride, pkt_len, lead, passes):
    """Every IPv6 kind (TCP / UDP / UDP without checksum, ICMPv6 echo / error / NDP / other types,
    extension-header chains inside and beyond the lane's window, Hop-by-Hop after the first, Fragment,
    opaque extension headers, malformed versions / lengths, corrupted bytes), alone (VER 6) or mixed
    with every IPv4 kind (VER 0), Rx verdicts and Tx bytes + verdicts against the oracle (chains past
    the lane's 96-B prologue finished inside the run-stream launches)."""
    netcsum.tune(netcsum.TUNE_TX_PASSES, passes)
    rng = random.Random(ver * 1000 + stride * 7 + pkt_len + lead * 131 + passes)
    n = 600 if stride < 5000 else 150
    udp_tx_csum = lead != 6
    buf = _batch_ip(rng, n, stride, pkt_len, lead, 1.0 if ver == 6 else 0.5)
    rx_w, tx_w, txf_w = _want_ip(buf, n, stride, pkt_len, lead, udp_tx_csum, ver)
    rx, tx, txf, d_rx, d_tx = _run_ip(buf, n, stride, pkt_len, lead, udp_tx_csum, ver)
    tag = "v6" if ver == 6 else "mixed"
    assert d_rx.startswith("pkt_stream_kernel") and f",rx,{tag}>" in d_rx and f",tx,{tag}>" in d_tx, (d_rx, d_tx)
    assert d_rx.endswith(" +inline_v6_walk"), d_rx
    assert d_tx.endswith(" +inline_v6_walk") and (" +pkt_scatter_kernel" in d_tx) == (passes == 2), d_tx
    bad = np.nonzero(rx != rx_w)[0]
    assert bad.size == 0, [(int(i), int(rx[i]), int(rx_w[i])) for i in bad[:6]]
    bad = np.nonzero(tx != tx_w)[0]
    assert bad.size == 0, [(int(j), (int(j) - lead) // stride, (int(j) - lead) % stride, int(tx[j]), int(tx_w[j]))
                           for j in bad[:8]]
    assert np.array_equal(txf, txf_w)
    if pkt_len >= 577:
        assert (rx_w & op.EXT_HDR).any() and ((rx_w & op.L4_OK) != 0).any()


@pytest.mark.parametrize("lead", list(range(16)))
@pytest.mark.parametrize("tile", [0, 8, 64])
def test_pkt_stream_v6_extension_chains_of_any_length(lead, tile):
    """Destination Options / Routing chains before TCP / UDP / ICMPv6 at every lead: one header of
    1..40 units (8..320 B, inside and past the lane's 96 - lead bytes) or 4..9 headers — every chain
    walked to its transport header (the batch kernel's window, then the walk: inside the Rx kernel by
    the wave's 16-lane groups, in the walk pass after Tx), Rx verdicts and Tx bytes + flags equal the
    oracle's, no EXT_HDR left. tile: datagrams per wave (0: the default; 8 / 64: many deferred
    datagrams per wave, up to four walked at once)."""
    netcsum.tune(netcsum.TUNE_TILE, tile if tile else -1)
    from packets import make_packet_v6
    rng = random.Random(900 + lead)
    stride = pkt_len = 1024
    pkts = []
    for units in list(range(1, 13)) + [20, 40]:
        for n_hdr in (1, 4, 9):
            inner = make_packet_v6(rng, rng.choice(["tcp", "udp", "icmp_echo"]), payload=rng.randint(24, 300))
            nh, ext = inner[6], b""
            for _k in range(n_hdr):
                u = units if n_hdr == 1 else rng.randint(1, 3)
                t = rng.choice([43, 60])
                ext = struct.pack("!BB", nh, u - 1) + ext_body(rng, t, u * 8 - 2) + ext
                nh = t
            body = ext + inner[40:]
            hdr = inner[:4] + struct.pack("!HB", len(body), nh) + inner[7:40]
            pkts.append(op.tx_finalize_v6(hdr + body)[0][:pkt_len])
    rng.shuffle(pkts)
    n = len(pkts)
    buf = np.frombuffer(rng.randbytes(lead + n * stride + 96), np.uint8).copy()
    for i, p in enumerate(pkts):
        buf[lead + i * stride:lead + i * stride + len(p)] = np.frombuffer(p, np.uint8)
    rx_w, tx_w, txf_w = _want_ip(buf, n, stride, pkt_len, lead, True, 6)
    rx, tx, txf, d_rx, _ = _run_ip(buf, n, stride, pkt_len, lead, True, 6)
    assert d_rx.startswith("pkt_stream_kernel"), d_rx
    assert np.array_equal(rx, rx_w) and np.array_equal(tx, tx_w) and np.array_equal(txf, txf_w)
    assert not (rx_w & op.EXT_HDR).any() and ((rx_w & op.L4_OK) != 0).all()


def test_pkt_stream_v6_c2_shape_round_trip_1M():
    """1 M x 1500-B TCP/IPv6 datagrams: Tx finalize, Rx accepts every one, one flipped byte per 1000
    (addresses included) is caught exactly, 4096 sampled datagrams equal the oracle's Tx bytes."""
    n, L = 1 << 20, 1500
    pk = torch.empty(n * L + 256, dtype=torch.uint8, device=DEV)
    netcsum.fill(pk, n * L, 0x5EED0006, 0)
    v = pk[: n * L].view(n, L)
    v[:, 0:8] = torch.tensor([0x60, 0, 0, 0, (L - 40) >> 8, (L - 40) & 0xFF, 6, 64], dtype=torch.uint8, device=DEV)
    v[:, 52] = 0x50                                                 # TCP data offset 5
    smp = np.sort(np.random.default_rng(6).choice(n, size=4096, replace=False))
    sidx = torch.from_numpy(smp).to(DEV)
    before = v[sidx].cpu().numpy()
    f = torch.zeros(n, dtype=torch.uint8, device=DEV)
    netcsum.tx_finalize_ipv6(pk, n, f, stride=L, pkt_len=L)
    torch.cuda.synchronize()
    assert netcsum.last_launch().startswith("pkt_stream_kernel"), netcsum.last_launch()
    after = v[sidx].cpu().numpy()
    for j in range(len(smp)):
        assert bytes(after[j]) == op.tx_finalize_v6(bytes(before[j]), True)[0], int(smp[j])
    netcsum.rx_validate_ipv6(pk, n, f, stride=L, pkt_len=L)
    torch.cuda.synchronize()
    ok = op.IP_OK | op.L4_OK | op.L4_CHECKED
    assert bool(((f & ok) == ok).all())
    bad = torch.arange(0, n, 1000, device=DEV)
    v[bad, 21] ^= 0x10                                              # a source-address byte
    netcsum.rx_validate_ipv6(pk, n, f, stride=L, pkt_len=L)
    torch.cuda.synchronize()
    failed = torch.nonzero((f & op.L4_OK) == 0).flatten()
    assert torch.equal(failed, bad)


@pytest.mark.parametrize("stride,pkt_len,run", [(1500, 1500, 8), (1000, 1000, 16), (577, 577, 32), (256, 200, 64),
                                                (128, 128, 64), (9000, 9000, 1), (2048, 2048, 5), (4096, 4096, 2),
                                                (8192, 8192, 1), (3000, 3000, 8), (1520, 1506, 16), (2048, 1984, 8)])
@pytest.mark.parametrize("copies", [1, 1000])
def test_pkt_stream_default_run_length_by_bytes(stride, pkt_len, run, copies):
    """Default run: about 20 KB of datagrams per wave for packed batches (the whole-span form 0, r2zq sweep) and
    24 KB of slots for the live-piece form 2 of other layouts (r4m ring probe), in multiples of 8, 8..64 — except
    packed runs whose bytes would be a multiple of 16 KiB or past 48 KiB, which take about 10 KiB (round 6,
    profiles/r6zu_pktlen.jsonl: 2 / 4 / 8 KiB and 9000-B datagrams in runs of 5 / 2 / 1 / 1) —, halved while
    the batch has fewer than 2048 runs (small bursts are latency-bound); results equal the lane-group kernel's.
    copies: the 300-datagram batch repeated (300 000 datagrams keep the full run). Layouts that are not
    packed run with TUNE_PKT_BOUND 2 here: by default their batches of >= 16 Ki datagrams take ring plans
    (the run the previous batch on the ring sampled; tests/test_gpu_ring_layouts.py)."""
    if stride != pkt_len:
        netcsum.tune(netcsum.TUNE_PKT_BOUND, 2)
    rng = random.Random(stride)
    n0 = 300
    buf0 = _batch(rng, n0, stride, pkt_len, 2)
    body = buf0[2:2 + n0 * stride]
    buf = np.concatenate([buf0[:2], np.tile(body, copies), buf0[2 + n0 * stride:]])
    n = n0 * copies
    spw = run
    while spw > 1 and n < 2048 * spw:
        spw //= 2
    netcsum.tune(netcsum.TUNE_KERNEL, 2)
    rx_ref, tx_ref, txf_ref, _, _ = _run(buf, n, stride, pkt_len, 2, True)
    netcsum.tune(netcsum.TUNE_KERNEL, 0)
    rx, tx, txf, d_rx, d_tx = _run(buf, n, stride, pkt_len, 2, True)
    assert f"pkts_per_wave={spw}" in d_rx and f"pkts_per_wave={spw}" in d_tx, (d_rx, d_tx)
    assert np.array_equal(rx, rx_ref) and np.array_equal(tx, tx_ref) and np.array_equal(txf, txf_ref)


def test_graph_capture_then_larger_uncaptured_batch_on_the_same_stream():
    """Scratch leases under stream capture (INTEGRATION §4 graph-capture note): a two-pass Tx batch is
    captured into a HIP graph after one uncaptured warm-up call (its record slot is then pinned to the
    graph); a LARGER uncaptured two-pass Tx batch on the same stream (1.1 MB of records: more than the
    1-MiB slot) takes a slot of its own instead of failing or growing the graph's; the graph, replayed
    afterwards, still finalizes its own batch. Every byte and flag equals the oracle's."""
    netcsum.tune(netcsum.TUNE_TX_PASSES, 2)
    rng = random.Random(5151)
    n1, n2, L = 600, 140000, 64
    buf1 = _batch(rng, n1, L, L, 0)
    buf2 = _batch(rng, n2, L, L, 0)
    _, tx1_w, txf1_w = _want(buf1, n1, L, L, 0, True)
    _, tx2_w, txf2_w = _want(buf2, n2, L, L, 0, True)
    s = torch.cuda.Stream(device=DEV)
    b1 = torch.from_numpy(buf1).to(DEV)
    f1 = torch.zeros(n1, dtype=torch.uint8, device=DEV)
    with torch.cuda.stream(s):
        netcsum.tx_finalize_ipv4(b1, n1, f1, stride=L, pkt_len=L, stream=s)      # uncaptured warm-up
    s.synchronize()
    b1.copy_(torch.from_numpy(buf1).to(DEV))
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        netcsum.tx_finalize_ipv4(b1, n1, f1, stride=L, pkt_len=L, stream=s)
    b2 = torch.from_numpy(buf2).to(DEV)
    f2 = torch.zeros(n2, dtype=torch.uint8, device=DEV)
    with torch.cuda.stream(s):
        netcsum.tx_finalize_ipv4(b2, n2, f2, stride=L, pkt_len=L, stream=s)
    s.synchronize()
    assert np.array_equal(b2.cpu().numpy(), tx2_w) and np.array_equal(f2.cpu().numpy(), txf2_w)
    b1.copy_(torch.from_numpy(buf1).to(DEV))
    f1.zero_()
    torch.cuda.synchronize()
    g.replay()
    torch.cuda.synchronize()
    assert np.array_equal(b1.cpu().numpy(), tx1_w) and np.array_equal(f1.cpu().numpy(), txf1_w)


@pytest.mark.parametrize("ver", [4, 6, 0])
@pytest.mark.parametrize("bound", [-1, 0, 1, 3])
@pytest.mark.parametrize("passes", [1, 2])
def test_pkt_stream_datagrams_ending_at_the_window_edge(ver, bound, passes):
    """The live forms sum a datagram whose bytes end inside the lane's 96-B header window from that
    window and leave it out of the stream (no sectors marked, no event walked): short datagrams at
    every window offset (stride 1521 walks the start through all 16 positions of a 16-B chunk),
    ending before, at and past the window's end, among longer ones, odd and even starts, against
    the oracle; form 0 (bound 0) keeps them in the stream and must agree."""
    from packets import KINDS6, make_packet_v6
    netcsum.tune(netcsum.TUNE_TX_PASSES, passes)
    netcsum.tune(netcsum.TUNE_PKT_BOUND, bound)
    try:
        rng = random.Random(4099 + 10 * ver + bound + 7 * passes)
        stride, pkt_len, lead, n = 1521, 1506, 5, 1600
        buf = np.frombuffer(rng.randbytes(lead + n * stride + 96), np.uint8).copy()
        for i in range(n):
            v6 = ver == 6 or (ver == 0 and rng.random() < 0.5)
            big = rng.random() < 0.15
            if v6:
                p = make_packet_v6(rng, rng.choice(KINDS6), payload=rng.randint(0, 1200 if big else 48))
            else:
                p = make_packet(rng, rng.choice(KINDS + ["udp", "tcp", "icmp"]), payload=rng.randint(0, 1200 if big else 70))
            p = bytearray(p[:pkt_len])
            if len(p) >= 12 and not v6 and rng.random() < 0.3:
                p[10:12] = rng.randbytes(2)                       # stale IP checksum field
            o = lead + i * stride
            buf[o:o + len(p)] = np.frombuffer(bytes(p), np.uint8)
        udp_tx_csum = True
        if ver == 4:
            rx_w, tx_w, txf_w = _want(buf, n, stride, pkt_len, lead, udp_tx_csum)
            rx, tx, txf, d_rx, d_tx = _run(buf, n, stride, pkt_len, lead, udp_tx_csum)
        else:
            rx_w, tx_w, txf_w = _want_ip(buf, n, stride, pkt_len, lead, udp_tx_csum, ver)
            rx, tx, txf, d_rx, d_tx = _run_ip(buf, n, stride, pkt_len, lead, udp_tx_csum, ver)
        assert d_rx.startswith("pkt_stream_kernel"), d_rx
        bad = np.nonzero(rx != rx_w)[0]
        assert bad.size == 0, [(int(i), int(rx[i]), int(rx_w[i])) for i in bad[:6]]
        bad = np.nonzero(tx != tx_w)[0]
        assert bad.size == 0, [(int(j), (int(j) - lead) // stride, (int(j) - lead) % stride) for j in bad[:8]]
        assert np.array_equal(txf, txf_w)
    finally:
        netcsum.tune(netcsum.TUNE_PKT_BOUND, -1)
